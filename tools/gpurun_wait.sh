#!/bin/bash
# Run ONE gpurun call, re-submitting it only while the pool reports no free box (exit 3: nothing ran,
# nothing charged); any other outcome -- success, failure, refusal, timeout -- ends here.
# usage: tools/gpurun_wait.sh TIMEOUT 'command'
to=$1; shift
for try in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@"; rc=$?
  [ $rc -ne 3 ] && exit $rc
  grep -q '"status": "transient"' /root/repo/gpurun_out/.last_call.json 2>/dev/null || exit $rc
  echo "[gpurun_wait] no free box (try $try); waiting 150 s"; sleep 150
done
exit 3
