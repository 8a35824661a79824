#!/bin/bash
# round-3 session i: the whole GPU suite with the f16x3 forward as the process default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3i}; mkdir -p $O
echo "== tests" >> $O/status.log
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.out 2> $O/tests.err; echo "   exit $?" >> $O/status.log
rc=$(tail -1 $O/status.log | grep -c "exit 0\|exit 1")
[ "$rc" = "1" ] || exit 1
echo "== bench" >> $O/status.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.out 2> $O/bench.err; echo "   exit $?" >> $O/status.log
echo done >> $O/status.log
