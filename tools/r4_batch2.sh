#!/bin/bash
# round-4 batch 2: full GPU suite, the headline + elasticity3Dbunny lines and profile, the Adam-gap
# variants (tools/diag_adam_gap2.py under --kernel-trace), PMC traffic passes, then (last: an
# experimental build) the same-box A/B of lib/ab A vs B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=${SESSION:-r4s}; O=gpurun_out/$S; mkdir -p $O
export TMPDIR=/tmp
SESSION=$S STEPS="${FIRST_STEPS:-tests bench prof}" CONFIGS="${CONFIGS:-elasticity3Dbunny}" bash tools/r4_session.sh || exit $?
for v in ${GAP_VARIANTS:-plateau noplateau noplanes add}; do
  echo "== gap $v" >> $O/status.log
  timeout -k 10 120 rocprofv3 --kernel-trace -d "$PWD/$O/gap_$v" -o run --output-format csv -- python tools/diag_adam_gap2.py --variant $v > $O/gap_$v.out 2>&1
  rc=$?; echo "   exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
done
if [ -n "${PMC:-}" ]; then
  SESSION=$S STEPS=pmc bash tools/gpu_session.sh || exit $?
fi
[ -n "${AB_ARGS:-}" ] || exit 0
SESSION=$S bash tools/r4_ab.sh || exit $?
