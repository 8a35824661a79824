#!/bin/bash
# same-box A/B of two library builds with tools/kbench.py: AB_ARGS (kbench args), libs under insr-pde_amd/lib/ab/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r4ab}; mkdir -p $O
for rep in 1 2; do
  for v in A B; do
    echo "== kbench $v rep $rep" >> $O/status.log
    timeout -k 10 300 python tools/kbench.py --lib insr-pde_amd/lib/ab/libinsr_hip_$v.so ${AB_ARGS} > $O/kbench_${v}_$rep.out 2> $O/kbench_${v}_$rep.err
    rc=$?; echo "   exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
  done
done
echo done >> $O/status.log
