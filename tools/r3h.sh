#!/bin/bash
# round-3 session h: f16x3 forward -- precision / wsplit / parity tests, kernel timings vs x6,
# precision errors, headline with the f16x3 forward
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3h}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 python -u -m pytest tests/test_gpu_wsplit.py tests/test_gpu_precision.py -q -x -m gpu --timeout 120 --timeout-method thread
run kb 300 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,grad,lap --sizes 8354,16708,66844 --variants x6,h3 --policies 0 --reps 20
run prec 300 python tools/prec_errors.py --nets fluid_pres,fluid_vel,advect,el2d --combos 1:1,4:1 --n 4000
echo done >> $O/status.log
