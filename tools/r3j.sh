#!/bin/bash
# round-3 session j: same-box A/B of the forward precision (x6 vs the f16x3 default), headline and
# fluid2DtlgnM, plus the precision tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3j}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 python -u -m pytest tests/test_gpu_precision.py -q -x -m gpu --timeout 300 --timeout-method thread
for rep in 1 2; do
  for c in fluid2Dtlgn fluid2DtlgnM; do
    INSR_JET_PREC_FWD=1 run ${c}_x6_$rep 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-roofline
    run ${c}_h3_$rep 300 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline --no-roofline
  done
done
echo done >> $O/status.log
