#!/bin/bash
# round-3 session d: resident / precision / C-ABI tests, hoist A/B (kbench --lib), small-batch value
# backward tile study, headline + fluid2DtlgnM bench lines.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3d}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_precision.py tests/test_capi.py -q -x -m gpu --timeout 120 --timeout-method thread
for rep in 1 2; do
run kbA$rep 300 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,lap --sizes 16708,66844 --variants x6 --policies 3 --bwd-only --reps 20 --lib insr-pde_amd/lib_exp/r3c_nohoist.so
run kbB$rep 300 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,lap --sizes 16708,66844 --variants x6 --policies 3 --bwd-only --reps 20
done
run kbT 300 python tools/kbench.py --nets fluid_vel --modes value --sizes 4178,8354,16708 --variants x6,x6_1,x6_2,x6_4 --policies 0,2 --reps 20
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run benchM 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline
run benchMmixed 300 python bench.py --config fluid2DtlgnM --precision mixed --steps 20 --warmup 3 --no-cpu-baseline
run stampsV16 120 python tools/diag_stamps.py --net fluid_vel --mode value --n 16708 --prec 1
run stampsV8 120 python tools/diag_stamps.py --net fluid_vel --mode value --n 8354 --prec 1
echo done >> $O/status.log
