#!/bin/bash
# round-3 session s: dynamic per-tile f16 scales of the forward's tangent / Laplacian planes and the
# wider static Laplacian factor of the backward's h operands (the Hessian stress test's NaN):
# targeted tests, the whole suite, precision record, forward A/B against the previous build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3s}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run t_quick 300 python -u -m pytest tests/test_gpu_hessian.py tests/test_gpu_precision.py tests/test_gpu_dw_f16.py tests/test_gpu_wsplit.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run prec 300 python tools/prec_errors.py --n 20000 --combos 4:1
for rep in 1 2; do
  run kb_new_$rep 200 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,grad,lap --sizes 16708,66844 --variants x6 --reps 20
  run kb_old_$rep 200 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,grad,lap --sizes 16708,66844 --variants x6 --reps 20 --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run bench40 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
