#!/bin/bash
# round-3 session n: fp16 products of the x6 backward (insr_jet_set_bwd_f16 masks): parity,
# the whole suite at the default (dW on), kernel and same-box bench A/B of the propagation bit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3n}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run t_f16 300 python -u -m pytest tests/test_gpu_dw_f16.py tests/test_gpu_wsplit.py tests/test_gpu_multi_bwd.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run tests 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
for m in 1 3 7; do
  run kb_val_$m 200 python tools/kbench.py --nets fluid_vel --modes value --sizes 8354,16708 --variants x6 --bwd-only --bwd-f16 $m
  run kb_lap_$m 200 python tools/kbench.py --nets fluid_pres --modes lap --sizes 8354,16708 --variants x6 --bwd-only --bwd-f16 $m
  run kb_grad_$m 200 python tools/kbench.py --nets el2d,el3d --modes grad --sizes 20400,32768 --variants x6 --bwd-only --bwd-f16 $m
done
for rep in 1 2; do
  for m in 1 3 7; do
    run bench_m${m}_$rep 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --bwd-f16 $m
    run el3d_m${m}_$rep 300 python bench.py --config elasticity3Dbunny --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --bwd-f16 $m
  done
done
INSR_TEST_BWD_F16=7 run tests7 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
echo done >> $O/status.log
