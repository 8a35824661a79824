#!/bin/bash
# round-3 session m: the fp16 dW GEMM of the two-kernel backward (insr_jet_set_dw_precision):
# its parity tests, the whole suite at the default, kernel A/B and same-box bench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3m}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run t_dw 300 python -u -m pytest tests/test_gpu_dw_f16.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run tests 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
for dw in 0 1; do
  run kb_lap_$dw 200 python tools/kbench.py --nets fluid_pres --modes lap --sizes 8354,16708,66844 --variants x6 --bwd-only --dw-f16 $dw
  run kb_grad_$dw 200 python tools/kbench.py --nets el2d,el3d --modes grad --sizes 20400,32768 --variants x6 --bwd-only --dw-f16 $dw
done
for rep in 1 2; do
  for dw in 0 1; do
    run bench_dw${dw}_$rep 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --dw-f16 $dw
    run el3d_dw${dw}_$rep 300 python bench.py --config elasticity3Dbunny --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --dw-f16 $dw
  done
done
echo done >> $O/status.log
