#!/bin/bash
# the drop-in (plain body) path: its GPU tests, then the plain bench lines
set -u
O=gpurun_out/${SESSION:-r5g13}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_plain_api.py tests/test_gpu_fullsize_phases.py tests/test_gpu_dp_capture.py tests/test_gpu_multi_bwd.py tests/test_gpu_phases.py tests/test_gpu_losses.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.out 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --api plain --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/plain_adv_$r.json 2>$O/err.txt || exit 1
  timeout -k 10 200 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/plain_$r.json 2>$O/err.txt || exit 1
done
