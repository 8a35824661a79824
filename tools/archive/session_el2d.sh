#!/bin/bash
# elasticity2Dstretch: backward-path A/B (--bwd-policy) and the elasticity GPU tests
set -u
O=gpurun_out/${SESSION:-r5g11}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_elastic.py tests/test_gpu_fullsize_phases.py tests/test_gpu_el3d_full.py -m gpu -x -q --timeout 120 --timeout-method thread -k "elastic or el2d or el3d or elasticity" > $O/tests.out 2>&1 || exit 1
for r in 1 2; do
  for p in 0 1 2 3 4 5; do
    timeout -k 10 200 python bench.py --config elasticity2Dstretch --bwd-policy $p --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/el2d_p${p}_$r.json 2>$O/err.txt || exit 1
  done
done
