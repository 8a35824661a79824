#!/bin/bash
# fluid2DtlgnM with --precision mixed (BASELINE configs[4]: "mixed fp32/bf16 MFMA"), its fp32-level line beside it
set -u
O=gpurun_out/${SESSION:-r5g17}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.out 2>&1 || exit 1
timeout -k 10 300 python bench.py --config fluid2DtlgnM --precision mixed --steps 20 --warmup 3 --no-cpu-baseline > $O/M_mixed.json 2>$O/err.txt || exit 1
timeout -k 10 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline > $O/M_fp32.json 2>$O/err.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_mixed" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --precision mixed --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof.out 2>&1 || exit 1
