#!/bin/bash
# rocprofv3 kernel stats of the elasticity configs + extra bench lines (plain API, bf16 precisions);
# stops at the first failing step (SESSION names the gpurun_out/ directory)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-cfg}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "elastic or el3d or phases" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_el2d -o run --output-format csv -- python bench.py --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_el2d.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_el3d -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 5 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_el3d.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config elasticity2Dstretch --steps 20 --warmup 3 --cpu-seconds 10 > $O/bench_el2d.log 2>&1 || exit $?
