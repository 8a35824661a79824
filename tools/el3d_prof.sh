#!/bin/bash
# elasticity3Dbunny bench + kernel trace (one GPU session)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-el3d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config elasticity3Dbunny --steps 10 --warmup 3 --cpu-seconds 5 > "$OUT/bench.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof.log" 2>&1
