#!/bin/bash
# kernel trace of elasticity2Dstretch and elasticity3Dbunny, fluid2DtlgnM and its 8-way shard at --steps 20
set -u
O=gpurun_out/${SESSION:-r5g10}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_el2d" -o run --output-format csv -- python bench.py --config elasticity2Dstretch --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/el2d.json 2>$O/el2d.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_el3d" -o run --output-format csv -- python bench.py --config elasticity3Dbunny --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/el3d.json 2>$O/el3d.err || exit 1
timeout -k 10 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline > $O/M.json 2>$O/M.err || exit 1
timeout -k 10 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/M8.json 2>$O/M8.err || exit 1
