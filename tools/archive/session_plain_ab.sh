#!/bin/bash
# plain (reference-body) fluid line next to the hand-fused one on the same box
set -u
O=gpurun_out/${SESSION:-r5g16}; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/fused_$r.json 2>$O/err.txt || exit 1
  timeout -k 10 200 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/plain_$r.json 2>$O/err.txt || exit 1
done
