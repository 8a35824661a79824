#!/bin/bash
# A/B of the bench's sustained untimed warm-up (--warm-ms): first timed timesteps vs the steady ones
set -u
O=gpurun_out/${SESSION:-r5g9}; mkdir -p $O
for r in 1 2; do
  for c in fluid2Dtlgn advect1D; do
    for w in 0 200 1000; do
      timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --warm-ms $w > $O/${c}_w${w}_$r.json 2>$O/err.txt || exit 1
    done
  done
done
