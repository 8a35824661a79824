#!/bin/bash
# A/B of the bench's graph unroll (same box): two lines each of --graph-unroll 1 and 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r4u}; mkdir -p $O
for rep in 1 2; do
  for u in 1 4; do
    echo "== bench unroll $u rep $rep" >> $O/status.log
    timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --graph-unroll $u > $O/bench_u${u}_$rep.out 2> $O/bench_u${u}_$rep.err
    rc=$?; echo "   exit $rc" >> $O/status.log; [ $rc -ne 0 ] && exit $rc
  done
done
echo done >> $O/status.log
