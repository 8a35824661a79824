#!/bin/bash
# round-3 session ad: bench.py with an untimed warm-up timestep (snapshots + phase loops in step()
# order) before the timed region -- headline and plain lines, the per-timestep times show whether
# the first timed timestep is still slower; bench launcher test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3ad}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2; do
  run bench_$rep 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 10
done
run plain 200 python bench.py --api plain --steps 20 --warmup 5 --no-cpu-baseline --no-roofline
run M 200 python bench.py --config fluid2DtlgnM --steps 20 --warmup 5 --no-cpu-baseline
run tests 300 python -u -m pytest tests/test_gpu_dp_graph.py tests/test_bench_launcher.py -q --timeout 200 --timeout-method thread -p no:cacheprovider
echo done >> $O/status.log
