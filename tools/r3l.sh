#!/bin/bash
# round-3 session l: whole GPU suite (batched reverse jets, device band samplers), headline bench
# with event-timed timesteps, the plain reference-API line and its per-step kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3l}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
for rep in 1 2; do
  run bench_$rep 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
  run plain_$rep 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
done
export TMPDIR=/tmp
run prof_plain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_plain" -o run --output-format csv -- python bench.py --api plain --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
