#!/bin/bash
# round-3 session y: HEAD after the dynamic fp16 scales (restored container): whole suite, precision
# record (default vs mask 0), headline + every config bench line, rocprof stats of the headline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3y}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
for m in 0 7; do
  run prec_$m 300 python tools/prec_errors.py --n 20000 --combos 4:1 --bwd-f16 $m
done
run bench 300 python bench.py --steps 20 --warmup 3
for c in fluid2DtlgnM advect1D elasticity2Dstretch elasticity3Dbunny; do
  run bench_$c 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 10
done
run plain 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
export TMPDIR=/tmp
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo done >> $O/status.log
