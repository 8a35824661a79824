#!/bin/bash
# round-3 session w (final build): whole suite + smoke, precision record, headline + every config
# bench line, plain-API line, per-rank shards, rocprof stats of the headline, PMC traffic passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3w}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run prec_7 300 python tools/prec_errors.py --n 20000 --combos 4:1 --bwd-f16 7
run bench 300 python bench.py --steps 20 --warmup 3
run bench40 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline
for c in fluid2DtlgnM advect1D elasticity2Dstretch elasticity3Dbunny; do
  run bench_$c 300 python bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 10
done
run mixed_M 300 python bench.py --config fluid2DtlgnM --precision mixed --steps 20 --warmup 3 --no-cpu-baseline
run plain 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run shard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run shard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
export TMPDIR=/tmp
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
PRX='jet_|dw_x6|reduce_'
B="python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline"
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_fetch" -o run --output-format csv -- $B
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_write" -o run --output-format csv -- $B
echo done >> $O/status.log
