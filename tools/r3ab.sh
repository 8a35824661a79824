#!/bin/bash
# round-3 session ab: value jets two-kernel from 24,576 points + the sampler draw plan: whole
# suite, smoke, headline / plain / fluid2DtlgnM 2-rank shard lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3ab}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
run plain 200 python bench.py --api plain --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
run shard2 200 python bench.py --config fluid2DtlgnM --shard-of 2 --steps 10 --warmup 3 --no-cpu-baseline
echo done >> $O/status.log
