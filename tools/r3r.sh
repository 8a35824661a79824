#!/bin/bash
# round-3 session r: whole suite after the routing change, fluid2DtlgnM line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3r}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_M 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --cpu-seconds 10
run bench 300 python bench.py --steps 20 --warmup 3
echo done >> $O/status.log
