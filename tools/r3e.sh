#!/bin/bash
# round-3 session e: full GPU suite, headline bench + rocprof, per-rank shards
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3e}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread
run bench 300 python bench.py --steps 20 --warmup 3
run shardM 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 50 --warmup 3 --no-cpu-baseline
run shardM4 300 python bench.py --config fluid2DtlgnM --shard-of 4 --steps 50 --warmup 3 --no-cpu-baseline
run shardM2 300 python bench.py --config fluid2DtlgnM --shard-of 2 --steps 50 --warmup 3 --no-cpu-baseline
export TMPDIR=/tmp
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline
run profM8 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/profM8" -o run --output-format csv -- python bench.py --config fluid2DtlgnM --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
