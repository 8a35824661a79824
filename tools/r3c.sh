#!/bin/bash
# round-3 session c: resident parity (fragment-order partials), backward-policy kernel sweep,
# precision pairs for 'mixed', per-rank shard benches.  Stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3c}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 400 python -u -m pytest tests/test_gpu_resident.py -q -x -m gpu --timeout 120 --timeout-method thread
run kb 400 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,lap --sizes 8354,16708,33092,65536,131072 --variants x6 --policies 0,3 --bwd-only --reps 20
run prec 300 python tools/prec_errors.py --nets fluid_pres,fluid_vel,advect --combos 1:1,2:3,3:2,2:2,1:3,3:1,3:3 --n 4000
run shardM 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 50 --warmup 3 --no-cpu-baseline
run shardB 300 python bench.py --config elasticity3Dbunny --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline
run shardM3 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 50 --warmup 3 --no-cpu-baseline --bwd-policy 3
echo done >> $O/status.log
