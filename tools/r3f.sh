#!/bin/bash
# round-3 session f: wsplit / parity / phase tests, propagation-prefetch A/B (kbench --lib), shard + headline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3f}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 600 python -u -m pytest tests/test_gpu_wsplit.py tests/test_gpu_parity.py tests/test_gpu_phases.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_phases.py -q -x -m gpu --timeout 120 --timeout-method thread
for rep in 1 2; do
run kbA$rep 300 python tools/kbench.py --nets fluid_pres --modes lap,grad --sizes 8354,16708,33092 --variants x6 --policies 0 --bwd-only --reps 20 --lib insr-pde_amd/lib_exp/r3e.so
run kbB$rep 300 python tools/kbench.py --nets fluid_pres --modes lap,grad --sizes 8354,16708,33092 --variants x6 --policies 0 --bwd-only --reps 20
done
run bench 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline
run shardM 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 50 --warmup 3 --no-cpu-baseline
run allreduce 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 tools/allreduce_cost.py
echo done >> $O/status.log
