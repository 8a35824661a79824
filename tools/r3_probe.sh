#!/bin/bash
# round-3 probe session: kernel stats per backward policy, precision combos, per-rank shard benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-probe}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -q -x --timeout 120 --timeout-method thread > $O/resident_tests.log 2>&1; echo "resident tests exit $?" >> $O/status.log
SESSION=${SESSION:-probe} POLICIES="${POLICIES:-0 2}" bash tools/prof_policies.sh || exit $?
timeout -k 10 300 python tools/prec_errors.py --nets fluid_pres,fluid_vel,advect --combos ${COMBOS:-2:3,3:2,1:3,3:1,2:2,3:3} --n 4000 > $O/prec.jsonl 2> $O/prec.err || exit $?
for c in fluid2DtlgnM elasticity3Dbunny; do
  timeout -k 10 300 python bench.py --config $c --shard-of 8 --steps 50 --warmup 3 --no-cpu-baseline --no-roofline > $O/shard8_$c.log 2>&1 || exit $?
done
