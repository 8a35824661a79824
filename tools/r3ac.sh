#!/bin/bash
# round-3 session ac: PMC traffic of the last build's headline kernels (separate FETCH / WRITE / SQ passes),
# the mixed-precision fluid2DtlgnM line, per-rank shards of the strong-scaling configs, and the
# value-backward launch shape under the fp16 products
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3ac}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
export TMPDIR=/tmp
PRX='jet_|dw_x6|reduce_'
B="python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline"
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_fetch" -o run --output-format csv -- $B
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_write" -o run --output-format csv -- $B
run pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$PRX" -d "$PWD/$O/pmc_sq" -o run --output-format csv -- $B
run mixed_M 300 python bench.py --config fluid2DtlgnM --precision mixed --steps 20 --warmup 3 --no-cpu-baseline
run shard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run shard_M4 300 python bench.py --config fluid2DtlgnM --shard-of 4 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
run shard_el3d8 300 python bench.py --config elasticity3Dbunny --shard-of 8 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
