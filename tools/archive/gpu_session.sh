#!/bin/bash
# One GPU-box session: parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / segfault / timeout (exit 124,134,137,139 or >128).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${SESSION:-s}
mkdir -p "$OUT"
# any failing GPU step ends the session: a fault in one step must not be followed by more GPU work
fatal() { [ "$1" -ne 0 ] && { echo "FATAL step exit $1 -- stopping" | tee -a "$OUT/status.log"; exit "$1"; }; return 0; }
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> "$OUT/status.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   $name exit $rc" >> "$OUT/status.log"
  fatal $rc
  return 0
}
for s in ${STEPS:-tests bench prof}; do
  case $s in
    tests) step tests ${TTO:-900} python -u -m pytest ${TESTFILES:-tests} -q -m gpu -x --timeout 120 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} ;;
    smoke) step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py --steps ${BSTEPS:-20} --warmup ${BWARM:-3} ;;
    configs) for c in ${CONFIGS:-advect1D elasticity2Dstretch elasticity3Dbunny fluid2DtlgnM}; do
               step bench_$c 400 python bench.py --config $c --steps ${CSTEPS:-10} --warmup ${BWARM:-3} --cpu-seconds 10
             done ;;
    kbench) step kbench 400 python tools/kbench.py --sizes ${KSIZES:-324,2048,8192,16384} --nets ${KNETS:-fluid_pres,fluid_vel} ;;
    dp2)   step dp2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --steps 5 --warmup 3 --no-cpu-baseline ;;
    eager) step eager 150 python bench.py --steps 5 --warmup 2 --no-graph --no-cpu-baseline ;;
    graph) step graph 150 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline ;;
    ab)    # same-box A/B of the backward-path policy (POLICIES, default "0 2 1"), 100 steps each, twice
           for rep in 1 2; do for pol in ${POLICIES:-0 2 1}; do
             step ab_p${pol}_$rep 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-roofline --bwd-policy $pol ${ABARGS:-}
           done; done ;;
    prof)  export TMPDIR=/tmp; step prof 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    pmc)   export TMPDIR=/tmp
           # HBM traffic of the jet kernels in the bench workload (eager: one counter sample per dispatch);
           # FETCH_SIZE and WRITE_SIZE need separate passes (TCC slots), SQ stall counters a third
           PRX='jet_|dw_x6|reduce_'
           step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$PRX" -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
           step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$PRX" -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline
           step pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "$PRX" -d "$PWD/$OUT/pmc_sq" -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-roofline ;;
  esac
done
echo done >> "$OUT/status.log"
