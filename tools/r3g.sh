#!/bin/bash
# round-3 session g: dynamic instruction mix of the x6 jets (SQ_INSTS_* per dispatch) on single jets
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3g}; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
KB="python tools/kbench.py --nets fluid_pres --modes value,lap --sizes 16708 --variants x6 --policies 0 --reps 3"
run mix1 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_CVT --kernel-include-regex "jet_|dw_x6" -d "$PWD/$O/mix1" -o run --output-format csv -- $KB
run mix2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "jet_|dw_x6" -d "$PWD/$O/mix2" -o run --output-format csv -- $KB
run plain 300 rocprofv3 --kernel-trace -d "$PWD/$O/plain" -o run --output-format csv -- python bench.py --api plain --steps 10 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
