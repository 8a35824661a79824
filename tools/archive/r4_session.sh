#!/bin/bash
# round-4 GPU session: STEPS (default "tests bench prof") with per-step time limits; stops at the first failure
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r4}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
export TMPDIR=/tmp
for s in ${STEPS:-tests bench prof}; do
  case $s in
    trec) run t_recompute 600 python -u -m pytest tests/test_gpu_recompute.py -x -v --timeout 120 --timeout-method thread ;;
    tests) run tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} ;;
    bench) run bench 300 python bench.py --steps ${BSTEPS:-20} --warmup 3 --no-cpu-baseline ;;
    benchcpu) run benchcpu 400 python bench.py --steps ${BSTEPS:-20} --warmup 3 ;;
    plain) run plain 300 python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    configs) for c in ${CONFIGS:-advect1D elasticity2Dstretch elasticity3Dbunny fluid2DtlgnM}; do
               run bench_$c 400 python bench.py --config $c --steps ${CSTEPS:-10} --warmup 3 --no-cpu-baseline; done ;;
    shards) run shard_M8 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline ;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    kbench) run kbench 400 python tools/kbench.py ${KARGS:---sizes 8192,16708,66844 --nets fluid_pres --modes lap --variants h3 --policies 0,2} ;;
  esac
done
echo done >> $O/status.log
