#!/bin/bash
# round-3 session z: sampler draw plan (one insr_sample_boxes launch per phase iteration of the
# reference-API phase bodies): its tests, same-box A/B of the plain-API line with / without the
# plan, rocprofv3 kernel trace of the plain step (kernel attribution)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3z}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 300 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_plain_api.py tests/test_gpu_dp_graph.py tests/test_gpu_phases.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
B="--api plain --steps 40 --warmup 3 --no-cpu-baseline --no-roofline"
for rep in 1 2 3; do
  run plan_$rep 200 python bench.py $B
  run noplan_$rep 200 python tools/ab_noplan.py $B
done
export TMPDIR=/tmp
run prof_plain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_plain" -o run --output-format csv -- python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
