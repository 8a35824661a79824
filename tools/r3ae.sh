#!/bin/bash
# round-3 session ae: Adam's first loads issued before the bias-correction pows -- optimiser /
# phase / parity tests, same-box A/B of the headline against the previous library (lib_exp)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3ae}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run tests 400 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_phases.py tests/test_gpu_parity.py tests/test_gpu_wsplit.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
B="bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-roofline"
for rep in 1 2 3; do
  run new_$rep 200 python $B
  run old_$rep 200 python $B --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
export TMPDIR=/tmp
run prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python $B
run prof_old 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_old" -o run --output-format csv -- python $B --lib insr-pde_amd/lib_exp/libinsr_hip.so
echo done >> $O/status.log
