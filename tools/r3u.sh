#!/bin/bash
# round-3 session u: Laplacian-only dynamic f16 forward scale: targeted tests, same-box headline A/B
# against the previous-commit library (static scales), then the whole suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3u}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
run t_quick 300 python -u -m pytest tests/test_gpu_hessian.py tests/test_gpu_precision.py tests/test_gpu_wsplit.py -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
for rep in 1 2 3; do
  run new_$rep 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
  run old_$rep 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
run tests 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
echo done >> $O/status.log
