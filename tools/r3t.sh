#!/bin/bash
# round-3 session t: same-box headline A/B, the current build vs the previous commit's (static f16
# Laplacian scale), alternating, 40-step lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3t}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2 3; do
  run new_$rep 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline
  run old_$rep 200 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
echo done >> $O/status.log
