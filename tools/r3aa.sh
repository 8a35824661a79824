#!/bin/bash
# round-3 session aa: value-jet backward routing re-measured with the f16x3 backward products --
# fused tile-split + partial rows (policy 1) vs two-kernel propagation + split-K dW (policy 2) vs
# auto (0), backward into .grad incl. reductions, fluid nets, 8K-66K points
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3aa}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2; do
  run kb_$rep 300 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value --sizes 4178,8354,16708,33092,66844 --variants x6 --policies 0,1,2 --bwd-only --reps 50
done
echo done >> $O/status.log
