#!/bin/bash
# round-3 session q: 6-wave (spilling) fp16 backward kernels vs the 4-wave default (kbench --lib),
# resident vs two-kernel f16 at the fluid2DtlgnM batch, and the plain reference-API step profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3q}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2; do
  run kb_w4_$rep 200 python tools/kbench.py --nets fluid_pres,el2d,el3d --modes lap,grad --sizes 8354,16708,32768 --variants x6 --bwd-only
  run kb_w6_$rep 200 python tools/kbench.py --nets fluid_pres,el2d,el3d --modes lap,grad --sizes 8354,16708,32768 --variants x6 --bwd-only --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
run kb_M 300 python tools/kbench.py --nets fluid_pres,fluid_vel --modes value,lap --sizes 66844 --variants x6 --bwd-only --policies 0,2
run bench_M_p2 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy 2
run bench_M_p0 300 python bench.py --config fluid2DtlgnM --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy 0
export TMPDIR=/tmp
run prof_plain 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_plain" -o run --output-format csv -- python bench.py --api plain --steps 20 --warmup 3 --no-cpu-baseline --no-roofline
echo done >> $O/status.log
