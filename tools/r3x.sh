#!/bin/bash
# round-3 session x: cost split of the dynamic fp16 scales -- same-box A/B of three libraries:
# both (working tree), forward-only (Laplacian-stream forward scale, static backward 2^-10), static
# (previous commit); headline lines + rocprof stats of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-r3x}; mkdir -p $O
run() { local name=$1 to=$2; shift 2; echo "== $name" >> $O/status.log
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "   exit $rc" >> $O/status.log
  [ $rc -ne 0 ] && exit $rc; return 0; }
B="bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-roofline"
for rep in 1 2 3; do
  run both_$rep 200 python $B
  run fwd_$rep 200 python $B --lib insr-pde_amd/lib_fwd/libinsr_hip.so
  run old_$rep 200 python $B --lib insr-pde_amd/lib_exp/libinsr_hip.so
done
export TMPDIR=/tmp
run prof_both 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_both" -o run --output-format csv -- python $B
run prof_fwd 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_fwd" -o run --output-format csv -- python $B --lib insr-pde_amd/lib_fwd/libinsr_hip.so
run prof_old 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_old" -o run --output-format csv -- python $B --lib insr-pde_amd/lib_exp/libinsr_hip.so
echo done >> $O/status.log
