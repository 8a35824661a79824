# 8-wave vs 4-wave (X6_MAX_WAVES=4, forward TU only) x6 forward study; results in profiles/r01/fwd_waves_study.
# Build the variant first: hipcc ... -mllvm -amdgpu-sched-strategy=max-ilp -DX6_MAX_WAVES=4 -c jet_x6_fwd.hip, link as lib/libinsr_hip_w4.so
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/s54; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
for v in base w4; do
  lib=insr-pde_amd/lib/libinsr_hip.so; [ $v = w4 ] && lib=insr-pde_amd/lib/libinsr_hip_w4.so
  timeout -k 10 150 python tools/kbench.py --nets fluid_pres,fluid_vel --sizes 324,16384 --variants x6 --reps 50 --lib $lib > $O/kb_$v.jsonl 2> $O/kb_$v.err; rc=$?; echo "kb $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
  INSR_HIP_LIB=$PWD/$lib timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_$v.jsonl 2>&1; rc=$?; echo "bench $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
done
echo done >> $O/status.log
