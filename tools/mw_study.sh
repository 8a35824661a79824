# Forward register-bound study (X6_FWD_MIN_WAVES=4: W = 128 forward held to 128 VGPRs) vs the
# unbounded build; results in profiles/r01/fwd_minwaves_study.  Build the variant first:
#   hipcc ... -mllvm -amdgpu-sched-strategy=max-ilp -DX6_FWD_MIN_WAVES=4 -c jet_x6_fwd.hip, link as lib/libinsr_hip_mw4.so
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${SESSION:-s57}; mkdir -p $O
for v in base mw4; do
  lib=insr-pde_amd/lib/libinsr_hip.so; [ $v = mw4 ] && lib=insr-pde_amd/lib/libinsr_hip_mw4.so
  timeout -k 10 200 python tools/kbench.py --nets fluid_pres,fluid_vel --sizes 324,16384 --variants x6,x6_1,x6_2,x6_4 --reps 50 --lib $lib > $O/kb_$v.jsonl 2> $O/kb_$v.err; rc=$?; echo "kb $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
  INSR_HIP_LIB=$PWD/$lib timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_$v.jsonl 2>&1; rc=$?; echo "bench $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
done
echo done >> $O/status.log
