# A/B of the W^T prefetch in the 1-tile value backward; results in profiles/r01/wpf_ab.  The
# default build has it off: for this A/B the main lib was built with -DX6_BWD_WPF=1 on the
# backward TU and lib/libinsr_hip_nopf.so without it.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${SESSION:-s74}; mkdir -p $O
for v in pf nopf pf nopf; do
  lib=insr-pde_amd/lib/libinsr_hip.so; [ $v = nopf ] && lib=insr-pde_amd/lib/libinsr_hip_nopf.so
  timeout -k 10 150 python tools/kbench.py --nets fluid_pres,fluid_vel --sizes 324 --variants x6 --reps 100 --lib $lib >> $O/kb_$v.jsonl 2>> $O/kb_$v.err; rc=$?; echo "kb $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
  INSR_HIP_LIB=$PWD/$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-roofline >> $O/bench_$v.jsonl 2>&1; rc=$?; echo "bench $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
done
echo done >> $O/status.log
