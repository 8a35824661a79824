# Machine-scheduler study (profiles/r01/flag_study).  Build the variants first:
#   make -C insr-pde_amd/csrc OUT=../lib/libinsr_hip_<s>.so OBJDIR=/tmp/obj_<s> EXTRA="-mllvm -amdgpu-sched-strategy=<s>"
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/flags
L=insr-pde_amd/lib
for v in base max-ilp max-memory-clause; do
  lib=$L/libinsr_hip_$v.so; [ $v = base ] && lib=$L/libinsr_hip.so
  timeout -k 10 150 python tools/kbench.py --nets fluid_pres,fluid_vel,el3d --sizes 16384 --variants x6 --reps 50 --lib $lib > gpurun_out/flags/kb_$v.jsonl
done
cp $L/libinsr_hip.so /tmp/base.so
for v in base max-ilp max-memory-clause base; do
  if [ $v = base ]; then cp /tmp/base.so $L/libinsr_hip.so; else cp $L/libinsr_hip_$v.so $L/libinsr_hip.so; fi
  timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline >> gpurun_out/flags/bench_$v.jsonl
done
