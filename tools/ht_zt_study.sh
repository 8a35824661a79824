# A/B of the x6 backward LDS writers (profiles/r01/s51).  Build the variants first:
#   make -C insr-pde_amd/csrc OUT=../lib/libinsr_hip_old.so OBJDIR=/tmp/obj_old EXTRA="-DX6_NO_HT"
#   make -C insr-pde_amd/csrc OUT=../lib/libinsr_hip_nozt.so OBJDIR=/tmp/obj_nozt   (HT, the default)
#   (main = a build with EXTRA=-DX6_ZT when re-running the ZT comparison)
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/s51; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
L=insr-pde_amd/lib
for v in old nozt main; do
  lib=$L/libinsr_hip_$v.so; [ $v = main ] && lib=$L/libinsr_hip.so
  timeout -k 10 150 python tools/kbench.py --nets fluid_pres,fluid_vel,el2d --sizes 324,16384 --variants x6 --reps 50 --lib $lib > $O/kb_$v.jsonl
done
timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench.jsonl
