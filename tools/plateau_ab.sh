# A/B of the Adam + plateau fusion on one box (INSR_FUSED_PLATEAU=0: separate plateau launch)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${SESSION:-s65}; mkdir -p $O
for v in 1 0 1 0; do
  INSR_FUSED_PLATEAU=$v timeout -k 10 150 python bench.py --no-cpu-baseline --no-roofline >> $O/bench_fp$v.jsonl 2>&1; rc=$?; echo "bench $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
done
echo done >> $O/status.log
