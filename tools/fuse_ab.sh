# A/B of the fused forward jets on one box (INSR_FUSE_FORWARDS=0: every jet its own launch)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${SESSION:-s72}; mkdir -p $O
for v in 1 0 1 0; do
  INSR_FUSE_FORWARDS=$v timeout -k 10 150 python bench.py --no-cpu-baseline --no-roofline >> $O/bench_f$v.jsonl 2>&1; rc=$?; echo "bench $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
  INSR_FUSE_FORWARDS=$v timeout -k 10 150 python bench.py --config fluid2DtlgnM --no-cpu-baseline --no-roofline >> $O/benchM_f$v.jsonl 2>&1; rc=$?; echo "benchM $v $rc" >> $O/status.log; [ $rc -ge 124 ] && exit $rc
done
echo done >> $O/status.log
