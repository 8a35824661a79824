# round-6 closing c3: the full GPU suite, smoke, the default bench line and every BASELINE config line
set -u
O=gpurun_out/c3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.out 2>&1; echo "tests $?" >> $O/status.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.out 2>&1 || { echo "smoke $?" >> $O/status.log; exit 2; }
timeout -k 10 600 python bench.py > $O/default.out 2> $O/default.err || { echo "default $?" >> $O/status.log; exit 3; }
timeout -k 10 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline > $O/advect1D.out 2> $O/advect1D.err || exit 4
for c in elasticity2Dstretch fluid2DtlgnM elasticity3Dbunny; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/$c.out 2> $O/$c.err || exit 5
done
timeout -k 10 300 python bench.py --config fluid2DtlgnM --shard-of 8 --steps 40 --warmup 3 --no-cpu-baseline --no-roofline > $O/shard_M8.out 2> $O/shard_M8.err || exit 6
echo done >> $O/status.log
