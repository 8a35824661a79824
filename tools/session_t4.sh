set -u
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/t4; mkdir -p $O
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --api plain --no-cpu-baseline > $O/bench_plain.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_fused.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_el2d -o run --output-format csv -- python bench.py --config elasticity2Dstretch --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_el2d.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof_plain -o run --output-format csv -- python bench.py --api plain --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof_plain.log 2>&1 || exit $?
