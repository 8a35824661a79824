set -u
O=gpurun_out/r6q1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_advect_iter.py tests/test_gpu_fullsize_phases.py tests/test_gpu_plain_api.py -m gpu -x -q --timeout 120 --timeout-method thread -k "advect or advection" > $O/tadv.out 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline > $O/A_$r.out 2> $O/A_$r.err || exit 2
  timeout -k 10 300 python bench.py --config advect1D --steps 40 --warmup 3 --no-cpu-baseline --lib insr-pde_amd/lib_exp/libinsr_hip.so > $O/B_$r.out 2> $O/B_$r.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof" -o run --output-format csv -- python bench.py --config advect1D --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > $O/prof.out 2>&1 || exit 4
