#!/bin/bash
# Same-box A/B of small-kernel launch shapes: kernel-trace stats of the headline bench with the
# current sources (A) and with the loss-group / sampler block shapes changed (B); sources restored.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-ab}; mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/$1 -o run --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline > $O/$1.log 2>&1; }
run A || exit $?
C=insr-pde_amd/csrc
cp $C/residual.hip /tmp/residual.hip.bak && cp $C/sampler.hip /tmp/sampler.hip.bak
sed -i 's/constexpr long kGroupPerBlock = 1024;/constexpr long kGroupPerBlock = 4096;/' $C/residual.hip
sed -i 's/constexpr int kSampThreads = 256;/constexpr int kSampThreads = 512;/' $C/sampler.hip
make -C $C -j16 > $O/build_B.log 2>&1 || { cp /tmp/residual.hip.bak $C/residual.hip; cp /tmp/sampler.hip.bak $C/sampler.hip; exit 1; }
run B; rc=$?
cp /tmp/residual.hip.bak $C/residual.hip && cp /tmp/sampler.hip.bak $C/sampler.hip
exit $rc
