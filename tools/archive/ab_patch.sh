#!/bin/bash
# Same-box A/B of a source patch: kernel-trace stats + bench line of the headline with the
# current sources (A) and with $PATCH applied (B; patch -p1, rebuilt on the box); reverted after.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-ab}; mkdir -p $O
export TMPDIR=/tmp
run() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/$1 -o run --output-format csv -- python bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-roofline > $O/$1.log 2>&1 || return $?
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-roofline > $O/bench_$1.log 2>&1
}
run A || exit $?
patch -p1 < "$PATCH" > $O/patch.log 2>&1 || exit 1
make -C insr-pde_amd/csrc -j16 > $O/build_B.log 2>&1 || { patch -R -p1 < "$PATCH"; exit 1; }
run B; rc=$?
patch -R -p1 < "$PATCH" >> $O/patch.log 2>&1
exit $rc
