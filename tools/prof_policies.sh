#!/bin/bash
# rocprofv3 kernel stats of the headline bench under each backward policy ($POLICIES), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${SESSION:-profpol}; mkdir -p $O
for pol in ${POLICIES:-0 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/p$pol" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy $pol ${ABARGS:-} > $O/p$pol.log 2>&1 || exit $?
done
