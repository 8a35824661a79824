#!/bin/bash
# Same-box A/B of the backward-path policies ($POLICIES) on $CONFIGS (bench.py lines) + the
# resident parity tests; stops at the first failing GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-abpol}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -q -x -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; exit 1; }
fi
for c in ${CONFIGS:-fluid2Dtlgn}; do
  for pol in ${POLICIES:-0 3 4}; do
    timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --bwd-policy $pol ${ABARGS:-} > $O/${c}_p$pol.json 2> $O/${c}_p$pol.err || { echo "bench $c $pol failed $?"; exit 1; }
    echo "$c p$pol $(python -c "import json,sys; d=json.loads(open('$O/${c}_p$pol.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['ms_per_step'], d['roofline']['avg_ms'] if d.get('roofline') else '')")" >> $O/summary.txt
  done
done
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  for pol in $PROF; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$O/prof_p$pol" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --bwd-policy $pol > $O/prof_p$pol.log 2>&1 || exit 1
  done
fi
