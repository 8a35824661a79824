#!/bin/bash
# Same-box A/B of run-time knobs: the headline bench with the default policy and with each
# "VAR=value" of $KNOBS (space separated), 100 steps each, alternating twice.
# (Tile-count overrides are no longer environment variables: tools/ab_tiles.py.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${SESSION:-abenv}; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-roofline > $O/default_$rep.log 2>&1 || exit $?
  for kv in $KNOBS; do
    timeout -k 10 200 env $kv python bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-roofline > $O/${kv//=/_}_$rep.log 2>&1 || exit $?
  done
done
