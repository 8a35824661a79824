#!/bin/bash
# round-4 batch: full GPU suite, bench + profile, the Adam-gap traces, then (last: an experimental
# build) the same-box A/B of two library builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S=${SESSION:-r4q}; O=gpurun_out/$S; mkdir -p $O
export TMPDIR=/tmp
SESSION=$S STEPS="${FIRST_STEPS:-tests bench prof}" bash tools/r4_session.sh || exit $?
echo "== adam gap traces" >> $O/status.log
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/$O/tr_normal" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > $O/tr_normal.out 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d "$PWD/$O/tr_noplanes" -o run --output-format csv -- python tools/diag_adam_gap.py --steps 10 --warmup 3 > $O/tr_noplanes.out 2>&1 || exit $?
echo "   ok" >> $O/status.log
[ -n "${AB_ARGS:-}" ] || exit 0
SESSION=$S bash tools/r4_ab.sh || exit $?
