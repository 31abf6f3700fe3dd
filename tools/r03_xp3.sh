#!/bin/bash
# GPU box: c3 A/B of the default library against the variants in B (3 reps), then the c4 rank bench
# (its roofline with pmc_c4.json's traffic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp3
REPS="${REPS:-1 2 3}" bash tools/ab_lib.sh || exit $?
timeout -k 10 600 python tools/c4_rank_bench.py --iters 5 > gpurun_out/xp3/c4_bench.log 2>&1 || exit $?
tail -1 gpurun_out/xp3/c4_bench.log | cut -c1-300 >&2
exit 0
