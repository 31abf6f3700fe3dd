#!/bin/bash
# GPU box: tools/r03_xp6.sh (tests on the variants in B, c3 and c5 A/Bs), then c2's A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r03_xp6.sh || exit $?
mkdir -p gpurun_out/ab_c5 && mv gpurun_out/ab/*.log gpurun_out/ab_c5/
REPS="${REPS:-1 2}" BENCH_ARGS="--config c2" bash tools/ab_lib.sh || exit $?
exit 0
