#!/bin/bash
# GPU box: tools/r03_v6.sh, then the fused-forward A/B (tools/ab_lib.sh) of the default library
# against the variants named in B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r03_v6.sh ${1:-r03_v6} || exit $?
B="${B:-g4096 g1024 u3}" REPS="1 2" bash tools/ab_lib.sh || exit $?
exit 0
