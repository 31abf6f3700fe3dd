#!/bin/bash
# Diagnostic ablations of the step (outputs are wrong by design; timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
A="--steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}"
for v in ${ABL:-0 1 2 4 8 6 15}; do
  FM_NO_OVERLAP=1 FM_ABLATE=$v timeout -k 10 300 python bench.py $A > gpurun_out/abl/a$v.log 2>&1 || exit $?
done
exit 0
