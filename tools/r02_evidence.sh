#!/bin/bash
# GPU box: the second half of a round's evidence -- the update's S-gather ablation PMC passes
# (tools/_variants base / nos), the c2 and c5 bench lines, then the c4 rank test + bench (+ rocprof).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
VARIANTS="base nos" bash tools/abl_pmc.sh || exit $?
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ev/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ev/bench_c5.log 2>&1 || exit $?
echo "c2/c5 done" >&2
PROF=1 bash tools/c4_round.sh
