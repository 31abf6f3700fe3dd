#!/bin/bash
# GPU box, round 4: PMC passes of the c2 line with the final forward (3 passes in flight at k <= 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_s}; mkdir -p $out
A="--steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0"
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" PMC_OUT=$out/pmc/c2_default BENCH_ARGS="--config c2 $A" \
    bash tools/pmc.sh || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0 --config c2 \
    > $out/bench_c2.log 2>&1 || exit $?
echo "c2 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c2.log | head -1)" >&2
exit 0
