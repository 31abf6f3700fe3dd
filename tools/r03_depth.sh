#!/bin/bash
# GPU box: prefetch depth 2 / 1 / 3 on the default library, the driver's command shape (20 steps,
# 5 warmup), three alternating reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/depth
for rep in 1 2 3; do
  for d in 2 1 3; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --prefetch-depth $d \
        > gpurun_out/depth/d${d}_$rep.log 2>&1 || exit $?
    echo "depth=$d rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/depth/d${d}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/depth/d${d}_$rep.log | head -1)" >&2
  done
done
exit 0
