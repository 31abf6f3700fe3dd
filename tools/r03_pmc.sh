#!/bin/bash
# GPU box: PMC passes (tools/pmc.sh) of the c3 (fused step), c2 and c5 bench lines, one directory each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
base=gpurun_out/${1:-r03_pmc}
for c in ${CONFIGS:-c3 c2 c5}; do
  PMC_OUT=$base/$c BENCH_ARGS="--config $c --steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0" \
      bash tools/pmc.sh || exit $?
  echo "== $c done" >&2
done
