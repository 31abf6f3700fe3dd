#!/bin/bash
# GPU box: PMC passes of the c3 (fused), c2 and c5 bench lines (tools/r03_pmc.sh, no c4), then an
# A/B of the per-phase HIP-event timing (--profile-kernels 1 / 0) at c3 and c5, alternating.
#   tools/r03_pmc_ab.sh OUTDIR [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=${1:-r03_pmc}; reps=${2:-2}
C4=0 bash tools/r03_pmc.sh $out || exit $?
mkdir -p gpurun_out/$out/ab
for rep in $(seq 1 $reps); do
  for c in c3 c5; do
    for p in 1 0; do
      timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0 \
          --profile-kernels $p > gpurun_out/$out/ab/${c}_p${p}_$rep.log 2>&1 || exit $?
      echo "$c prof=$p rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$out/ab/${c}_p${p}_$rep.log | head -1)" \
           "$(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/$out/ab/${c}_p${p}_$rep.log | head -1)" >&2
    done
  done
done
exit 0
