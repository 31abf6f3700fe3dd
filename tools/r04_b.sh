#!/bin/bash
# GPU box, round 4: A/B of the grouping sort (LSD passes + split vs the bucket sort with the split
# folded in) at c3 / c2 / c5, the fused sharded owner step on and off at world 1, three alternating
# reps each (bench.py lines, 20 steps, 5 warmup).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_b}; mkdir -p $out
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
ms() { echo "$(grep -o '"ms_per_step": [0-9.]*' $1 | head -1 | cut -d' ' -f2) $(grep -o '"median_ms_per_step": [0-9.]*' $1 | head -1 | cut -d' ' -f2)"; }
for rep in ${REPS:-1 2 3}; do
  for c in ${CONFIGS:-c3 c2 c5}; do
    for s in lsd default; do
      timeout -k 10 300 python bench.py $B --config $c --sort $s > $out/ab_${c}_${s}_$rep.log 2>&1 || exit $?
      echo "$c sort=$s rep$rep $(ms $out/ab_${c}_${s}_$rep.log)" >&2
    done
  done
  if [ "${SHARDED:-1}" = "1" ]; then
    for f in off on; do
      timeout -k 10 300 python bench.py $B --force-sharded --fuse $f > $out/ab_sh1_fuse${f}_$rep.log 2>&1 || exit $?
      echo "sharded1 fuse=$f rep$rep $(ms $out/ab_sh1_fuse${f}_$rep.log)" >&2
    done
  fi
done
exit 0
