#!/bin/bash
# GPU box, round 4: unfused forward with 3 passes in flight (fu3), the update loading 2 entries ahead
# at k = 5..8 (d2) and k = 13..16 (d4), against this tree: alternating reps at c2 / c5 / c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_o}; mkdir -p $out
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2; do
  for cv in c2:tree c2:fu3 c2:d2 c5:tree c5:fu3 c5:d4 c3:tree c3:d4; do
    c=${cv%%:*}; v=${cv#*:}
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config $c > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
    echo "$c $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1)" >&2
  done
done
exit 0
