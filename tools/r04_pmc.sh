#!/bin/bash
# GPU box, round 4: PMC passes (tools/pmc.sh, one counter group per pass) of the c3 (fused step, bucket
# sort), c2, c5 and world-1 sharded (fused owner step) bench lines, converted to profiles/pmc_*.json
# with the kernels one step launches (bench.py step_traffic reads "per_step").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
base=gpurun_out/${1:-r04_pmc}
tag=${2:-r04}
A="--steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0"
BK='"k_radix_count": 1, "k_radix_scan_rows": 1, "k_radix_scatter": 1, "k_bucket_order": 1, "k_bucket_sort": 1'
for c in ${CONFIGS:-c3 c2 c5 sh1}; do
  args="--config $c"
  [ $c = sh1 ] && args="--config c3 --force-sharded"
  PMC_OUT=$base/$c BENCH_ARGS="$args $A" bash tools/pmc.sh || exit $?
  case $c in
    c3) meta="{\"num_features\": 100000000, \"k\": 16, \"batch_rows\": 262144, \"fused\": true, \"timed_steps\": 5, \"build\": \"$tag (bucket sort with the split, tags at the step)\", \"per_step\": {\"k_forward\": 1, \"k_segment_update\": 1, \"k_segment_combine\": 1, \"k_tag_runs\": 1, $BK, \"k_bucket_offsets\": 1, \"k_bucket_compact\": 1}}"; f=pmc_c3_fused.json ;;
    c2) meta="{\"num_features\": 1000000, \"k\": 8, \"batch_rows\": 65536, \"fused\": false, \"timed_steps\": 5, \"build\": \"$tag (bucket sort)\", \"per_step\": {\"k_forward\": 1, \"k_segment_update\": 1, \"k_segment_combine\": 1, $BK}}"; f=pmc_c2.json ;;
    c5) meta="{\"num_features\": 1000000, \"k\": 16, \"batch_rows\": 65536, \"fused\": false, \"timed_steps\": 5, \"build\": \"$tag (bucket sort)\", \"per_step\": {\"k_forward\": 1, \"k_segment_update\": 1, \"k_segment_combine\": 1, $BK}}"; f=pmc_c5.json ;;
    sh1) meta="{\"num_features\": 100000000, \"k\": 16, \"batch_rows\": 262144, \"fused\": true, \"mode\": \"sharded\", \"world\": 1, \"timed_steps\": 5, \"build\": \"$tag (fused owner step)\"}"; f=pmc_c3_sharded1.json ;;
  esac
  python tools/pmc_to_json.py $base/$c profiles/$f "$meta" || exit $?
  echo "== $c done -> profiles/$f" >&2
done
