#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE of the update kernel per ablation variant (tools/_variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for v in ${VARIANTS:-$(ls tools/_variants)}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    tag=$(echo $c | cut -d' ' -f1)
    FM_HIP_LIB=tools/_variants/$v/libfm_hip.so FM_ABLATE=1 timeout -k 10 120 rocprofv3 --pmc $c \
        --kernel-include-regex "k_segment_update|k_forward" -T --output-format csv \
        -d gpurun_out/abl/$v-$tag -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-prefetch \
        > gpurun_out/abl/$v-$tag.log 2>&1 || { tail -5 gpurun_out/abl/$v-$tag.log >&2; exit 1; }
  done
  echo "$v done" >&2
done
exit 0
