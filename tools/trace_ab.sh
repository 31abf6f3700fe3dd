#!/bin/bash
# GPU box: kernel traces of the c3 bench with the LSD sort and with the bucket sort (timeline analysis:
# tools/timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tr
for m in ${MODES:-0 1}; do
  FM_SORT_BUCKET=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/tr/b$m -o run \
    -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/tr/b$m.log 2>&1 || exit $?
  echo "bucket=$m $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/tr/b$m.log)" >&2
done
