#!/bin/bash
# GPU box: singleton fusion -- its tests, then an alternating c3 step A/B: unfused (FM_FUSE_SINGLE=0)
# vs fused with the next batch sorted 1 or 2 steps ahead (median of 40 steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fuse
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_sort.py -q -x \
    --timeout 120 --timeout-method thread > gpurun_out/fuse/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/fuse/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in "0 1" "1 1" "1 2"; do
    set -- $v
    FM_FUSE_SINGLE=$1 timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --prefetch-depth $2 \
        > gpurun_out/fuse/f$1_d$2_$rep.log 2>&1 || exit $?
    echo "fuse=$1 depth=$2 rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/fuse/f$1_d$2_$rep.log | tr '\n' ' ')" >&2
  done
done
