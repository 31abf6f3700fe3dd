#!/bin/bash
# GPU box: fusion tests, then alternating c3 steps: unfused, fused (default build), fused with the
# forward capped at 5 waves/SIMD (tools/_variants/minw5); the next batch sorted 2 steps ahead.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/f2
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/f2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/f2/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in unfused fused minw5; do
    lib=fm_spark_amd/lib/libfm_hip.so; fz=1
    [ $v = unfused ] && fz=0
    [ $v = minw5 ] && lib=tools/_variants/minw5/libfm_hip.so
    FM_FUSE_SINGLE=$fz FM_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline \
        --prefetch-depth 2 --host-path-steps 0 > gpurun_out/f2/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/f2/${v}_$rep.log | head -1) $(grep -o '"forward": {[^}]*}, "update": {[^}]*}' gpurun_out/f2/${v}_$rep.log)" >&2
  done
done
