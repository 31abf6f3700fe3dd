#!/bin/bash
# GPU box, round 4: the fused step's split scan + scatter on an aux stream beside the forward (this
# tree) against all of the split on the main stream (tools/_variants/noaux): fused / parity / fit
# tests, alternating c3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_t}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_resident_fit.py \
    tests/test_gpu_bucket.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in tree noaux; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
exit 0
