#!/bin/bash
# GPU box, round 4: the fused step without the split's scatter (the update walks the whole sorted
# view, skipping singleton runs): GPU tests, the fused-vs-unfused bitwise probe, an A/B against the
# previous commit's library (tools/_variants/prev: the multi view), then the final evidence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_j}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_resident_fit.py tests/test_gpu_bucket.py \
    tests/test_gpu_parity.py tests/test_gpu_group.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fuse_bitwise_probe.py > $out/bitwise.json 2> $out/bitwise.err || exit $?
cat $out/bitwise.json >&2
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in tree prev; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
exit 0
