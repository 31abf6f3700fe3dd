#!/bin/bash
# GPU box, round 4: the fused step's split back at the step (main stream, tags written by its count
# pass) against the split in fm_batch_prepare + a tag pass (tools/_variants/sideplit): fused GPU
# tests, alternating c3 reps, then c3 with the fit leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_i}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_resident_fit.py tests/test_gpu_parity.py \
    -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in tree sideplit; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 full $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
exit 0
