#!/bin/bash
# GPU box, round 4: the split's count and scatter passes loading a wave's whole chunk at once (this
# tree) against the committed one-row-per-round-trip passes (base): the fused, sharded, resident-fit
# and full-size GPU tests on this tree, then alternating c3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_z}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fuse.py tests/test_gpu_shard.py tests/test_gpu_resident_fit.py tests/test_gpu_fullsize.py > $out/tests_tree.log 2>&1 || { tail -20 $out/tests_tree.log >&2; exit 1; }
tail -1 $out/tests_tree.log >&2
B="--steps 30 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in base tree; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config c3 > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c3 -o run --output-format csv -- \
    python bench.py $B --config c3 > $out/prof_c3.log 2>&1 || exit $?
exit 0
