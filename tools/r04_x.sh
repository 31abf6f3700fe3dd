#!/bin/bash
# GPU box, round 4: the split's one-block scan loading 48 chunk counts per thread, one round for a c3 batch (sp48), against this
# tree's separate one-block scan launch: fused/shard GPU tests on the variant, then alternating c3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_x}; mkdir -p $out
V=tools/_variants/sp48/libfm_hip.so
FM_HIP_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_fuse.py tests/test_gpu_shard.py tests/test_gpu_resident_fit.py > $out/tests_sp48.log 2>&1 || { tail -20 $out/tests_sp48.log >&2; exit 1; }
tail -1 $out/tests_sp48.log >&2
B="--steps 30 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in tree sp48; do
    lib=""; [ $v != tree ] && lib=$V
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config c3 > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
exit 0
