#!/bin/bash
# GPU box, round 4: the split's whole-chunk loads in the count pass only (b1), the scatter pass only
# (b2), both (b3), against this tree (neither): the fused and sharded GPU tests on b1 and b2, then
# alternating c3 reps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_za}; mkdir -p $out
for v in b1 b2; do
  FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_fuse.py tests/test_gpu_shard.py > $out/tests_$v.log 2>&1 || { tail -20 $out/tests_$v.log >&2; exit 1; }
  echo "$v $(tail -1 $out/tests_$v.log)" >&2
done
B="--steps 30 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2 3; do
  for v in tree b1 b2 b3; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config c3 > $out/ab_c3_${v}_$rep.log 2>&1 || exit $?
    echo "c3 $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_c3_${v}_$rep.log | head -1)" >&2
  done
done
exit 0
