#!/bin/bash
# GPU box, round 4: stream priorities -- the step's stream high, the side stream lowest (this tree,
# bench --main-priority high) against no priorities (tools/_variants/nopri, --main-priority default):
# alternating reps at c3 / c2 / c5 and world-1 sharded, after the fused / parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_l}; mkdir -p $out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_resident_fit.py \
      -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
  rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
fi
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in ${REPS:-1 2 3}; do
  for c in ${CONFIGS:-c3 c2 c5 sh1}; do
    for v in tree nopri; do
      lib=""; pr=high; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so && pr=default
      a="--config $c"; [ $c = sh1 ] && a="--config c3 --force-sharded"
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B $a --main-priority $pr > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1)" >&2
    done
  done
done
exit 0
