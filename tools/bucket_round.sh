#!/bin/bash
# GPU box: the bucket sort against rocPRIM (tools/sort_bench, several sizes / skews), the GPU tests
# with it on, then an alternating step A/B of the LSD passes (FM_SORT_BUCKET=0) and the bucket sort.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bkt
sb() {  # n bits skew
  SORT_CHECK_ONLY=${CHECK_ONLY:-} timeout -k 10 120 tools/sort_bench "$@" > "gpurun_out/bkt/sort_$1_$2_$3.log" 2>&1
  local rc=$?
  echo "sort $* rc=$rc: $(grep -E 'fm_hip|mism' gpurun_out/bkt/sort_$1_$2_$3.log | tr '\n' ' ')" >&2
  return $rc
}
sb 10223616 27 0 && sb 10223616 27 1 && sb 2555904 20 0 && sb 9953280 28 0 && \
  CHECK_ONLY=1 sb 100000 20 0 && CHECK_ONLY=1 sb 3000 13 0 && CHECK_ONLY=1 sb 1500000 27 2 || exit $?
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  FM_SORT_BUCKET=1 timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/bkt/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/bkt/pytest.log >&2
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
for rep in 1 2; do
  for m in 0 1; do
    FM_SORT_BUCKET=$m timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/bkt/bench_b${m}_$rep.log 2>&1 || exit $?
    echo "bucket=$m rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/bkt/bench_b${m}_$rep.log)" >&2
  done
done
exit 0
