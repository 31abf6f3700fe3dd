#!/bin/bash
# GPU box: quick bucket-sort iteration -- correctness against rocPRIM at c3 / c4 / skewed shapes,
# rocprof kernel stats of the standalone sort, the sort tests, a step A/B (LSD vs bucket).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/bq
sb() {
  SORT_CHECK_ONLY=${CHECK_ONLY:-} timeout -k 10 120 tools/sort_bench "$@" > "gpurun_out/bq/sort_$1_$2_$3.log" 2>&1
  local rc=$?
  echo "sort $* rc=$rc: $(grep -E 'fm_hip|mism' gpurun_out/bq/sort_$1_$2_$3.log | tr '\n' ' ')" >&2
  return $rc
}
sb 10223616 27 0 && sb 10223616 27 3 && sb 9953280 28 3 && CHECK_ONLY=1 sb 100000 20 0 && \
  CHECK_ONLY=1 sb 1500000 27 2 || exit $?
SORT_CHECK_ONLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/bq/prof -o sb -- tools/sort_bench 10223616 27 3 \
  > gpurun_out/bq/prof.log 2>&1 || exit $?
FM_SORT_BUCKET=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -q -rf --timeout 120 --timeout-method thread \
  > gpurun_out/bq/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/bq/pytest.log >&2; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for rep in 1 2; do
  for m in 0 1; do
    FM_SORT_BUCKET=$m timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/bq/bench_b${m}_$rep.log 2>&1 || exit $?
    echo "bucket=$m rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/bq/bench_b${m}_$rep.log)" >&2
  done
done
exit 0
