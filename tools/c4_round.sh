#!/bin/bash
# GPU box: the c4 rank test and the c4 rank bench (+ rocprof kernel stats of the bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4.py -m gpu -x -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/c4_test.log 2>&1
rc=$?; echo "c4 test rc=$rc" >&2; tail -n 25 gpurun_out/c4_test.log >&2
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/c4_rank_bench.py --iters 5 > gpurun_out/c4_bench.log 2>&1
rc=$?; echo "c4 bench rc=$rc" >&2; tail -n 5 gpurun_out/c4_bench.log >&2
[ $rc -ne 0 ] && exit $rc
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/c4prof -o run \
    -- python tools/c4_rank_bench.py --iters 5 > gpurun_out/c4_rocprof.log 2>&1
  rc=$?; echo "c4 rocprof rc=$rc" >&2; tail -n 3 gpurun_out/c4_rocprof.log >&2
fi
exit $rc
