#!/bin/bash
# GPU box: all GPU tests, then the sharded (world 1) bench with and without the prefetch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sh
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread > gpurun_out/sh/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/sh/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-sharded > gpurun_out/sh/bench_sh.log 2>&1 || exit $?
tail -1 gpurun_out/sh/bench_sh.log >&2
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-sharded --no-prefetch > gpurun_out/sh/bench_sh_nopf.log 2>&1 || exit $?
tail -1 gpurun_out/sh/bench_sh_nopf.log >&2
exit 0
