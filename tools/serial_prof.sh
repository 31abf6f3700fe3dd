#!/bin/bash
# GPU box: kernel trace of a serial step (no sort prefetch, no sort/forward overlap) so every
# kernel's duration is its own, plus the standalone sort comparison (tools/sort_bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/serial
if [ -x tools/sort_bench ]; then
  timeout -k 10 120 ./tools/sort_bench > gpurun_out/serial/sort_bench.log 2>&1 || exit $?
  cat gpurun_out/serial/sort_bench.log >&2
fi
FM_NO_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/serial/prof -o run \
  -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-prefetch ${BENCH_ARGS:-} > gpurun_out/serial/bench.log 2>&1 || exit $?
tail -1 gpurun_out/serial/bench.log >&2
exit 0
