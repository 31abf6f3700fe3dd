#!/bin/bash
# GPU-box runner: parity tests, smoke, bench.  Stops at the first crash / fault / timeout;
# plain test failures (pytest exit 1) do not stop the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-20}"
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >&2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 30 "gpurun_out/$name.log" >&2
  return $rc
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
run bench 600 python bench.py --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} || exit $?
if [ "${SHARDED:-0}" = "1" ]; then
  run bench_sharded 600 python bench.py --steps "$STEPS" --warmup 3 --force-sharded --no-cpu-baseline || exit $?
fi
if [ "${PROF:-0}" = "1" ]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run \
      -- python bench.py --steps "$STEPS" --warmup 3 --no-cpu-baseline ${BENCH_ARGS_PROF:-} || exit $?
fi
exit 0
