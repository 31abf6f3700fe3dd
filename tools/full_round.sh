#!/bin/bash
# GPU box: the whole evidence set for one build -- GPU tests, smoke, default bench, rocprof kernel
# trace + stats of the same bench command, PMC passes (tools/pmc.sh), world-1 sharded bench and the
# R = 8 phase simulator.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/full
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 3 "$OUT/$name.log" | cut -c1-400 >&2
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -rf --timeout 200 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py --steps 20 --warmup 3 || exit $?
step rocprof 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof -o run \
    -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit $?
BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-prefetch --batches 2 --profile-kernels 0" step pmc 900 bash tools/pmc.sh || exit $?
step bench_sharded 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --force-sharded || exit $?
step sim8 600 python tools/shard_sim_bench.py --ranks 8 || exit $?
exit 0
