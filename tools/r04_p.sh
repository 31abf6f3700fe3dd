#!/bin/bash
# GPU box, round 4: the final tree (3 forward passes for k <= 8): the whole GPU suite, smoke, the
# driver's bench command, c2 / c5 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_p}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log >&2
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_default.log | head -1) $(grep -o '"fit_ms_per_iter_steady": [0-9.]*' $out/bench_default.log | head -1)" >&2
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for c in c2 c5; do
  timeout -k 10 300 python bench.py $B --config $c > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
done
exit 0
