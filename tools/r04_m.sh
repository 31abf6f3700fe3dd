#!/bin/bash
# GPU box, round 4: the final tree -- the whole GPU suite, smoke(), and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_m}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log >&2
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | head -1 | cut -c1-300 >&2
exit 0
