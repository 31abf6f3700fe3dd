#!/bin/bash
# GPU box, round 4: the whole GPU suite (incl. the full-size tests) and smoke().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_h}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log >&2; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -2 $out/smoke.log >&2
exit $rc
