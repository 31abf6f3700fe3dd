#!/bin/bash
# GPU box: the whole GPU test suite, then smoke() -- what the driver runs at round end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=${OUT:-gpurun_out/suite}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
    > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log >&2
exit 0
