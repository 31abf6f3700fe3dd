#!/bin/bash
# GPU box: the fused-step and parity tests on the default library, then the c3 A/B against the
# variants named in B (tools/ab_lib.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp2
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py -x -v -rf \
    --timeout 300 --timeout-method thread > gpurun_out/xp2/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/xp2/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
REPS="${REPS:-1 2 3}" bash tools/ab_lib.sh || exit $?
exit 0
