#!/bin/bash
# GPU box: fused-step tests on the variant, then the c3 A/B of the default library against B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp4
for v in ${B}; do
  FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py -x -q \
      --timeout 200 --timeout-method thread > gpurun_out/xp4/pytest_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/xp4/pytest_$v.log >&2; [ $rc -ne 0 ] && exit $rc
done
REPS="${REPS:-1 2 3}" bash tools/ab_lib.sh || exit $?
exit 0
