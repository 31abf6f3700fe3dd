#!/bin/bash
# GPU box: fused-step tests on every variant in B, then the c3 A/B (three reps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp10
for v in default ${B}; do
  lib=fm_spark_amd/lib/libfm_hip.so; [ "$v" != default ] && lib=tools/_variants/$v/libfm_hip.so
  FM_HIP_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py -x -q --timeout 200 --timeout-method thread \
      > gpurun_out/xp10/pytest_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/xp10/pytest_$v.log >&2; [ $rc -ne 0 ] && exit $rc
done
REPS="1 2 3" bash tools/ab_lib.sh || exit $?
exit 0
