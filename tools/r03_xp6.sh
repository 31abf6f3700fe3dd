#!/bin/bash
# GPU box: fused-step and parity tests on the variants in B, then c3 and c5 A/Bs against them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp6
for v in ${B}; do
  FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py \
      tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/xp6/pytest_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/xp6/pytest_$v.log >&2; [ $rc -ne 0 ] && exit $rc
done
REPS="${REPS:-1 2 3}" bash tools/ab_lib.sh || exit $?
mkdir -p gpurun_out/ab_c3 && mv gpurun_out/ab/*.log gpurun_out/ab_c3/
REPS="${REPS:-1 2 3}" BENCH_ARGS="--config c5" bash tools/ab_lib.sh || exit $?
exit 0
