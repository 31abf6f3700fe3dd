#!/bin/bash
# GPU box: the whole GPU suite + smoke after the bucket sort's removal; the one-launch count scan for
# small sorts (FM_SCAN_SMALL) checked on the parity tests and timed against the tree at c2 / c5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05_d}; mkdir -p $out
OUT=$out/suite bash tools/gpu_suite.sh || exit $?
FM_HIP_LIB=fm_spark_amd/lib/variants/scansmall/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_fp64_inputs.py tests/test_gpu_fuse.py -x -q --timeout 300 --timeout-method thread > $out/pytest_scansmall.log 2>&1
rc=$?; tail -1 $out/pytest_scansmall.log >&2; [ $rc -ne 0 ] && exit $rc
OUT=$out/ab VARIANTS="default scansmall" CONFIGS="c2 c5" REPS="1 2 3" bash tools/ab.sh || exit $?
exit 0
