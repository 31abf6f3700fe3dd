#!/bin/bash
# GPU box: A/B of the whole-record fused forward (32- and 64-lane teams) at c3, and of the prepared
# batch's sort wait moved before the forward at c2 / c5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05_h}; mkdir -p $out
FM_HIP_LIB=fm_spark_amd/lib/variants/whole32/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py \
    -x -q --timeout 300 --timeout-method thread > $out/pytest_whole32.log 2>&1
rc=$?; tail -1 $out/pytest_whole32.log >&2; [ $rc -ne 0 ] && exit $rc
OUT=$out/ab VARIANTS="default whole32 whole" CONFIGS="c3" REPS="1 2 3" bash tools/ab.sh || exit $?
OUT=$out/ab VARIANTS="default waitearly" CONFIGS="c2 c5" REPS="1 2 3" bash tools/ab.sh || exit $?
exit 0
