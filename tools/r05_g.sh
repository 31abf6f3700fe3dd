#!/bin/bash
# GPU box: the fused forward on whole-record gathers (FM_FWD_WHOLE build): the fused / full-size /
# resident-fit parity tests on it, then alternating c3 A/B against the tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05_g}; mkdir -p $out
FM_HIP_LIB=fm_spark_amd/lib/variants/whole32/libfm_hip.so timeout -k 10 800 python -u -m pytest tests/test_gpu_fuse.py \
    tests/test_gpu_fullsize.py tests/test_gpu_resident_fit.py tests/test_gpu_parity.py -x -v --timeout 300 \
    --timeout-method thread > $out/pytest_whole.log 2>&1
rc=$?; tail -1 $out/pytest_whole.log >&2; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/pytest_whole.log | head >&2; exit $rc; }
OUT=$out/ab VARIANTS="default whole32 whole" CONFIGS="c3" REPS="1 2 3" bash tools/ab.sh || exit $?
exit 0
