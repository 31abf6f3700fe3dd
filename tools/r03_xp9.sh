#!/bin/bash
# GPU box: the GPU tests of the fused step, parity, bench and group paths on the default library, then
# the c3 A/B against the variants in B (tools/ab_lib.sh) and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/xp9
timeout -k 10 700 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_bench.py \
    tests/test_gpu_group.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/xp9/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/xp9/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
REPS="${REPS:-1 2 3}" bash tools/ab_lib.sh || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/xp9/bench_c3.log 2>&1 || exit $?
echo "driver cmd: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/xp9/bench_c3.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/xp9/bench_c3.log | head -1)" >&2
exit 0
