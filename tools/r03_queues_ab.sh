#!/bin/bash
# GPU box: hardware-queue count A/B (GPU_MAX_HW_QUEUES 4 = HIP's default, 8 = bench.py's) on the c3
# single-table step and the world-1 sharded step, after the multi-GPU tests; then a kernel trace of
# the sharded bench (which queue each stream's kernels ran on).  Usage: tools/r03_queues_ab.sh OUTDIR [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-queues_ab}; reps=${2:-2}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_bench.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0"
for rep in $(seq 1 $reps); do
  for q in 4 8; do
    for v in c3 sharded; do
      args=""; [ $v = sharded ] && args="--force-sharded"
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 $B $args > $out/${v}_q${q}_$rep.log 2>&1 || exit $?
      echo "$v q=$q rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_q${q}_$rep.log | head -1) $(grep -o '"prepare_ms_median": [0-9.]*' $out/${v}_q${q}_$rep.log)" >&2
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_sharded -o run \
    -- python bench.py --steps 20 --warmup 5 --force-sharded --no-cpu-baseline --host-path-steps 0 \
    > $out/rocprof_sharded.log 2>&1 || exit $?
