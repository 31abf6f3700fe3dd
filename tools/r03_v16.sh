#!/bin/bash
# GPU box: the bench GPU tests, then the driver's command and the c2 / c5 lines on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03_v16}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_fuse.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/bench_c3.log | head -1)" >&2
for c in c2 c5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline --host-path-steps 0 > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
done
exit 0
