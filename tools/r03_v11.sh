#!/bin/bash
# GPU box: the bench GPU tests, then the driver's bench command (c3, 20 steps, 5 warmup) twice, the
# world-1 sharded and the c5 lines.   tools/r03_v11.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=${1:-r03_v11}; out=gpurun_out/$name
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v -rf --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/c3_$rep.log 2>&1 || exit $?
  echo "c3 rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $out/c3_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/c3_$rep.log | head -1)" >&2
done
for v in sharded c5; do
  args="--config $v"; [ $v = sharded ] && args="--force-sharded"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 $args > $out/$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $out/$v.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/$v.log | head -1)" >&2
done
exit 0
