#!/bin/bash
# GPU box: the fused-step tests, then alternating c3 benches: fused (depth 2), unfused (depth 2),
# fused (depth 1).  Usage: tools/r03_ab.sh OUTDIR [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-ab}; reps=${2:-2}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_group.py tests/test_gpu_bench.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in $(seq 1 $reps); do
  for v in fused unfused fused_d1; do
    args="--fuse on --prefetch-depth 2"
    [ $v = unfused ] && args="--fuse off --prefetch-depth 2"
    [ $v = fused_d1 ] && args="--fuse on --prefetch-depth 1"
    timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0 $args \
        > $out/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1) $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}' $out/${v}_$rep.log)" >&2
  done
done
