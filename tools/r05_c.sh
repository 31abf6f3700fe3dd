#!/bin/bash
# GPU box: the multi-GPU tests after the fused owner step's removal, the bench's default command, and
# c4's owner slot sort (28-bit slots) with the LSD passes against the bucket sort, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_c}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_shard.py -x -v --timeout 300 \
    --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | cut -c1-300 >&2
for rep in 1 2; do
  for s in lsd bucket; do
    timeout -k 10 600 python -u tools/c4_rank_bench.py --iters 5 --sort $s > $out/c4_${s}_$rep.log 2>&1 || exit $?
    grep '^{' $out/c4_${s}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$s', $rep, {k: round(v['avg_ms'], 3) for k, v in d['phases'].items()})" >&2
  done
done
exit 0
