#!/bin/bash
# GPU box, round 4: the fit loop with splits gathered two iterations ahead (fit_diag + the bench
# leg), the R = 8 sharded shapes simulated on one GPU (tools/shard_sim_bench.py), and c4's rank 0 at
# full size (tools/c4_rank_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_k}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident_fit.py -x -v --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fit_diag.py 8 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
python -c "import json; d=json.load(open('$out/fit_diag.json')); print({k: (v['ms_per_iter'] if isinstance(v, dict) else v) for k, v in d.items() if k != 'rows'})" >&2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
timeout -k 10 400 python -u tools/shard_sim_bench.py --ranks 8 > $out/sim8.log 2>&1 || exit $?
tail -12 $out/sim8.log >&2
timeout -k 10 600 python -u tools/c4_rank_bench.py --iters 5 > $out/c4_bench.log 2>&1 || exit $?
tail -6 $out/c4_bench.log >&2
exit 0
