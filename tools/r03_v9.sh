#!/bin/bash
# GPU box: the fused-step and parity tests, two c3 bench lines, the R = 8 shard simulation, the
# fused c3 PMC passes.   tools/r03_v9.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=${1:-r03_v9}; out=gpurun_out/$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_bench.py -x -v -rf \
    --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --host-path-steps 0 > $out/c3_$rep.log 2>&1 || exit $?
  echo "c3 rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $out/c3_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/c3_$rep.log | head -1)" >&2
done
timeout -k 10 300 python tools/shard_sim_bench.py --ranks 8 > $out/sim8.log 2>&1 || exit $?
tail -6 $out/sim8.log >&2
CONFIGS="c3" C4=0 bash tools/r03_pmc.sh $name/pmc || exit $?
exit 0
