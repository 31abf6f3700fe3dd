#!/bin/bash
# GPU box: the sharded / group GPU tests, world-1 sharded and c3 bench lines (two each), then the
# c4 rank's PMC passes (tools/r03_pmc.sh, c4 only) and its bench with the traffic attached.
#   tools/r03_v7.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=${1:-r03_v7}; out=gpurun_out/$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_group.py tests/test_gpu_bench.py \
    tests/test_gpu_multirank.py -x -v -rf --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --host-path-steps 0"
for rep in 1 2; do
  for v in sharded c3; do
    args="--config $v"; [ $v = sharded ] && args="--force-sharded"
    timeout -k 10 300 $B $args > $out/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1)" \
         "$(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1)" >&2
  done
done
if [ "${C4:-1}" = "1" ]; then
  CONFIGS="" bash tools/r03_pmc.sh $name/pmc || exit $?
fi
exit 0
