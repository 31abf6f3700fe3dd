#!/bin/bash
# GPU box: the sharded / group / bench GPU tests, then c3, c5 and world-1 sharded bench lines (two
# each), then the PMC passes of the world-1 sharded step (owner kernels).  First failure ends it.
#   tools/r03_v6.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=${1:-r03_v6}; out=gpurun_out/$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_group.py tests/test_gpu_bench.py \
    tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -v -rf --timeout 200 --timeout-method thread \
    > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 40 --warmup 5 --no-cpu-baseline --host-path-steps 0"
for rep in 1 2; do
  for v in c3 c5 sharded; do
    args="--config $v"; [ $v = sharded ] && args="--force-sharded"
    timeout -k 10 300 $B $args > $out/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1)" \
         "$(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1)" \
         "$(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}' $out/${v}_$rep.log)" >&2
  done
done
PMC_OUT=$out/pmc_sharded1 BENCH_ARGS="--force-sharded --steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0" \
    KREGEX="k_segment_update|k_forward|k_radix_scatter|k_segment_combine|k_pack_srec|k_shard_combine|k_route_keys|k_pair_table|k_sample_mask" \
    PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;TCC_HIT_sum TCC_MISS_sum" \
    bash tools/pmc.sh || exit $?
exit 0
