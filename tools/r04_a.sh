#!/bin/bash
# GPU box, round 4 first pass: the changed GPU tests (fused flush fix, bucket sort, resident fit, fused
# sharded owner step), the random-gather request ceiling (tools/gather_ceiling.hip + one TCC PMC pass),
# then the driver's bench command, the world-1 sharded line and a rocprof kernel-stats pass of c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_a}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_fuse.py tests/test_gpu_resident_fit.py \
    tests/test_gpu_ml.py tests/test_gpu_group.py tests/test_gpu_shard.py -x -v \
    --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for sk in 3 0 2; do
  SORT_CHECK_ONLY=1 timeout -k 10 120 ./tools/_bin_sort_bench 10223616 27 $sk >> $out/sort_bench.log 2>&1
  rc=$?; [ $rc -gt 1 ] && exit $rc
done
grep -E "ms|mismatch" $out/sort_bench.log >&2
timeout -k 10 120 ./tools/_bin_gather_ceiling > $out/gather.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gather -T --output-format csv \
    -d $out/gather_pmc -o run -- ./tools/_bin_gather_ceiling > $out/gather_pmc.log 2>&1 || exit $?
python tools/gather_ceiling.py $out/gather.log $out/gather_pmc $out/gather_ceiling.json >&2 || exit $?
cp $out/gather_ceiling.json profiles/gather_ceiling.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-sharded --no-cpu-baseline --host-path-steps 0 \
    > $out/bench_sharded1.log 2>&1 || exit $?
echo "sharded1 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sharded1.log | head -1)" >&2
for c in c2 c5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline --host-path-steps 0 --fit-iters 0 \
      > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_c3 -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0 > $out/prof_c3.log 2>&1 || exit $?
exit 0
