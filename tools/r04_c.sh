#!/bin/bash
# GPU box, round 4: the manual fm_shard_* tests (fused owner step with and without fusion), then the
# sort bench, the gather ceiling and the bench lines (c3 with the fit leg, world-1 sharded, c2, c5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_c}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -v --timeout 300 --timeout-method thread \
    > $out/pytest_shard.log 2>&1
rc=$?; tail -1 $out/pytest_shard.log >&2; [ $rc -gt 1 ] && exit $rc
for sk in 3 0 2; do
  SORT_CHECK_ONLY=1 timeout -k 10 120 ./tools/_bin_sort_bench 10223616 27 $sk 2>&1 | grep -E "fm_hip|rocprim|mismatch" >> $out/sort_bench.log
  rc=$?; [ $rc -gt 1 ] && exit $rc
done
cat $out/sort_bench.log >&2
timeout -k 10 120 ./tools/_bin_gather_ceiling > $out/gather.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gather -T --output-format csv \
    -d $out/gather_pmc -o run -- ./tools/_bin_gather_ceiling > $out/gather_pmc.log 2>&1 || exit $?
python tools/gather_ceiling.py $out/gather.log $out/gather_pmc $out/gather_ceiling.json >&2 || exit $?
cp $out/gather_ceiling.json profiles/gather_ceiling.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
for c in c2 c5; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline --host-path-steps 0 --fit-iters 0 \
      > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-sharded --no-cpu-baseline --host-path-steps 0 --fit-iters 0 \
    > $out/bench_sharded1.log 2>&1 || exit $?
echo "sharded1 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sharded1.log | head -1)" >&2
exit 0
