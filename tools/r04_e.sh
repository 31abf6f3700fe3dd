#!/bin/bash
# GPU box, round 4: LSD sort by default with the tile-major counts, the bucket sort's big path
# writing the dense multi view, the owner singleton pass reading V of untagged rows only.  GPU tests,
# the fit loop's diagnosis, the sort bench, bench lines (c3 with the fit leg, c2, c5, world-1
# sharded with the fused owner step off / on), PMC passes and a kernel trace of c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_e}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_shard.py \
    tests/test_gpu_resident_fit.py tests/test_gpu_fuse.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fit_diag.py 8 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
cat $out/fit_diag.json >&2
for sk in 3 2; do
  SORT_CHECK_ONLY=1 timeout -k 10 120 ./tools/_bin_sort_bench 10223616 27 $sk > $out/sort_bench_$sk.log 2>&1
  rc=$?; grep -E "fm_hip" $out/sort_bench_$sk.log >&2; [ $rc -ne 0 ] && exit $rc
done
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
for c in c2 c5; do
  timeout -k 10 300 python bench.py $B --config $c --fit-iters 0 > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
done
for f in off on; do
  timeout -k 10 300 python bench.py $B --force-sharded --fuse $f --fit-iters 0 > $out/bench_sh1_fuse$f.log 2>&1 || exit $?
  echo "sharded1 fuse=$f $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sh1_fuse$f.log | head -1)" >&2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c3 -o run --output-format csv -- \
    python bench.py $B --fit-iters 0 --profile-kernels 0 > $out/prof_c3.log 2>&1 || exit $?
CASES="c3:default c2:default c5:default" bash tools/r04_pmc2.sh ${1:-r04_e}_pmc r04_e || exit $?
exit 0
