#!/bin/bash
# GPU box, round 4: refilled batches grow with slack (the fit loop), the fused owner step on request
# only, and an A/B of 8192-key sort tiles on 1024-thread blocks (tools/_variants/sb1024) against the
# 4096-key tiles: GPU tests, the fit diagnosis, sort benches, bench lines (alternating reps), a
# kernel trace of c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_f}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_group.py tests/test_gpu_resident_fit.py \
    tests/test_gpu_bucket.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/fit_diag.py 8 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
python -c "import json; d=json.load(open('$out/fit_diag.json')); print({k: (v['ms_per_iter'] if isinstance(v, dict) else v) for k, v in d.items() if k != 'rows'})" >&2
for sk in 3 0; do
  for v in 512:./tools/_bin_sort_bench 1024:./tools/_variants/sb1024/sort_bench; do
    SORT_CHECK_ONLY=1 timeout -k 10 120 ${v#*:} 10223616 27 $sk > $out/sort_bench_${v%%:*}_$sk.log 2>&1
    rc=$?; echo "block=${v%%:*} $(grep -E 'fm_hip lsd' $out/sort_bench_${v%%:*}_$sk.log)" >&2; [ $rc -ne 0 ] && exit $rc
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in ${REPS:-1 2}; do
  for c in c3 c2 c5; do
    for v in t512 sb1024; do
      lib=""; [ $v = sb1024 ] && lib=tools/_variants/sb1024/libfm_hip.so
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config $c > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1)" >&2
    done
  done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 full $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
timeout -k 10 300 python bench.py $B --force-sharded > $out/bench_sh1.log 2>&1 || exit $?
echo "sharded1 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sh1.log | head -1)" >&2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c3 -o run --output-format csv -- \
    python bench.py $B --profile-kernels 0 > $out/prof_c3.log 2>&1 || exit $?
exit 0
