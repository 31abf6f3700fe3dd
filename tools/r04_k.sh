#!/bin/bash
# GPU box, round 4: the sort's count and level-1 scan in one kernel (A/B against the two-kernel
# build, tools/_variants/cc0; sort benches checked against rocPRIM), the fit loop with splits
# gathered two iterations ahead (fit_diag + the bench leg), the R = 8 sharded shapes simulated on one
# GPU (tools/shard_sim_bench.py), and c4's rank 0 at full size (tools/c4_rank_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_k}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident_fit.py tests/test_gpu_parity.py tests/test_gpu_bucket.py \
    tests/test_gpu_fuse.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for sk in 3 0 2; do
  for v in tree:./tools/_bin_sort_bench cc0:./tools/_variants/cc0/sort_bench; do
    SORT_CHECK_ONLY=1 timeout -k 10 120 ${v#*:} 10223616 27 $sk > $out/sort_bench_${v%%:*}_$sk.log 2>&1
    rc=$?; echo "${v%%:*} skew$sk $(grep -E 'fm_hip lsd' $out/sort_bench_${v%%:*}_$sk.log) $(grep -c 'mismatches.*: 0' $out/sort_bench_${v%%:*}_$sk.log)" >&2; [ $rc -ne 0 ] && exit $rc
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in 1 2; do
  for c in c3 c2 c5; do
    for v in tree cc0; do
      lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config $c > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1)" >&2
    done
  done
done
timeout -k 10 300 python tools/fit_diag.py 8 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
python -c "import json; d=json.load(open('$out/fit_diag.json')); print({k: (v['ms_per_iter'] if isinstance(v, dict) else v) for k, v in d.items() if k != 'rows'})" >&2
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 > $out/bench_c3.log 2>&1 || exit $?
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_c3.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_c3.log | head -1)" >&2
timeout -k 10 400 python -u tools/shard_sim_bench.py --ranks 8 > $out/sim8.log 2>&1 || exit $?
tail -12 $out/sim8.log >&2
exit 0
