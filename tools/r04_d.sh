#!/bin/bash
# GPU box, round 4: the bucket sort with the multi-block big path -- its GPU tests, the sort bench
# (checked against rocPRIM) on c3-like / hot / one-key-dominated keys, then bench lines at c3
# (bucket and LSD, with the fit leg), c2, c5 and world-1 sharded, and a kernel trace of c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_d}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread \
    > $out/pytest_bucket.log 2>&1
rc=$?; tail -1 $out/pytest_bucket.log >&2; [ $rc -ne 0 ] && exit $rc
for sk in 3 0 2; do
  for v in 512:./tools/_bin_sort_bench 1024:./tools/_variants/bb1024/sort_bench; do
    SORT_CHECK_ONLY=1 timeout -k 10 120 ${v#*:} 10223616 27 $sk > $out/sort_bench_${v%%:*}_$sk.log 2>&1
    rc=$?; echo "bb=${v%%:*}" >&2; grep -E "fm_hip|mismatch" $out/sort_bench_${v%%:*}_$sk.log >&2; [ $rc -ne 0 ] && exit $rc
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0"
for c in c3 c2 c5; do
  for s in default lsd bb1024; do
    fi=0; [ $c = c3 ] && [ $s = default ] && fi=8
    lib=""; srt=$s; [ $s = bb1024 ] && lib=tools/_variants/bb1024/libfm_hip.so && srt=default
    FM_HIP_LIB=$lib timeout -k 10 400 python bench.py $B --config $c --sort $srt --fit-iters $fi > $out/bench_${c}_$s.log 2>&1 || exit $?
    echo "$c $s $(grep -o '"ms_per_step": [0-9.]*' $out/bench_${c}_$s.log | head -1) $(grep -o '"sort": {"avg_ms": [0-9.]*' $out/bench_${c}_$s.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_${c}_$s.log | head -1)" >&2
  done
done
for f in off on; do
  timeout -k 10 300 python bench.py $B --force-sharded --fuse $f --fit-iters 0 > $out/bench_sh1_fuse$f.log 2>&1 || exit $?
  echo "sharded1 fuse=$f $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sh1_fuse$f.log | head -1)" >&2
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_c3 -o run --output-format csv -- \
    python bench.py $B --fit-iters 0 --profile-kernels 0 > $out/prof_c3.log 2>&1 || exit $?
exit 0
