set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
o=gpurun_out/r05_l; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_resident_fit.py tests/test_gpu_shard.py > $o/tests.log 2>&1; rc=$?; tail -2 $o/tests.log; [ $rc -ne 0 ] && exit $rc
for v in default oldsplit base; do
  lib=fm_spark_amd/lib/libfm_hip.so; [ $v != default ] && lib=fm_spark_amd/lib/variants/$v/libfm_hip.so
  for c in c3 c5; do
    FM_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/prof_${v}_$c -o run --output-format csv -- \
      python bench.py --config $c --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline > $o/prof_${v}_$c.log 2>&1 || exit $?
  done
done
OUT=$o/ab VARIANTS="default oldsplit base" CONFIGS="c3 c5 c2" REPS="1 2 3" tools/ab.sh || exit $?
