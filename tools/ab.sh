#!/bin/bash
# GPU box: A/B of library builds inside one call, alternating.  Each variant is a build of libfm_hip.so:
# "default" = fm_spark_amd/lib/libfm_hip.so, any other name = fm_spark_amd/lib/variants/<name>/libfm_hip.so
# (python -m fm_spark_amd.build --out fm_spark_amd/lib/variants/<name>/libfm_hip.so -D <MACRO>), loaded
# through FM_HIP_LIB.  Per rep, config and variant: one bench.py run; prints mean and median ms/step.
#   OUT=gpurun_out/ab VARIANTS="default x" CONFIGS="c3 c2" REPS="1 2 3" STEPS=40 BENCH_ARGS=... tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=${OUT:-gpurun_out/ab}; mkdir -p $out
for rep in ${REPS:-1 2 3}; do
  for c in ${CONFIGS:-c3}; do
    for v in ${VARIANTS:-default}; do
      lib=fm_spark_amd/lib/libfm_hip.so; [ "$v" != default ] && lib=fm_spark_amd/lib/variants/$v/libfm_hip.so
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline \
          --fit-iters 0 --host-path-steps 0 ${BENCH_ARGS:-} > $out/${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"median_ms_per_step": [0-9.]*' $out/${c}_${v}_$rep.log | tr '\n' ' ')" >&2
    done
  done
done
exit 0
