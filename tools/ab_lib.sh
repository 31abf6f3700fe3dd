#!/bin/bash
# GPU box: alternating c3 step A/B of the default library against tools/_variants/$B (median of 40 steps;
# B may name several variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in ${REPS:-1 2 3}; do
  for v in default ${B}; do
    lib=fm_spark_amd/lib/libfm_hip.so; [ "$v" != default ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
        > gpurun_out/ab/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' gpurun_out/ab/${v}_$rep.log | tr '\n' ' ')" >&2
  done
done
