#!/bin/bash
# GPU box, round 4: LSD digit width A/B -- 9/10-bit digits (this tree) against 7-bit (tools/_variants/rb7:
# 4 passes at c3, 3 at c2 / c5; 16x longer digit runs per tile) and 8-bit (rb8) -- sort benches
# checked against rocPRIM, then alternating bench reps, then one TCC pass per variant at c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_g}; mkdir -p $out
VS=${VARIANTS:-"tree rb7 rb8"}
for sk in 3 0; do
  for v in $VS; do
    bin=./tools/_bin_sort_bench; [ $v != tree ] && bin=./tools/_variants/$v/sort_bench
    SORT_CHECK_ONLY=1 timeout -k 10 120 $bin 10223616 27 $sk > $out/sort_bench_${v}_$sk.log 2>&1
    rc=$?; echo "$v skew$sk $(grep -E 'fm_hip lsd' $out/sort_bench_${v}_$sk.log) $(grep -c 'mismatches.*: 0' $out/sort_bench_${v}_$sk.log)" >&2; [ $rc -ne 0 ] && exit $rc
  done
done
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for rep in ${REPS:-1 2}; do
  for c in ${CONFIGS:-c3 c2 c5}; do
    for v in $VS; do
      lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config $c > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1) $(grep -o '"median_ms_per_step": [0-9.]*' $out/ab_${c}_${v}_$rep.log | head -1)" >&2
    done
  done
done
for v in $VS; do
  lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
  FM_HIP_LIB=$lib PMC_OUT=$out/pmc_$v BENCH_ARGS="--steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0" \
      PMC_GROUPS="TCC_HIT_sum TCC_MISS_sum" bash tools/pmc.sh || exit $?
done
exit 0
