#!/bin/bash
# GPU box, round 4: A/B of the grouping sort at c3 / c2 / c5 -- the LSD passes + split ("lsd"), the
# bucket sort with 1024-thread phase-2 blocks ("b1024", this tree's library) and with 512-thread
# blocks (a build with -DFM_BKT_BB=512, tools/_variants/bb512) -- then the fused sharded owner step
# off and on at world 1; three alternating reps each (bench.py lines, 20 steps, 5 warmup).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_b}; mkdir -p $out
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
V512=tools/_variants/bb512/libfm_hip.so
ms() { echo "$(grep -o '"ms_per_step": [0-9.]*' $1 | head -1 | cut -d' ' -f2) $(grep -o '"median_ms_per_step": [0-9.]*' $1 | head -1 | cut -d' ' -f2) $(grep -o '"sort": {"avg_ms": [0-9.]*' $1 | head -1 | cut -d' ' -f3)"; }
for sk in 3 0 2; do
  timeout -k 10 120 ./tools/_variants/bb512/sort_bench 10223616 27 $sk 2>&1 | grep -E "fm_hip|mismatch" >> $out/sort_bench_512.log
  rc=$?; [ $rc -gt 1 ] && exit $rc
done
cat $out/sort_bench_512.log >&2
for rep in ${REPS:-1 2 3}; do
  for c in ${CONFIGS:-c3 c2 c5}; do
    vs="lsd b1024 b512"
    [ $c != c3 ] && vs="$vs fon"   # c2 / c5: the fused step now that the split left the main stream
    for v in $vs; do
      lib=""; srt=default; fz=auto
      [ $v = lsd ] && srt=lsd
      [ $v = b512 ] && lib=$V512
      [ $v = fon ] && fz=on
      FM_HIP_LIB=$lib timeout -k 10 300 python bench.py $B --config $c --sort $srt --fuse $fz > $out/ab_${c}_${v}_$rep.log 2>&1 || exit $?
      echo "$c $v rep$rep $(ms $out/ab_${c}_${v}_$rep.log)" >&2
    done
  done
  if [ "${SHARDED:-1}" = "1" ]; then
    for f in off on; do
      timeout -k 10 300 python bench.py $B --force-sharded --fuse $f > $out/ab_sh1_fuse${f}_$rep.log 2>&1 || exit $?
      echo "sharded1 fuse=$f rep$rep $(ms $out/ab_sh1_fuse${f}_$rep.log)" >&2
    done
  fi
done
exit 0
