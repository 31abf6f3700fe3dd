#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass per counter group, kernel-trace only) on a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0}"
REGEX="${KREGEX:-k_segment_update|k_forward|k_radix_scatter|k_radix_count|k_radix_chunk|k_segment_combine|k_split|k_pack_srec}"
CMD="${PMC_CMD:-python bench.py $ARGS}"
GROUPS_DEFAULT=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
                "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum")
if [ -n "${PMC_GROUPS:-}" ]; then IFS=';' read -ra GROUPS_RUN <<< "$PMC_GROUPS"; else GROUPS_RUN=("${GROUPS_DEFAULT[@]}"); fi
i=0
for grp in "${GROUPS_RUN[@]}" ${EXTRA_PMC:-}; do
  i=$((i+1))
  echo "== pass $i: $grp" >&2
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" -T --output-format csv \
      -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  echo "== pass $i rc=$rc" >&2
  [ $rc -ne 0 ] && { tail -20 $OUT/p$i.log >&2; exit $rc; }
done
exit 0
