#!/bin/bash
# GPU box: PMC passes (tools/pmc.sh) of the c3 (fused step), c2 and c5 bench lines, one directory each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
base=gpurun_out/${1:-r03_pmc}
for c in ${CONFIGS:-c3 c2 c5}; do
  PMC_OUT=$base/$c BENCH_ARGS="--config $c --steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0" \
      bash tools/pmc.sh || exit $?
  echo "== $c done" >&2
done
if [ "${C4:-1}" = "1" ]; then  # c4: one full rank (tools/c4_rank_bench.py), traffic and wait counters
  PMC_OUT=$base/c4 PMC_CMD="python tools/c4_rank_bench.py --iters 3" \
      KREGEX="k_segment_update|k_forward|k_radix_scatter|k_segment_combine|k_pack_srec|k_shard_combine" \
      PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
      bash tools/pmc.sh || exit $?
  echo "== c4 done" >&2
fi
