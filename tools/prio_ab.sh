#!/bin/bash
# GPU box: side-stream priority x sort block shape A/B on the c3 step (3 alternating reps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prio
for rep in 1 2 3; do
  for v in ${VARIANTS:-base s256}; do
    for p in ${PRIOS:-0 1}; do
      FM_SIDE_PRIO=$p FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 300 python bench.py --steps 40 --warmup 3 \
          --no-cpu-baseline --host-path-steps 0 > gpurun_out/prio/$v-$p-$rep.log 2>&1 || { tail -5 gpurun_out/prio/$v-$p-$rep.log >&2; exit 1; }
      echo "$v prio $p rep $rep: $(tail -1 gpurun_out/prio/$v-$p-$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["median_ms_per_step"],4), {k: round(v["avg_ms"],3) for k,v in d["kernels"].items()})')" >&2
    done
  done
done
