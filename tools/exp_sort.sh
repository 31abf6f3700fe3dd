#!/bin/bash
# GPU box: sort tile-shape A/B.  Standalone sort per tools/_variants/sb_* build, then the c3 step
# per tools/_variants/lib_* library, alternating variants so box drift hits all of them alike.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sortexp
for v in ${SB:-$(cd tools/_variants && ls -d sb_* 2>/dev/null)}; do
  timeout -k 10 120 ./tools/_variants/$v/sort_bench > gpurun_out/sortexp/$v.log 2>&1 || { cat gpurun_out/sortexp/$v.log >&2; exit 1; }
  echo "== $v" >&2; grep -E "fm_hip radix_sort_pairs64|mismatches|rocprim radix_sort_pairs" gpurun_out/sortexp/$v.log >&2
  grep -q "mismatches vs rocprim (both stable): 0$" gpurun_out/sortexp/$v.log || { echo "$v: sort output differs" >&2; exit 1; }
done
for rep in 1 2 3; do
  for v in ${LIBS:-$(cd tools/_variants && ls -d lib_* 2>/dev/null)}; do
    FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline \
        > gpurun_out/sortexp/$v-$rep.log 2>&1 || { tail -5 gpurun_out/sortexp/$v-$rep.log >&2; exit 1; }
    echo "$v rep $rep: $(tail -1 gpurun_out/sortexp/$v-$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), {k: round(x["avg_ms"],4) for k, x in d.get("kernels", {}).items()})')" >&2
  done
done
exit 0
