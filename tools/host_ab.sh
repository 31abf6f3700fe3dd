#!/bin/bash
# GPU box: host-path (fm_step with a host CSR, PCIe-inclusive) A/B between the in-tree library and
# tools/_variants/* builds, alternating; 5 device steps each (the leg runs after them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hostab
for rep in 1 2 3; do
  for v in tree ${VARIANTS:-$(cd tools/_variants && ls)}; do
    lib=""; [ "$v" != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-path-steps 24 \
        > gpurun_out/hostab/$v-$rep.log 2>&1 || { tail -5 gpurun_out/hostab/$v-$rep.log >&2; exit 1; }
    echo "$v rep $rep: $(tail -1 gpurun_out/hostab/$v-$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["host_path_ms_per_step"], d["host_path"]["mean_ms_per_step"])')" >&2
  done
done
