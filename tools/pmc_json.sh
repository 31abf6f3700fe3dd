#!/bin/bash
# profiles/pmc_*.json from the raw PMC passes of tools/pmc.sh (run here, on the passes merged back
# under gpurun_out/): tools/pmc_json.sh <base dir> <tag> [config ...]  (passes in <base dir>/<config>)
set -eu
cd "$(dirname "$0")/.."
base=$1; tag=$2; shift 2
for c in ${@:-c3 c2 c5}; do
  meta=$(python - $c "$tag" <<'PY'
import json, sys
import bench
c, tag = sys.argv[1:3]
F, k, B, _, _ = bench.CONFIGS[c]
fused = c == "c3"
print(json.dumps({"num_features": F, "k": k, "batch_rows": B, "fused": fused, "timed_steps": 5,
                  "grouping": "lsd", "build": f"{tag} (lsd sort{', fused step' if fused else ''})",
                  "per_step": bench.step_kernels(F, fused)}))
PY
)
  f=profiles/pmc_${c}$([ $c = c3 ] && echo _fused || true)_lsd.json
  python tools/pmc_to_json.py $base/$c $f "$meta"
  echo "$c -> $f"
done
