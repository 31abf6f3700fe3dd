#!/bin/bash
# profiles/pmc_*.json from the raw PMC passes of tools/pmc.sh (run here, on the passes merged back
# under gpurun_out/): tools/pmc_json.sh <base dir> <tag> [config:sort ...]
set -eu
cd "$(dirname "$0")/.."
base=$1; tag=$2; shift 2
for cs in "${@:-c3:default c2:default c5:default}"; do
  c=${cs%%:*}; s=${cs#*:}
  meta=$(python - $c $s "$tag" <<'PY'
import json, sys
import bench
c, s, tag = sys.argv[1:4]
F, k, B, _, _ = bench.CONFIGS[c]
fused = c == "c3"
n = int(39 * B)
g = bench.grouping(s, n, F)
print(json.dumps({"num_features": F, "k": k, "batch_rows": B, "fused": fused, "timed_steps": 5,
                  "grouping": g, "build": f"{tag} ({g} sort{', fused step' if fused else ''})",
                  "per_step": bench.step_kernels(F, n, s, fused)}))
PY
)
  g=$(echo "$meta" | python -c "import json,sys; print(json.load(sys.stdin)['grouping'])")
  f=profiles/pmc_${c}$([ $c = c3 ] && echo _fused || true)_$g.json
  python tools/pmc_to_json.py $base/${c}_$s $f "$meta"
  echo "$c $s -> $f"
done
