#!/bin/bash
# GPU box, round 4: PMC passes (tools/pmc.sh, one counter group per pass) of bench lines, converted to
# profiles/pmc_*.json with the launches per step of every kernel (bench.py step_kernels) and the
# grouping sort they were counted with.  Cases: "c3:default c3:lsd c2:default c5:default" (config:sort).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
base=gpurun_out/${1:-r04_pmc2}
tag=${2:-r04}
A="--steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0"
for cs in ${CASES:-c3:default c3:lsd c2:default c5:default}; do
  c=${cs%%:*}; s=${cs#*:}
  PMC_OUT=$base/${c}_$s BENCH_ARGS="--config $c --sort $s $A" bash tools/pmc.sh || exit $?
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
) || exit $?
  f=profiles/pmc_${c}$([ $c = c3 ] && echo _fused)_$(echo "$meta" | python -c "import json,sys; print(json.load(sys.stdin)['grouping'])").json
  python tools/pmc_to_json.py $base/${c}_$s $f "$meta" || exit $?
  echo "== $c $s done -> $f" >&2
done
