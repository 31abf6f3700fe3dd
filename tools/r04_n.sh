#!/bin/bash
# GPU box, round 4: the driver's bench command twice (the fit leg's spread), then fit_diag.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_n}; mkdir -p $out
for rep in 1 2; do
  timeout -k 10 400 python bench.py > $out/bench_default_$rep.log 2>&1 || exit $?
  echo "rep$rep $(grep -o '"ms_per_step": [0-9.]*' $out/bench_default_$rep.log | head -1) $(grep -o '"fit_ms_per_iter": [0-9.]*' $out/bench_default_$rep.log | head -1) $(grep -o '"fit_ms_per_iter_steady": [0-9.]*' $out/bench_default_$rep.log | head -1)" >&2
done
timeout -k 10 300 python tools/fit_diag.py 16 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
python -c "import json; d=json.load(open('$out/fit_diag.json')); print({k: (v['ms_per_iter'] if isinstance(v, dict) else v) for k, v in d.items() if k != 'rows'})" >&2
exit 0
