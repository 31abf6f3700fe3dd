#!/bin/bash
# GPU box, round 4: the select kernel over a flat entry range (this tree) against the 16-lane team
# per row (tools/_variants/prev): the resident-fit GPU tests, fit_diag alternating, a rocprof kernel
# trace of fit_diag for the select kernel's time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_r}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident_fit.py -x -v --timeout 300 --timeout-method thread \
    > $out/pytest.log 2>&1
rc=$?; tail -1 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in tree prev; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python tools/fit_diag.py 16 > $out/fit_diag_${v}_$rep.json 2> $out/fit_diag_${v}_$rep.err || exit $?
    python -c "import json; d=json.load(open('$out/fit_diag_${v}_$rep.json')); print('$v rep$rep', {k: (round(v['ms_per_iter'], 3) if isinstance(v, dict) else v) for k, v in d.items() if k not in ('rows', 'iters')})" >&2
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_fit -o run --output-format csv -- \
    python tools/fit_diag.py 16 > $out/prof_fit.log 2>&1 || exit $?
exit 0
