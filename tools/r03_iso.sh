#!/bin/bash
# GPU box: the fused-step tests, then the step's kernels in isolation (tools/fwd_iso.py) and the
# c3 step A/B fused / unfused.  Usage: tools/r03_iso.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-iso}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fwd_iso.py > $out/iso.log 2>&1 || exit $?
grep '^{' $out/iso.log >&2
for v in on off; do
  timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0 --fuse $v \
      > $out/bench_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"median_ms_per_step": [0-9.]*' $out/bench_$v.log) $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}' $out/bench_$v.log)" >&2
done
