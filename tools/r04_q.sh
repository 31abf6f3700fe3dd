#!/bin/bash
# GPU box, round 4: the resident fit loop's host side -- the host thread pool at 16 threads (this
# tree) against 8 (tools/_variants/ht8): fit_diag and the bench's fit leg, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_q}; mkdir -p $out
nproc >&2; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >&2
cat /sys/fs/cgroup/cpu.max 2>/dev/null >&2 || true
for rep in 1 2; do
  for v in tree ht8; do
    lib=""; [ $v != tree ] && lib=tools/_variants/$v/libfm_hip.so
    FM_HIP_LIB=$lib timeout -k 10 300 python tools/fit_diag.py 16 > $out/fit_diag_${v}_$rep.json 2> $out/fit_diag_${v}_$rep.err || exit $?
    python -c "import json; d=json.load(open('$out/fit_diag_${v}_$rep.json')); print('$v rep$rep', {k: (round(v['ms_per_iter'], 3) if isinstance(v, dict) else v) for k, v in d.items() if k not in ('rows', 'iters')}, {k: v['host_ms_per_iter'] for k, v in d.items() if k == 'pipelined_1'})" >&2
  done
done
exit 0
