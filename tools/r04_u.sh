#!/bin/bash
# GPU box, round 4 close: the driver's bench command on the final tree and rocprof's kernel-trace
# stats of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_u}; mkdir -p $out
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | head -1 | cut -c1-300 >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_default -o run --output-format csv -- \
    python bench.py > $out/prof_default.log 2>&1 || exit $?
exit 0
