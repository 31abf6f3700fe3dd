#!/bin/bash
# GPU box, round 4 close (the 48-wide split scan): the whole GPU suite, smoke, the driver's bench
# command and rocprof's kernel-trace stats of the same command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_y}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20 >&2
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log >&2
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | head -1 | cut -c1-300 >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_default -o run --output-format csv -- \
    python bench.py > $out/prof_default.log 2>&1 || exit $?
exit 0
