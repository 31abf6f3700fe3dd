#!/bin/bash
# GPU box: the whole GPU suite + smoke on this tree (split views, sort count without the alignment
# copy), the bench's default command, then the 256-thread chunk scan A/B at c3 / c2 / c5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05_b}; mkdir -p $out
OUT=$out/suite bash tools/gpu_suite.sh || exit $?
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | cut -c1-300 >&2
grep -o '"fit_ms_per_iter[a-z_]*": [0-9.]*\|"vs_step": [0-9.]*\|"steady_vs_step": [0-9.]*' $out/bench_default.log >&2
OUT=$out/ab VARIANTS="default scan256" CONFIGS="c3 c2 c5" REPS="1 2 3" bash tools/ab.sh || exit $?
exit 0
