#!/bin/bash
# GPU box, a round's closing evidence for one tree: the whole GPU suite + smoke, the driver's bench
# command, rocprofv3 kernel-trace stats of the default leg alone (every k_forward launch in the timed
# pipeline: the line's roofline is reproducible from them), and the PMC passes of c3 / c2 / c5
# (tools/pmc.sh; tools/pmc_json.sh turns them into profiles/pmc_*.json here).
#   tools/evidence.sh <out name> [skip-suite]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-evidence}; mkdir -p $out
if [ "${2:-}" != skip-suite ]; then
  OUT=$out/suite bash tools/gpu_suite.sh || exit $?
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | cut -c1-300 >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_leg -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline > $out/prof_leg.log 2>&1 || exit $?
grep '^{' $out/prof_leg.log | cut -c1-200 >&2
for c in c3 c2 c5; do
  PMC_OUT=$out/pmc/$c BENCH_ARGS="--config $c --steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0" \
      bash tools/pmc.sh || exit $?
done
exit 0
