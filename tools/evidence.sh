#!/bin/bash
# GPU box, a round's closing evidence for one tree: the whole GPU suite + smoke, the driver's bench
# command, rocprofv3 kernel-trace stats of the default leg alone (every k_forward launch in the timed
# pipeline: the line's roofline is reproducible from them), and the PMC passes of c3 / c2 / c5
# (tools/pmc.sh; tools/pmc_json.sh turns them into profiles/pmc_*.json here); bench lines of c2, c5 and
# the world-1 sharded protocol, and the R = 8 owner phases (tools/shard_sim_bench.py).
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
for c in c2 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline \
      > $out/bench_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --force-sharded --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline \
    > $out/bench_sh1.log 2>&1 || exit $?
timeout -k 10 300 python tools/shard_sim_bench.py --ranks 8 --reps 2 > $out/sim8.log 2>&1 || exit $?
grep -h -o '"config": {"workload": "[^"]*\|"ms_per_step": [0-9.]*' $out/bench_c2.log $out/bench_c5.log $out/bench_sh1.log >&2
grep "owner phases" $out/sim8.log >&2
for c in c3 c2 c5; do
  PMC_OUT=$out/pmc/$c BENCH_ARGS="--config $c --steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0" \
      bash tools/pmc.sh || exit $?
done
exit 0
