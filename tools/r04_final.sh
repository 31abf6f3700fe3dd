#!/bin/bash
# GPU box, round 4 evidence: the driver's bench command, rocprof kernel-trace stats of that same
# command, bench lines of c2 / c5 / world-1 sharded, then PMC passes (c3, c2, c5, world-1 sharded;
# tools/pmc_json.sh turns them into profiles/pmc_*.json here) -- smoke first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r04_final}; mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log >&2
timeout -k 10 400 python bench.py > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | head -1 | cut -c1-400 >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_default -o run --output-format csv -- \
    python bench.py > $out/prof_default.log 2>&1 || exit $?
B="--steps 20 --warmup 5 --no-cpu-baseline --host-path-steps 0 --fit-iters 0"
for c in c2 c5; do
  timeout -k 10 300 python bench.py $B --config $c > $out/bench_$c.log 2>&1 || exit $?
  echo "$c $(grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.log | head -1)" >&2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$c -o run --output-format csv -- \
      python bench.py $B --config $c > $out/prof_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py $B --force-sharded > $out/bench_sh1.log 2>&1 || exit $?
echo "sharded1 $(grep -o '"ms_per_step": [0-9.]*' $out/bench_sh1.log | head -1)" >&2
timeout -k 10 300 python tools/fit_diag.py 8 > $out/fit_diag.json 2> $out/fit_diag.err || exit $?
export PMC_GROUPS="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum"
A="--steps 5 --warmup 2 --no-cpu-baseline --profile-kernels 0 --host-path-steps 0 --fit-iters 0"
for c in c3 c2 c5; do
  PMC_OUT=$out/pmc/${c}_default BENCH_ARGS="--config $c $A" bash tools/pmc.sh || exit $?
done
PMC_OUT=$out/pmc/sh1 BENCH_ARGS="--config c3 --force-sharded $A" bash tools/pmc.sh || exit $?
exit 0
