#!/bin/bash
# GPU box: the round's evidence.  Every GPU step has its own time limit; the first crash / fault /
# time limit ends the script (plain test failures, pytest rc 1, do not stop the benches).
#   tools/r03_evidence.sh OUTDIR [parts]   parts: any of tests bench prof multi (default: all)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r03_ev}; parts=${2:-"tests bench prof multi"}
mkdir -p $out
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(tail -c 400 $out/$name.log | tr '\n' ' ' | cut -c1-400)" >&2
  return $rc
}
B="python bench.py --steps 20 --warmup 5"
for part in $parts; do
  case $part in
  tests)
    run pytest_gpu 1100 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
  bench)
    run bench_c3 600 $B || exit $?
    run bench_c2 300 $B --config c2 --no-cpu-baseline --host-path-steps 0 || exit $?
    run bench_c5 300 $B --config c5 --no-cpu-baseline --host-path-steps 0 || exit $? ;;
  prof)
    for c in c3 c2 c5; do
      run rocprof_$c 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_$c -o run \
          -- python bench.py --steps 20 --warmup 5 --config $c --no-cpu-baseline --host-path-steps 0 || exit $?
    done ;;
  multi)
    run bench_sharded1 300 $B --force-sharded --no-cpu-baseline --host-path-steps 0 || exit $?
    run bench_repl_c2 300 $B --config c2 --parallel replicated --no-cpu-baseline --host-path-steps 0 || exit $?
    run rocprof_sharded1 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $out/prof_sharded1 -o run \
        -- python bench.py --steps 20 --warmup 5 --force-sharded --no-cpu-baseline --host-path-steps 0 || exit $? ;;
  esac
done
exit 0
