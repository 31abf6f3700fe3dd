#!/bin/bash
# GPU box: c2 / c5 with the fused step forced on against the library's default (unfused for tables
# inside the Infinity Cache), alternating; a c5 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_e}; mkdir -p $out
for rep in 1 2 3; do
  for c in c2 c5; do
    for f in auto on; do
      timeout -k 10 300 python bench.py --config $c --steps 40 --warmup 5 --no-cpu-baseline --fit-iters 0 \
          --host-path-steps 0 --fuse $f > $out/${c}_fuse${f}_$rep.log 2>&1 || exit $?
      echo "$c fuse=$f rep=$rep $(grep -o '"ms_per_step": [0-9.]*\|"median_ms_per_step": [0-9.]*' $out/${c}_fuse${f}_$rep.log | tr '\n' ' ')" >&2
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace_c5 -o run --output-format csv -- \
    python bench.py --config c5 --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline > $out/trace_c5.log 2>&1 || exit $?
exit 0
