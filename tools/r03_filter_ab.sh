#!/bin/bash
# GPU box: the singleton filter before the sort (this build) against the full sort + split of the
# saved build tools/_variants/lib_sortsplit.so: fused-step / filter tests, isolated kernels of both,
# then alternating c3 benches (new fused, old fused, new unfused with and without the filter) and
# the world-1 sharded step with and without it.  Usage: tools/r03_filter_ab.sh OUTDIR [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-filter_ab}; reps=${2:-2}
mkdir -p $out
OLD=$PWD/tools/_variants/lib_sortsplit.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py tests/test_gpu_group.py -x -q \
    --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fwd_iso.py --variants on,off > $out/iso_new.log 2>&1 || exit $?
grep '^{' $out/iso_new.log >&2
FM_HIP_LIB=$OLD timeout -k 10 200 python tools/fwd_iso.py --variants on > $out/iso_old.log 2>&1 || exit $?
grep '^{' $out/iso_old.log >&2
B="python bench.py --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0"
for rep in $(seq 1 $reps); do
  for v in new old unf_filter unf_full shard_filter shard_full; do
    lib=""; args="--fuse on"
    case $v in
      old) lib=$OLD ;;
      unf_filter) args="--fuse off --sort-filter on" ;;
      unf_full) args="--fuse off --sort-filter off" ;;
      shard_filter) args="--force-sharded --sort-filter on" ;;
      shard_full) args="--force-sharded --sort-filter off" ;;
    esac
    FM_HIP_LIB=$lib timeout -k 10 300 $B $args > $out/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1) $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}' $out/${v}_$rep.log)" >&2
  done
done
