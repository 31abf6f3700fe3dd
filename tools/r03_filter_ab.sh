#!/bin/bash
# GPU box: the singleton filter before the sort (this build) against the full sort + split of the
# saved build tools/_variants/lib_sortsplit.so: fused-step tests, isolated kernels of both, then
# alternating c3 benches (new fused, old fused, new unfused).  Usage: tools/r03_filter_ab.sh OUTDIR [reps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-filter_ab}; reps=${2:-2}
mkdir -p $out
OLD=$PWD/tools/_variants/lib_sortsplit.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_fuse.py tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -3 $out/pytest.log >&2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fwd_iso.py --variants on > $out/iso_new.log 2>&1 || exit $?
grep '^{' $out/iso_new.log >&2
FM_HIP_LIB=$OLD timeout -k 10 200 python tools/fwd_iso.py --variants on > $out/iso_old.log 2>&1 || exit $?
grep '^{' $out/iso_old.log >&2
for rep in $(seq 1 $reps); do
  for v in new old new_unfused; do
    lib=""; args="--fuse on"
    [ $v = old ] && lib=$OLD
    [ $v = new_unfused ] && args="--fuse off"
    FM_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline --host-path-steps 0 \
        $args > $out/${v}_$rep.log 2>&1 || exit $?
    echo "$v rep=$rep $(grep -o '"median_ms_per_step": [0-9.]*' $out/${v}_$rep.log | head -1) $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}[^}]*}[^}]*}' $out/${v}_$rep.log)" >&2
  done
done
