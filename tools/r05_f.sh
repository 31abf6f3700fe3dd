#!/bin/bash
# GPU box: c3's forward stream replayed (tools/gather_ceiling.hip) incl. the skeleton in the forward's
# 4-lane shape, with the TCC request counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_f}; mkdir -p $out
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_ceiling.hip -o /tmp/gather_ceiling > $out/build_gc.log 2>&1 || exit $?
timeout -k 10 200 python tools/c3_stream.py /tmp/c3_stream.bin > $out/c3_stream.log 2>&1 || exit $?
timeout -k 10 200 /tmp/gather_ceiling 100000000 /tmp/c3_stream.bin > $out/gather.log 2>&1 || exit $?
cat $out/gather.log >&2
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d $out/gather_pmc -o run -- \
    /tmp/gather_ceiling 100000000 /tmp/c3_stream.bin > $out/gather_pmc.log 2>&1 || exit $?
python tools/gather_ceiling.py $out/gather.log $out/gather_pmc $out/gather_ceiling.json >&2 || exit $?
exit 0
