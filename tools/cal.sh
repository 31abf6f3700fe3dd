#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE calibration passes for tools/traffic_cal (known byte counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cal
timeout -k 10 120 ./tools/traffic_cal > gpurun_out/cal/plain.log 2>&1 || exit $?
cat gpurun_out/cal/plain.log >&2
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -T --output-format csv -d gpurun_out/cal/p$i -o run -- ./tools/traffic_cal \
      > gpurun_out/cal/p$i.log 2>&1 || exit $?
done
exit 0
