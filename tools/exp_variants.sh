#!/bin/bash
# GPU box: parity tests on the default build, then a short bench per variant in tools/_variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/var/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/var/pytest.log >&2
  [ $rc -ne 0 ] && exit $rc
fi
for v in ${VARIANTS:-$(ls tools/_variants)}; do
  FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/var/$v.log) $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}' gpurun_out/var/$v.log)" >&2
  [ $rc -ne 0 ] && exit $rc
done
exit 0
