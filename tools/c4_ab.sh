set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/c4ab
FM_HIP_LIB=tools/_variants/${TESTLIB:-p8d1}/libfm_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c4ab/pytest.log 2>&1 || { tail -20 gpurun_out/c4ab/pytest.log >&2; exit 1; }
tail -1 gpurun_out/c4ab/pytest.log >&2
for rep in 1 2; do
for v in ${VARIANTS:-base d1 p8d1}; do
  FM_HIP_LIB=tools/_variants/$v/libfm_hip.so timeout -k 10 300 python -u tools/c4_rank_bench.py --iters 5 > gpurun_out/c4ab/$v-$rep.log 2>&1 || { tail -5 gpurun_out/c4ab/$v-$rep.log >&2; exit 1; }
  echo "$v $rep $(tail -1 gpurun_out/c4ab/$v-$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: round(v["avg_ms"],4) for k, v in d["phases"].items()})')" >&2
done
done
