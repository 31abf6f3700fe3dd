set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_tuning.py -x -v -s --timeout 600 --timeout-method thread > gpurun_out/tuning.log 2>&1 || { tail -30 gpurun_out/tuning.log; exit 1; }
tail -3 gpurun_out/tuning.log
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --host-path-steps 0 > gpurun_out/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --force-sharded --no-cpu-baseline > gpurun_out/bench_sharded.log 2>&1 || exit 1
bash tools/pmc.sh && VARIANTS="base nos" bash tools/abl_pmc.sh
