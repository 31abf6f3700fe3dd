PROF=1 BENCH_ARGS=--no-cpu-baseline bash tools/gpu_round.sh && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --features 1000000 > gpurun_out/bench_f1m.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --features 10000000 > gpurun_out/bench_f10m.log 2>&1
