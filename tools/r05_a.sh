#!/bin/bash
# GPU box, round 5 first call: the changed paths' GPU tests, the driver's bench command, rocprof stats
# of the default leg alone, c3's own gather stream, the R = 8 owner step fused / unfused, the update's
# counters with nothing beside it, and a c2 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_a}; mkdir -p $out $out/upd_iso
timeout -k 10 600 python -u -m pytest tests/test_gpu_resident_fit.py tests/test_gpu_shard.py tests/test_gpu_group.py \
    tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -1 $out/pytest_gpu.log >&2; [ $rc -ne 0 ] && { grep -E "FAILED|ERROR|Error" $out/pytest_gpu.log | head -20 >&2; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench_default.log 2>&1 || exit $?
grep '^{' $out/bench_default.log | cut -c1-400 >&2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_leg -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline > $out/prof_leg.log 2>&1 || exit $?
grep '^{' $out/prof_leg.log | cut -c1-300 >&2
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gather_ceiling.hip -o /tmp/gather_ceiling > $out/build_gc.log 2>&1 || exit $?
timeout -k 10 200 python tools/c3_stream.py /tmp/c3_stream.bin > $out/c3_stream.log 2>&1 || exit $?
timeout -k 10 200 /tmp/gather_ceiling 100000000 /tmp/c3_stream.bin > $out/gather.log 2>&1 || exit $?
cat $out/gather.log >&2
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d $out/gather_pmc -o run -- \
    /tmp/gather_ceiling 100000000 /tmp/c3_stream.bin > $out/gather_pmc.log 2>&1 || exit $?
python tools/gather_ceiling.py $out/gather.log $out/gather_pmc $out/gather_ceiling.json >&2 || exit $?
timeout -k 10 500 python tools/shard_sim_bench.py --fuse off,on --reps 3 > $out/sim8.log 2>&1 || exit $?
grep -E "R=|owner phases" $out/sim8.log >&2
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_segment_update|k_forward" -T --output-format csv \
      -d $out/upd_iso/p$i -o run -- python tools/fwd_iso.py --variants on --steps 10 > $out/upd_iso/p$i.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/fwd_iso.py --variants on --steps 10 > $out/upd_iso/plain.log 2>&1 || exit $?
cat $out/upd_iso/plain.log >&2
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/trace_c2 -o run --output-format csv -- \
    python bench.py --config c2 --steps 20 --warmup 5 --fit-iters 0 --host-path-steps 0 --no-cpu-baseline > $out/trace_c2.log 2>&1 || exit $?
grep '^{' $out/trace_c2.log | cut -c1-300 >&2
exit 0
