#!/bin/bash
# M=192 decode-GEMM kernels, then the flagship bench at 384 failures per GPU per step
# split over 2 shards (192-row buckets) and 3 shards (128-row buckets).
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_decode or gate_up_silu" > gpurun_out/wave_tests.log 2>&1 || { echo "kernel tests failed"; tail -30 gpurun_out/wave_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -2 gpurun_out/wave_tests.log
: > gpurun_out/wave_sweep.jsonl
for C in ${CONFIGS:-2:384 3:384}; do   # shards:failures-per-GPU-per-step
  S=${C%%:*}; B=${C##*:}
  timeout -k 10 ${TMO:-400} python -u bench.py --shards $S --batch $B --max-batch $B \
    --steps ${STEPS:-3} --warmup ${WARMUP:-1} >> gpurun_out/wave_sweep.jsonl 2> gpurun_out/wave_${S}_$B.err \
    || { echo "bench shards=$S failed"; tail -20 gpurun_out/wave_${S}_$B.err; exit 1; }
done
cut -c1-400 gpurun_out/wave_sweep.jsonl
