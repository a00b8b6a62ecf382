#!/bin/bash
# fp8 (e4m3fn) KV cache: kernel + engine tests, then the flagship bench with the fp8
# cache and with the default bf16 cache.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fp8kv.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_fp8kv.log; exit 1; }
tail -1 gpurun_out/pytest_fp8kv.log
: > gpurun_out/bench_fp8kv.jsonl
for D in fp8 auto; do
  timeout -k 10 400 python -u bench.py --kv-dtype $D --steps 3 --warmup 1 >> gpurun_out/bench_fp8kv.jsonl 2> gpurun_out/bench_fp8kv_$D.err || { echo "bench $D failed"; tail -20 gpurun_out/bench_fp8kv_$D.err; exit 1; }
done
cut -c1-300 gpurun_out/bench_fp8kv.jsonl
