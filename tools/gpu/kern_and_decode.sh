#!/bin/bash
# kernel + llama GPU tests, decode-step microbench at B=256, short flagship bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kern_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/kern_gpu.log; exit 1; }
tail -1 gpurun_out/kern_gpu.log
timeout -k 10 300 python -u tools/bench_components.py --batches 256 --prompt 1024 --skip-scan > gpurun_out/decode_b256.log 2>&1 || { echo "components failed"; tail -20 gpurun_out/decode_b256.log; exit 1; }
grep '"bench"' gpurun_out/decode_b256.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.log gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
