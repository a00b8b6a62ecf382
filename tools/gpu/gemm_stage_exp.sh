#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k gemm_decode -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gemm_test.log 2>&1 || { tail -20 gpurun_out/gemm_test.log; exit 1; }
tail -2 gpurun_out/gemm_test.log
timeout -k 10 500 python -u tools/bench_gemm.py --m 128,256 > gpurun_out/gemm_ns4.jsonl 2>&1 || { tail -20 gpurun_out/gemm_ns4.jsonl; exit 1; }
cat gpurun_out/gemm_ns4.jsonl
