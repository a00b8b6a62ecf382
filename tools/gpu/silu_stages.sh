#!/bin/bash
# Fused gate|up+SwiGLU decode GEMM: LDS ring depth 3 vs 4 at M = 64/128 (numerics test, then timing).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "gate_up_silu or gemm_decode" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/silu_test.log 2>&1 || { tail -20 gpurun_out/silu_test.log; exit 1; }
tail -2 gpurun_out/silu_test.log
timeout -k 10 400 python -u tools/bench_gemm.py --m 64,128,256 --shapes gate_up > gpurun_out/silu_stages.jsonl 2>&1 || { tail -20 gpurun_out/silu_stages.jsonl; exit 1; }
cat gpurun_out/silu_stages.jsonl
