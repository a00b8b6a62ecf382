#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "skinny or gate_up_silu or gemm_decode" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/skinny_test.log 2>&1 || { tail -30 gpurun_out/skinny_test.log; exit 1; }
tail -2 gpurun_out/skinny_test.log
cp operator_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
timeout -k 10 500 python -u tools/bench_skinny.py --write-table gpurun_out/gemm_tuned.json > gpurun_out/skinny.jsonl 2>&1 || { tail -20 gpurun_out/skinny.jsonl; exit 1; }
cat gpurun_out/skinny.jsonl
