#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cp operator_amd/ops/gemm_tuned.json gpurun_out/gemm_tuned.json
timeout -k 10 500 python -u tools/bench_skinny.py --write-table gpurun_out/gemm_tuned.json > gpurun_out/skinny.jsonl 2>&1 || { tail -20 gpurun_out/skinny.jsonl; exit 1; }
grep per_step gpurun_out/skinny.jsonl
cp gpurun_out/gemm_tuned.json operator_amd/ops/gemm_tuned.json
PYTHONPATH=$PWD timeout -k 10 300 python -u tools/bench_components.py --skip-scan --batches 1,4,16,32 --ctx 128 > gpurun_out/components_small.jsonl 2> gpurun_out/components.err || { tail -20 gpurun_out/components.err; exit 1; }
cat gpurun_out/components_small.jsonl
