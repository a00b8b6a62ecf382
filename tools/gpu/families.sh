#!/bin/bash
# New-family kernels (prefill v3 / decode for GQA groups 3, 5, 6, 7; q/k/v bias) and
# the flagship pipeline bench on Qwen2.5-7B and Mistral-7B (random-init, bf16).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_llama_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_families.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_families.log; exit 1; }
tail -1 gpurun_out/pytest_families.log
: > gpurun_out/bench_families.jsonl
for m in qwen2.5-7b mistral-7b; do
  timeout -k 10 400 python -u bench.py --model $m --steps 2 --warmup 1 >> gpurun_out/bench_families.jsonl 2> gpurun_out/bench_$m.err || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.err; exit 1; }
done
cat gpurun_out/bench_families.jsonl
