#!/bin/bash
# BASELINE configs 2, 3 and 5 on one MI355X (config 4 = bench.py).
set -o pipefail
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 500 python -u tools/bench_components.py > gpurun_out/components.jsonl 2> gpurun_out/components.err || { tail -20 gpurun_out/components.err; exit 1; }
cat gpurun_out/components.jsonl
timeout -k 10 400 python -u tools/bench_tp.py --model llama3-70b --weights fp8 --batch 16 --prompt 1024 --gen 64 > gpurun_out/tp70b.jsonl 2> gpurun_out/tp70b.err || { tail -20 gpurun_out/tp70b.err; exit 1; }
cat gpurun_out/tp70b.jsonl
