#!/bin/bash
# Decode window length (engine.multi_step) with the default two shards.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/multistep.jsonl
for M in ${MS:-16 8}; do
  timeout -k 10 450 python -u bench.py --multi-step $M --steps 3 --warmup 1 >> gpurun_out/multistep.jsonl 2> gpurun_out/multistep.err || { echo "bench $M failed"; tail -20 gpurun_out/multistep.err; exit 1; }
done
cut -c1-200 gpurun_out/multistep.jsonl
