#!/bin/bash
# Flagship bench with 2 operator shards per GPU vs 1 (256 failures per GPU per step either way).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shards.jsonl
for S in ${SHARDS:-2 1}; do
  timeout -k 10 ${TMO:-500} python -u bench.py --shards $S --steps ${STEPS:-3} --warmup ${WARMUP:-1} >> gpurun_out/shards.jsonl 2> gpurun_out/shards_$S.err || { echo "bench shards=$S failed"; tail -20 gpurun_out/shards_$S.err; exit 1; }
done
cut -c1-330 gpurun_out/shards.jsonl
