#!/bin/bash
# Flagship bench at prefill batch sizes 32k / 16k (default) tokens.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/prefill_tokens.jsonl
for T in ${TS:-32768 16384}; do
  timeout -k 10 400 python -u bench.py --prefill-tokens $T --steps 3 --warmup 1 >> gpurun_out/prefill_tokens.jsonl 2> gpurun_out/prefill_tokens_$T.err || { echo "bench T=$T failed"; tail -20 gpurun_out/prefill_tokens_$T.err; exit 1; }
done
cut -c1-300 gpurun_out/prefill_tokens.jsonl
