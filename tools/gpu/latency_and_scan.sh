#!/bin/bash
# Open-loop latency (one operator, Poisson arrivals) and BASELINE config 2 end to end,
# after the LogFactory fix (injected signatures always from the scanned library).
set -o pipefail
mkdir -p gpurun_out
( while sleep 30; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python -u tools/bench_scan.py --docs 4096 --iters 10 --arms profiled > gpurun_out/scan_e2e2.jsonl 2>&1 || { tail -20 gpurun_out/scan_e2e2.jsonl; exit 1; }
grep '"bench' gpurun_out/scan_e2e2.jsonl
timeout -k 10 700 python -u tools/bench_latency.py --rates 2,8,16,24 --seconds 30 --warmup-s 5 > gpurun_out/lat.jsonl 2> gpurun_out/lat.err || { tail -20 gpurun_out/lat.err; exit 1; }
cat gpurun_out/lat.jsonl
