#!/bin/bash
# Scan tests + BASELINE config 2 (1.19 GB x 1000 patterns): kernel rate and end-to-end analyze.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/scan_test.log 2>&1 || { tail -30 gpurun_out/scan_test.log; exit 1; }
tail -1 gpurun_out/scan_test.log
timeout -k 10 300 python -u tools/bench_scan.py --docs 4096 --iters 10 --arms profiled > gpurun_out/scan_e2e.jsonl 2>&1 || { tail -20 gpurun_out/scan_e2e.jsonl; exit 1; }
grep '"bench' gpurun_out/scan_e2e.jsonl
