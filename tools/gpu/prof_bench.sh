#!/bin/bash
# rocprofv3 kernel trace + stats of a short flagship bench run; summary of the timed window.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 --json-out gpurun_out/prof_bench.json > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -30 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python3 tools/prof_summary.py "$f" --window-json gpurun_out/prof_bench.json --top 40 > gpurun_out/prof_summary.txt
cp $(find gpurun_out/prof -name '*kernel_stats.csv' | head -1) gpurun_out/prof_kernel_stats.csv
gzip -c "$f" > gpurun_out/kernel_trace.csv.gz; rm -f "$f"
head -60 gpurun_out/prof_summary.txt
