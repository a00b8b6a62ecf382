#!/bin/bash
# Kernel + roctx marker trace of a short flagship bench run (host-side gaps analysis).
set -o pipefail
mkdir -p gpurun_out/profm
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/profm -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 --json-out gpurun_out/profm_bench.json > gpurun_out/profm_bench.log 2>&1 || { echo "rocprof bench failed"; tail -30 gpurun_out/profm_bench.log; exit 1; }
tail -1 gpurun_out/profm_bench.log
for f in $(find gpurun_out/profm -name '*_trace.csv'); do gzip -f "$f"; done
find gpurun_out/profm -name '*.csv.gz' | xargs ls -la
