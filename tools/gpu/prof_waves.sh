#!/bin/bash
# Kernel trace of a 4-wave pipelined bench; per-wave timeline.
set -o pipefail
mkdir -p gpurun_out/profw
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/profw -o run --output-format csv -- python3 -u bench.py --steps 4 --warmup 1 ${BENCH_ARGS:-} --json-out gpurun_out/profw_bench.json > gpurun_out/profw_bench.log 2>&1 || { echo "rocprof bench failed"; tail -30 gpurun_out/profw_bench.log; exit 1; }
f=$(find gpurun_out/profw -name '*kernel_trace.csv' | head -1)
python3 tools/wave_gaps.py "$f" --window-json gpurun_out/profw_bench.json
gzip -f "$f"; for m in $(find gpurun_out/profw -name "*marker_api_trace.csv"); do gzip -f "$m"; done
