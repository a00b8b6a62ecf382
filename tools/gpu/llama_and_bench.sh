#!/bin/bash
# llama GPU tests, a short bench, then a kernel/marker-traced bench step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_llama_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/llama_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/llama_gpu.log; exit 1; }
tail -1 gpurun_out/llama_gpu.log
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.log gpurun_out/bench.err; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-330
bash tools/gpu/prof_markers.sh > /dev/null && python3 tools/trace_phases.py gpurun_out/profm/run_kernel_trace.csv.gz --window-json gpurun_out/profm_bench.json --gaps 100
