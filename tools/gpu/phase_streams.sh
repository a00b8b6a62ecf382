#!/bin/bash
# Engine phase streams (prefill normal / decode high priority) with two operator shards.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_llama_gpu.py -x -q -k "pipelined" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_phase.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_phase.log; exit 1; }
tail -1 gpurun_out/pytest_phase.log
: > gpurun_out/phase_streams.jsonl
for P in "--phase-streams" ""; do
  timeout -k 10 450 python -u bench.py $P --steps 3 --warmup 1 >> gpurun_out/phase_streams.jsonl 2> gpurun_out/phase_streams.err || { echo "bench $P failed"; tail -20 gpurun_out/phase_streams.err; exit 1; }
done
cut -c1-200 gpurun_out/phase_streams.jsonl
