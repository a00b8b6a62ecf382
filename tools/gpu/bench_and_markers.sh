#!/bin/bash
# Short flagship bench + a kernel/marker-traced single step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 "$@" > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash tools/gpu/prof_markers.sh
