#!/bin/bash
# GPU test tier + smoke + the driver's bench shape (20 timed steps, 5 warmup).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_full.log 2> gpurun_out/bench_full.err || { echo "bench failed"; tail -30 gpurun_out/bench_full.log gpurun_out/bench_full.err; exit 1; }
tail -1 gpurun_out/bench_full.log
