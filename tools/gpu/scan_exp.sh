#!/bin/bash
# ac_scan: profiled state order vs BFS (BASELINE config 2) + GPU scan tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_scan.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_scan.log; exit 1; }
tail -3 gpurun_out/pytest_scan.log
timeout -k 10 400 python -u tools/bench_scan.py "$@" > gpurun_out/bench_scan.log 2>&1 || { echo "bench_scan failed"; tail -30 gpurun_out/bench_scan.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_scan.log
