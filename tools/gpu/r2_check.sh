#!/bin/bash
# GPU test tier + smoke + config-2 scan + short flagship bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for docs in 4096 256; do
  timeout -k 10 120 python -u tools/bench_scan.py --docs $docs --iters 10 --arms profiled > gpurun_out/scan_$docs.log 2>&1 || { echo "scan failed"; tail -20 gpurun_out/scan_$docs.log; exit 1; }
  grep '"bench"' gpurun_out/scan_$docs.log
done
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
