#!/bin/bash
# Round-2 first GPU pass: gpu test tier, smoke, prefill/decode overlap experiment.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u tools/bench_pd_overlap.py > gpurun_out/pd_overlap.log 2>&1 || { echo "pd_overlap failed"; tail -30 gpurun_out/pd_overlap.log; exit 1; }
cat gpurun_out/pd_overlap.log | grep -v amdgpu.ids
