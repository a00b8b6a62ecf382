#!/bin/bash
# ac_scan: scan GPU tests, then BASELINE config 2 (1.19 GB x 1000 patterns) for v2 (BFS / profiled
# state order) and v1, at 1.19 GB and 70 MB of text.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/scan_sweep.jsonl
: > $out
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_scan.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_scan.log; exit 1; }
tail -1 gpurun_out/pytest_scan.log
for v in v2 v1; do for docs in 4096 256; do
  OAMD_SCAN=$v timeout -k 10 120 python -u tools/bench_scan.py --docs $docs --iters 10 > gpurun_out/sweep_one.log 2>&1 || { echo "run $v failed"; tail -20 gpurun_out/sweep_one.log; exit 1; }
  grep '"bench"' gpurun_out/sweep_one.log | sed "s/^{/{\"kernel\": \"$v\", /" >> $out
done; done
python3 -c "
import json
for l in open('$out'):
    d=json.loads(l); print(d['kernel'], d['arm'], d['bytes']//2**20, 'MiB', d['kernel_ms'], 'ms', d['kernel_GBps'], 'GB/s', d['raw_matches'], d['same_matches_as_first_arm'], 'analyze', d['analyze_s'])
"
