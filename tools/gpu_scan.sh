# One GPU call: the scan GPU tests, then BASELINE config 2 (tools/bench_scan.py, profiled arm).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/scan_tests.log 2>&1 || { tail -30 gpurun_out/scan_tests.log; exit 1; }
tail -2 gpurun_out/scan_tests.log
timeout -k 10 400 python -u tools/bench_scan.py --arms profiled --iters 20 > gpurun_out/scan_bench.jsonl
cat gpurun_out/scan_bench.jsonl
