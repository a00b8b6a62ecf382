#!/bin/bash
# Driver-shaped flagship bench (20 timed / 5 warmup steps, default shape), then a
# rocprofv3 kernel trace + stats of a short default run (both operator shards'
# processes are traced: the child shard inherits the profiler).
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/bench20.json > gpurun_out/bench20.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench20.log; exit 1; }
tail -1 gpurun_out/bench20.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 -u bench.py --steps 2 --warmup 1 --json-out gpurun_out/prof_bench.json > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof bench failed"; tail -30 gpurun_out/prof_bench.log; exit 1; }
tail -1 gpurun_out/prof_bench.log
python3 tools/two_proc_summary.py $(find gpurun_out/prof -name '*kernel_trace.csv') --window-json gpurun_out/prof_bench.json --top 16 > gpurun_out/prof_summary.txt
i=0; for f in $(find gpurun_out/prof -name '*kernel_stats.csv'); do cp "$f" gpurun_out/prof_kernel_stats_$i.csv; i=$((i+1)); done
for f in $(find gpurun_out/prof -name '*.csv'); do rm -f "$f"; done
cat gpurun_out/prof_summary.txt
