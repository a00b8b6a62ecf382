#!/bin/bash
# operator.sink_concurrency sweep on the flagship bench (3 timed steps each).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sink_sweep.jsonl
for sc in ${SCS:-0 8 32}; do
  timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --sink-concurrency $sc > gpurun_out/ss.log 2>&1 || { echo "bench sc=$sc failed"; tail -20 gpurun_out/ss.log; exit 1; }
  tail -1 gpurun_out/ss.log | python3 -c "import json,sys; o=json.loads(sys.stdin.read()); o['sink_concurrency']=$sc; print(json.dumps(o))" >> gpurun_out/sink_sweep.jsonl
  tail -1 gpurun_out/sink_sweep.jsonl | python3 -c "import json,sys; o=json.loads(sys.stdin.read()); print('sc', o['sink_concurrency'], o['value'], o['p50_explanation_latency_ms'])"
done
