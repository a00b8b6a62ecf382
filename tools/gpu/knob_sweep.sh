#!/bin/bash
# Flagship bench knob sweep (3 timed steps each): decode window length, prefill batch size.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/knobs.jsonl
for arm in "" "--multi-step 16" "--prefill-tokens 65536" "--multi-step 4"; do
  timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 $arm > gpurun_out/kn.log 2>&1 || { echo "bench $arm failed"; tail -20 gpurun_out/kn.log; exit 1; }
  tail -1 gpurun_out/kn.log | python3 -c "import json,sys; o=json.loads(sys.stdin.read()); print(json.dumps({'arm': '$arm' or 'default', 'value': o['value'], 'p50_ms': o['p50_explanation_latency_ms']}))" | tee -a gpurun_out/knobs.jsonl
done
