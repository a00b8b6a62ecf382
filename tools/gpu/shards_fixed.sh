#!/bin/bash
# Re-measure operator-shard configurations after the LogFactory fix (every shard and
# rank now injects signatures of the scanned library: equal work per failure).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shards_fixed.jsonl
for cfg in "--shards 2" "--shards 1" "--shards 3 --batch 384 --max-batch 384"; do
  timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 $cfg > gpurun_out/sf.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/sf.log; exit 1; }
  tail -1 gpurun_out/sf.log >> gpurun_out/shards_fixed.jsonl
  python3 -c "import json,sys; o=json.loads(open('gpurun_out/shards_fixed.jsonl').read().splitlines()[-1]); d=o['detail']; n=sum(d['outcomes'].values()); print('$cfg', o['value'], o['p50_explanation_latency_ms'], 'prompt tok/analysis', round(d['prefill_tokens_per_gpu']/n,1))"
done
