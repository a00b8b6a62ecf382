#!/bin/bash
# bench.py knob sweep on one GPU; one JSON line per variant in gpurun_out/sweep.jsonl
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sweep.jsonl
for args in "$@"; do
  timeout -k 10 400 python -u bench.py $args > gpurun_out/sweep_one.log 2>&1 || { echo "FAILED: $args"; tail -5 gpurun_out/sweep_one.log; exit 1; }
  echo "{\"args\": \"$args\", \"result\": $(tail -1 gpurun_out/sweep_one.log)}" >> gpurun_out/sweep.jsonl
  python -c "import json;d=json.loads(open('gpurun_out/sweep.jsonl').read().splitlines()[-1]);r=d['result'];print(d['args'],r['value'],r['p50_explanation_latency_ms'])"
done
