#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_order.log
for args in "--spread 0" "--spread 0 --shuffle" "--spread 0.45" "--spread 0.45 --shuffle" "--spread 0.45 --shuffle --sort desc" "--spread 0.45 --shuffle --sort asc"; do
  timeout -k 10 120 python -u tools/bench_attn.py --ctx 1100 --splits 1 --variants 0 $args >> gpurun_out/attn_order.log 2>&1 || { echo "failed: $args"; tail -5 gpurun_out/attn_order.log; exit 1; }
done
grep ctx gpurun_out/attn_order.log
