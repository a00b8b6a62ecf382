#!/bin/bash
# Open-loop (Poisson) latency with two operator shards on one GPU: each shard process
# gets half of the offered rate; the union of their latencies is reported.
set -o pipefail
mkdir -p gpurun_out
RATES=${RATES:-12,16}   # per shard
START=$(python3 -c "import time; print(time.time() + 200)")
( while sleep 30; do date >> gpurun_out/lat_heartbeat.txt; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for i in 0 1; do
  ( timeout -k 10 700 python -u tools/bench_latency.py --rates $RATES --seconds ${SECS:-40} --warmup-s 8 --max-batch 128 --kv-gb 48 --seed $((5 + i)) --start-at $START --dump-lat gpurun_out/lat_shard$i.json > gpurun_out/lat_shard$i.log 2> gpurun_out/lat_shard$i.err ) &
  eval P$i=\$!
done
wait $P0 || { echo "shard 0 failed"; tail -20 gpurun_out/lat_shard0.err; exit 1; }
wait $P1 || { echo "shard 1 failed"; tail -20 gpurun_out/lat_shard1.err; exit 1; }
python3 - <<'PY'
import json, statistics
a, b = (json.load(open(f"gpurun_out/lat_shard{i}.json")) for i in (0, 1))
for r in a:
    lat = a[r]["lat"] + b[r]["lat"]
    lat.sort()
    span = max(a[r]["span"], b[r]["span"])
    q = lambda p: lat[min(len(lat) - 1, int(round(p / 100 * (len(lat) - 1))))]
    print(json.dumps({"bench": "open-loop latency, 2 operator shards", "offered_rate": 2 * float(r),
                      "completed": len(lat), "analyses_per_s": round(len(lat) / span, 2),
                      "p50_ms": round(statistics.median(lat) * 1e3, 1), "p90_ms": round(q(90) * 1e3, 1),
                      "p99_ms": round(q(99) * 1e3, 1)}))
PY
