#!/bin/bash
# GPU-side concurrency across processes: decode-step graph replays (C++ launch, no
# host load) of one B=256 engine vs two B=128 engines in two processes at once.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/procs_decode.jsonl
timeout -k 10 200 python -u tools/bench_graph_contention.py --batch 256 --steps 400 >> gpurun_out/procs_decode.jsonl 2>gpurun_out/procs_decode_a.err || exit 1
timeout -k 10 200 python -u tools/bench_graph_contention.py --batch 128 --steps 400 >> gpurun_out/procs_decode.jsonl 2>gpurun_out/procs_decode_b.err || exit 1
( timeout -k 10 300 python -u tools/bench_graph_contention.py --batch 128 --steps 400 --sync-start 2 > gpurun_out/pd_p0.json 2>gpurun_out/pd_p0.err ) &
P0=$!
( timeout -k 10 300 python -u tools/bench_graph_contention.py --batch 128 --steps 400 --sync-start 2 > gpurun_out/pd_p1.json 2>gpurun_out/pd_p1.err ) &
P1=$!
wait $P0 || exit 1
wait $P1 || exit 1
cat gpurun_out/procs_decode.jsonl gpurun_out/pd_p0.json gpurun_out/pd_p1.json
