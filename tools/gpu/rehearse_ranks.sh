#!/bin/bash
# Rehearse the driver's multi-GPU launch shape (torch.distributed.run, one process per
# rank) on a one-GPU box: N ranks share cuda:0 (OAMD_BENCH_SHARE_GPU=1, gloo timing
# collectives). Checks the rendezvous, the per-rank operators and the rank-0 JSON line.
set -o pipefail
mkdir -p gpurun_out
N=${N:-2}
OAMD_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --steps 2 --warmup 1 \
  > gpurun_out/rehearse_n$N.json 2> gpurun_out/rehearse_n$N.err || { echo "rehearsal failed"; tail -30 gpurun_out/rehearse_n$N.err; exit 1; }
cat gpurun_out/rehearse_n$N.json
