#!/bin/bash
# Two engines sharing one GPU at the flagship's concurrency (2 x 128 failures in flight)
set -o pipefail
mkdir -p gpurun_out
OAMD_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${N:-2} \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus ${N:-2} --steps 3 --warmup 1 --batch ${B:-128} --max-batch ${B:-128} \
  > gpurun_out/rehearse_n${N:-2}_b${B:-128}.json 2> gpurun_out/rehearse_n${N:-2}_b${B:-128}.err || { echo "failed"; tail -30 gpurun_out/rehearse_n${N:-2}_b${B:-128}.err; exit 1; }
cat gpurun_out/rehearse_n${N:-2}_b${B:-128}.json
