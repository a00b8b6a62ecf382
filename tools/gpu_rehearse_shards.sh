# Rehearse the multi-GPU bench topology on ONE GPU: torchrun with N ranks that share cuda:0
# (gloo for the bench's barriers), rank r = operator shard r of N, all against one REST API
# server process that rank 0 starts. Numbers are not a scaling result (ranks share a GPU).
#   bash tools/gpu_rehearse_shards.sh [N] [bench args...]
set -e
cd $GRAFT_REPO_ROOT
N=${1:-2}; shift || true
OAMD_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus $N ${@:---steps 2 --warmup 1} \
  > gpurun_out/rehearse_rest.json 2> gpurun_out/rehearse_rest.err
grep '"metric"' gpurun_out/rehearse_rest.json | tail -1 | cut -c1-1500
