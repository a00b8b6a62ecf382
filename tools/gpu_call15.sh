set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_rehearse_shards.sh 2
bash tools/profile_flagship.sh --steps 2 --warmup 1
