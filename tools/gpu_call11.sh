set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_scan.sh
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 10,11,12,5,1 > gpurun_out/gtv2.jsonl
cat gpurun_out/gtv2.jsonl
