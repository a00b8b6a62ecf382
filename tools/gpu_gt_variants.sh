set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/gemm_tile_variants.py --variants 1,2,4,5 > gpurun_out/gtv.jsonl
timeout -k 10 200 python -u tools/gemm_tile_variants.py --variants 1,2,4,5 --m 16384 --n 6144 --k 4096 >> gpurun_out/gtv.jsonl
cat gpurun_out/gtv.jsonl
bash tools/pmc_gemm_tile.sh "4 5" && cat gpurun_out/pmc_summary.txt
