set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 13,14,15,16,2 > gpurun_out/gtv3.jsonl
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 13,14,15,16,2 --m 16384 --n 6144 --k 4096 >> gpurun_out/gtv3.jsonl
cat gpurun_out/gtv3.jsonl
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE" bash tools/pmc_gemm_tile.sh "13"
cat gpurun_out/pmc_summary.txt
