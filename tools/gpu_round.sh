# One GPU call: the GPU test tier, a short flagship bench, then a gemm_tile PMC pass.
#   bash tools/gpu_round.sh [bench args...]
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE" bash tools/pmc_gemm_tile.sh "1 2 blas"
cat gpurun_out/pmc_summary.txt
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants ${GTV:-1,2,3} > gpurun_out/gtv.jsonl
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants ${GTV:-1,2,3} --m 16384 --n 6144 --k 4096 >> gpurun_out/gtv.jsonl
cat gpurun_out/gtv.jsonl
