set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_tile" > gpurun_out/gt_tests.log 2>&1 || { tail -30 gpurun_out/gt_tests.log; exit 1; }
tail -1 gpurun_out/gt_tests.log
GT_VARIANT_EXTRA=4 timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 1,4,2 > gpurun_out/gtv4.jsonl
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 1,4,2 --m 16384 --n 6144 --k 4096 >> gpurun_out/gtv4.jsonl
cat gpurun_out/gtv4.jsonl
bash tools/profile_flagship.sh --steps 2 --warmup 1
