# One GPU call: gemm_tile numerics, then the 4-wave ring (variant 1) vs the 8-wave
# 2-segment schedule (variant 2) vs hipBLASLt on the prefill shapes and the lm_head.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gemm_tile_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gt_tests.log 2>&1 || { tail -30 gpurun_out/gt_tests.log; exit 1; }
tail -2 gpurun_out/gt_tests.log
timeout -k 10 400 python -u tools/bench_gemm_tile.py --m ${GT_M:-8192,32768} --lm-m 256 --variant 2 --alt 1 --rounds 3 --out gpurun_out/gt_bench.jsonl
