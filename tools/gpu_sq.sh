# silu_quantize_fp8 with compile-time slab counts: numerics + TP=8 simulated decode
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "silu_quantize or fp8" --timeout 120 --timeout-method thread > gpurun_out/sq_tests.log 2>&1 || { tail -30 gpurun_out/sq_tests.log; exit 1; }
tail -1 gpurun_out/sq_tests.log
for i in 1 2; do
timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp8_sq.log 2>&1 || { tail -20 gpurun_out/tp8_sq.log; exit 1; }
grep -o '"p50_ms_per_token": [0-9.]*' gpurun_out/tp8_sq.log
done
