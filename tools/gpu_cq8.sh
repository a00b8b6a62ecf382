# combine_q8 with LDS-staged split statistics: numerics, TP=8 simulated decode, then the
# BASELINE config-4 shape (39 waves x 256 = 9,984 failures) on one GPU
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn_decode" --timeout 120 --timeout-method thread > gpurun_out/cq8_tests.log 2>&1 || { tail -30 gpurun_out/cq8_tests.log; exit 1; }
tail -1 gpurun_out/cq8_tests.log
timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp8_cq8.log 2>&1 || { tail -20 gpurun_out/tp8_cq8.log; exit 1; }
grep '"bench"' gpurun_out/tp8_cq8.log
timeout -k 10 900 python -u bench.py --gpus 1 --steps 39 --warmup 1 > gpurun_out/config4.json 2> gpurun_out/config4.err || { tail -5 gpurun_out/config4.err; exit 1; }
tail -c 1200 gpurun_out/config4.json
