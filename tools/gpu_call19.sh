set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_prefix_sharing_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "prefill or prefix" > gpurun_out/c19_tests.log 2>&1 || { tail -30 gpurun_out/c19_tests.log; exit 1; }
tail -1 gpurun_out/c19_tests.log
timeout -k 10 300 python -u tools/bench_prefill_attn.py --variants 3,4,5,6,7 --shapes 16x1024,4x4096,mixed > gpurun_out/pfa_opt.jsonl
cat gpurun_out/pfa_opt.jsonl
G=gpurun_out/gtv_shapes.jsonl
timeout -k 10 200 python -u tools/gemm_tile_variants.py --variants 1,4 --m 32768 --n 6144 --k 4096 > $G
timeout -k 10 200 python -u tools/gemm_tile_variants.py --variants 1,4 --m 32768 --n 4096 --k 4096 >> $G
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 1,4 --m 32768 --n 28672 --k 4096 --silu >> $G
timeout -k 10 300 python -u tools/gemm_tile_variants.py --variants 1,4 --m 32768 --n 4096 --k 14336 >> $G
timeout -k 10 200 python -u tools/gemm_tile_variants.py --variants 1,4 --m 8192 --n 28672 --k 4096 --silu >> $G
cat $G
