set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_prefix_sharing_gpu.py tests/test_llama_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t16.log 2>&1 || { tail -40 gpurun_out/t16.log; exit 1; }
tail -2 gpurun_out/t16.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench16.json 2> gpurun_out/bench16.err
cut -c1-3000 gpurun_out/bench16.json
bash tools/gpu_rehearse_shards.sh 2
