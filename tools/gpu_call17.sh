set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err
cut -c1-2500 gpurun_out/bench20.json
