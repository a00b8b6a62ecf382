# GPU tier + short flagship bench + prefill attention timing (session health check).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps ${STEPS:-3} --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 1500 gpurun_out/bench.json
timeout -k 10 300 python -u tools/bench_prefill_attn.py --variants 3,4 --shapes 16x1024,4x4096,mixed > gpurun_out/pattn.jsonl 2> gpurun_out/pattn.err
cat gpurun_out/pattn.jsonl
