# GPU tier + short flagship benches (fresh-session health check; admission-wait A/B).
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 > gpurun_out/bench_a20.json 2> gpurun_out/bench_a20.err
tail -c 1500 gpurun_out/bench_a20.json
timeout -k 10 400 python -u bench.py --steps 3 --warmup 2 --admit-wait-ms 5 > gpurun_out/bench_a5.json 2> gpurun_out/bench_a5.err
tail -c 600 gpurun_out/bench_a5.json
timeout -k 10 300 python -u tools/bench_prefill_attn.py --variants 3,4,5,6,7 --shapes 16x1024,4x4096,mixed > gpurun_out/pattn.jsonl 2> gpurun_out/pattn.err
cat gpurun_out/pattn.jsonl
