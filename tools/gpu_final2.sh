# End-of-session check: GPU tier, smoke(), flagship bench, TP=8 simulated decode.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp8_final.log 2>&1 || { tail -20 gpurun_out/tp8_final.log; exit 1; }
grep '"bench"' gpurun_out/tp8_final.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-5} --warmup ${WARM:-2} > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
tail -c 1600 gpurun_out/bench_final.json
