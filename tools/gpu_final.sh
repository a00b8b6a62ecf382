# Round-end rehearsal: GPU tier, smoke(), and the driver-shaped 20-step flagship bench.
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARM:-5} > gpurun_out/bench20.json 2> gpurun_out/bench20.err || { tail -20 gpurun_out/bench20.err; exit 1; }
tail -c 2500 gpurun_out/bench20.json
