# One GPU call: the whole GPU test tier, then a short flagship bench.
#   bash tools/gpu_check.sh [bench args...]
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
