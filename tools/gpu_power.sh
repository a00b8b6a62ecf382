# Flagship bench with the GPU's clock / power sampled every second (rocm-smi): is the
# decode phase running at a power-limited clock?
set -e
cd $GRAFT_REPO_ROOT
( for i in $(seq 1 150); do date +%s.%N; rocm-smi -c -P -t --json 2>/dev/null || rocm-smi -c -P 2>/dev/null; sleep 1; done ) > gpurun_out/power_samples.txt 2>&1 &
mon=$!
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_power.json 2> gpurun_out/bench_power.err || { kill $mon; tail -5 gpurun_out/bench_power.err; exit 1; }
kill $mon || true
tail -c 300 gpurun_out/bench_power.json
head -c 1500 gpurun_out/power_samples.txt
