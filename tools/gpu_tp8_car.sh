# TP=8 simulated per-rank decode (llama3-70b fp8, B=64): one-shot AR+RMSNorm workgroups 32 vs 64.
set -e
cd $GRAFT_REPO_ROOT
for nb in 32 64; do
  OAMD_CAR_BLOCKS=$nb timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp_car$nb.log 2>&1 || { tail -20 gpurun_out/tp_car$nb.log; exit 1; }
  echo "car_blocks $nb $(grep -o '"p50_ms_per_token": [0-9.]*' gpurun_out/tp_car$nb.log)"
done
