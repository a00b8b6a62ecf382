# prefill attention v3 schedule variants; flagship kernel trace (idle + decode-window gaps); TP=8 simulated decode trace
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_prefill_attn.py --variants 3,4,5,6,7 --shapes 16x1024,4x4096,mixed > gpurun_out/pattn.jsonl 2> gpurun_out/pattn.err
cat gpurun_out/pattn.jsonl
bash tools/profile_flagship.sh --steps 2 --warmup 1
cat gpurun_out/fl_window_gaps.jsonl
head -4 gpurun_out/fl_idle.jsonl
bash tools/gpu_tp8.sh
