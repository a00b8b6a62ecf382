# rocprofv3 kernel trace of the flagship bench, reduced on the GPU box to
#   gpurun_out/fl_trace_summary.txt  (kernel x grid: calls, total, median)
#   gpurun_out/fl_wave_gaps.jsonl    (per-wave prefill / decode spans and the GPU-idle gap before each wave)
#   gpurun_out/fl_idle.jsonl         (every GPU-idle gap of the timed window by wave phase)
#   gpurun_out/fl_window_gaps.jsonl  (idle after each token D2H copy: decode-window hand-offs)
# and the multi-GB trace deleted before gpurun copies gpurun_out/ back.
#   bash tools/profile_flagship.sh [bench args...]     (default: --steps 2 --warmup 1)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_fl
args=${@:---steps 2 --warmup 1}
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/prof_fl -o run --output-format csv -- python3 bench.py $args > gpurun_out/fl.json 2> gpurun_out/fl.err
python3 tools/trace_summary.py gpurun_out/prof_fl/run_kernel_trace.csv --out gpurun_out/fl_trace_summary.txt --top 80
python3 tools/wave_gaps.py gpurun_out/prof_fl/run_kernel_trace.csv --window-json gpurun_out/fl.json > gpurun_out/fl_wave_gaps.jsonl
python3 tools/idle_breakdown.py gpurun_out/prof_fl/run_kernel_trace.csv --window-json gpurun_out/fl.json --context 6 > gpurun_out/fl_idle.jsonl
python3 tools/window_gaps.py gpurun_out/prof_fl/run_kernel_trace.csv --window-json gpurun_out/fl.json > gpurun_out/fl_window_gaps.jsonl
rm -f gpurun_out/prof_fl/run_kernel_trace.csv
tail -c 400 gpurun_out/fl.json
