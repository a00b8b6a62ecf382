# TP=8 simulated per-rank decode (llama3-70b fp8, B=64): timing + rocprofv3 kernel trace summary.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp8.log 2>&1 || { tail -20 gpurun_out/tp8.log; exit 1; }
grep '"bench"' gpurun_out/tp8.log
rm -rf gpurun_out/prof_tp8
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_tp8 -o run --output-format csv -- python3 tools/bench_tp.py --simulate-tp 8 --model llama3-70b --weights fp8 --batch 64 --prompt 1024 --gen 48 > gpurun_out/tp8_prof.log 2>&1
python3 tools/trace_summary.py gpurun_out/prof_tp8/run_kernel_trace.csv --out gpurun_out/tp8_trace_summary.txt --top 40
rm -f gpurun_out/prof_tp8/run_kernel_trace.csv
head -25 gpurun_out/tp8_trace_summary.txt
