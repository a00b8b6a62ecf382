# Marker + kernel trace of the flagship bench, reduced on the box to the per-wave host
# timeline (gpurun_out/wave_host_timeline.jsonl); the big traces are deleted.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_mk
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d gpurun_out/prof_mk -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/mk.json 2> gpurun_out/mk.err
ls gpurun_out/prof_mk > gpurun_out/prof_mk_files.txt
python3 tools/wave_host_timeline.py --markers gpurun_out/prof_mk/run_marker_api_trace.csv --kernels gpurun_out/prof_mk/run_kernel_trace.csv > gpurun_out/wave_host_timeline.jsonl
head -c 2000 gpurun_out/prof_mk/run_marker_api_trace.csv > gpurun_out/marker_head.csv
rm -f gpurun_out/prof_mk/run_kernel_trace.csv gpurun_out/prof_mk/run_marker_api_trace.csv
