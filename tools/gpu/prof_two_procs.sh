#!/bin/bash
# Kernel traces of two bench ranks sharing one GPU (2 x 128 failures in flight), one
# rocprofv3 per rank; tools/two_proc_summary.py compares kernel times and overlap.
set -o pipefail
mkdir -p gpurun_out/p2r0 gpurun_out/p2r1
export TMPDIR=/tmp OAMD_BENCH_SHARE_GPU=1 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29633
for r in 0 1; do
  ( RANK=$r LOCAL_RANK=$r timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/p2r$r -o run --output-format csv -- python3 -u bench.py --gpus 2 --steps 2 --warmup 1 --batch 128 --max-batch 128 --json-out gpurun_out/p2r${r}_bench.json > gpurun_out/p2r${r}.log 2>&1 ) &
  eval P$r=\$!
done
wait $P0 || { echo "rank0 failed"; tail -20 gpurun_out/p2r0.log; exit 1; }
wait $P1 || { echo "rank1 failed"; tail -20 gpurun_out/p2r1.log; exit 1; }
cat gpurun_out/p2r0_bench.json | head -c 600; echo
python3 tools/two_proc_summary.py gpurun_out/p2r0 gpurun_out/p2r1 --window-json gpurun_out/p2r0_bench.json > gpurun_out/two_proc_summary.txt
cat gpurun_out/two_proc_summary.txt
for f in $(find gpurun_out/p2r0 gpurun_out/p2r1 -name '*kernel_trace.csv'); do gzip -f "$f"; done
