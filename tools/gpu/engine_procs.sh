#!/bin/bash
# Flagship bench with the engines in 1 (in-process) or 2 engine processes per GPU.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/engine_procs.jsonl
for P in ${PROCS:-2 1}; do
  timeout -k 10 400 python -u bench.py --engine-procs $P --steps ${STEPS:-3} --warmup 1 ${EXTRA:-} >> gpurun_out/engine_procs.jsonl 2> gpurun_out/engine_procs_$P.err || { echo "bench procs=$P failed"; tail -20 gpurun_out/engine_procs_$P.err; exit 1; }
done
cut -c1-420 gpurun_out/engine_procs.jsonl
