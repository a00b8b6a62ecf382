#!/bin/bash
# CPU quota / throttling of the box's cgroup around one short bench run.
mkdir -p gpurun_out
echo "nproc=$(nproc) cpus_allowed=$(grep Cpus_allowed_list /proc/self/status)"
for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.stat; do echo "== $f"; cat $f 2>/dev/null; done
env | grep -i -E "RAYON|TOKENIZERS|OMP_NUM|MKL_NUM" 
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench_cg.log 2> gpurun_out/bench_cg.err
tail -1 gpurun_out/bench_cg.log | cut -c1-200
echo "== after"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null
