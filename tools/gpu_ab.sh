# Same-box A/B/C: ab_old/ and ab_mid/ (other builds of this tree) vs the current tree,
# alternating flagship benches.
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for arm in ${ARMS:-old mid new}; do
    if [ $arm = new ]; then b=bench.py; else b=ab_$arm/bench.py; fi
    timeout -k 10 300 python -u $b --steps ${STEPS:-3} --warmup 2 > gpurun_out/ab_${arm}_$i.json 2> gpurun_out/ab_${arm}_$i.err || { tail -5 gpurun_out/ab_${arm}_$i.err; exit 1; }
    echo "$arm $i $(grep -o '"value": [0-9.]*' gpurun_out/ab_${arm}_$i.json) $(grep -o '"p50_explanation_latency_ms": [0-9.]*' gpurun_out/ab_${arm}_$i.json)"
  done
done
