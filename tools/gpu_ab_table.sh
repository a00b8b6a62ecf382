# Same-box flagship A/B: the tuned decode GEMM table vs a fewer-split-K-slabs table
# (qkv 2 slabs instead of 4, down 4 instead of 8): does less slab traffic pay in the power-bound run?
set -e
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for arm in tuned fewer; do
    if [ $arm = fewer ]; then export OAMD_GEMM_TABLE=$GRAFT_REPO_ROOT/tools/gemm_table_fewer_slabs.json; else unset OAMD_GEMM_TABLE; fi
    timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 > gpurun_out/abt_${arm}_$i.json 2> gpurun_out/abt_${arm}_$i.err || { tail -5 gpurun_out/abt_${arm}_$i.err; exit 1; }
    echo "$arm $i $(grep -o '"value": [0-9.]*' gpurun_out/abt_${arm}_$i.json) $(grep -o '"p50_explanation_latency_ms": [0-9.]*' gpurun_out/abt_${arm}_$i.json)"
  done
done
