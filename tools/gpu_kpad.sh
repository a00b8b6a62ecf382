# prefill attention K-tile layout A/B (ab_old/: XOR-swizzled 256-B rows; tree: 272-B padded rows)
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_prefix_sharing_gpu.py -x -q -k "attn_prefill or prefix" --timeout 120 --timeout-method thread > gpurun_out/kpad_tests.log 2>&1 || { tail -30 gpurun_out/kpad_tests.log; exit 1; }
tail -1 gpurun_out/kpad_tests.log
for i in 1 2; do
  for arm in old new; do
    if [ $arm = old ]; then t=ab_old/tools/bench_prefill_attn.py; else t=tools/bench_prefill_attn.py; fi
    timeout -k 10 200 python -u $t --variants 3,4 --shapes 16x1024,4x4096,mixed > gpurun_out/kpad_${arm}_$i.jsonl 2>/dev/null
    grep -v SDPA gpurun_out/kpad_${arm}_$i.jsonl | sed "s/^/$arm $i /"
  done
done
