set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_prefix_sharing_gpu.py tests/test_llama_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t16.log 2>&1 || { tail -40 gpurun_out/t16.log; exit 1; }
tail -2 gpurun_out/t16.log
for args in "" "--no-prefix-sharing" "--page-size 16" "--page-size 32"; do
  timeout -k 10 400 python -u bench.py --steps 4 --warmup 2 $args > gpurun_out/b16.json 2> gpurun_out/b16.err
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/b16.json').read().strip().splitlines()[-1])
print(json.dumps({'args': sys.argv[1], 'value': d['value'], 'p50_ms': d['p50_explanation_latency_ms'], 'prompt_tok': d['detail']['prompt_tokens_per_analysis'], 'prefill_tok': d['detail']['prefill_tokens_per_gpu'], 'shared': d['detail'].get('shared_prefix'), 'eager': d['detail']['prefill_eager_batches']}))" "$args" | tee -a gpurun_out/b16_ab.jsonl
done
bash tools/gpu_rehearse_shards.sh 2
