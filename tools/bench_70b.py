"""Llama-3-70B explanation decode on ONE MI355X with fp8 (e4m3fn W8A8) projection
weights — the large-model path of BASELINE config 5 (which names TP=8 over
xGMI; one 288 GB GPU holds the 70 GB of fp8 weights, so TP=1 runs here).

Random-init weights of the exact architecture; prefill of B prompts then
hipGraph decode. Prints one JSON line per batch size."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.llm import GenRequest, LLMEngine  # noqa: E402
from operator_amd.models.config import get_config  # noqa: E402
from operator_amd.models.kv_cache import PagedKVCache  # noqa: E402
from operator_amd.models.llama import LlamaModel  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3-70b")
ap.add_argument("--weights", default="fp8", choices=["fp8", "bfloat16"])
ap.add_argument("--batches", default="1,16,64")
ap.add_argument("--prompt", type=int, default=1024)
ap.add_argument("--gen", type=int, default=64)
ap.add_argument("--kv-gb", type=float, default=80.0)
a = ap.parse_args()

cfg = get_config(a.model)
t0 = time.perf_counter()
m = LlamaModel(cfg, device="cuda", weight_dtype=a.weights).init_random(0)
torch.cuda.synchronize()
init_s = time.perf_counter() - t0
pages = PagedKVCache.pages_for_budget(int(a.kv_gb * 1e9), cfg.layers, cfg.kv_heads, 128, 64)
kv = PagedKVCache(cfg.layers, pages, cfg.kv_heads, 128, 64, device="cuda")
print(json.dumps({"model": a.model, "weights": a.weights, "weight_gb": round(m.weight_bytes() / 1e9, 1),
                  "init_s": round(init_s, 1), "kv_pages": pages,
                  "hbm_allocated_gb": round(torch.cuda.memory_allocated() / 1e9, 1)}), flush=True)
for B in [int(x) for x in a.batches.split(",")]:
    eng = LLMEngine(m, kv, max_batch=B, max_context=a.prompt + a.gen + 64, use_graphs=True)
    eng.warmup([next(b for b in eng.buckets if b >= B)])
    reqs = [GenRequest(list(range(1, a.prompt + 1)), max_tokens=a.gen, temperature=0.3, seed=i, ignore_eos=True)
            for i in range(B)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in reqs:
        eng.submit(r)
    while eng.waiting:
        eng.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gen0 = sum(len(r.output) for r in reqs)
    while eng.running:
        eng.step()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    toks = sum(len(r.output) for r in reqs) - gen0
    print(json.dumps({"bench": "70b-decode", "batch": B, "prompt": a.prompt, "prefill_s": round(t1 - t0, 3),
                      "prefill_tok_s": round(B * a.prompt / (t1 - t0), 1),
                      "ms_per_token_step": round((t2 - t1) / max(toks / B, 1) * 1e3, 2),
                      "decode_tok_s": round(toks / (t2 - t1), 1)}), flush=True)
    del eng
