"""Llama-3-8B decode steps at batch 256, eager (one dispatch per kernel, so rocprofv3 --pmc
can attribute counters per kernel): the GEMM -> consumer pairs of a real decode step
(qkv -> rope_kv, o -> rmsnorm, gate|up, down -> rmsnorm) with their production plans.
For byte accounting of the split-K fp32 slabs:

    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum ... -- python3 tools/decode_step_pmc.py
    python3 tools/pmc_summary.py <counter_collection.csv> --grid
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.llm import GenRequest, LLMEngine  # noqa: E402
from operator_amd.models.config import get_config  # noqa: E402
from operator_amd.models.kv_cache import PagedKVCache  # noqa: E402
from operator_amd.models.llama import LlamaModel  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3-8b")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--prompt", type=int, default=512)
ap.add_argument("--steps", type=int, default=3)
ap.add_argument("--layers", type=int, default=0, help="truncate the model (0 = all layers)")
a = ap.parse_args()
cfg = get_config(a.model)
if a.layers:
    import dataclasses

    cfg = dataclasses.replace(cfg, layers=a.layers)
m = LlamaModel(cfg, device="cuda").init_random(0)
pages = PagedKVCache.pages_for_budget(int(40e9), cfg.layers, cfg.kv_heads, cfg.head_dim, 16)
kv = PagedKVCache(cfg.layers, pages, cfg.kv_heads, cfg.head_dim, 16, device="cuda")
eng = LLMEngine(m, kv, max_batch=a.batch, max_context=a.prompt + a.steps + 64, use_graphs=False,
                prefix_sharing=False)
reqs = [GenRequest([(7 * i + j) % 30000 + 1 for j in range(a.prompt)], max_tokens=a.steps + 2, temperature=0.3,
                   seed=i, ignore_eos=True) for i in range(a.batch)]
for r in reqs:
    eng.submit(r)
while eng.waiting or eng._pf is not None:
    eng.step()
torch.cuda.synchronize()
for _ in range(a.steps):
    eng.step()
torch.cuda.synchronize()
print("decode steps done", eng.stats.steps, flush=True)
