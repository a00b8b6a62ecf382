"""Component microbenchmarks on one GPU: 8B decode step per batch bucket,
prefill tokens/s, and the log-scan GB/s. Writes JSON lines to stdout."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.llm import GenRequest, LLMEngine  # noqa: E402
from operator_amd.models.config import get_config
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import LlamaModel


def bench_llm(model_name, batches, ctx, prompt_len, max_context):
    cfg = get_config(model_name)
    m = LlamaModel(cfg, device="cuda").init_random(0)
    pages = PagedKVCache.pages_for_budget(int(60e9), cfg.layers, cfg.kv_heads, 128, 64)
    kv = PagedKVCache(cfg.layers, pages, cfg.kv_heads, 128, 64, device="cuda")
    for B in batches:
        eng = LLMEngine(m, kv, max_batch=B, max_context=max_context, use_graphs=True)
        eng.warmup([B])
        reqs = [GenRequest(list(range(1, prompt_len + 1)), max_tokens=ctx, temperature=0.3, seed=i, ignore_eos=True)
                for i in range(B)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in reqs:
            eng.submit(r)
        while eng.waiting or eng._pf is not None:   # admitted + the pipelined prefill finished
            eng.step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        n = 0
        gen0 = sum(len(r.output) for r in reqs)
        while eng.running:
            eng.step()
            n += 1
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        toks = sum(len(r.output) for r in reqs) - gen0
        print(json.dumps({"bench": "llm", "model": model_name, "batch": B, "prompt": prompt_len,
                          "prefill_s": round(t1 - t0, 4), "prefill_tok_s": round(B * prompt_len / (t1 - t0), 1),
                          "engine_steps": n, "decode_tokens": toks,
                          "ms_per_token_step": round((t2 - t1) / max(toks / B, 1) * 1e3, 3),
                          "decode_tok_s": round(toks / (t2 - t1), 1)}), flush=True)


def bench_scan(n_docs, doc_kb, n_patterns):
    from operator_amd.engine.match import MatchEngine
    from operator_amd.patterns.synth import LogFactory, synthetic_library
    ps = synthetic_library(n_patterns)
    fac = LogFactory(n_patterns=n_patterns, seed=1)
    docs, _ = fac.batch(n_docs, doc_kb * 1024, n_failures=3)
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024)
    eng.scan_gpu(docs)
    torch.cuda.synchronize()
    total = sum(map(len, docs))
    # kernel-only timing
    from operator_amd.ops import kernels
    C = kernels()
    seg = eng.last_seg
    n_segs = eng._text.numel() // seg
    tot_pad = sum(((len(d) + 1 + seg - 1) // seg) * seg for d in docs)
    ev0, ev1 = torch.cuda.Event(True), torch.cuda.Event(True)
    ev0.record()
    for _ in range(5):
        eng._count.zero_()
        C.ac_scan(eng._text[:tot_pad], seg, eng.cls_map, eng.table, eng.log2c, eng.hot_states, eng.out_off,
                  eng.out_ids, eng._matches, eng._count, eng._seg_nl, 0, eng.hot_table, eng.chain)
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 5
    t0 = time.perf_counter()
    res = eng.analyze(docs)
    t1 = time.perf_counter()
    print(json.dumps({"bench": "scan", "bytes": total, "patterns": n_patterns, "states": eng.dfa_states,
                      "kernel_ms": round(ms, 3), "kernel_GBps": round(tot_pad / ms / 1e6, 1),
                      "analyze_s": round(t1 - t0, 3), "analyses_per_s": round(len(docs) / (t1 - t0), 1),
                      "raw_matches": eng.stats.raw_matches}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batches", default="1,16,64,128,256")
    ap.add_argument("--ctx", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--max-context", type=int, default=2048)
    ap.add_argument("--scan-docs", type=int, default=4096)
    ap.add_argument("--scan-kb", type=int, default=256)
    ap.add_argument("--skip-llm", action="store_true")
    ap.add_argument("--skip-scan", action="store_true")
    a = ap.parse_args()
    if not a.skip_scan:
        bench_scan(a.scan_docs, a.scan_kb, 1000)
    if not a.skip_llm:
        bench_llm(a.model, [int(x) for x in a.batches.split(",")], a.ctx, a.prompt, a.max_context)
