"""Prefill/decode overlap on one MI355X: can a compute-bound prefill (hipBLASLt
GEMMs at M = 16k tokens) run beside the HBM-bound decode step (paged attention
over 256 x ~1.1k-token contexts) on a second HIP stream?

Times (a) N decode-graph replays alone, (b) P prefill forwards alone, (c) both
issued together on two streams (decode stream at high priority, or equal), and
prints one JSON line per arm. Llama-3-8B, random-init weights, bf16.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402
from operator_amd.engine.llm import GenRequest, LLMEngine  # noqa: E402
from operator_amd.models.config import get_config  # noqa: E402
from operator_amd.models.kv_cache import PagedKVCache  # noqa: E402
from operator_amd.models.llama import ForwardBatch  # noqa: E402
from operator_amd.models.llama import LlamaModel  # noqa: E402


def prefill_batch(eng, lens, pages_per):
    kv, dev = eng.kv, eng.device
    P = kv.page_size
    ar = [np.arange(n, dtype=np.int64) for n in lens]
    rng = np.random.default_rng(0)
    ids = np.concatenate([rng.integers(1, 120000, n) for n in lens]).astype(np.int64)
    pos = np.concatenate(ar)
    pg = [np.asarray(kv.allocator.alloc(pages_per), dtype=np.int64) for _ in lens]
    slots = np.concatenate([p[a // P] * P + a % P for p, a in zip(pg, ar)])
    cu = np.zeros(len(lens) + 1, dtype=np.int64)
    cu[1:] = np.cumsum(lens)
    var = ops.prefill_variant(eng.model.hq, eng.model.hkv)
    ws, wq = ops.prefill_work_list(lens, ops.prefill_block_q(eng.model.hq, eng.model.hkv, var))
    t = lambda x, dt=torch.long: torch.as_tensor(np.asarray(x)).to(dtype=dt).to(dev)  # noqa: E731
    work = (t(cu, torch.int32), t(ws, torch.int32), t(wq, torch.int32), var)
    return ForwardBatch(t(ids), t(pos), t(slots), True, t(cu[1:] - 1), seq_lens=lens, prefill_work=work)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=1100)
    ap.add_argument("--decode-steps", type=int, default=200)
    ap.add_argument("--prefills", type=int, default=4)
    ap.add_argument("--prefill-tokens", type=int, default=16384)
    a = ap.parse_args()
    cfg = get_config("llama3-8b")
    m = LlamaModel(cfg, device="cuda").init_random(0)
    pages = PagedKVCache.pages_for_budget(int(120e9), cfg.layers, cfg.kv_heads, 128, 64)
    kv = PagedKVCache(cfg.layers, pages, cfg.kv_heads, 128, 64, device="cuda")
    eng = LLMEngine(m, kv, max_batch=a.batch, max_context=a.ctx + a.decode_steps * 4 + 64, use_graphs=True)
    reqs = [GenRequest(list(range(1, a.ctx + 1)), max_tokens=a.decode_steps * 4, temperature=0.3, seed=i,
                       ignore_eos=True) for i in range(a.batch)]
    for r in reqs:
        eng.submit(r)
    while eng.waiting:
        eng.step()
    B = len(eng.running)
    bp = next(b for b in eng.buckets if b >= B)
    splits = ops.decode_splits(a.ctx + a.decode_steps * 4, bp, eng.hkv)
    g = eng._graph(bp, splits)
    g.st.load(eng.running, eng.max_pages)
    plen = 900
    lens = [plen] * (a.prefill_tokens // plen)
    fb = prefill_batch(eng, lens, eng.kv.pages_needed(plen))
    torch.cuda.synchronize()

    st = g.st

    def dec(n):
        # each replay appends its token to st.hist[:, st.step]: the column index must
        # wrap every multi_step replays exactly as LLMEngine._launch does
        for i in range(n):
            if i % eng.multi_step == 0:
                st.step.zero_()
            g.graph.replay()

    def pre(n):
        for _ in range(n):
            m.forward(fb, kv)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    print(json.dumps({"setup": "ok", "B": B, "bucket": bp, "splits": splits}), flush=True)
    dec(3)
    pre(1)
    td = timed(lambda: dec(a.decode_steps))
    tp = timed(lambda: pre(a.prefills))
    out = {"decode_steps": a.decode_steps, "decode_ms": round(td, 1), "decode_ms_per_step": round(td / a.decode_steps, 3),
           "prefills": a.prefills, "prefill_tokens": sum(lens) * a.prefills, "prefill_ms": round(tp, 1),
           "sum_ms": round(td + tp, 1)}
    print(json.dumps({"arm": "alone", **out}), flush=True)
    for prio in ((0, 0), (-1, 0)):
        sd = torch.cuda.Stream(priority=prio[0])
        sp = torch.cuda.Stream(priority=prio[1])
        ed, ep = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        sd.wait_event(e0)
        sp.wait_event(e0)
        with torch.cuda.stream(sp):
            pre(a.prefills)
            ep.record()
        with torch.cuda.stream(sd):
            dec(a.decode_steps)
            ed.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"arm": "concurrent", "prio_decode": prio[0], "prio_prefill": prio[1],
                          "wall_ms": round(wall, 1), "decode_done_ms": round(e0.elapsed_time(ed), 1),
                          "prefill_done_ms": round(e0.elapsed_time(ep), 1),
                          "gain_vs_serial": round((td + tp) / wall, 3)}), flush=True)


if __name__ == "__main__":
    main()
