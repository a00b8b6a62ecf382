"""Decode-attention microbenchmark: time per call and effective HBM GB/s.

--spread S draws each sequence's context uniformly from [ctx (1 - S), ctx (1 + S)]
(the serving mix; 0 = every sequence at ctx); --shuffle scatters the page table
(pages allocated over time are not contiguous)."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--ctx", type=str, default="545,1024,2048")
ap.add_argument("--hq", type=int, default=32)
ap.add_argument("--hkv", type=int, default=8)
ap.add_argument("--page", type=int, default=64)
ap.add_argument("--splits", type=str, default="need")
ap.add_argument("--variants", type=str, default="0,2")
ap.add_argument("--pages-total", type=int, default=0)
ap.add_argument("--spread", type=float, default=0.0)
ap.add_argument("--shuffle", action="store_true")
ap.add_argument("--sort", choices=["none", "desc", "asc"], default="none",
                help="order the batch rows by context length (the engine can order its rows)")
a = ap.parse_args()
D = 128
for ctx in [int(c) for c in a.ctx.split(",")]:
    B = a.batch
    g = torch.Generator().manual_seed(0)
    lens = torch.full((B,), ctx, dtype=torch.int32)
    if a.spread > 0:
        lo, hi = int(ctx * (1 - a.spread)), int(ctx * (1 + a.spread))
        lens = torch.randint(max(1, lo), hi + 1, (B,), generator=g, dtype=torch.int32)
        if a.sort != "none":
            lens = lens.sort(descending=a.sort == "desc").values
    per = (int(lens.max()) + a.page - 1) // a.page
    total = a.pages_total or B * per + 8
    kc = torch.randn(total, a.hkv, a.page, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    order = torch.randperm(B * per, generator=g) if a.shuffle else torch.arange(B * per)
    bt = order.to(torch.int32).reshape(B, per).cuda()
    sl = lens.cuda()
    q = torch.randn(B, a.hq, D, device="cuda", dtype=torch.bfloat16)
    for sp in a.splits.split(","):
      for var in [int(x) for x in a.variants.split(",")]:
        ns = ops.decode_splits(int(lens.max()), B, a.hkv) if sp == "need" else int(sp)
        ws = ops.decode_workspace(B, a.hq, ns, "cuda")
        out = torch.empty_like(q)
        for _ in range(3):
            ops.attn_decode(q, kc, vc, bt, sl, 1 / math.sqrt(D), ns, out=out, workspace=ws, variant=var)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        n = 20
        e0.record()
        for _ in range(n):
            ops.attn_decode(q, kc, vc, bt, sl, 1 / math.sqrt(D), ns, out=out, workspace=ws, variant=var)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        byts = int(lens.sum()) * a.hkv * D * 2 * 2
        print(json.dumps({"ctx": ctx, "spread": a.spread, "sort": a.sort, "shuffle": a.shuffle, "B": B, "splits": ns, "variant": var, "us": round(us, 1),
                          "GBps": round(byts / us / 1e3, 1)}), flush=True)
    del kc, vc
