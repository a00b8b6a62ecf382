"""Prefill attention microbenchmark: the three attn_prefill variants (v1 per-query-head,
v2 GQA-grouped 16-row waves, v3 swapped-operand 32x32 MFMA) against PyTorch SDPA on the same
packed causal batch (Llama-3-8B heads: Hq 32, Hkv 8, D 128). One JSON line per (shape, kernel).

    python tools/bench_prefill_attn.py --out gpurun_out/prefill_attn.jsonl
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="16x1024,64x256,4x4096,mixed")
ap.add_argument("--hq", type=int, default=32)
ap.add_argument("--hkv", type=int, default=8)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--out", default=None)
ap.add_argument("--variants", default="1,2,3", help="attn_prefill variants")
a = ap.parse_args()

dev = "cuda:0"
D = 128
rows = []


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


for shape in a.shapes.split(","):
    if shape == "mixed":  # prompt lengths like the bench's rendered prompts (300..1024)
        g = torch.Generator().manual_seed(0)
        lens = [int(x) for x in torch.randint(300, 1025, (24,), generator=g)]
    else:
        b, L = (int(x) for x in shape.split("x"))
        lens = [L] * b
    T = sum(lens)
    torch.manual_seed(0)
    q = torch.randn(T, a.hq, D, device=dev, dtype=torch.bfloat16)
    k = torch.randn(T, a.hkv, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(T, a.hkv, D, device=dev, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    flops = 4 * D * a.hq * sum(L * (L + 1) / 2 for L in lens)
    cu = [0]
    for L in lens:
        cu.append(cu[-1] + L)
    it = lambda x: torch.tensor(x, dtype=torch.int32, device=dev)  # noqa: E731
    o = torch.empty_like(q)
    outs = {}
    for var in tuple(int(x) for x in a.variants.split(",")):
        ws, wq = ops.prefill_work_list(lens, ops.prefill_block_q(a.hq, a.hkv, var))
        work = (it(cu), it(ws), it(wq), var)
        ms = timed(lambda: ops.attn_prefill(q, k, v, lens, scale, out=o, work=work), a.iters)
        outs[var] = o.clone()
        rows.append({"shape": shape, "tokens": T, "kernel": f"attn_prefill v{var}", "ms": round(ms, 4),
                     "tflops": round(flops / ms / 1e9, 1), "work_items": len(ws)})

    def sdpa():
        s0 = 0
        for L in lens:  # per sequence (SDPA has no packed varlen form); equal lengths use one call
            qs = q[s0:s0 + L].transpose(0, 1).unsqueeze(0)
            ks = k[s0:s0 + L].transpose(0, 1).unsqueeze(0)
            vs = v[s0:s0 + L].transpose(0, 1).unsqueeze(0)
            F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True)
            s0 += L

    def sdpa_batched():
        B, L = len(lens), lens[0]
        qs = q.view(B, L, a.hq, D).transpose(1, 2)
        ks = k.view(B, L, a.hkv, D).transpose(1, 2)
        vs = v.view(B, L, a.hkv, D).transpose(1, 2)
        F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True)

    fn = sdpa_batched if len(set(lens)) == 1 else sdpa
    ms = timed(fn, a.iters)
    rows.append({"shape": shape, "tokens": T, "kernel": "torch SDPA", "ms": round(ms, 4),
                 "tflops": round(flops / ms / 1e9, 1)})
    ref = outs.get(3)
    for var, out in outs.items():   # every variant equals v3 (the production kernel)
        if ref is not None and var != 3:
            err = (out.float() - ref.float()).abs().max().item()
            assert err < 5e-2, (shape, var, err)

for r in rows:
    print(json.dumps(r))
if a.out:
    with open(a.out, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
