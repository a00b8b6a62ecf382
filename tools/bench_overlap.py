"""Can decode attention (HBM-bound) and a decode GEMM (latency/MFMA-bound) share the
GPU? Times each alone and both on two streams concurrently (micro-batch overlap)."""
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

B, ctx, P, D, Hq, Hkv = 128, 1100, 64, 128, 32, 8
per = (ctx + P - 1) // P
kc = torch.randn(B * per + 8, Hkv, P, D, device="cuda", dtype=torch.bfloat16)
vc = torch.randn_like(kc)
bt = torch.arange(B * per, device="cuda", dtype=torch.int32).reshape(B, per)
sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
out = torch.empty_like(q)
ws = ops.decode_workspace(B, Hq, 1, "cuda")
M = 128
x = torch.randn(M, 4096, device="cuda", dtype=torch.bfloat16)
wl = [torch.randn(28672, 4096, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(4)]
y = torch.empty(M, 28672, device="cuda", dtype=torch.bfloat16)
n_attn, n_gemm = 20, 20


def attn():
    for _ in range(n_attn):
        ops.attn_decode(q, kc, vc, bt, sl, 1 / math.sqrt(D), 1, out=out, workspace=ws)


def gemm(kind):
    for i in range(n_gemm):
        if kind == "blas":
            F.linear(x, wl[i % 4], out=y)
        else:
            ops.kernels().gemm_decode(x, wl[i % 4], y, None, 1, 128, 128, False, False, 3)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def both(kind):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        attn()
    with torch.cuda.stream(s2):
        gemm(kind)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


for kind in ("ours", "blas"):
    ta = timed(attn)
    tg = timed(lambda: gemm(kind))
    tb = timed(lambda: both(kind))
    print(json.dumps({"gemm": kind, "attn_us": round(ta, 1), "gemm_us": round(tg, 1), "sum_us": round(ta + tg, 1),
                      "concurrent_us": round(tb, 1), "overlap_gain": round((ta + tg) / tb, 3)}), flush=True)
