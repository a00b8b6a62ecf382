"""A/B: gemm_decode with row-major W vs W stored in [N/64][K/64][64][64] tiles
(each LDS-DMA piece a contiguous 1 KB). Same plan per shape (tuned table)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def tile(w):
    N, K = w.shape
    return w.view(N // 64, 64, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K)


def timeit(fn, wl, it=32):
    for w in wl:
        fn(w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for i in range(it):
        fn(wl[i % len(wl)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for name, (N, K) in shapes.items():
    n = max(1, min(16, -(-(1 << 30) // (N * K * 2))))
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(n)]
    wt = [tile(w) for w in ws]
    for M in (64, 128, 256):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        plan = ops.gemm_plan(M, N, K) or (min(M, 256), 128 if N >= 192 * 128 else 64, 1)
        bm, bn, S = plan
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = torch.empty(max(1, S) * M * N, device="cuda", dtype=torch.float32)
        C = ops.kernels()
        run = lambda w, t: C.gemm_decode(x, w, y, part if S > 1 else None, S, bn, bm, False, t)  # noqa: E731
        run(wt[0], True)
        err = (y.float() - F.linear(x, ws[0]).float()).abs().max().item()
        a = timeit(lambda w: run(w, False), ws)
        b = timeit(lambda w: run(w, True), wt)
        print(json.dumps({"gemm": name, "M": M, "plan": plan, "rowmajor_us": round(a, 1), "tiled_us": round(b, 1),
                          "tiled_maxerr": round(err, 4)}), flush=True)
    del ws, wt
