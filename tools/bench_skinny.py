"""Small-bucket decode GEMMs (M <= 32): gfx950 gemm_skinny (every split count, and the
fused gate|up + SwiGLU) vs hipBLASLt, on the Llama-3-8B projection shapes. Weights
rotate through >= 1 GB of copies so nothing is served from the 256 MB MALL.

--write-table merges the winners into operator_amd/ops/gemm_tuned.json as
``skinny,M,N,K -> S | "blas"`` and ``silu,M,N,K -> [0] | "blas"``."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402
from operator_amd.ops import kernels  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", default="1,2,4,8,16,32")
ap.add_argument("--model", default="8b", choices=["8b", "70b"])
ap.add_argument("--write-table", default=None)
a = ap.parse_args()
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
if a.model == "70b":
    shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
              "lm_head": (128256, 8192)}
ws = {k: [torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02
          for _ in range(max(1, min(16, -(-(1 << 30) // (n * kk * 2)))))] for k, (n, kk) in shapes.items()}


def timeit(fn, wl, it=48):
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


DEFERRED = ("o", "down")  # models/llama.py: defer=True projections (split-K slabs summed by rmsnorm)
table = {}
for M in [int(x) for x in a.m.split(",")]:
    tot = {"hipblaslt": 0.0, "best": 0.0}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        mult = 1 if name == "lm_head" else 32
        res = {"hipblaslt": timeit(lambda w: F.linear(x, w), ws[name])}
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        part = torch.empty(8 * M * N, device="cuda", dtype=torch.float32)
        ref = F.linear(x, ws[name][0]).float()
        for S in (1, 2, 4, 8):
            if K % (128 * S):
                continue
            kernels().gemm_skinny(x, ws[name][0], y, part if S > 1 else None, S, False)
            err = (y.float() - ref).abs().max().item()
            if err > 0.1:
                print("BAD", name, M, S, err, flush=True)
                continue
            # o / down hand their slabs to the next rmsnorm in the model: no reduce kernel
            yy = None if (S > 1 and name in DEFERRED) else y
            res[f"s{S}"] = timeit(lambda w: kernels().gemm_skinny(x, w, yy, part if S > 1 else None, S, False),
                                  ws[name])
        best = min(res, key=res.get)
        if best != "hipblaslt" and res[best] < 0.97 * res["hipblaslt"]:
            table[f"skinny,{M},{N},{K}"] = int(best[1:])
        else:
            table[f"skinny,{M},{N},{K}"] = "blas"
            best = "hipblaslt"
        tot["hipblaslt"] += res["hipblaslt"] * mult
        tot["best"] += res[best] * mult
        print(json.dumps({"M": M, "gemm": name, "N": N, "K": K, "best": best,
                          "best_TBps_w": round(N * K * 2 / res[best] / 1e6, 2),
                          **{k: round(v, 1) for k, v in res.items()}}), flush=True)
    N, K = shapes["gate_up"]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    yo = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    res = {"blas+silu": timeit(lambda w: ops.silu_mul(F.linear(x, w), block=64), ws["gate_up"]),
           "fused": timeit(lambda w: kernels().gemm_skinny(x, w, yo, None, 1, True), ws["gate_up"])}
    table[f"silu,{M},{N},{K}"] = [0] if res["fused"] < 0.97 * res["blas+silu"] else "blas"
    print(json.dumps({"M": M, "gemm": "gate_up+silu", **{k: round(v, 1) for k, v in res.items()}}), flush=True)
    print(json.dumps({"M": M, "per_step_gemm_ms_hipblaslt": round(tot["hipblaslt"] / 1e3, 3),
                      "per_step_gemm_ms_best": round(tot["best"] / 1e3, 3)}), flush=True)
if a.write_table:
    old = json.load(open(a.write_table)) if os.path.exists(a.write_table) else {}
    old.update(table)
    with open(a.write_table, "w") as f:
        json.dump(dict(sorted(old.items())), f, indent=1)
