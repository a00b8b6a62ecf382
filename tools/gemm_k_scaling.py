#!/usr/bin/env python3
"""Per-tile overhead vs per-K-step cost of the prefill GEMMs: time gemm_tile variants and
hipBLASLt at fixed M x N over several K (random operands, interleaved rounds in one
process). The slope over K is the K-step cost, the intercept the per-tile fill / epilogue.

    python tools/gemm_k_scaling.py --m 32768 --n 4096 --k 1024,2048,4096,8192 --variants 1,5
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from operator_amd import ops  # noqa: E402


def timeit(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", default="1024,2048,4096,8192")
    ap.add_argument("--variants", default="1,5")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    C = ops.kernels()
    M, N = a.m, a.n
    variants = [int(v) for v in a.variants.split(",")]
    for K in (int(k) for k in a.k.split(",")):
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        flops = 2.0 * M * N * K
        iters = max(3, min(200, int(2e13 / flops)))
        arms = {f"v{v}": (lambda v=v: C.gemm_tile(x, w, y, None, False, v)) for v in variants}
        arms["blas"] = lambda: F.linear(x, w, out=y)
        t = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                t[k].append(timeit(fn, iters))
        med = {k: statistics.median(v) for k, v in t.items()}
        print(json.dumps({"M": M, "N": N, "K": K, **{f"{k}_us": round(v, 1) for k, v in med.items()},
                          **{f"{k}_tflops": round(flops / v / 1e6, 1) for k, v in med.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
