#!/usr/bin/env python3
"""Decode split-K choice judged with its consumer: the M=256 o / down projections
(Llama-3-8B) followed by the residual RMSNorm that sums their fp32 split-K slabs, as
the model runs them (ops.linear(defer_reduce=True) -> ops.rmsnorm). The tuned table
picks splits by GEMM time alone; every slab is written and read back once more by
the norm, so fewer splits can win the pair. Cold weights (4 rotating copies).
One JSON line per projection: us per (GEMM + norm) for every variant."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from operator_amd import ops  # noqa: E402
from operator_amd.ops import SplitK  # noqa: E402

SHAPES = [("o", 4096, 4096), ("down", 4096, 14336)]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    C = ops.kernels()
    M = a.m
    for name, N, K in SHAPES:
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(4)]
        nw = torch.ones(N, device="cuda", dtype=torch.bfloat16)
        res = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        P = torch.empty(16 * M * N, dtype=torch.float32, device="cuda")
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        it = {"i": 0}

        def nxt():
            it["i"] += 1
            return ws[it["i"] % 4]

        def dec(bm, bn, S):
            def f():
                d = ops.linear(x, nxt(), splits=S, bm=bm, bn=bn, partial=P, defer_reduce=S > 1)
                ops.rmsnorm(d, nw, 1e-5, residual=res)
            return f

        def pp(bm, S):
            def f():
                C.gemm_pp(x, nxt(), None if S > 1 else y, P if S > 1 else None, S, bm, False, True)
                ops.rmsnorm(SplitK(P, S, M, N) if S > 1 else y, nw, 1e-5, residual=res)
            return f

        def table():
            d = ops.linear(x, nxt(), defer_reduce=True)
            ops.rmsnorm(d, nw, 1e-5, residual=res)

        cands = {"table": table}
        for bm in (128, 256):
            for bn in (64, 128):
                for S in (1, 2, 4, 8):
                    if K % (64 * S) == 0:
                        cands[f"dec_bm{bm}_bn{bn}_s{S}"] = dec(bm, bn, S)
            for S in (1, 2, 4, 8):
                cands[f"pp_bm{bm}_s{S}"] = pp(bm, S)
        t = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, f in cands.items():
                t[k].append(timeit(f, a.iters))
        med = {k: round(statistics.median(v), 2) for k, v in t.items()}
        best = min(med, key=med.get)
        print(json.dumps({"M": M, "shape": name, "N": N, "K": K, "best": best, "best_us": med[best],
                          "table_us": med["table"], "plan": ops.gemm_plan(M, N, K),
                          "us": dict(sorted(med.items(), key=lambda kv: kv[1]))}), flush=True)


if __name__ == "__main__":
    main()
