#!/usr/bin/env python3
"""Decode-bucket projections of Llama-3-8B at M = 256 (qkv, o, down, gate|up + SwiGLU):
the production plan (ops.linear / ops.gate_up_silu as the model calls them, split-K slabs
deferred to the consumer), alone and paired with the consumer that sums its slabs. Weights are COLD as in a real decode step (each step streams 16 GB of weights +
the KV cache through a 256 MiB Infinity Cache): every call uses the next of enough
rotating weight copies to exceed 512 MB. Interleaved rounds, medians. (Round 4 also timed a
deep-weight-stream kernel here, gemm_dw: slower on every shape,
profiles/decode_gemm_dw_vs_table_m256_cold.jsonl, and deleted.)
One JSON line per shape.

    python tools/bench_decode_gemm.py [--m 256] [--rounds 5]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from operator_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("down", 4096, 14336, False),
          ("gate_up+silu", 28672, 4096, True)]


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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default="qkv,o,down,gate_up+silu")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tile", action="store_true",
                    help="also time the 256x256-tile kernel (gemm_tile) with split-K S = 1, 2, 4, 8, 16")
    a = ap.parse_args()
    M = a.m
    rows = []
    for name, N, K, silu in SHAPES:
        if name not in a.shapes.split(","):
            continue
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ncopy = max(2, -(-512 * 2**20 // (N * K * 2)))
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
        it = {"i": 0}

        def nxt():
            it["i"] += 1
            return ws[it["i"] % ncopy]

        cands = {}
        if silu:
            cands["table"] = lambda: ops.gate_up_silu(x, nxt(), ops.GU_BLOCK)
        else:
            # "+norm": the pair as the model runs it, the projection then a residual RMSNorm that
            # reads its output (summing the fp32 slabs of a split-K plan)
            nw = torch.ones(N, device="cuda", dtype=torch.bfloat16)
            res = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
            yn = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            norm = lambda r: ops.rmsnorm(r, nw, 1e-5, residual=res, out=yn)  # noqa: E731
            cands["table"] = lambda: ops.linear(x, nxt(), defer_reduce=True)
            cands["table+norm"] = lambda: norm(ops.linear(x, nxt(), defer_reduce=True))
        if a.tile:
            C = ops.kernels()
            P = torch.empty(16 * M * N, dtype=torch.float32, device="cuda")
            for S in (1, 2, 4, 8, 16):
                if K % (64 * S):
                    continue
                if silu:
                    y2 = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
                    cands[f"tile_s{S}"] = (lambda S=S, y2=y2: C.gemm_tile(x, nxt(), y2, None, True, 0, S,
                                                                         P if S > 1 else None))
                elif S == 1:
                    y1 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
                    cands["tile_s1+norm"] = lambda y1=y1: (C.gemm_tile(x, nxt(), y1, None, False, 0, 1, None),
                                                           norm(y1))
                else:
                    cands[f"tile_s{S}+norm"] = (lambda S=S: (C.gemm_tile(x, nxt(), None, None, False, 0, S, P),
                                                             norm(ops.SplitK(P, S, M, N))))
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn, a.iters))
        us = {k: round(statistics.median(v), 2) for k, v in times.items()}
        r = {"M": M, "shape": name, "N": N, "K": K, "weight_copies": ncopy, "us": us,
             "weight_tb_s": round(N * K * 2 / us["table"] / 1e6, 2)}
        print(json.dumps(r), flush=True)
        rows.append(r)
        del ws
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
