#!/usr/bin/env python3
"""Decode-bucket GEMMs (M = 64 / 128 / 256, Llama-3-8B projections): the LDS-DMA
split-K gemm_decode (tuned table, what ops.linear / gate_up_silu pick) vs the
256x256-tile gemm_tile at split-K S in {1, 2, 4, 8, 16}, interleaved rounds in one
process, random operands. One JSON line per (M, shape)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from operator_amd import ops  # noqa: E402

SHAPES = [("gate_up+silu", 28672, 4096, True), ("qkv", 6144, 4096, False), ("o", 4096, 4096, False),
          ("down", 4096, 14336, False), ("lm_head", 128256, 4096, False)]


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
    ap.add_argument("--m", default="64,128,256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tile", action="store_true", help="also time gemm_tile split-K")
    ap.add_argument("--shapes", default="gate_up+silu,qkv,o,down", help="comma list (lm_head: the vocab projection)")
    a = ap.parse_args()
    C = ops.kernels()
    for M in [int(x) for x in a.m.split(",")]:
        for name, N, K, silu in SHAPES:
            if name not in a.shapes.split(","):
                continue
            torch.manual_seed(0)
            x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
            nw = 2 if N * K > (1 << 28) else 4   # rotating weight copies (the vocab projection is 1 GB each)
            ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(nw)]
            y = torch.empty(M, N // 2 if silu else N, dtype=torch.bfloat16, device="cuda")
            P = torch.empty((4 if N > 65536 else 16) * M * N, dtype=torch.float32, device="cuda")
            it = {"i": 0}

            def cur():
                w = ws[it["i"] % len(ws)]
                it["i"] += 1
                return ops.gate_up_silu(x, w, 64) if silu else ops.linear(x, w)

            def tile(S):
                def f():
                    w = ws[it["i"] % len(ws)]
                    it["i"] += 1
                    C.gemm_tile(x, w, y, None, silu, 0, S, P if S > 1 else None)
                return f

            def pp(S, bm, nt, one=False):
                def f():
                    w = ws[it["i"] % len(ws)]
                    it["i"] += 1
                    C.gemm_pp(x, w, y, P if S > 1 else None, S, bm, silu, nt, one)
                return f

            cands = {"decode": cur}
            if a.tile:
                for S in (1, 2, 4, 8, 16):
                    if K % (64 * S) == 0 and S * M * N <= P.numel():
                        cands[f"tile_s{S}"] = tile(S)
            for bm in ((128, 256) if M > 128 else (128,)):
                for S in ((1,) if silu else (1, 2) if N > 65536 else (1, 2, 4, 8)):
                    if K % (64 * S) == 0:
                        for nt in (True, False):
                            cands[f"pp_bm{bm}_s{S}{'_nt' if nt else ''}"] = pp(S, bm, nt)
                        if bm == 256:
                            cands[f"pp_bm256_s{S}_one"] = pp(S, bm, True, True)
            t = {k: [] for k in cands}
            for _ in range(a.rounds):
                for k, f in cands.items():
                    t[k].append(timeit(f, a.iters))
            med = {k: round(statistics.median(v), 2) for k, v in t.items()}
            # numerics: tile vs the current path
            ref = cur()
            errs = {}
            for S in ((1,) if silu else (1, 4)):
                C.gemm_pp(x, ws[(it["i"] - 1) % len(ws)], y, P if S > 1 else None, S, 128, silu, True)
                errs[f"pp_s{S}"] = round((y.float() - ref.float()).abs().max().item(), 4)
            best = min(med, key=med.get)
            wb = N * K * 2
            print(json.dumps({"M": M, "shape": name, "N": N, "K": K, "us": med, "best": best,
                              "best_weight_tb_s": round(wb / med[best] / 1e6, 2), "max_diff_vs_decode": errs}),
                  flush=True)


if __name__ == "__main__":
    main()
