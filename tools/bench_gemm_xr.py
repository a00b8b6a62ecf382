#!/usr/bin/env python3
"""gemm_xr (register-streamed activations, csrc/kernels/gemm_xr.hip) against the production
decode plan (ops.linear / ops.gate_up_silu as of round 5: gemm_tn / gemm_pp) on the Llama-3-8B
projections at M = 256, COLD weights (rotating copies > 512 MB, as in a real decode step),
random operands, interleaved rounds in one process. gemm_xr reads X in the tiled layout; the
tile pass is timed separately (the model's producers write it directly). One JSON line per
shape and split count.

    python tools/bench_gemm_xr.py [--rounds 5] [--splits 1,2,4,8]
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--splits", default="1,2,4,8")
    ap.add_argument("--shapes", default="qkv,o,down,gate_up+silu")
    ap.add_argument("--ablate", type=int, default=0, help="also time the ablation arms at this split count")
    a = ap.parse_args()
    M = 256
    C = ops.kernels()
    for name, N, K, silu in SHAPES:
        if name not in a.shapes.split(","):
            continue
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        xt = torch.empty_like(x)
        C.tile_rows(x, xt)
        ncopy = max(2, -(-512 * 2**20 // (N * K * 2)))
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
        it = {"i": 0}

        def nxt():
            it["i"] += 1
            return ws[it["i"] % ncopy]

        P = torch.empty(8 * M * N, dtype=torch.float32, device="cuda")
        cands = {}
        if silu:
            y = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
            cands["table"] = lambda: ops.gate_up_silu(x, nxt(), ops.GU_BLOCK)
            cands["xr_s1_tiled"] = lambda: C.gemm_xr(xt, nxt(), y, None, 1, 3)
        else:
            cands["table"] = lambda: ops.linear(x, nxt(), defer_reduce=True)
            for S in (int(v) for v in a.splits.split(",")):
                if K % (64 * S) == 0:
                    cands[f"xr_s{S}"] = (lambda S=S: C.gemm_xr(xt, nxt(), None, P, S, 0))
        cands["tile_rows"] = lambda: C.tile_rows(x, xt)
        if a.ablate and not silu:   # timing-only arms (wrong results): which stream bounds the kernel
            S = a.ablate
            for e, nm in ((10, "abl_noX"), (11, "abl_noW"), (12, "abl_mfma_only")):
                cands[nm] = (lambda e=e: C.gemm_xr(xt, nxt(), None, P, S, e))
        t = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                t[k].append(timeit(fn, a.iters))
        med = {k: round(statistics.median(v), 2) for k, v in t.items()}
        best = min((v, k) for k, v in med.items() if k.startswith("xr"))
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "us": med, "best_xr": best[1],
                          "speedup_vs_table": round(med["table"] / best[0], 3),
                          "weight_tb_s_best": round(N * K * 2 / best[0] / 1e6, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
