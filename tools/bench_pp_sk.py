#!/usr/bin/env python3
"""Stream-K vs per-tile gemm_pp for the M = 256 gate|up + SwiGLU decode GEMM of Llama-3-8B
(csrc/kernels/gemm_pp.hip SK: one block per CU over the flattened (tile, K-step) stream vs one
block per 128-feature tile, 224 of 256 CUs). Cold weights (rotating copies > 512 MB, as in a
decode step), random operands, interleaved rounds, medians. One JSON line.

    python tools/bench_pp_sk.py [--m 256] [--rounds 7]
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


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=28672)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N, K = a.m, a.n, a.k
    kern = ops.kernels()
    torch.manual_seed(0)
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    ncopy = max(2, -(-512 * 2**20 // (N * K * 2)))
    ws_ = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
    y = torch.empty(M, N // 2, dtype=torch.bfloat16, device="cuda")
    skw = torch.empty(N // 128 * 32768, dtype=torch.float32, device="cuda")
    skf = torch.zeros(N // 128, dtype=torch.int32, device="cuda")
    arms = {
        "per_tile": lambda w: kern.gemm_pp(x, w, y, None, 1, 256, True, True),
        "stream_k": lambda w: kern.gemm_pp(x, w, y, None, 1, 256, True, True, False, skw, skf),
    }
    times: dict[str, list[float]] = {k: [] for k in arms}
    for _ in range(a.rounds):
        for name, fn in arms.items():
            it = 0
            fn(ws_[0])
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(a.iters):
                fn(ws_[it % ncopy])
                it += 1
            e.record()
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / a.iters * 1e3)
    med = {k: round(statistics.median(v), 2) for k, v in times.items()}
    print(json.dumps({"shape": "gate_up+silu", "M": M, "N": N, "K": K,
                      "sk_grid": kern.gemm_pp_sk_grid(N // 128, K // 64), "tiles": N // 128,
                      "us_median": med, "us_all": {k: [round(t, 2) for t in v] for k, v in times.items()},
                      "speedup": round(med["per_tile"] / med["stream_k"], 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
