#!/usr/bin/env python3
"""LDS ring depth sweep of the M = 256 decode GEMMs (gemm_tn, csrc/kernels/gemm.hip): a CU
ingests about its LDS-DMA bytes in flight per ~2 us (MI355X guide, decode-GEMM notes in
README), so deeper rings of smaller tiles (5 stages x 32 KiB for 128 x 128, 6 x 24 KiB for
64 x 128) trade X re-reads for bytes in flight. Cold weights (rotating copies > 512 MB),
random operands, interleaved rounds, medians; split-K slabs left to the consumer (as the
model runs them), so plans with the same S compare directly. One JSON line per shape.

    python tools/bench_decode_stages.py [--shapes o,qkv,down] [--rounds 5]
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

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}
LDS = 160 * 1024


def plans(N: int, K: int):
    out = []
    for bm in (64, 128, 256):
        for bn in (64, 128):
            if N % bn:
                continue
            for ns in (3, 4, 5, 6):
                stage = (bm + bn) * 128
                if ns * stage > LDS or (ns == 4 and bm + bn > 320) or (ns == 5 and bm + bn > 256) \
                        or (ns == 6 and bm + bn > 192):
                    continue
                for S in (1, 2, 3, 4, 5, 6, 8):
                    if K // 64 < S:
                        continue
                    wgs = (N // bn) * S * (256 // bm)
                    if wgs < 128 or wgs > 1024:
                        continue
                    out.append((bm, bn, S, ns))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="o,qkv,down")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M = 256
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ncopy = max(2, -(-512 * 2**20 // (N * K * 2)))
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(ncopy)]
        prod = ops.gemm_plan(M, N, K)
        cands = plans(N, K)
        times: dict[str, list[float]] = {}
        for _ in range(a.rounds):
            for (bm, bn, S, ns) in cands:
                key = f"bm{bm}_bn{bn}_S{S}_ns{ns}"
                part = torch.empty(S * M * N, dtype=torch.float32, device="cuda")
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                it = [0]

                def call():
                    w = ws[it[0] % ncopy]
                    it[0] += 1
                    return ops.linear(x, w, splits=S, bn=bn, bm=bm, stages=ns, partial=part, defer_reduce=S > 1)

                call()
                torch.cuda.synchronize()
                s.record()
                for _ in range(a.iters):
                    call()
                e.record()
                torch.cuda.synchronize()
                times.setdefault(key, []).append(s.elapsed_time(e) / a.iters * 1e3)
        med = {k: round(statistics.median(v), 2) for k, v in times.items()}
        best = sorted(med.items(), key=lambda kv: kv[1])[:8]
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "production_plan": prod,
                          "best": best, "all_us": med}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
