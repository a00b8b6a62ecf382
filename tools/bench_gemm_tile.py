#!/usr/bin/env python3
"""gfx950 gemm_tile (csrc/kernels/gemm_tile.hip) vs hipBLASLt (torch F.linear) on the
Llama-3-8B prefill projections and the lm_head, uniform random operands, interleaved
rounds in one process (cdna_hip_programming.md §5.4 rules 24/25). One JSON line per shape.

    python tools/bench_gemm_tile.py [--m 4096,16384,32768] [--rounds 5]
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

SHAPES = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up+silu", 28672, 4096, True),
          ("down", 4096, 14336, False)]
LM = [("lm_head", 128256, 4096, False)]


def timeit(fn, iters: int) -> float:
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="4096,16384,32768")
    ap.add_argument("--lm-m", default="1,16,32,64,128,256")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--variant", type=int, default=0, help="gemm_tile schedule (0 = default)")
    ap.add_argument("--alt", type=int, default=None, help="also time this gemm_tile variant")
    a = ap.parse_args()
    C = ops.kernels()
    rows = []
    cases = [(int(m), *s) for m in a.m.split(",") if m for s in SHAPES] + \
            [(int(m), *s) for m in a.lm_m.split(",") if m for s in LM]
    for M, name, N, K, silu in cases:
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        y = torch.empty(M, N // 2 if silu else N, dtype=torch.bfloat16, device="cuda")
        yb = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        flops = 2.0 * M * N * K
        iters = max(3, min(200, int(2e13 / flops)))
        mine = lambda: C.gemm_tile(x, w, y, None, silu, a.variant)  # noqa: E731
        alt = lambda: C.gemm_tile(x, w, y, None, silu, a.alt)  # noqa: E731
        blas = (lambda: ops.silu_mul(F.linear(x, w, out=yb), block=64, out=y)) if silu else \
            (lambda: F.linear(x, w, out=yb))  # noqa: E731
        tm, tb, ta = [], [], []
        for _ in range(a.rounds):
            tm.append(timeit(mine, iters))
            tb.append(timeit(blas, iters))
            if a.alt is not None:
                ta.append(timeit(alt, iters))
        # numerics spot check against hipBLASLt
        if not silu:
            mine()
            blas()
            err = (y.float() - yb.float()).abs().max().item()
        else:
            err = None
        m_us, b_us = statistics.median(tm), statistics.median(tb)
        r = {"shape": name, "M": M, "N": N, "K": K, "gemm_tile_us": round(m_us, 1), "hipblaslt_us": round(b_us, 1),
             "gemm_tile_tflops": round(flops / m_us / 1e6, 1), "hipblaslt_tflops": round(flops / b_us / 1e6, 1),
             "speedup": round(b_us / m_us, 3), "min_us": [round(min(tm), 1), round(min(tb), 1)],
             "max_abs_diff_vs_blas": err,
             "weight_tb_s": round(N * K * 2 / m_us / 1e6, 2)}
        if ta:
            r[f"variant{a.alt}_us"] = round(statistics.median(ta), 1)
            r[f"variant{a.alt}_tflops"] = round(flops / statistics.median(ta) / 1e6, 1)
        if silu:
            r["hipblaslt_includes"] = "separate silu_mul kernel"
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
