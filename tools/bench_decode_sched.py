#!/usr/bin/env python3
"""M = 256 decode projections of Llama-3-8B: the production plan against gemm_pp's
schedules (0 ping-pong, 1 one segment, 2 lock-step) at every split count, each split-K
candidate also timed together with the RMSNorm that sums its fp32 slabs (the pair the
model runs). Cold weights as in a decode step (rotating copies > 512 MB), interleaved
rounds in one process, medians. One JSON line per shape.

    python tools/bench_decode_sched.py [--rounds 5] [--shapes qkv,o,down,gate_up+silu]
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
    ap.add_argument("--scheds", default="0,2,4,6,7,8")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    M = a.m
    C = ops.kernels()
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

        y = torch.empty(M, N // 2 if silu else N, dtype=torch.bfloat16, device="cuda")
        P = torch.empty(8 * M * N, dtype=torch.float32, device="cuda")
        nw = torch.ones(N, device="cuda", dtype=torch.bfloat16)
        res = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        yn = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        cands = {}
        if silu:
            cands["table"] = lambda: ops.gate_up_silu(x, nxt(), ops.GU_BLOCK)
            for sc in [int(v) for v in a.scheds.split(",")]:
                cands[f"pp256_sched{sc}"] = (lambda sc=sc: C.gemm_pp(x, nxt(), y, None, 1, 256, True, True, sc))
        else:
            norm = lambda r: ops.rmsnorm(r, nw, 1e-5, residual=res, out=yn)  # noqa: E731
            cands["table"] = lambda: ops.linear(x, nxt(), defer_reduce=True)
            cands["table+norm"] = lambda: norm(ops.linear(x, nxt(), defer_reduce=True))
            for sc in [int(v) for v in a.scheds.split(",")]:
                for S in (1, 2, 4, 8):
                    if K % (64 * S):
                        continue
                    if S == 1:
                        cands[f"s1_sched{sc}+norm"] = (lambda sc=sc: norm(
                            (C.gemm_pp(x, nxt(), y, None, 1, 256, False, True, sc), y)[1]))
                    else:
                        def f(S=S, sc=sc):
                            C.gemm_pp(x, nxt(), None, P, S, 256, False, True, sc)
                            return norm(ops.SplitK(P, S, M, N))
                        cands[f"s{S}_sched{sc}+norm"] = f
        times = {k: [] for k in cands}
        for _ in range(a.rounds):
            for k, fn in cands.items():
                times[k].append(timeit(fn, a.iters))
        us = {k: round(statistics.median(v), 2) for k, v in times.items()}
        best = min((k for k in us if silu or k.endswith("+norm")), key=us.get)
        r = {"M": M, "shape": name, "N": N, "K": K, "weight_copies": ncopy, "us": us, "best": best}
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
