#!/usr/bin/env python3
"""Interleaved timing of gemm_tile schedules (csrc/kernels/gemm_tile.hip `variant`) and
hipBLASLt on one prefill shape, uniform random operands (cdna_hip_programming.md §5.4
rules 24/25). Variant 5 is a timing-only experiment (no loads in the loop).

    python tools/gemm_tile_variants.py --variants 1,2,3 [--m 16384 --n 4096 --k 14336]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=16384)
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--k", type=int, default=14336)
ap.add_argument("--variants", default="1,2,3")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--silu", action="store_true", help="fused SwiGLU epilogue (the gate_up GEMM; N = 2 x intermediate)")
a = ap.parse_args()
C = ops.kernels()
x = (torch.rand(a.m, a.k, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(a.n, a.k, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
y = torch.empty(a.m, a.n // 2 if a.silu else a.n, dtype=torch.bfloat16, device="cuda")
flops = 2.0 * a.m * a.n * a.k
iters = max(3, min(100, int(2e13 / flops)))


def timeit(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


arms = {f"v{v}": (lambda v=int(v): C.gemm_tile(x, w, y, None, a.silu, v)) for v in a.variants.split(",")}
if a.silu:   # hipBLASLt arm: the plain GEMM into a scratch output (no epilogue)
    y2 = torch.empty(a.m, a.n, dtype=torch.bfloat16, device="cuda")
    arms["blas"] = lambda: F.linear(x, w, out=y2)
    ref = None   # the fused arms are checked against the first one
else:
    arms["blas"] = lambda: F.linear(x, w, out=y)
    ref = F.linear(x, w)
t = {k: [] for k in arms}
for _ in range(a.rounds):
    for k, fn in arms.items():
        t[k].append(timeit(fn))
out = {"M": a.m, "N": a.n, "K": a.k}
for k, v in t.items():
    us = statistics.median(v)
    arms[k]()
    if ref is None and k != "blas":
        ref = y.clone()
    err = (y.float() - ref.float()).abs().max().item() if k != "blas" or not a.silu else 0.0
    out[k] = {"us": round(us, 1), "tflops": round(flops / us / 1e6, 1), "max_abs_err": round(err, 4)}
print(json.dumps(out), flush=True)
