"""Run one decode GEMM config repeatedly (for rocprofv3 --pmc): y = x W^T."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=256)
ap.add_argument("--n", type=int, default=28672)
ap.add_argument("--k", type=int, default=4096)
ap.add_argument("--bm", type=int, default=256)
ap.add_argument("--bn", type=int, default=128)
ap.add_argument("--s", type=int, default=1)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
x = torch.randn(a.m, a.k, device="cuda", dtype=torch.bfloat16)
ws = [torch.randn(a.n, a.k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(4)]
y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
p = torch.empty(max(1, a.s) * a.m * a.n, device="cuda", dtype=torch.float32)
for i in range(a.iters):
    ops.kernels().gemm_decode(x, ws[i % 4], y, p if a.s > 1 else None, a.s, a.bn, a.bm, False, False, 3)
torch.cuda.synchronize()
