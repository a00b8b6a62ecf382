"""Run one gemm_tile shape repeatedly (for rocprofv3 --pmc): y = x W^T, random operands."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=16384)
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--k", type=int, default=14336)
ap.add_argument("--variant", type=int, default=4)
ap.add_argument("--blas", action="store_true")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
x = (torch.rand(a.m, a.k, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(a.n, a.k, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
y = torch.empty(a.m, a.n, device="cuda", dtype=torch.bfloat16)
for i in range(a.iters):
    if a.blas:
        torch.nn.functional.linear(x, w, out=y)
    else:
        ops.kernels().gemm_tile(x, w, y, None, False, a.variant)
torch.cuda.synchronize()
