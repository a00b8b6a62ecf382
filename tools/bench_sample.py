"""Sampler microbenchmark: the decode step's Gumbel-max sampling of B rows of a
128k-vocab bf16 logits matrix (Llama-3 lm_head output), us per call."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--vocab", type=int, default=128256)
ap.add_argument("--scale", type=float, default=1.0, help="logit std (a trained model's rows are peaked: larger)")
a = ap.parse_args()
x = (torch.randn(a.batch, a.vocab, device="cuda") * a.scale).to(torch.bfloat16)
t = torch.full((a.batch,), 0.3, device="cuda")
sd = torch.arange(a.batch, device="cuda")
ps = torch.arange(a.batch, device="cuda")
for _ in range(3):
    ops.sample(x, t, sd, ps)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
n = 50
e0.record()
for _ in range(n):
    ops.sample(x, t, sd, ps)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / n * 1e3
print(json.dumps({"bench": "sample", "batch": a.batch, "vocab": a.vocab, "scale": a.scale, "us": round(us, 1),
                  "GBps": round(x.numel() * 2 / us / 1e3, 1)}))
