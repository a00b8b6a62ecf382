"""Decode-shape GEMM microbenchmark: hipBLASLt default heuristic vs TunableOp-tuned
(hipBLASLt + rocBLAS solution search). y[M,N] = x[M,K] @ W[N,K]^T, bf16."""
import argparse
import json
import os

import torch
import torch.nn.functional as F

ap = argparse.ArgumentParser()
ap.add_argument("--m", default="1,16,64,128,256")
ap.add_argument("--tune", action="store_true")
ap.add_argument("--file", default="gpurun_out/tunableop_results.csv")
a = ap.parse_args()
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
if a.tune:
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.file)
    tun.set_max_tuning_duration(200)
    tun.set_max_tuning_iterations(30)
# rotate through enough weight copies (>=1 GB) that nothing is served from the 256 MB MALL,
# as in a real 32-layer decode step
ws = {k: [torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02
          for _ in range(max(1, min(16, -(-(1 << 30) // (n * kk * 2)))))] for k, (n, kk) in shapes.items()}
for M in [int(x) for x in a.m.split(",")]:
    tot = 0.0
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        wl = ws[name]
        for w in wl:
            F.linear(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        it = 32
        e0.record()
        for i in range(it):
            F.linear(x, wl[i % len(wl)])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / it * 1e3
        tot += us * (1 if name == "lm_head" else 32)
        print(json.dumps({"M": M, "gemm": name, "N": N, "K": K, "us": round(us, 1),
                          "TFLOPs": round(2 * M * N * K / us / 1e6, 1), "TBps_w": round(N * K * 2 / us / 1e6, 2),
                          "tuned": a.tune}), flush=True)
    print(json.dumps({"M": M, "per_step_gemm_ms": round(tot / 1e3, 3), "tuned": a.tune}), flush=True)
if a.tune:
    import torch.cuda.tunable as tun
    tun.write_file()
