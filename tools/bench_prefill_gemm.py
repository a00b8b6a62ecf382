"""Prefill-shape GEMMs (M = prefill chunk tokens): hipBLASLt default heuristic vs
TunableOp-tuned. y = x @ W^T, bf16. Writes the TunableOp results CSV."""
import argparse
import json

import torch
import torch.nn.functional as F

ap = argparse.ArgumentParser()
ap.add_argument("--m", default="16384")
ap.add_argument("--tune", action="store_true")
ap.add_argument("--file", default="gpurun_out/tunableop_prefill.csv")
a = ap.parse_args()
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
if a.tune:
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.file)
    tun.set_max_tuning_duration(500)
    tun.set_max_tuning_iterations(50)
    tun.set_rotating_buffer_size(512)
tot = 0.0
for M in [int(x) for x in a.m.split(",")]:
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        for _ in range(3):
            F.linear(x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(10):
            F.linear(x, w)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 10 * 1e3
        tot += us
        print(json.dumps({"M": M, "gemm": name, "us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1),
                          "tuned": a.tune}), flush=True)
print(json.dumps({"layer_us": round(tot, 1), "tuned": a.tune}))
if a.tune:
    import torch.cuda.tunable as tun
    for r in tun.get_results():
        print("tuned:", r, flush=True)
