"""Decode-shape GEMM microbenchmark: y[M,N] = x[M,K] @ W[N,K]^T, bf16.

Compares hipBLASLt (F.linear, default heuristic or --tune TunableOp) with the
gfx950 gemm_decode kernel at every split-K count. Weights rotate through enough
copies (>= 1 GB) that nothing is served from the 256 MB MALL, as in a real
32-layer decode step."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", default="64,128,256")
ap.add_argument("--tune", action="store_true")
ap.add_argument("--no-custom", action="store_true")
ap.add_argument("--file", default="gpurun_out/tunableop_results.csv")
ap.add_argument("--write-table", default=None, help="write the best (bm, bn, splits) per shape as JSON")
ap.add_argument("--tp", type=int, default=1, help="also cover the TP-sharded shapes of this degree")
ap.add_argument("--fp8", action="store_true", help="also time the W8A8 e4m3fn gemm_fp8 path")
ap.add_argument("--model", default="8b", choices=["8b", "70b"])
ap.add_argument("--hot", action="store_true",
                help="one weight copy (served from the 256 MB MALL after the first call): the cache-resident bound")
ap.add_argument("--shapes", default=None, help="comma list of projections to time (default: all)")
a = ap.parse_args()
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}
if a.model == "70b":
    shapes = {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
              "lm_head": (128256, 8192)}
if a.tp > 1:
    t = a.tp
    shapes = {f"{k}_tp{t}": ((n // t, kk) if k in ("qkv", "gate_up", "lm_head") else (n, kk // t))
              for k, (n, kk) in shapes.items()}
if a.shapes:
    shapes = {k: v for k, v in shapes.items() if k.split("_tp")[0] in a.shapes.split(",")}
table = {}
if a.tune:
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(a.file)
    tun.set_max_tuning_duration(200)
    tun.set_max_tuning_iterations(30)
    tun.set_rotating_buffer_size(1024)
ws = {k: [torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02
          for _ in range(1 if a.hot else max(1, min(16, -(-(1 << 30) // (n * kk * 2)))))]
      for k, (n, kk) in shapes.items()}


def timeit(fn, wl, it=32):
    for w in wl:
        fn(w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for i in range(it):
        fn(wl[i % len(wl)])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for M in [int(x) for x in a.m.split(",")]:
    tot = {"hipblaslt": 0.0, "best": 0.0}
    for name, (N, K) in shapes.items():
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        mult = 1 if name == "lm_head" else 32
        res = {"hipblaslt": timeit(lambda w: F.linear(x, w), ws[name])}
        if not a.no_custom and M in ops.GEMM_DECODE_M:
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            part = torch.empty(8 * M * N, device="cuda", dtype=torch.float32)
            ref = F.linear(x, ws[name][0]).float()
            for bm in (64, 128, 256):
                for bn in (64, 128):
                    for S in (1, 2, 4, 8):
                        for ns in ((2, 3, 4) if bm <= 128 else (3, 4) if bm + bn <= 320 else (3,)):
                            if bm > M or K % (64 * S) or N % bn:
                                continue
                            got = ops.linear(x, ws[name][0], out=y, splits=S, partial=part, bn=bn, bm=bm,
                                             stages=ns).float()
                            err = (got - ref).abs().max().item()
                            if err > 0.1:
                                print("BAD", name, M, bm, bn, S, ns, err, flush=True)
                                continue
                            key = f"m{bm}n{bn}s{S}x{ns}"
                            res[key] = timeit(lambda w: ops.linear(x, w, out=y, splits=S, partial=part, bn=bn, bm=bm,
                                                                   stages=ns), ws[name])
        if a.fp8:
            # enough quantized copies (>= 1 GB) that nothing is served from the MALL
            n8 = max(1, min(16, -(-(1 << 30) // (N * K))))
            w8s = [ops.quantize_fp8(ws[name][i % len(ws[name])]) for i in range(n8)]
            q, sx = ops.quantize_fp8(x)
            y8 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            bm, bn, S = ops.fp8_plan(M, N, K)
            part = torch.empty(S * M * N, device="cuda", dtype=torch.float32) if S > 1 else None
            fp8_us = timeit(lambda wp: ops.kernels().gemm_fp8(q, wp[0], sx, wp[1], y8, part, S, bn, bm), w8s)
            quant_us = timeit(lambda _: ops.quantize_fp8(x), [None])
            print(json.dumps({"M": M, "gemm": name, "fp8_us": round(fp8_us, 1), "fp8_quant_us": round(quant_us, 1),
                              "fp8_plan": [bm, bn, S], "fp8_TBps_w": round(N * K / fp8_us / 1e6, 2)}), flush=True)
            del w8s
        times = dict(res)
        best = min(times, key=times.get)
        if M in ops.GEMM_DECODE_M:
            # the custom kernel must win by >= 3 % to displace hipBLASLt (noise margin)
            if best != "hipblaslt" and times[best] < 0.97 * times["hipblaslt"]:
                bm_, rest = best[1:].split("n")
                bn_, rest = rest.split("s")
                s_, ns_ = rest.split("x")
                table[f"{M},{N},{K}"] = [int(bm_), int(bn_), int(s_), int(ns_)]
            else:
                table[f"{M},{N},{K}"] = "blas"
                best = "hipblaslt"
        tot["hipblaslt"] += res["hipblaslt"] * mult
        tot["best"] += times[best] * mult
        out = {"M": M, "gemm": name, "N": N, "K": K, "best": best,
               "best_TBps_w": round(N * K * 2 / times[best] / 1e6, 2)}
        top = sorted(times.items(), key=lambda kv: kv[1])[:4]
        out.update({"hipblaslt": round(res["hipblaslt"], 1), "top": [(k, round(v, 1)) for k, v in top]})
        print(json.dumps(out), flush=True)
    # fused gate|up + SwiGLU vs hipBLASLt + silu_mul (interleaved layout)
    if not a.no_custom and M in ops.GEMM_DECODE_M and "gate_up" in shapes:
        N, K = shapes["gate_up"]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        res = {"blas+silu": timeit(lambda w: ops.silu_mul(F.linear(x, w), block=64), ws["gate_up"])}
        yo = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
        for bm in (64, 128, 256):
            for ns in ((2, 3, 4) if bm == 64 else (3, 4) if bm == 128 else (3,)):
                if bm <= M:
                    res[f"fused_m{bm}x{ns}"] = timeit(
                        lambda w: ops.kernels().gemm_decode(x, w, yo, None, 1, 128, bm, True, False, ns), ws["gate_up"])
        best = min(res, key=res.get)
        table[f"silu,{M},{N},{K}"] = ([int(v) for v in best.split("_m")[1].split("x")] if best != "blas+silu" and
                                      res[best] < 0.97 * res["blas+silu"] else "blas")
        print(json.dumps({"M": M, "gemm": "gate_up+silu", "best": best,
                          **{k: round(v, 1) for k, v in res.items()}}), flush=True)
    print(json.dumps({"M": M, "per_step_gemm_ms_hipblaslt": round(tot["hipblaslt"] / 1e3, 3),
                      "per_step_gemm_ms_best": round(tot["best"] / 1e3, 3)}), flush=True)
if a.write_table:
    old = {}
    if os.path.exists(a.write_table):
        with open(a.write_table) as f:
            old = json.load(f)
    old.update(table)
    with open(a.write_table, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)
if a.tune:
    import torch.cuda.tunable as tun
    for r in tun.get_results():
        print("tuned:", r, flush=True)
