"""fp8 W8A8 decode GEMM plans at the TP=8 per-rank shapes of Llama-3-70B (M = 64 rows).

Times ``ops.linear_fp8(..., defer_reduce=True)`` (the production mode: the fp32 split-K
slabs go to the next kernel) for every (bn, splits) plan, from cold weights (enough
rotating copies to overflow the 256 MB MALL), plus the same plan followed by a plain
slab sum (the extra reading a consumer pays for more slabs). One JSON line per shape.

  python tools/bench_fp8_plans.py [--m 64] [--iters 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

SHAPES = {"qkv": (1280, 8192), "o": (8192, 1024), "gate_up": (7168, 8192), "down": (8192, 3584)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--hot", action="store_true", help="one weight copy (L2/MALL-resident): isolates the cold-HBM cost")
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = "cuda"
    M = a.m
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        copies = 1 if a.hot else max(2, (640 << 20) // (N * K))
        ws = [ops.quantize_fp8(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for _ in range(copies)]
        x = ops.quantize_fp8(torch.randn(M, K, device=dev, dtype=torch.bfloat16))
        ref = (x[0].float() * x[1][:, None]) @ (ws[0][0].float() * ws[0][1][:, None]).t()
        res = {"shape": name, "M": M, "N": N, "K": K, "weight_copies": copies, "us": {}, "us_with_slab_sum": {},
               "default_plan": list(ops.fp8_plan(M, N, K))}
        for bn in (64, 128):
            if N % bn:
                continue
            for S in (1, 2, 4, 8):   # the kernel takes S | 8
                if K % (128 * S):
                    continue
                plan = (64 if M <= 64 else 128 if M <= 128 else 256, bn, S)
                try:
                    y = ops.linear_fp8(x, ws[0][0], ws[0][1], plan=plan)
                except Exception as e:  # noqa: BLE001 - a plan the kernel does not take
                    res["us"][f"bn{bn}_s{S}"] = f"refused: {e}"[:80]
                    continue
                err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                assert err < 2e-2, (name, plan, err)
                for with_sum in (False, True):
                    def run(i):
                        w = ws[i % copies]
                        r = ops.linear_fp8(x, w[0], w[1], plan=plan, defer_reduce=True)
                        if with_sum and S > 1:
                            r.p.view(S, -1).sum(0)
                    # the calls are captured in one graph: host launch cost (tens of us per
                    # Python call) would otherwise hide kernels of a few us
                    s_ = torch.cuda.Stream()
                    s_.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s_):
                        for i in range(3):
                            run(i)
                    torch.cuda.current_stream().wait_stream(s_)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        for i in range(a.iters):
                            run(i)
                    g.replay()
                    torch.cuda.synchronize()
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record()
                    g.replay()
                    en.record()
                    torch.cuda.synchronize()
                    us = st.elapsed_time(en) * 1e3 / a.iters
                    (res["us_with_slab_sum"] if with_sum else res["us"])[f"bn{bn}_s{S}"] = round(us, 2)
        best = min((v, k) for k, v in res["us"].items() if isinstance(v, float))
        res["best"] = best[1]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
