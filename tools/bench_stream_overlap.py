"""Does splitting a latency-bound decode batch over two HIP streams pay? (VERDICT r4 "next"
item 3(b): two micro-batches on two streams inside the captured decode graph.)

Proxy of the TP=8 70B fp8 decode layer's GEMM chain (per layer: QKV, O, gate|up, down at
the per-rank shapes, W8A8 with the production plans, bf16 outputs so each split-K plan
also runs its slab reduce) over --layers distinct weight sets (cold-ish: > the MALL),
captured in one hipGraph per arm and replayed:
  * one:  the whole batch (M rows) on one stream;
  * two:  two halves of M/2 rows on two streams forked and joined inside the graph.
If the per-kernel fixed costs (launch, ramp, drain) dominate, the two-stream arm hides
one half's fixed cost under the other's and takes well under the one-stream time.

  python tools/bench_stream_overlap.py [--m 64] [--layers 8] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402

SHAPES = (("qkv", 1280, 8192), ("o", 8192, 1024), ("gate_up", 7168, 8192), ("down", 8192, 3584))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = "cuda"
    W = [{n: ops.quantize_fp8(torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02) for n, N, K in SHAPES}
         for _ in range(a.layers)]

    def inputs(m):
        return {K: ops.quantize_fp8(torch.randn(m, K, device=dev, dtype=torch.bfloat16)) for K in (8192, 1024, 3584)}

    def chain(x):
        out = None
        for layer in W:
            for n, N, K in SHAPES:
                out = ops.linear_fp8(x[K], layer[n][0], layer[n][1])
        return out

    def timed(g):
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(a.iters):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    res = {"bench": "stream_overlap", "m": a.m, "layers": a.layers, "kernels_per_layer": None}
    # arm one: M rows, one stream
    x = inputs(a.m)
    chain(x)
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1, stream=s0):
        chain(x)
    res["one_stream_us"] = round(timed(g1), 1)
    # arm two: M/2 rows on each of two streams, forked and joined inside the graph
    xa, xb = inputs(a.m // 2), inputs(a.m // 2)
    chain(xa)
    torch.cuda.synchronize()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s0):
        fork = torch.cuda.Event()
        fork.record(s0)
        s1.wait_event(fork)
        with torch.cuda.stream(s1):
            chain(xb)
        chain(xa)
        join = torch.cuda.Event()
        join.record(s1)
        s0.wait_event(join)
    res["two_streams_us"] = round(timed(g2), 1)
    # arm half: M/2 rows, one stream (the per-kernel floor)
    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g3, stream=s0):
        chain(xa)
    res["half_one_stream_us"] = round(timed(g3), 1)
    res["per_layer_us"] = {k: round(res[k] / a.layers, 2) for k in ("one_stream_us", "two_streams_us",
                                                                   "half_one_stream_us")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
