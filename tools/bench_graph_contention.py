"""Does host-side contention stall a captured decode step on MI355X?

Replays the Llama-3-8B B=256 decode-step graph N times (contexts ~1.1k) and
reports ms per step in three arms: (a) nothing else running, (b) one Python
thread spinning on pure-Python work beside the engine thread (GIL contention,
the operator's pipeline threads), (c) the same spinner while the steps are
launched from C++ with the GIL released (operator_amd._C.graph_launch).
Random-init weights, bf16.
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd import ops  # noqa: E402
from operator_amd.engine.llm import GenRequest, LLMEngine  # noqa: E402
from operator_amd.models.config import get_config  # noqa: E402
from operator_amd.models.kv_cache import PagedKVCache  # noqa: E402
from operator_amd.models.llama import LlamaModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=1100)
    ap.add_argument("--steps", type=int, default=160)
    ap.add_argument("--sync-start", type=int, default=0,
                    help="N processes run together: each waits at a file barrier under /tmp before timing")
    ap.add_argument("--only-alone", action="store_true")
    ap.add_argument("--order", default="py,c", help="arm order of the alone runs")
    a = ap.parse_args()
    cfg = get_config("llama3-8b")
    m = LlamaModel(cfg, device="cuda").init_random(0)
    pages = PagedKVCache.pages_for_budget(int(100e9), cfg.layers, cfg.kv_heads, 128, 64)
    kv = PagedKVCache(cfg.layers, pages, cfg.kv_heads, 128, 64, device="cuda")
    eng = LLMEngine(m, kv, max_batch=a.batch, max_context=a.ctx + 4 * a.steps + 64, use_graphs=True,
                    prefill_graphs=False)
    reqs = [GenRequest(list(range(1, a.ctx + 1)), max_tokens=4 * a.steps, temperature=0.3, seed=i, ignore_eos=True)
            for i in range(a.batch)]
    for r in reqs:
        eng.submit(r)
    while eng.waiting:
        eng.step()
    B = len(eng.running)
    bp = next(b for b in eng.buckets if b >= B)
    g = eng._graph(bp, ops.decode_splits(a.ctx + 4 * a.steps, bp, eng.hkv))
    g.st.load(eng.running, eng.max_pages)
    C = ops.kernels()
    stream = torch.cuda.current_stream().cuda_stream

    def py_replays(n):
        for i in range(n):
            if i % eng.multi_step == 0:
                g.st.step.zero_()
            g.graph.replay()

    def c_replays(n, chunk=None):
        done = 0
        while done < n:
            k = min(eng.multi_step, n - done)
            g.st.step.zero_()
            if chunk is None:
                C.graph_launch(g.graph.raw_cuda_graph_exec(), k, stream)
            else:
                for j in range(0, k, chunk):
                    C.graph_launch(g.graph.raw_cuda_graph_exec(), min(chunk, k - j), stream)
            done += k

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(a.steps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    stop = threading.Event()

    def spin():
        x = 0
        while not stop.is_set():
            for i in range(1000):
                x += i * i

    py_replays(8)
    torch.cuda.synchronize()
    if a.sync_start:   # crude cross-process start barrier: every process touches a file, waits for N
        d = "/tmp/oamd_sync_start"
        os.makedirs(d, exist_ok=True)
        open(os.path.join(d, str(os.getpid())), "w").close()
        t_end = time.time() + 120
        while len(os.listdir(d)) < a.sync_start and time.time() < t_end:
            time.sleep(0.01)
    out = {"B": B, "bucket": bp, "ctx": a.ctx, "procs": max(1, a.sync_start)}
    if a.sync_start:
        t0 = time.perf_counter()
        c_replays(a.steps * 2)
        torch.cuda.synchronize()
        out["together_c_ms"] = round((time.perf_counter() - t0) * 1e3 / (a.steps * 2), 3)
        print(json.dumps(out), flush=True)
        return
    for arm in a.order.split(","):
        if arm == "py":
            out["alone_py_ms"] = round(timed(py_replays), 3)
        elif arm == "c":
            out["alone_c_ms"] = round(timed(c_replays), 3)
        elif arm == "c1":
            out["alone_c1_ms"] = round(timed(lambda n: c_replays(n, 1)), 3)
    if a.only_alone:
        print(json.dumps(out), flush=True)
        return
    th = [threading.Thread(target=spin, daemon=True) for _ in range(4)]
    for t in th:
        t.start()
    out["spin4_py_ms"] = round(timed(py_replays), 3)
    out["spin4_c_ms"] = round(timed(c_replays), 3)
    stop.set()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
