"""scan_gpu per batch, eager launches vs the captured scan graph, at the flagship wave
shape (256 logs x 64 KiB x 1000 patterns) and a 64-log match-service batch."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.match import MatchEngine  # noqa: E402
from operator_amd.patterns.synth import LogFactory, synthetic_library  # noqa: E402

ps = synthetic_library(1000, seed=0)
fac = LogFactory(n_patterns=1000, seed=1)
for n in (64, 256):
    batches = [fac.batch(n, 64 * 1024, n_failures=3, seed=s)[0] for s in range(4)]
    row = {"bench": "scan_graph", "docs": n, "log_kib": 64}
    for arm in ("eager", "graph"):
        eng = MatchEngine(ps, device="cuda", seg_bytes=1024, scan_graphs=arm == "graph")
        for b in batches:            # profile + capture
            eng.scan_gpu(b)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            for b in batches:
                t0 = time.perf_counter()
                eng.scan_gpu(b)
                ts.append(time.perf_counter() - t0)
        ts.sort()
        row[arm + "_ms_p50"] = round(1e3 * ts[len(ts) // 2], 3)
        row[arm + "_ms_min"] = round(1e3 * ts[0], 3)
        if arm == "graph":
            row["graph_replays"] = eng.graph_replays
    print(json.dumps(row), flush=True)
