"""Tensor-parallel explanation decode benchmark (BASELINE config 5: Llama-3-70B,
TP=8 over xGMI, fp8 MFMA path). Launch one process per GPU:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29531 tools/bench_tp.py --model llama3-70b --weights fp8 --batch 64

The TP group is the whole world. Rank 0 is the engine leader (it submits the
requests); every other rank mirrors its steps (operator_amd/engine/tp.py).
Decode all-reduces up to ``--oneshot-mb`` go through the one-shot IPC kernel
(parallel/custom_ar.py), larger ones through RCCL. Random-init weights, synthetic
prompts, generation always runs to ``--gen`` tokens. Rank 0 prints one JSON line.
On the CPU tier the same script runs with gloo and a tiny model (tests/test_parallel.py).

``--simulate-tp N`` (one process, one GPU): rank 0's shard of a TP=N replica —
70B per-rank shapes — with every all-reduce launched as the world-1 one-shot kernel
(fused with the residual + RMSNorm), so the per-rank step time can be measured on a
single MI355X and compared with the weight-streaming floor of the shard
(``weight_floor_ms``: shard weight bytes / 6.3 TB/s). xGMI transfer time is NOT
included (no peers): it is the part only an 8-GPU node can measure.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.engine.llm import GenRequest  # noqa: E402
from operator_amd.engine.tp import TPLLMEngine, control_group  # noqa: E402
from operator_amd.models.config import get_config  # noqa: E402
from operator_amd.models.kv_cache import PagedKVCache  # noqa: E402
from operator_amd.models.llama import LlamaModel  # noqa: E402
from operator_amd.parallel.comm import init_from_env, split_groups  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3-70b")
ap.add_argument("--weights", default="fp8", choices=["fp8", "bfloat16"])
ap.add_argument("--cpu", action="store_true", help="run on the CPU (gloo) even where a GPU is visible")
ap.add_argument("--dtype", default="bfloat16")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--prompt", type=int, default=1024)
ap.add_argument("--gen", type=int, default=128)
ap.add_argument("--kv-gb", type=float, default=64.0)
ap.add_argument("--oneshot-mb", type=float, default=8.0, help="0 = RCCL for every all-reduce")
ap.add_argument("--oneshot-max-kb", type=float, default=0.0,
                help="one-shot / two-shot crossover override; 0 = calibrate on the node (engine default)")
ap.add_argument("--no-graphs", action="store_true")
ap.add_argument("--simulate-tp", type=int, default=0,
                help="one process: rank 0's shard of a TP=N replica, collectives as world-1 one-shot kernels")
a = ap.parse_args()

info = init_from_env()
gpu = torch.cuda.is_available() and not a.cpu
dev = torch.device("cuda", info.local_rank) if gpu else torch.device("cpu")
if gpu:
    torch.cuda.set_device(dev)
if a.simulate_tp > 1:
    if info.world > 1:
        raise SystemExit("--simulate-tp runs as ONE process")
    from operator_amd.parallel.comm import SimulatedTPGroup  # noqa: E402

    tp = SimulatedTPGroup(a.simulate_tp, dev)
    oneshot = tp.car is not None
    ctrl = None
else:
    tp, _ = split_groups(info.world)
    oneshot = bool(gpu and a.oneshot_mb > 0 and tp.enable_oneshot(dev, int(a.oneshot_mb * (1 << 20)),
                                                                   int(a.oneshot_max_kb * 1024) or None))
    ctrl = control_group(tp) if tp.world > 1 else None

cfg = get_config(a.model)
calibration = None
if oneshot and a.simulate_tp <= 1 and a.oneshot_max_kb <= 0:   # the engine's own start-up measurement
    from operator_amd.engine.factory import calibrate_allreduce  # noqa: E402

    calibration = calibrate_allreduce(tp, cfg.hidden, a.batch)
dtype = getattr(torch, a.dtype)
t0 = time.perf_counter()
m = LlamaModel(cfg, device=dev, tp=tp, dtype=dtype, weight_dtype=a.weights if gpu else "bfloat16").init_random(0)
pages = PagedKVCache.pages_for_budget(int(a.kv_gb * 1e9), cfg.layers, m.hkv, cfg.head_dim, 64,
                                      torch.finfo(dtype).bits // 8)
kv = PagedKVCache(cfg.layers, pages, m.hkv, cfg.head_dim, 64, device=dev, dtype=dtype)
if a.simulate_tp > 1:   # no peers to lock-step with: the plain engine drives the shard
    from operator_amd.engine.llm import LLMEngine  # noqa: E402

    eng = LLMEngine(m, kv, max_batch=a.batch, max_context=a.prompt + a.gen + 64, use_graphs=gpu and not a.no_graphs)
    eng.leader, eng.follow = True, None
else:
    eng = TPLLMEngine(m, kv, tp_group=tp, ctrl_group=ctrl, max_batch=a.batch, max_context=a.prompt + a.gen + 64,
                      use_graphs=gpu and not a.no_graphs)
eng.warmup([next(b for b in eng.buckets if b >= a.batch)])
init_s = time.perf_counter() - t0


def sync():
    if gpu:
        torch.cuda.synchronize()
    if tp.world > 1 and a.simulate_tp <= 1:
        torch.distributed.barrier()


sync()
if not eng.leader:
    eng.follow()
    sync()
    torch.distributed.destroy_process_group()
    sys.exit(0)

reqs = [GenRequest([1 + (7 * i + j) % (cfg.vocab_size - 2) for j in range(a.prompt)], max_tokens=a.gen,
                   temperature=0.3, seed=i, ignore_eos=True) for i in range(a.batch)]
t0 = time.perf_counter()
for r in reqs:
    eng.submit(r)
while any(not r.output for r in reqs):
    eng.step()
if gpu:
    torch.cuda.synchronize()
t1 = time.perf_counter()
gen0 = sum(len(r.output) for r in reqs)
step_ms = []
while any(not r.done for r in reqs):
    s0 = time.perf_counter()
    n0 = sum(len(r.output) for r in reqs)
    eng.step()
    n1 = sum(len(r.output) for r in reqs)
    if n1 > n0:
        step_ms.append((time.perf_counter() - s0) * 1e3 * a.batch / (n1 - n0))
if gpu:
    torch.cuda.synchronize()
t2 = time.perf_counter()
if hasattr(eng, "close"):
    eng.close()
toks = sum(len(r.output) for r in reqs) - gen0
wbytes = m.weight_bytes()
print(json.dumps({"bench": "tp-decode", "model": a.model, "weights": a.weights if gpu else "bfloat16",
                  "tp": tp.world, "batch": a.batch, "prompt": a.prompt, "gen": a.gen,
                  "oneshot_allreduce": oneshot, "hipgraph": eng.use_graphs, "init_s": round(init_s, 1),
                  "prefill_tok_s": round(a.batch * a.prompt / (t1 - t0), 1),
                  "decode_tok_s": round(toks / (t2 - t1), 1),
                  "p50_ms_per_token": round(statistics.median(step_ms), 3) if step_ms else None,
                  "latency_s": round(t2 - t0, 3),
                  "simulated_tp": a.simulate_tp if a.simulate_tp > 1 else None,
                  "allreduce_calibration": calibration,
                  "rank_weight_gb": round(wbytes / 1e9, 2),
                  "weight_floor_ms": round(wbytes / 6.3e12 * 1e3, 3)}), flush=True)
sync()
if tp.world > 1 and a.simulate_tp <= 1:
    torch.distributed.destroy_process_group()
