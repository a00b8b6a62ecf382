"""Tensor parallelism beyond world 2 on the CPU tier (gloo): TP = 4 and TP = 8 of a
70B-shaped head layout (tiny-tp8: GQA 16/8, every dimension divisible by 8) must
reproduce TP = 1 — prefill logits and greedy + sampled generation through the
lock-stepped TPLLMEngine leader/followers (SURVEY.md §4.2 "Distributed", P3).
Also: a step error on the TP leader only is fatal for the replica (no local abort
that would leave the followers inside a collective)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


PROMPTS = [[5, 6, 7, 8], list(range(20, 61))]


def _reqs():
    from operator_amd.engine.llm import GenRequest

    return [GenRequest(list(PROMPTS[0]), max_tokens=8, temperature=0.0, ignore_eos=True),
            GenRequest(list(PROMPTS[1]), max_tokens=8, temperature=0.8, seed=11, ignore_eos=True)]


def _tp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from operator_amd.engine.tp import TPLLMEngine, control_group
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch, LlamaModel
    from operator_amd.parallel.comm import init_from_env, split_groups

    init_from_env(backend="gloo")
    tp, _ = split_groups(world)
    cfg = get_config("tiny-tp8")
    m = LlamaModel(cfg, device="cpu", tp=tp, dtype=torch.float32).init_random(seed=21)
    assert m.hq == cfg.heads // world and m.hkv == cfg.kv_heads // world
    kv = PagedKVCache(cfg.layers, 64, m.hkv, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    ids = torch.arange(3, 40) % cfg.vocab_size
    T = ids.numel()
    fb = ForwardBatch(ids, torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None, seq_lens=[T])
    logits = tp.all_gather(m.forward(fb, kv), dim=1)
    eng = TPLLMEngine(m, kv, tp_group=tp, ctrl_group=control_group(tp), max_batch=4, max_context=256,
                      use_graphs=False)
    if tp.rank == 0:
        reqs = _reqs()
        for r in reqs:
            eng.submit(r)
        while any(not r.done for r in reqs):
            eng.step()
        eng.close()
        torch.save({"logits": logits, "out": [r.output for r in reqs]}, os.path.join(out_dir, "tp.pt"))
    else:
        eng.follow()
    dist.barrier()
    dist.destroy_process_group()


def _reference():
    from operator_amd.engine.llm import LLMEngine
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch, LlamaModel

    cfg = get_config("tiny-tp8")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=21)
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    ids = torch.arange(3, 40) % cfg.vocab_size
    T = ids.numel()
    fb = ForwardBatch(ids, torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None, seq_lens=[T])
    ref = m.forward(fb, kv)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    reqs = _reqs()
    eng.generate(reqs)
    return ref, [r.output for r in reqs]


@pytest.mark.parametrize("world", [4, 8])
def test_tp_matches_tp1(world, tmp_path):
    mp.start_processes(_tp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(tmp_path / "tp.pt", weights_only=True)
    ref, outs = _reference()
    torch.testing.assert_close(got["logits"], ref, atol=1e-4, rtol=1e-4)
    assert got["out"] == outs


def _fail_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from operator_amd.engine.explain import EngineLoop
    from operator_amd.engine.llm import GenRequest
    from operator_amd.engine.tp import TPLLMEngine, control_group
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import LlamaModel
    from operator_amd.parallel.comm import init_from_env, split_groups

    init_from_env(backend="gloo", timeout_s=20)
    tp, _ = split_groups(world)
    cfg = get_config("tiny-tp8")
    m = LlamaModel(cfg, device="cpu", tp=tp, dtype=torch.float32).init_random(seed=2)
    kv = PagedKVCache(cfg.layers, 64, m.hkv, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = TPLLMEngine(m, kv, tp_group=tp, ctrl_group=control_group(tp), max_batch=4, max_context=256,
                      use_graphs=False)
    if tp.rank == 0:
        real, calls = m.forward, {"n": 0}

        def flaky(fb, kv_):
            calls["n"] += 1
            if calls["n"] == 3:   # a leader-only failure mid-generation (e.g. OOM on this rank)
                raise RuntimeError("HIP out of memory (injected on the leader)")
            return real(fb, kv_)

        m.forward = flaky
        loop = EngineLoop(eng)
        loop.start()
        r = GenRequest(list(range(1, 20)), max_tokens=8, temperature=0.0, ignore_eos=True)
        eng.submit(r)
        loop.notify()
        assert r.event.wait(60)
        loop.join(30)
        res = {"fatal": loop.fatal is not None, "alive": loop.is_alive(), "error": r.error or ""}
        torch.save(res, os.path.join(out_dir, "fail.pt"))
    else:
        try:
            eng.follow()     # the leader never arrives for the step it failed: the collective times out
        except Exception:  # noqa: BLE001
            pass
    os._exit(0)   # the replica is dead by design; no clean process-group teardown


def test_tp_leader_failure_is_fatal(tmp_path):
    mp.start_processes(_fail_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = torch.load(tmp_path / "fail.pt", weights_only=True)
    assert res["fatal"] and not res["alive"] and "out of memory" in res["error"]


def test_bench_tp_simulate_runs_one_rank_shard():
    """tools/bench_tp.py --simulate-tp 8: one process drives rank 0's TP=8 shard (per-rank
    shapes, simulated collectives) and reports the shard's weight floor."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "bench_tp.py"), "--simulate-tp", "8", "--model",
                        "tiny-tp8", "--dtype", "float32", "--weights", "bfloat16", "--cpu", "--batch", "3", "--prompt", "24", "--gen", "6", "--kv-gb",
                        "0.05"], capture_output=True, text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert out["simulated_tp"] == 8 and out["tp"] == 8 and out["decode_tok_s"] > 0 and out["weight_floor_ms"] > 0


SHARED_HEAD = list(range(100, 140))


def _shared_reqs():
    from operator_amd.engine.llm import GenRequest

    return [GenRequest(SHARED_HEAD + list(range(3 + i, 10 + 2 * i)), max_tokens=6, temperature=0.0, ignore_eos=True)
            for i in range(6)]


def _tp_prefix_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from operator_amd.engine.tp import TPLLMEngine, control_group
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import LlamaModel
    from operator_amd.parallel.comm import init_from_env, split_groups

    init_from_env(backend="gloo")
    tp, _ = split_groups(world)
    cfg = get_config("tiny-tp8")
    m = LlamaModel(cfg, device="cpu", tp=tp, dtype=torch.float32).init_random(seed=22)
    kv = PagedKVCache(cfg.layers, 96, m.hkv, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = TPLLMEngine(m, kv, tp_group=tp, ctrl_group=control_group(tp), max_batch=2, max_context=256,
                      use_graphs=False, prefix_sharing=True)
    if tp.rank == 0:
        reqs = _shared_reqs()
        for r in reqs:
            eng.submit(r)
        while any(not r.done for r in reqs):
            eng.step()
        eng.close()
        torch.save({"out": [r.output for r in reqs], "builds": eng.stats.prefix_builds,
                    "hits": eng.stats.prefix_hits}, os.path.join(out_dir, "tp_pfx.pt"))
    else:
        eng.follow()
        torch.save({"builds": eng.stats.prefix_builds, "hits": eng.stats.prefix_hits},
                   os.path.join(out_dir, f"tp_pfx_{tp.rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_tp_prefix_sharing_matches_tp1(tmp_path):
    """Shared prompt-prefix pages under TP = 4: the prefix is built at the same step on
    every rank (admission replays the leader's submissions deterministically), the
    followers share it exactly as the leader does, and greedy outputs equal a TP = 1
    engine with sharing."""
    from operator_amd.engine.llm import LLMEngine
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import LlamaModel

    world = 4
    mp.start_processes(_tp_prefix_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = torch.load(tmp_path / "tp_pfx.pt", weights_only=True)
    assert got["builds"] == 1 and got["hits"] >= 3
    for r in range(1, world):
        f = torch.load(tmp_path / f"tp_pfx_{r}.pt", weights_only=True)
        assert (f["builds"], f["hits"]) == (got["builds"], got["hits"])
    cfg = get_config("tiny-tp8")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=22)
    kv = PagedKVCache(cfg.layers, 96, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=2, max_context=256, use_graphs=False, prefix_sharing=True)
    reqs = _shared_reqs()
    eng.generate(reqs)
    assert got["out"] == [r.output for r in reqs]
