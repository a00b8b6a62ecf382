"""Tensor / data parallel logic on the CPU tier: gloo, world_size 2 (SURVEY.md §4.2
"Distributed"). TP=2 must reproduce the TP=1 model (logits and greedy/sampled
tokens), and the collective wrappers must behave like their definitions."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from operator_amd.engine.llm import GenRequest, LLMEngine
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch, LlamaModel
    from operator_amd.parallel.comm import Group, init_from_env, split_groups

    init_from_env(backend="gloo")
    tp, dp = split_groups(world)
    g = Group()
    # collectives sanity
    t = torch.tensor([float(rank + 1)])
    g.all_reduce_(t)
    assert t.item() == sum(range(1, world + 1))
    ag = g.all_gather(torch.tensor([rank]), dim=0)
    assert ag.tolist() == list(range(world))

    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", tp=tp, dtype=torch.float32).init_random(seed=9)
    kv = PagedKVCache(cfg.layers, 64, m.hkv, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    ids = torch.arange(3, 40) % cfg.vocab_size
    T = ids.numel()
    fb = ForwardBatch(ids, torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None, seq_lens=[T])
    logits_local = m.forward(fb, kv)
    logits = tp.all_gather(logits_local, dim=1)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    reqs = [GenRequest([5, 6, 7, 8], max_tokens=10, temperature=0.0, ignore_eos=True),
            GenRequest(list(range(20, 45)), max_tokens=10, temperature=0.9, seed=4, ignore_eos=True)]
    eng.generate(reqs)
    if rank == 0:
        torch.save({"logits": logits, "out": [r.output for r in reqs]}, os.path.join(out_dir, "tp.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_matches_tp1(tmp_path):
    from operator_amd.engine.llm import GenRequest, LLMEngine
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch, LlamaModel

    port = _free_port()
    mp.start_processes(_tp_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    got = torch.load(tmp_path / "tp.pt", weights_only=True)
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=9)
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    ids = torch.arange(3, 40) % cfg.vocab_size
    T = ids.numel()
    fb = ForwardBatch(ids, torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None, seq_lens=[T])
    ref = m.forward(fb, kv)
    torch.testing.assert_close(got["logits"], ref, atol=1e-4, rtol=1e-4)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    reqs = [GenRequest([5, 6, 7, 8], max_tokens=10, temperature=0.0, ignore_eos=True),
            GenRequest(list(range(20, 45)), max_tokens=10, temperature=0.9, seed=4, ignore_eos=True)]
    eng.generate(reqs)
    assert got["out"] == [r.output for r in reqs]


def test_bench_tp_script_two_ranks():
    """tools/bench_tp.py (BASELINE config 5 launcher) under torch.distributed.run:
    leader + follower lock-step through TPLLMEngine over gloo."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "tools", "bench_tp.py"),
           "--model", "tiny-gqa4", "--dtype", "float32", "--batch", "3", "--prompt", "24", "--gen", "6",
           "--kv-gb", "0.05"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["tp"] == 2 and out["decode_tok_s"] > 0


def test_oneshot_disabled_without_gpu():
    from operator_amd.parallel.comm import Group

    g = Group.single()
    assert g.enable_oneshot("cpu") is False
    t = torch.ones(4)
    assert g.all_reduce_(t) is t


def test_bench_self_launches_ranks():
    """`python bench.py --gpus 2` with no outer torchrun starts its two rank processes
    itself (127.0.0.1 rendezvous); the JSON line reports the 2-rank job, not one rank."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu", "--steps", "1", "--warmup", "1",
           "--model", "tiny", "--batch", "3", "--max-tokens", "4", "--prompt-tokens", "128", "--log-kb", "4",
           "--patterns", "40"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["detail"]["rccl_world"] == 2 and out["detail"]["launcher"] == "bench.py"
    assert len(out["detail"]["per_rank_elapsed_s"]) == 2
    assert out["detail"]["outcomes"] == {"ai-complete": 3}   # rank 0's own wave


def test_bench_refuses_missing_gpus():
    """Without --cpu, --gpus N on a host with fewer than N GPUs fails instead of
    measuring one device."""
    import subprocess
    import sys

    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("host has the GPUs")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, cwd=root, env=env)
    assert r.returncode != 0 and "visible GPUs" in r.stderr


@pytest.mark.parametrize("shards,apiserver", [(1, "auto"), (2, "inproc")])
def test_bench_two_ranks_gloo(shards, apiserver):
    """bench.py as the driver launches it for N > 1 (torch.distributed.run, one rank per
    device, 127.0.0.1 rendezvous), on the CPU tier with gloo and a tiny model: rank 0
    prints exactly one JSON line with whole-job numbers. Default (auto): the ranks are
    the shards of ONE operator deployment on ONE REST API server process (run
    --shard-per-gpu); inproc with 2 operator shards per rank (a child process each):
    the counts cover both shards."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--model", "tiny", "--batch", str(3 * shards),
           "--max-tokens", "4", "--prompt-tokens", "128", "--log-kb", "4", "--patterns", "40", "--shards", str(shards),
           "--apiserver", apiserver]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 6 * shards and out["config"]["parallelism"] == "dp2"
    assert out["config"]["operator_shards_per_gpu"] == shards
    assert out["detail"]["outcomes"] == {"ai-complete": 6 * shards} and out["value"] > 0
    assert out["config"]["apiserver"].startswith("1 REST API server process(es)" if apiserver == "auto" else "in-process")


def test_bench_eight_ranks_gloo_one_apiserver():
    """The N = 8 launch exactly as the driver starts it (torch.distributed.run, 8 ranks,
    127.0.0.1 rendezvous), on the CPU tier: rank 0 starts the REST API servers (one per 4
    ranks: 2) and broadcasts their URLs, every rank is one operator shard of its server's
    group, the world is checked against --gpus, and every failure of every rank is analysed
    exactly once (the servers' own Event records, merged)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "8", "--steps", "1", "--warmup", "1", "--model", "tiny", "--batch", "3",
           "--max-tokens", "4", "--prompt-tokens", "128", "--log-kb", "4", "--patterns", "40"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=root, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 24
    assert out["detail"]["rccl_world"] == 8 and len(out["detail"]["per_rank_elapsed_s"]) == 8
    assert out["config"]["apiserver"].startswith("2 REST API server process(es), 4 ranks each")
    assert out["detail"]["outcomes"] == {"ai-complete": 3}              # rank 0's own timed wave
    assert out["detail"]["outcomes_all_ranks"] == {"ai-complete": 24}   # 8 ranks x 3 failures
    # the one API server's record: every pod of every rank (warmup waves too) has exactly one
    # PodmortemAnalysisComplete Event -- each failure analysed once, by one operator shard
    audit = out["detail"]["apiserver_audit"]
    assert audit == {"pods_with_complete_event": 48, "max_complete_events_per_pod": 1, "expected_pods": 48,
                     "apiservers": 2}
    assert out["value"] > 0


def test_allreduce_dispatch_table_selection():
    """custom_ar.choose_protocols: the fastest IPC protocol per size, the group backend
    (RCCL) only when it beats both by the margin, runs merged, NaN = unavailable; and
    lookup_protocol routes any message size through the table (past the end: last entry)."""
    from operator_amd.parallel.custom_ar import (PROTO_BACKEND, PROTO_ONESHOT, PROTO_TWOSHOT, choose_protocols,
                                                 lookup_protocol)

    sizes = [8192, 16384, 65536, 262144, 1 << 20, 4 << 20]
    times = {PROTO_ONESHOT: [5e-6, 5.5e-6, 7e-6, 12e-6, 40e-6, 150e-6],
             PROTO_TWOSHOT: [8e-6, 8.5e-6, 9e-6, 11e-6, 25e-6, 80e-6],
             PROTO_BACKEND: [30e-6, 30e-6, 31e-6, 33e-6, 26e-6, 60e-6]}
    table = choose_protocols(sizes, times)
    assert table == [(65536, PROTO_ONESHOT), (1 << 20, PROTO_TWOSHOT), (4 << 20, PROTO_BACKEND)]
    assert lookup_protocol(table, 100) == PROTO_ONESHOT
    assert lookup_protocol(table, 65536) == PROTO_ONESHOT
    assert lookup_protocol(table, 65537) == PROTO_TWOSHOT
    assert lookup_protocol(table, 3 << 20) == PROTO_BACKEND
    assert lookup_protocol(table, 64 << 20) == PROTO_BACKEND
    # within the margin the IPC kernel keeps the size (RCCL 1 % faster at 1 MB: not enough)
    t2 = dict(times)
    t2[PROTO_BACKEND] = [30e-6, 30e-6, 31e-6, 33e-6, 24.8e-6, 100e-6]
    assert choose_protocols(sizes, t2) == [(65536, PROTO_ONESHOT), (4 << 20, PROTO_TWOSHOT)]
    # a protocol that could not be timed (NaN) never wins; no IPC timing at all -> backend
    t3 = {PROTO_ONESHOT: [float("nan")] * 6, PROTO_TWOSHOT: times[PROTO_TWOSHOT]}
    assert choose_protocols(sizes, t3) == [(4 << 20, PROTO_TWOSHOT)]
    assert choose_protocols(sizes[:2], {}) == [(16384, PROTO_BACKEND)]
    assert choose_protocols([], times) == []
    # the LL protocol competes where it was timed (NaN past its half-capacity limit)
    from operator_amd.parallel.custom_ar import PROTO_LL

    t4 = dict(times)
    t4[PROTO_LL] = [3e-6, 3.5e-6, 6e-6, float("nan"), float("nan"), float("nan")]
    assert choose_protocols(sizes, t4) == [(65536, PROTO_LL), (1 << 20, PROTO_TWOSHOT), (4 << 20, PROTO_BACKEND)]


def test_allreduce_route_keeps_ll_within_capacity():
    """route(): a forced or tabled LL protocol falls back to one-shot for messages whose
    LL packets (twice the bytes) would not fit the receive slots."""
    from operator_amd.parallel.custom_ar import PROTO_LL, PROTO_ONESHOT, OneShotAllReduce

    car = OneShotAllReduce.__new__(OneShotAllReduce)
    car.max_bytes, car.oneshot_max_bytes, car.forced, car.table = 8 << 20, 512 << 10, PROTO_LL, None
    assert car.route(4 << 20) == PROTO_LL
    assert car.route((4 << 20) + 16) == PROTO_ONESHOT
    car.forced, car.table = None, [(8 << 20, PROTO_LL)]
    assert car.route(1 << 20) == PROTO_LL and car.route(6 << 20) == PROTO_ONESHOT


def test_decode_message_sizes_follow_buckets():
    from operator_amd.engine.factory import decode_message_sizes

    assert decode_message_sizes(8192, 64) == [r * 8192 * 2 for r in (1, 2, 4, 8, 16, 32, 64)]
    assert decode_message_sizes(4096, 1) == [8192]
