"""Tensor parallelism on the GPU kernels: TP = 2 and 4 as ranks sharing the one MI355X of
the box (cuda:0), the decode all-reduces through the IPC kernels between them (the fused
all-reduce + residual + RMSNorm, and with fp8 weights its e4m3fn epilogue), gloo only
for the handle exchange (RCCL refuses two ranks on one device). The sharded model's
prefill logits and one paged decode step (the decode RoPE folded into attention, the
per-rank kv-head shard) are checked against the fp32 PyTorch path of the same global
weights on the host (as tests/test_llama_gpu.py does for TP = 1), with a bf16- / fp8-sized
tolerance, and against the TP = 1 model on the same kernels. The CPU tier pins TP = 4 / 8
to TP = 1 exactly in fp32 (tests/test_tp_scale.py) (SURVEY.md §4.2 "Distributed")."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

LENS = [200, 90, 33]   # 323 prefill rows: the planned hipBLASLt projections too
P, PER = 16, 16


def _cfg():
    from operator_amd.models.config import LlamaConfig

    return LlamaConfig(name="tp-gpu", vocab_size=4096, hidden=2048, intermediate=4096, layers=2, heads=16,
                       kv_heads=8, max_position=4096, bos_id=4000, eos_ids=(4001,))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu_copy(m):
    """The fp32 host model with the same (global, TP = 1) weights."""
    from operator_amd.models.llama import LayerWeights, LlamaModel

    c = LlamaModel(m.cfg, device="cpu", dtype=torch.float32)
    c.embed, c.final_norm, c.lm_head = m.embed.float().cpu(), m.final_norm.float().cpu(), m.lm_head.float().cpu()
    c.layers = [LayerWeights(*(t.float().cpu() for t in (l.wqkv, l.wo, l.wgu, l.wd, l.attn_norm, l.mlp_norm)))
                for l in m.layers]
    return c


def _run(m, hkv: int, dev: str = "cuda"):
    """Prefill LENS, then one decode step: (last-token prefill logits, decode logits), the
    rank's vocab shard, on the CPU."""
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import ForwardBatch

    B = len(LENS)
    kv = PagedKVCache(m.cfg.layers, B * PER, hkv, 128, P, device=dev,
                      **({} if dev == "cuda" else {"dtype": torch.float32}))
    bt = torch.arange(B * PER, dtype=torch.int32).reshape(B, PER)
    ids = [torch.randint(0, m.cfg.vocab_size, (L,), generator=torch.Generator().manual_seed(i))
           for i, L in enumerate(LENS)]
    pos = torch.cat([torch.arange(L) for L in LENS])
    slots = torch.cat([bt[i, torch.arange(L) // P].long() * P + torch.arange(L) % P for i, L in enumerate(LENS)])
    last = torch.tensor(LENS).cumsum(0) - 1
    fb = ForwardBatch(torch.cat(ids).to(dev), pos.to(dev), slots.to(dev), True, last.to(dev), seq_lens=LENS)
    pre = m.forward(fb, kv).float().cpu()
    nxt = torch.tensor([int(x[-1]) for x in ids])
    dpos = torch.tensor(LENS)
    dslots = torch.stack([bt[i, L // P].long() * P + L % P for i, L in enumerate(LENS)])
    fb = ForwardBatch(nxt.to(dev), dpos.to(dev), dslots.to(dev), False, None, block_tables=bt.to(dev),
                      context_lens=(dpos + 1).int().to(dev), num_splits=1)
    dec = m.forward(fb, kv).float().cpu()
    if dev == "cuda":
        torch.cuda.synchronize()
    return pre, dec


def _worker(rank: int, world: int, port: int, wdt: str, q) -> None:
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK="0")
        import torch.distributed as dist

        from operator_amd.models.llama import LlamaModel
        from operator_amd.parallel.comm import init_from_env, split_groups

        init_from_env(backend="gloo")
        torch.cuda.set_device(0)
        tp, _ = split_groups(world)
        assert tp.enable_oneshot(torch.device("cuda", 0))
        m = LlamaModel(_cfg(), device="cuda", tp=tp, weight_dtype=wdt).init_random(seed=7)
        pre, dec = _run(m, m.hkv)
        tp.oneshot.check()
        dist.barrier()
        tp.oneshot.close()
        dist.destroy_process_group()
        q.put((rank, "ok", pre.numpy(), dec.numpy()))   # by value: the child exits before the get
    except BaseException:  # noqa: BLE001
        import traceback

        q.put((rank, "error", traceback.format_exc(), None))


@pytest.mark.parametrize("wdt,world", [("bfloat16", 2), ("fp8", 2), ("bfloat16", 4)])
def test_tp_on_one_gpu_tracks_tp1(wdt, world):
    import torch.multiprocessing as mp

    from operator_amd.models.llama import LlamaModel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, wdt, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, status, a, b = q.get(timeout=300)
            assert status == "ok", a
            got[rank] = (torch.from_numpy(a), torch.from_numpy(b))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    pre = torch.cat([got[r][0] for r in range(world)], dim=1)   # vocab shards in rank order
    dec = torch.cat([got[r][1] for r in range(world)], dim=1)
    m1 = LlamaModel(_cfg(), device="cuda", weight_dtype=wdt).init_random(seed=7)
    pre1, dec1 = _run(m1, m1.hkv)
    del m1
    mb = LlamaModel(_cfg(), device="cuda").init_random(seed=7)   # the same global bf16 weights
    with torch.inference_mode():
        pref, decf = _run(_cpu_copy(mb), mb.hkv, dev="cpu")
    del mb
    # against the fp32 host path: bf16 rounding through 2 layers, or with fp8 weights the
    # e4m3fn weight/activation quantization (per-shard channel scales of the row-parallel
    # weights) on top
    tol = 0.02 if wdt == "bfloat16" else 0.08   # measured: 0.0065 (TP=2, 4) and 0.056 (fp8)
    errs = {}
    for name, got_, want in (("prefill", pre, pref), ("decode", dec, decf)):
        assert got_.shape == want.shape
        errs[name] = float((got_ - want).abs().max() / want.abs().max())
    errs1 = {n: float((a - b).abs().max() / b.abs().max()) for n, a, b in (("prefill", pre1, pref),
                                                                        ("decode", dec1, decf))}
    print(f"TP={world} {wdt}: max-logit error vs fp32 host {errs}; TP=1 on the same kernels {errs1}")
    for n in errs:
        assert errs[n] < tol, (n, errs, errs1)
        # the sharding adds no error beyond what the kernels' precision already has at TP=1
        assert errs[n] < 1.5 * errs1[n] + 0.005, (n, errs, errs1)
    # the decode step's greedy token is the fp32 path's for rows whose top-2 logits are
    # not a near tie
    top2 = decf.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 0.02 * decf.abs().max()
    assert torch.equal(dec.argmax(1)[clear], decf.argmax(1)[clear])
    assert torch.equal(pre.argmax(1), pref.argmax(1)) or wdt == "fp8"
