"""Shared prompt-prefix KV pages (engine/llm.py ``_SharedPrefix``): requests whose
prompts start with the same whole KV pages map one set of pages computed once, and
prefill only their own tokens against the cached prefix K/V. The CPU tier checks the
attention reference and the engine end to end against engines without sharing; the
GPU tier checks the HIP kernel path (tests/test_prefix_sharing_gpu.py)."""
import torch

from operator_amd import ops
from operator_amd.engine.llm import GenRequest, LLMEngine
from operator_amd.models.config import get_config
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import LlamaModel
from operator_amd.ops import reference


def test_reference_prefix_attention_equals_full_causal_rows():
    """Attention of a sequence's own rows over [prefix K/V ++ own K/V] == the last rows of
    plain causal attention over the whole sequence (prefix lengths 0, 16 and 32)."""
    torch.manual_seed(0)
    Hq, Hkv, D = 8, 2, 32
    P = 32
    pk, pv = torch.randn(P, Hkv, D), torch.randn(P, Hkv, D)
    own = [5, 17, 9]
    pl = [16, 0, 32]
    q = torch.randn(sum(own), Hq, D)
    k, v = torch.randn(sum(own), Hkv, D), torch.randn(sum(own), Hkv, D)
    cu = [0, 5, 22, 31]
    out = reference.attn_prefill(q, k, v, cu, 0.17, prefix=(pk, pv, pl))
    for i, (a, b) in enumerate(zip(cu[:-1], cu[1:])):
        n = pl[i]
        qf = torch.cat([torch.randn(n, Hq, D), q[a:b]])
        kf, vf = torch.cat([pk[:n], k[a:b]]), torch.cat([pv[:n], v[a:b]])
        full = reference.attn_prefill(qf, kf, vf, [0, n + b - a], 0.17)
        torch.testing.assert_close(out[a:b], full[n:], rtol=1e-5, atol=1e-5)
    # the ops entry point takes the same prefix on the CPU
    o2 = ops.attn_prefill(q, k, v, own, 0.17, prefix=(pk, pv, None, pl))
    torch.testing.assert_close(o2, out)


def _engine(m, cfg, sharing):
    kv = PagedKVCache(cfg.layers, 96, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=torch.float32)
    return kv, LLMEngine(m, kv, max_batch=2, max_context=256, use_graphs=False, prefix_sharing=sharing)


def test_engine_shares_prefix_pages_and_matches_unshared():
    """Six prompts with a common 40-token head (two whole 16-token pages), admitted two at
    a time: once the head has been seen twice it is computed once and the later
    requests map its pages and prefill only their own tokens. Greedy outputs equal an
    engine without sharing; every request's own pages come back, the prefix keeps its 2."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=11)
    head = list(range(100, 140))
    prompts = [head + list(range(3 + i, 3 + i + 7 + 3 * i)) for i in range(6)]
    outs = {}
    for sharing in (False, True):
        kv, eng = _engine(m, cfg, sharing)
        reqs = [GenRequest(p, max_tokens=8, temperature=0.0, ignore_eos=True) for p in prompts]
        eng.generate(reqs)
        outs[sharing] = [r.output for r in reqs]
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages
        if sharing:
            assert eng.stats.prefix_builds == 1 and eng.prefix_pages == 2
            assert eng.stats.prefix_hits == 4 and eng.stats.prefix_tokens == 4 * 32
            assert eng.stats.prefill_tokens == sum(map(len, prompts)) - 4 * 32
    assert outs[True] == outs[False]


def test_engine_prefix_replaced_only_when_unused():
    """A different common head replaces the shared prefix once no request holds the old
    one; prompts that do not start with the current prefix run unshared."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=12)
    kv, eng = _engine(m, cfg, True)
    a = [GenRequest(list(range(200, 240)) + [i + 1, i + 2], max_tokens=3, temperature=0.0, ignore_eos=True)
         for i in range(4)]
    eng.generate(a)
    first = eng._pfx
    assert first is not None and first.tokens == tuple(range(200, 232))
    b = [GenRequest(list(range(300, 340)) + [i + 1], max_tokens=3, temperature=0.0, ignore_eos=True)
         for i in range(4)]
    eng.generate(b)
    assert eng._pfx is not first and eng._pfx.tokens == tuple(range(300, 332))
    assert first.retired and first.users == 0
    assert kv.allocator.free + eng.prefix_pages == kv.num_pages
    # sharing off: nothing is built
    kv2, eng2 = _engine(m, cfg, False)
    eng2.generate([GenRequest(list(range(200, 240)), max_tokens=2, temperature=0.0, ignore_eos=True)
                   for _ in range(4)])
    assert eng2.stats.prefix_builds == 0 and eng2.prefix_pages == 0


def test_prefix_build_failure_releases_its_pages():
    """A forward that raises while the shared prefix is computed returns the prefix's
    pages (they belong to no request yet, so nothing else would free them); the engine
    then carries on and builds the prefix once the forward works again."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=13)
    kv, eng = _engine(m, cfg, True)
    head = list(range(100, 140))
    real = m.forward

    def boom(fb, cache):
        if fb.kv_sink is not None:
            raise RuntimeError("injected prefix forward failure")
        return real(fb, cache)

    m.forward = boom
    reqs = [GenRequest(head + [i + 1], max_tokens=2, temperature=0.0, ignore_eos=True) for i in range(4)]
    for r in reqs:
        eng.submit(r)
    raised = False
    try:
        for _ in range(100):
            eng.step()
    except RuntimeError:
        raised = True
    assert raised and eng._pfx is None
    held = sum(len(r.pages) for r in reqs)   # admitted requests (running or mid-prefill)
    assert kv.allocator.free + held == kv.num_pages   # nothing leaked by the failed build
    m.forward = real
    while any(not r.done for r in reqs):
        eng.step()
    assert kv.allocator.free + eng.prefix_pages == kv.num_pages


def test_idle_prefix_gives_way_to_admission():
    """When a request's pages do not fit only because an idle shared prefix (no users)
    holds them, the prefix is dropped and the request admitted, not refused."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=14)
    kv = PagedKVCache(cfg.layers, 12, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=2, max_context=256, use_graphs=False, prefix_sharing=True)
    head = list(range(100, 140))
    eng.generate([GenRequest(head + [i + 1], max_tokens=2, temperature=0.0, ignore_eos=True) for i in range(4)])
    assert eng.prefix_pages == 2
    # 12 pages, 2 held by the idle prefix: a request needing 11 fits only without it
    big = GenRequest(list(range(500, 500 + 160)), max_tokens=16, temperature=0.0, ignore_eos=True)
    assert kv.pages_needed(len(big.prompt) + big.max_tokens) == 11
    eng.generate([big])
    assert big.error is None and len(big.output) == 16
    assert eng.prefix_pages == 0 and kv.allocator.free == kv.num_pages
