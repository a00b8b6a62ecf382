"""Shared prompt-prefix KV on MI355X: the v3 prefill attention kernel with a cached
prefix against the fp32 reference, and the engine (eager and graph-captured prefill,
graph decode) with and without prefix sharing."""
import pytest
import torch

from operator_amd import ops
from operator_amd.engine.llm import GenRequest, LLMEngine
from operator_amd.models.config import get_config
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import LlamaModel
from operator_amd.ops import reference

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("var", [3, 4])
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (28, 4)])
def test_prefill_attention_with_prefix_matches_fp32(Hq, Hkv, var):
    """attn_prefill variants 3 / 4 with pk / pv / seq_pfx == fp32 attention over [prefix ++ own]
    keys (prefix 0 - 192 keys per sequence, partial last prefix tiles included; own
    lengths around the 32-row blocks)."""
    if var == 4 and Hq // Hkv > 4:
        pytest.skip("v4 (4-wave workgroups) takes GQA groups <= 4")
    torch.manual_seed(3)
    D, P = 128, 256
    own = [1, 33, 64, 200, 97, 5, 40]
    pl = [64, 0, 192, 96, 128, 0, 112]   # whole 64-key tiles and partial ones (page sizes 32, 16)
    T = sum(own)
    r = lambda *s: (torch.randn(*s, device="cuda") * 0.5).to(torch.bfloat16)  # noqa: E731
    q, k, v = r(T, Hq, D), r(T, Hkv, D), r(T, Hkv, D)
    pk, pv = r(P, Hkv, D), r(P, Hkv, D)
    cu = [0]
    for n in own:
        cu.append(cu[-1] + n)
    ws, wq = ops.prefill_work_list(own, ops.prefill_block_q(Hq, Hkv, var))
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")  # noqa: E731
    work = (i32(cu), i32(ws), i32(wq), var)
    o = ops.attn_prefill(q, k, v, own, D ** -0.5, work=work, prefix=(pk, pv, i32(pl), None))
    ref = reference.attn_prefill(q.float().cpu(), k.float().cpu(), v.float().cpu(), cu, D ** -0.5,
                                 prefix=(pk.float().cpu(), pv.float().cpu(), pl))
    torch.testing.assert_close(o.float().cpu(), ref, atol=2e-2, rtol=2e-2)
    # no prefix through the same kernel == the plain call
    o0 = ops.attn_prefill(q, k, v, own, D ** -0.5, work=work, prefix=(pk, pv, i32([0] * len(own)), None))
    torch.testing.assert_close(o0, ops.attn_prefill(q, k, v, own, D ** -0.5, work=work), atol=0, rtol=0)


@pytest.mark.parametrize("graphs", [False, True])
def test_engine_prefix_sharing_matches_unshared(graphs):
    """Eight prompts sharing a 130-token head (two whole 64-token pages), two admitted per
    batch: with sharing, the later ones map the prefix pages and prefill only their own
    tokens (eager or graph-captured prefill); greedy outputs match an engine without
    (7 of 8: the prefix K/V come from a 128-row prefill whose GEMM plans may sum in
    another order than the full prompts' batch)."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cuda").init_random(seed=9)
    head = [(7 * i) % 900 + 5 for i in range(130)]
    prompts = [head + [(11 * j + i) % 900 + 3 for j in range(200 + 5 * i)] for i in range(8)]
    outs = {}
    for sharing in (False, True):
        kv = PagedKVCache(cfg.layers, 256, cfg.kv_heads, 128, 64, device="cuda")
        # 512-token prefill batches: with the prefix the pairs of own tokens (404-474) replay
        # the 512 graph bucket; without, each prompt (330-365) runs eagerly
        eng = LLMEngine(m, kv, max_batch=2, max_prefill_tokens=512, max_context=1024, use_graphs=graphs,
                        prefix_sharing=sharing)
        reqs = [GenRequest(p, max_tokens=12, temperature=0.0, ignore_eos=True) for p in prompts]
        eng.generate(reqs)
        outs[sharing] = [r.output for r in reqs]
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages
        if sharing:
            assert eng.stats.prefix_builds == 1 and eng.stats.prefix_hits >= 6
            assert not graphs or eng.stats.prefill_graph_replays > 0
    agree = sum(a == b for a, b in zip(outs[True], outs[False]))
    assert agree >= 7, (outs[True], outs[False])


def test_shared_prefix_kv_equals_full_prompt_kv():
    """What sharing changes numerically, pinned: the shared prefix's K/V (one prefill of
    just the head tokens, captured by the engine into _pk / _pv) against the same head
    tokens' K/V inside a prefill of a whole prompt. Causality makes them the same math;
    only the GEMM plans' summation order differs (128 vs 330+ rows), so they agree to a
    bf16 rounding step or two -- which is also why a greedy output can occasionally flip
    (test above: 7 of 8 must agree; outputs are NOT guaranteed identical with sharing)."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cuda").init_random(seed=9)
    head = [(7 * i) % 900 + 5 for i in range(130)]
    prompts = [head + [(11 * j + i) % 900 + 3 for j in range(200 + 5 * i)] for i in range(4)]
    kv = PagedKVCache(cfg.layers, 256, cfg.kv_heads, 128, 64, device="cuda")
    eng = LLMEngine(m, kv, max_batch=2, max_prefill_tokens=512, max_context=1024, use_graphs=False,
                    prefix_sharing=True)
    eng.generate([GenRequest(p, max_tokens=2, temperature=0.0, ignore_eos=True) for p in prompts])
    pf = eng._pfx
    assert pf is not None and pf.n == 128
    full = prompts[0]
    n = len(full)
    cap_k = torch.zeros(cfg.layers, n, cfg.kv_heads, 128, dtype=torch.bfloat16, device="cuda")
    cap_v = torch.zeros_like(cap_k)

    def sink(i, k, v):
        cap_k[i].copy_(k.reshape(n, cfg.kv_heads, 128))
        cap_v[i].copy_(v.reshape(n, cfg.kv_heads, 128))

    kv2 = PagedKVCache(cfg.layers, 64, cfg.kv_heads, 128, 64, device="cuda")
    var = ops.prefill_variant(m.hq, m.hkv)
    ws, wq = ops.prefill_work_list([n], ops.prefill_block_q(m.hq, m.hkv, var))
    i32 = lambda x: torch.tensor(x, dtype=torch.int32, device="cuda")  # noqa: E731
    from operator_amd.models.llama import ForwardBatch

    fb = ForwardBatch(torch.tensor(full, dtype=torch.long, device="cuda"), torch.arange(n, device="cuda"),
                      torch.arange(n, device="cuda"), True, torch.tensor([n - 1], device="cuda"), seq_lens=[n],
                      prefill_work=(i32([0, n]), i32(ws), i32(wq), var), kv_sink=sink)
    m.forward(fb, kv2)
    for name, got, ref in (("k", eng._pk[:, :pf.n], cap_k[:, :pf.n]), ("v", eng._pv[:, :pf.n], cap_v[:, :pf.n])):
        err = (got.float() - ref.float()).abs()
        scale = ref.float().abs().amax()
        assert float(err.amax()) <= 0.03 * float(scale) + 1e-3, (name, float(err.amax()), float(scale))
