"""Explanation model correctness on CPU (reference ops): architecture parity with
HuggingFace transformers' LlamaForCausalLM, and KV-cached decode == full recompute."""
import pytest
import torch

from operator_amd.engine.llm import GenRequest, LLMEngine
from operator_amd.models.config import get_config
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import ForwardBatch, LlamaModel


def _tiny(name="tiny-gqa4", dtype=torch.float32):
    cfg = get_config(name)
    m = LlamaModel(cfg, device="cpu", dtype=dtype).init_random(seed=7)
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=dtype)
    return cfg, m, kv


def _full_logits(m, kv, ids):
    T = len(ids)
    fb = ForwardBatch(torch.tensor(ids), torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None,
                      seq_lens=[T])
    return m.forward(fb, kv)


def test_matches_transformers_llama():
    transformers = pytest.importorskip("transformers")
    cfg, m, kv = _tiny()
    hf_cfg = transformers.LlamaConfig(
        vocab_size=cfg.vocab_size, hidden_size=cfg.hidden, intermediate_size=cfg.intermediate,
        num_hidden_layers=cfg.layers, num_attention_heads=cfg.heads, num_key_value_heads=cfg.kv_heads,
        head_dim=cfg.head_dim, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps,
        max_position_embeddings=cfg.max_position, tie_word_embeddings=False, attention_bias=False, mlp_bias=False)
    hf = transformers.LlamaForCausalLM(hf_cfg).eval().float()
    D, H = cfg.head_dim, cfg.hidden
    sd = {"model.embed_tokens.weight": m.embed, "model.norm.weight": m.final_norm, "lm_head.weight": m.lm_head}
    for i, lw in enumerate(m.layers):
        q, k, v = torch.split(lw.wqkv, [cfg.heads * D, cfg.kv_heads * D, cfg.kv_heads * D])
        g, u = m.split_gate_up(lw.wgu)
        p = f"model.layers.{i}."
        sd.update({p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                   p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": lw.wo,
                   p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u, p + "mlp.down_proj.weight": lw.wd,
                   p + "input_layernorm.weight": lw.attn_norm, p + "post_attention_layernorm.weight": lw.mlp_norm})
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    assert not [k for k in missing if "rotary" not in k], missing
    ids = torch.randint(0, cfg.vocab_size, (1, 37))
    with torch.no_grad():
        ref = hf(ids).logits[0]
    ours = _full_logits(m, kv, ids[0].tolist())
    torch.testing.assert_close(ours, ref, atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("name", ["tiny", "tiny-gqa4"])
def test_cached_decode_equals_recompute(name):
    cfg, m, kv = _tiny(name)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    prompts = [[5, 9, 13, 2, 7], list(range(40, 80)), [3]]
    reqs = [GenRequest(p, max_tokens=12, temperature=0.0, ignore_eos=True) for p in prompts]
    eng.generate(reqs)
    for r in reqs:
        seq = list(r.prompt)
        for _ in range(12):
            nxt = int(torch.argmax(_full_logits(m, kv, seq)[-1]))
            seq.append(nxt)
        assert r.output == seq[len(r.prompt):], (r.output, seq[len(r.prompt):])
    assert kv.allocator.free + eng.prefix_pages == kv.num_pages  # every page returned


def test_sampling_is_seeded_and_batch_invariant():
    cfg, m, kv = _tiny("tiny")
    eng = LLMEngine(m, kv, max_batch=8, max_context=128, use_graphs=False)
    a = eng.generate([GenRequest([1, 2, 3], max_tokens=8, temperature=0.8, seed=11, ignore_eos=True)])[0].output
    b = eng.generate([GenRequest([1, 2, 3], max_tokens=8, temperature=0.8, seed=11, ignore_eos=True),
                      GenRequest([4, 5], max_tokens=3, temperature=0.8, seed=3, ignore_eos=True)])[0].output
    c = eng.generate([GenRequest([1, 2, 3], max_tokens=8, temperature=0.8, seed=12, ignore_eos=True)])[0].output
    assert a == b
    assert a != c


def test_fp8_weight_model_tracks_bf16():
    cfg = get_config("tiny-gqa4")
    logits = {}
    for wd in ("bfloat16", "fp8"):
        m = LlamaModel(cfg, device="cpu", dtype=torch.float32, weight_dtype=wd).init_random(seed=7)
        kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=torch.float32)
        logits[wd] = _full_logits(m, kv, list(range(3, 40)))
        if wd == "fp8":
            assert m.layers[0].wqkv.dtype == torch.float8_e4m3fn and m.layers[0].sqkv is not None
            eng = LLMEngine(m, kv, max_batch=2, max_context=256, use_graphs=False)
            r = eng.generate([GenRequest([5, 6, 7], max_tokens=5, temperature=0.0, ignore_eos=True)])[0]
            assert len(r.output) == 5
    cos = torch.nn.functional.cosine_similarity(logits["fp8"].flatten(), logits["bfloat16"].flatten(), dim=0)
    assert cos > 0.98, float(cos)


def test_fp8_kv_cache_tracks_bf16_cache():
    """An e4m3fn KV cache (stored x / scale): cached decode logits stay close to the
    full-precision cache; prefill attention never reads the cache."""
    cfg = get_config("tiny-gqa4")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=7)
    prompt = list(range(10, 60))
    outs = {}
    for name, dt, sc in (("f32", torch.float32, 1.0), ("fp8", torch.float8_e4m3fn, 0.5)):
        kv = PagedKVCache(cfg.layers, 16, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=dt,
                          k_scale=sc, v_scale=sc)
        eng = LLMEngine(m, kv, max_batch=2, max_context=256, use_graphs=False)
        r = eng.generate([GenRequest(prompt, max_tokens=6, temperature=0.0, ignore_eos=True)])[0]
        assert kv.k.dtype == dt
        outs[name] = r.output
    # greedy tokens from fp8 keys/values agree with the fp32 cache on a random model
    assert sum(a == b for a, b in zip(outs["f32"], outs["fp8"])) >= 4, outs


def test_engine_prefill_failure_releases_pages():
    """A step that raises during the PREFILL (the batch is off `waiting`, pages
    allocated, not yet `running`) still returns every page and fails the batch."""
    from operator_amd.engine.explain import EngineLoop

    cfg = get_config("tiny")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=4)
    kv = PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    real, calls = m.forward, {"n": 0}

    def flaky(fb, kv_):
        calls["n"] += 1
        if calls["n"] == 1:
            assert fb.is_prefill
            raise RuntimeError("HIP out of memory (injected in prefill)")
        return real(fb, kv_)

    m.forward = flaky
    loop = EngineLoop(eng)
    loop.start()
    try:
        first = [GenRequest(list(range(1, 30)), max_tokens=8, temperature=0.0, ignore_eos=True) for _ in range(3)]
        for r in first:
            eng.submit(r)
        loop.notify()
        for r in first:
            assert r.event.wait(60)
        assert all(r.error and "out of memory" in r.error for r in first)
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages and loop.fatal is None
        again = GenRequest(list(range(1, 30)), max_tokens=4, temperature=0.0, ignore_eos=True)
        eng.submit(again)
        loop.notify()
        assert again.event.wait(60) and again.error is None and len(again.output) == 4
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages
    finally:
        loop.stop()
        loop.join(10)


def test_engine_step_failure_releases_pages_and_keeps_serving():
    """A step that raises (e.g. out of memory) fails the requests it held, returns
    their KV pages and leaves the engine loop serving the next requests."""
    from operator_amd.engine.explain import EngineLoop

    cfg = get_config("tiny")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=4)
    kv = PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
    real, calls = m.forward, {"n": 0}

    def flaky(fb, kv_):
        calls["n"] += 1
        if calls["n"] == 3:   # fail mid-generation, with pages held
            raise RuntimeError("HIP out of memory (injected)")
        return real(fb, kv_)

    m.forward = flaky
    loop = EngineLoop(eng)
    loop.start()
    try:
        first = [GenRequest(list(range(1, 30)), max_tokens=8, temperature=0.0, ignore_eos=True) for _ in range(3)]
        for r in first:
            eng.submit(r)
        loop.notify()
        for r in first:
            assert r.event.wait(60)
        assert all(r.error and "out of memory" in r.error for r in first)
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages and loop.fatal is None and loop.is_alive()
        again = GenRequest(list(range(1, 30)), max_tokens=8, temperature=0.0, ignore_eos=True)
        eng.submit(again)
        loop.notify()
        assert again.event.wait(60) and again.error is None and len(again.output) == 8
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages
    finally:
        loop.stop()
        loop.join(10)


def test_pipelined_prefill_batches_match_one_at_a_time():
    """Several prefill batches in a row (max_prefill_tokens forces one prompt per
    batch): each batch is launched before the previous one's first tokens are read,
    and every request still generates exactly what it generates alone."""
    cfg, m, kv = _tiny("tiny-gqa4")
    prompts = [list(range(3, 40)), list(range(50, 75)), list(range(9, 39)), list(range(100, 135))]
    alone = []
    for p in prompts:
        e1 = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False)
        alone.append(e1.generate([GenRequest(p, max_tokens=6, temperature=0.0, ignore_eos=True)])[0].output)
    eng = LLMEngine(m, kv, max_batch=4, max_prefill_tokens=40, max_context=256, use_graphs=False)
    reqs = [GenRequest(p, max_tokens=6, temperature=0.0, ignore_eos=True) for p in prompts]
    for r in reqs:
        eng.submit(r)
    launched = []
    real = eng._prefill

    def spy(batch):
        launched.append((len(batch), eng._pf is not None))   # a previous batch still pending?
        return real(batch)

    eng._prefill = spy
    while any(not r.done for r in reqs):
        eng.step()
    assert [r.output for r in reqs] == alone
    assert len(launched) == 4 and sum(p for _, p in launched) == 3   # batches 2-4 queued behind a pending one
    assert kv.allocator.free + eng.prefix_pages == kv.num_pages


def test_pipelined_prefill_failure_releases_both_batches():
    """A launch that raises while the previous prefill batch is still pending fails
    and releases both batches (pages allocated, rows not yet running)."""
    from operator_amd.engine.explain import EngineLoop

    cfg = get_config("tiny")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=4)
    kv = PagedKVCache(cfg.layers, 32, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=4, max_prefill_tokens=32, max_context=256, use_graphs=False)
    real, calls = m.forward, {"n": 0}

    def flaky(fb, kv_):
        calls["n"] += 1
        if calls["n"] == 2:
            assert fb.is_prefill and eng._pf is not None
            raise RuntimeError("HIP out of memory (injected in the second prefill)")
        return real(fb, kv_)

    m.forward = flaky
    reqs = [GenRequest(list(range(1, 30)), max_tokens=4, temperature=0.0, ignore_eos=True) for _ in range(2)]
    for r in reqs:
        eng.submit(r)
    loop = EngineLoop(eng)
    loop.start()
    try:
        loop.notify()
        for r in reqs:
            assert r.event.wait(60)
        assert all(r.error and "out of memory" in r.error for r in reqs)
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages and loop.fatal is None and eng._pf is None
        again = GenRequest(list(range(1, 30)), max_tokens=4, temperature=0.0, ignore_eos=True)
        eng.submit(again)
        loop.notify()
        assert again.event.wait(60) and again.error is None and len(again.output) == 4
        assert kv.allocator.free + eng.prefix_pages == kv.num_pages
    finally:
        loop.stop()
        loop.join(10)


@pytest.mark.parametrize("wd", ["bfloat16", "fp8"])
def test_weight_cache_roundtrip(tmp_path, wd):
    """engine.weight_cache_dir: the first start builds and writes the shard, the next maps
    it back (identical tensors); another seed / dtype is a different key, never a hit."""
    import os

    from operator_amd.models import weight_cache

    cfg = get_config("tiny-gqa4")
    a = LlamaModel(cfg, device="cpu", dtype=torch.float32, weight_dtype=wd)
    assert weight_cache.load_or_build(a, str(tmp_path), None, 7) == "miss"
    files = os.listdir(tmp_path)
    assert len(files) == 1 and files[0].endswith("-r0of1.safetensors")
    b = LlamaModel(cfg, device="cpu", dtype=torch.float32, weight_dtype=wd)
    assert weight_cache.load_or_build(b, str(tmp_path), None, 7) == "hit"
    assert len(b.layers) == len(a.layers)
    for t0, t1 in [(a.embed, b.embed), (a.lm_head, b.lm_head), (a.final_norm, b.final_norm)]:
        assert torch.equal(t0, t1)
    for la, lb in zip(a.layers, b.layers):
        for f in weight_cache.LAYER_FIELDS:
            x, y = getattr(la, f), getattr(lb, f)
            assert (x is None) == (y is None)
            if x is not None:
                assert x.dtype == y.dtype and torch.equal(x.view(torch.uint8), y.view(torch.uint8)), f
    c = LlamaModel(cfg, device="cpu", dtype=torch.float32, weight_dtype=wd)
    assert weight_cache.load_or_build(c, str(tmp_path), None, 8) == "miss"   # another seed: new key
    assert len(os.listdir(tmp_path)) == 2
    assert weight_cache.load_or_build(LlamaModel(cfg, device="cpu", dtype=torch.float32), None, None, 7) == "off"
    # a damaged file is rebuilt, not trusted
    p = os.path.join(tmp_path, files[0])
    with open(p, "r+b") as fh:
        fh.truncate(100)
    d = LlamaModel(cfg, device="cpu", dtype=torch.float32, weight_dtype=wd)
    assert weight_cache.load_or_build(d, str(tmp_path), None, 7) == "miss"
    assert torch.equal(d.embed, a.embed)


def test_weight_cache_key_tracks_layout_code(tmp_path):
    """A change to the code that lays a shard out (sharding / packing / quantization) is a
    new cache key: an old file is never mapped back with a stale layout."""
    from operator_amd.models import weight_cache

    cfg = get_config("tiny-gqa4")
    a = LlamaModel(cfg, device="cpu", dtype=torch.float32)
    assert weight_cache.load_or_build(a, str(tmp_path), None, 7) == "miss"

    class Relaid(LlamaModel):   # same everything, but a different shard layout routine
        def _shard_layer(self, *args, **kw):
            lw = super()._shard_layer(*args, **kw)
            return lw

    assert weight_cache.layout_version(Relaid) != weight_cache.layout_version(LlamaModel)
    b = Relaid(cfg, device="cpu", dtype=torch.float32)
    assert weight_cache.cache_path(str(tmp_path), b, "random:7") != weight_cache.cache_path(str(tmp_path), a, "random:7")
    assert weight_cache.load_or_build(b, str(tmp_path), None, 7) == "miss"


def test_tile_out_ok_rejects_outputs_gemm_tile_cannot_write():
    """linear(): an explicit output gemm_tile's binding would refuse (row stride not a
    multiple of 4, misaligned base, strided columns) falls back instead of raising."""
    from operator_amd import ops

    base = torch.empty(64, 132, dtype=torch.bfloat16)
    assert ops.tile_out_ok(None) and ops.tile_out_ok(base[:, :128])
    assert not ops.tile_out_ok(torch.empty(64, 130, dtype=torch.bfloat16)[:, :128])   # row stride 130
    assert not ops.tile_out_ok(base[:, 1:129])                                        # base 2 B off
    assert not ops.tile_out_ok(base.t())                                               # column stride
    assert not ops.tile_out_ok(torch.empty(64, 128, dtype=torch.float32))


def test_prefill_bucket_sizes_bound_padding():
    """Prefill graph buckets: 512-token steps to 4096, then quarter-octave steps, capped
    at max_prefill_tokens; any batch <= the cap fits a bucket padded by < 512 tokens or
    <= 20 % (so no batch cut at a bucket runs eagerly)."""
    from operator_amd.engine.llm import _prefill_bucket_sizes

    b = _prefill_bucket_sizes(32768)
    assert b[:8] == [512 * i for i in range(1, 9)] and b[-1] == 32768
    assert b == sorted(set(b))
    for t in range(1, 32769, 97):
        T = next(x for x in b if x >= t)
        assert T - t < 512 or (T - t) <= 0.2 * T
    assert _prefill_bucket_sizes(1000) == [512, 1000]


def test_decode_window_columns_wrap():
    """A decode window's tokens sit in hist columns (s0 + i) % multi_step (the device step
    counter is not reset per window); _consume reads them in step order across the wrap."""
    import torch

    from operator_amd.engine.llm import GenRequest, LLMEngine, _Window

    eng = LLMEngine.__new__(LLMEngine)
    eng.multi_step, eng.eos, eng.token_hook = 8, set(), None

    class _S:
        decode_tokens = 0
    eng.stats = _S()
    reqs = [GenRequest([1], ignore_eos=True), GenRequest([1], ignore_eos=True)]
    host = torch.arange(16).reshape(2, 8)            # row r, column c -> 8 r + c
    eng._consume(_Window(None, reqs, 2, 4, host, None, 6))
    assert reqs[0].output == [6, 7, 0, 1] and reqs[1].output == [14, 15, 8, 9]
    eng._consume(_Window(None, reqs, 2, 2, host, None, 2))
    assert reqs[0].output[-2:] == [2, 3]


def test_decode_buckets_skip_the_skinny_row_counts():
    """9-64 decode rows share the 64-row bucket (llm.SKIP_BUCKETS: the 16 / 32-row buckets
    would put the bf16 GEMMs on gemm_skinny); an engine whose max_batch is one of them
    keeps it as its largest bucket."""
    from operator_amd.engine.llm import _buckets

    assert _buckets(256) == [1, 2, 4, 8, 64, 128, 256]
    assert _buckets(64) == [1, 2, 4, 8, 64]
    assert _buckets(32) == [1, 2, 4, 8, 32]
    assert _buckets(16) == [1, 2, 4, 8, 16]
    assert _buckets(48) == [1, 2, 4, 8, 48]
