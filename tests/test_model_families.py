"""Model families beyond Llama-3 (models/config.py): HF config.json parsing, Qwen2
(q/k/v bias, GQA group 7) and Mistral parity with transformers on the CPU reference
path, a safetensors checkpoint round trip through the engine factory, and the
checkpoint-tokenizer rules (no double BOS, add_bos, chat templates)."""
import json

import pytest
import torch

from operator_amd.config import load_settings
from operator_amd.models.config import PRESETS, config_from_hf, get_config
from operator_amd.models.kv_cache import PagedKVCache
from operator_amd.models.llama import ForwardBatch, LlamaModel


def _logits(m, ids):
    cfg = m.cfg
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, page_size=16, device="cpu", dtype=m.dtype)
    T = len(ids)
    fb = ForwardBatch(torch.tensor(ids), torch.arange(T), torch.full((T,), -1, dtype=torch.long), True, None,
                      seq_lens=[T])
    return m.forward(fb, kv)


def _hf_state_dict(m: LlamaModel) -> dict:
    cfg, D = m.cfg, m.cfg.head_dim
    sd = {"model.embed_tokens.weight": m.embed, "model.norm.weight": m.final_norm, "lm_head.weight": m.lm_head}
    sizes = [cfg.heads * D, cfg.kv_heads * D, cfg.kv_heads * D]
    for i, lw in enumerate(m.layers):
        q, k, v = torch.split(lw.wqkv, sizes)
        g, u = m.split_gate_up(lw.wgu)
        p = f"model.layers.{i}."
        sd.update({p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                   p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": lw.wo,
                   p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u, p + "mlp.down_proj.weight": lw.wd,
                   p + "input_layernorm.weight": lw.attn_norm, p + "post_attention_layernorm.weight": lw.mlp_norm})
        if lw.bqkv is not None:
            bq, bk, bv = torch.split(lw.bqkv, sizes)
            sd.update({p + "self_attn.q_proj.bias": bq, p + "self_attn.k_proj.bias": bk,
                       p + "self_attn.v_proj.bias": bv})
    return {k: v.contiguous() for k, v in sd.items()}


def _hf_config_dict(cfg) -> dict:
    d = {"model_type": cfg.arch, "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden,
         "intermediate_size": cfg.intermediate, "num_hidden_layers": cfg.layers, "num_attention_heads": cfg.heads,
         "num_key_value_heads": cfg.kv_heads, "head_dim": cfg.head_dim, "rope_theta": cfg.rope_theta,
         "rms_norm_eps": cfg.rms_eps, "max_position_embeddings": cfg.max_position,
         "tie_word_embeddings": cfg.tie_embeddings, "bos_token_id": cfg.bos_id, "eos_token_id": list(cfg.eos_ids)}
    if cfg.arch == "qwen2":
        d.update(use_sliding_window=False, sliding_window=cfg.max_position)
    if cfg.arch == "mistral":
        d["sliding_window"] = None
    return d


def test_presets_param_counts():
    # published sizes of the released checkpoints
    for name, billions in (("qwen2.5-7b", 7.62), ("qwen2.5-3b", 3.09), ("mistral-7b", 7.25), ("llama3.2-3b", 3.21),
                           ("llama3-8b", 8.03), ("llama3.1-70b", 70.55)):
        assert abs(PRESETS[name].param_count() / 1e9 - billions) < 0.01, name


def test_config_from_hf(tmp_path):
    for name in ("qwen2.5-7b", "mistral-7b", "llama3.1-8b", "llama3.2-3b"):
        ref = PRESETS[name]
        d = tmp_path / name
        d.mkdir()
        hc = _hf_config_dict(ref)
        if ref.rope_scaling:
            hc["rope_scaling"] = ref.rope_scaling
        (d / "config.json").write_text(json.dumps(hc))
        c = config_from_hf(str(d), name=name)
        for f in ("arch", "vocab_size", "hidden", "intermediate", "layers", "heads", "kv_heads", "rope_theta",
                  "rms_eps", "max_position", "tie_embeddings", "qkv_bias", "add_bos", "eos_ids", "bos_id"):
            assert getattr(c, f) == getattr(ref, f), (name, f)
        assert c.rope_scaling == ref.rope_scaling
    # generation_config eos ids are merged in
    d = tmp_path / "qwen2.5-7b"
    (d / "generation_config.json").write_text(json.dumps({"eos_token_id": [151645, 151643, 151999]}))
    assert config_from_hf(str(d)).eos_ids == (151645, 151643, 151999)
    # a Mistral-v0.1-style sliding window caps the context (full attention == SWA inside it)
    hc = _hf_config_dict(PRESETS["mistral-7b"])
    hc["sliding_window"] = 4096
    (tmp_path / "m01").mkdir()
    (tmp_path / "m01" / "config.json").write_text(json.dumps(hc))
    assert config_from_hf(str(tmp_path / "m01")).max_position == 4096
    # shapes the kernels do not serve are refused, not silently mis-run
    for bad in ({"model_type": "gemma"}, {"head_dim": 64}, {"num_key_value_heads": 1, "num_attention_heads": 32}):
        hc = {**_hf_config_dict(PRESETS["llama3-8b"]), **bad}
        p = tmp_path / f"bad{len(list(tmp_path.iterdir()))}"
        p.mkdir()
        (p / "config.json").write_text(json.dumps(hc))
        with pytest.raises(ValueError):
            config_from_hf(str(p))


@pytest.mark.parametrize("arch", ["qwen2", "mistral"])
def test_matches_transformers(arch):
    transformers = pytest.importorskip("transformers")
    if arch == "qwen2":
        cfg = get_config("tiny-qwen")
        hf_cfg = transformers.Qwen2Config(**{k: v for k, v in _hf_config_dict(cfg).items() if k != "model_type"})
        hf_cls = transformers.Qwen2ForCausalLM
    else:
        cfg = get_config("tiny-gqa4", arch="mistral", rope_theta=1e6)
        hf_cfg = transformers.MistralConfig(**{k: v for k, v in _hf_config_dict(cfg).items() if k != "model_type"})
        hf_cls = transformers.MistralForCausalLM
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=7)
    hf = hf_cls(hf_cfg).eval().float()
    missing, unexpected = hf.load_state_dict(_hf_state_dict(m), strict=False)
    assert not [k for k in missing if "rotary" not in k], missing
    assert not unexpected, unexpected
    ids = torch.randint(0, cfg.vocab_size, (1, 41))
    with torch.no_grad():
        ref = hf(ids).logits[0]
    torch.testing.assert_close(_logits(m, ids[0].tolist()), ref, atol=2e-3, rtol=2e-3)


def test_checkpoint_roundtrip_through_factory(tmp_path):
    """A Qwen2-style safetensors checkpoint directory is served through the engine
    factory: config.json defines the model, biases load, logits match the source."""
    from safetensors.torch import save_file

    from operator_amd.engine.factory import build_llm

    cfg = get_config("tiny-qwen")
    src = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=3)
    save_file(_hf_state_dict(src), str(tmp_path / "model.safetensors"))
    (tmp_path / "config.json").write_text(json.dumps(_hf_config_dict(cfg)))
    s = load_settings(env={}, overrides={"engine.model_path": str(tmp_path), "engine.device": "cpu",
                                         "engine.dtype": "float32", "engine.kv_cache_gb": 0.01,
                                         "engine.use_graphs": False, "engine.max_batch": 4})
    model, kv, llm, tok = build_llm(s)
    assert model.cfg.arch == "qwen2" and model.cfg.qkv_bias and not tok.add_bos
    assert model.layers[0].bqkv is not None
    ids = list(range(5, 30))
    torch.testing.assert_close(_logits(model, ids), _logits(src, ids), atol=1e-5, rtol=1e-5)


def _checkpoint_tokenizer(path, with_bos_processor=True):
    import tokenizers
    from tokenizers import models, pre_tokenizers, processors

    vocab = {"<s>": 0, "</s>": 1, "<unk>": 2, "<|user|>": 3, "<|assistant|>": 4}
    for i, w in enumerate("pod failed with OOMKilled exit code 137 the container".split()):
        vocab[w] = 5 + i
    tk = tokenizers.Tokenizer(models.WordLevel(vocab, unk_token="<unk>"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    tk.add_special_tokens(["<s>", "</s>", "<|user|>", "<|assistant|>"])
    if with_bos_processor:  # what Llama-3's tokenizer.json does: prepend BOS itself
        tk.post_processor = processors.TemplateProcessing(single="<s> $A", special_tokens=[("<s>", 0)])
    tk.save(str(path))
    return vocab


def test_checkpoint_tokenizer_single_bos_and_chat_template(tmp_path):
    from operator_amd.engine.tokenizer import Tokenizer, load_chat_template

    f = tmp_path / "tokenizer.json"
    vocab = _checkpoint_tokenizer(f)
    t = Tokenizer(100, 0, 1, path=str(f))
    ids = t.encode("pod failed with OOMKilled")
    assert ids == [0, vocab["pod"], vocab["failed"], vocab["with"], vocab["OOMKilled"]]  # one BOS, not two
    assert Tokenizer(100, 0, 1, path=str(f), add_bos=False).encode("pod failed") == [vocab["pod"], vocab["failed"]]
    assert t.decode(ids + [1]) == "pod failed with OOMKilled"
    # chat template from tokenizer_config.json ("auto"): BOS and turn markers come from the template
    tpl = ("{{ bos_token }}{% for m in messages %}<|{{ m.role }}|> {{ m.content }} {% endfor %}"
           "{% if add_generation_prompt %}<|assistant|>{% endif %}")
    (tmp_path / "tokenizer_config.json").write_text(json.dumps({"chat_template": tpl}))
    assert load_chat_template("auto", str(tmp_path)) == tpl
    assert load_chat_template("none", str(tmp_path)) is None
    assert load_chat_template("auto", None) is None
    tc = Tokenizer(100, 0, 1, path=str(f), chat_template=load_chat_template("auto", str(tmp_path)))
    assert tc.encode("pod failed") == [0, vocab["<|user|>"], vocab["pod"], vocab["failed"], vocab["<|assistant|>"]]
    with pytest.raises(Exception):
        Tokenizer(100, 0, 1, path=str(f), chat_template="{{ raise_exception('no system role') }}").encode("x")


def test_several_local_models_routed_by_model_id(tmp_path):
    """engine.extra_models: each local model its own engine; an AIProvider's modelId
    picks it (case-insensitive), anything else goes to engine.model; the AIProvider
    controller reports which engine serves the provider."""
    from operator_amd.api.models import AIProviderConfig, AnalysisResult, AnalysisSummary
    from operator_amd.controller.aiprovider import AIProviderReconciler
    from operator_amd.engine.factory import build_explain_service
    from operator_amd.engine.providers import ProviderRouter
    from operator_amd.kube.fake import FakeKube

    s = load_settings(env={}, overrides={"engine.model": "tiny", "engine.extra_models": ["tiny-gqa4"],
                                         "engine.device": "cpu", "engine.dtype": "float32",
                                         "engine.kv_cache_gb": 0.04, "engine.use_graphs": False,
                                         "engine.max_batch": 4, "engine.max_context": 512})
    svc = build_explain_service(s)
    try:
        assert svc.models == ["tiny", "tiny-gqa4"]
        res = AnalysisResult(pod_name="p", pod_namespace="default",
                             summary=AnalysisSummary(highest_severity="HIGH", significant_events=1))
        st = {m: svc.services[m].ee.llm.stats for m in svc.models}
        before = {m: st[m].decode_tokens for m in svc.models}
        svc.explain(res, AIProviderConfig(model_id="TINY-GQA4", max_tokens=5, caching_enabled=False))
        assert st["tiny-gqa4"].decode_tokens > before["tiny-gqa4"] and st["tiny"].decode_tokens == before["tiny"]
        svc.explain(res, AIProviderConfig(model_id="gpt-4o", max_tokens=5, caching_enabled=False))
        assert st["tiny"].decode_tokens > before["tiny"]   # unknown model -> the default engine
        out = svc.explain_many([(res, AIProviderConfig(model_id=m, max_tokens=3, caching_enabled=False))
                                for m in ("tiny", "tiny-gqa4", "tiny")])
        assert [o.tokens_generated for o in out] == [3, 3, 3]
        rec = AIProviderReconciler(FakeKube(), ProviderRouter(svc), "tiny")
        msg = rec.reconcile({"metadata": {"name": "a", "namespace": "default"},
                             "spec": {"providerId": "local", "modelId": "tiny-gqa4"}}).status["message"]
        assert msg == "Served by on-node engine (tiny-gqa4)"
        msg = rec.reconcile({"metadata": {"name": "b", "namespace": "default"},
                             "spec": {"providerId": "local", "modelId": "other"}}).status["message"]
        assert msg.endswith("requested modelId other is mapped to tiny")
    finally:
        svc.close()


def test_streaming_detokenization_with_checkpoint_special_tokens(tmp_path):
    """A checkpoint-style byte-level BPE with special tokens (Llama-3 ships 256 <|...|> ids):
    decode() skips them, so the byte table maps them to no bytes and streaming stays on."""
    import random

    import tokenizers
    from tokenizers import decoders, models, pre_tokenizers, trainers

    from operator_amd.engine.tokenizer import Tokenizer

    tk = tokenizers.Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=400, show_progress=False, initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tk.train_from_iterator(["pod failed with OOMKilled", "Back-off restarting failed container"] * 50, trainer=tr)
    tk.add_special_tokens(["<|begin_of_text|>", "<|eot_id|>"] + [f"<|reserved_special_token_{i}|>" for i in range(8)])
    f = tmp_path / "tokenizer.json"
    tk.save(str(f))
    t = Tokenizer(tk.get_vocab_size(), tk.token_to_id("<|begin_of_text|>"), tk.token_to_id("<|eot_id|>"), path=str(f))
    assert t.byte_table() is not None
    specials = [tk.token_to_id(f"<|reserved_special_token_{i}|>") for i in range(8)]
    rng = random.Random(5)
    for _ in range(10):
        ids = [rng.randrange(0, t.n_vocab) for _ in range(60)] + specials
        rng.shuffle(ids)
        buf = bytearray()
        t.feed(buf, ids)
        assert t.text_of(buf) == t.decode(ids)


def test_streaming_detokenization_is_exact_or_off(tmp_path):
    """Tokenizer.byte_table: a byte-level BPE streams each request's bytes per decode window
    (LLMEngine.token_hook) and its text equals decode() for any ids (ids past the vocabulary,
    BOS/EOS, invalid UTF-8 included); a tokenizer whose decoding is not plain byte
    concatenation (WordLevel joins with spaces) is detected and keeps decode_batch."""
    import random

    import torch

    from operator_amd.engine.llm import GenRequest, LLMEngine
    from operator_amd.engine.tokenizer import Tokenizer
    from operator_amd.models.config import get_config
    from operator_amd.models.kv_cache import PagedKVCache
    from operator_amd.models.llama import LlamaModel

    f = tmp_path / "tokenizer.json"
    _checkpoint_tokenizer(f)
    assert Tokenizer(100, 0, 1, path=str(f)).byte_table() is None
    cfg = get_config("tiny")
    tok = Tokenizer(cfg.vocab_size, cfg.bos_id, cfg.eos_ids[0])
    assert tok.byte_table() is not None
    rng = random.Random(3)
    for _ in range(20):
        ids = [rng.randrange(0, cfg.vocab_size + 50) for _ in range(rng.randrange(1, 200))]
        buf = bytearray()
        for w in range(0, len(ids), 8):
            tok.feed(buf, ids[w:w + 8])
        assert tok.text_of(buf) == tok.decode(ids)
    # through the engine: the per-window hook sees every appended token exactly once
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32).init_random(seed=2)
    kv = PagedKVCache(cfg.layers, 64, cfg.kv_heads, cfg.head_dim, 16, device="cpu", dtype=torch.float32)
    eng = LLMEngine(m, kv, max_batch=4, max_context=256, use_graphs=False, multi_step=4)

    def hook(reqs):
        for r in reqs:
            if r.detok is None:
                r.detok = bytearray()
            tok.feed(r.detok, r.output[r.detok_pos:])
            r.detok_pos = len(r.output)

    eng.token_hook = hook
    reqs = [GenRequest(list(range(3, 20 + 7 * i)), max_tokens=13 + i, temperature=0.7, seed=i, ignore_eos=True)
            for i in range(3)]
    eng.generate(reqs)
    for r in reqs:
        hook([r])
        assert tok.text_of(r.detok) == tok.decode(r.output)
