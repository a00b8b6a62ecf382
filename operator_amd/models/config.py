"""Explanation-model configurations (Llama-architecture families, head_dim 128).

The reference delegates explanation to an external LLM via its ai-interface
service (J/service/AIInterfaceClient.java:45-59; AIProvider.spec.modelId), so
whichever model a user had behind that hop must be servable on-node. Supported
architectures share one decoder (pre-norm RMSNorm, RoPE, GQA, SwiGLU):

  llama    Llama-2/3/3.1/3.2 (llama3 rope scaling, tied embeddings for 3.2)
  mistral  Mistral-7B v0.2/v0.3 (no sliding window in those releases)
  qwen2    Qwen2 / Qwen2.5 (bias on the q/k/v projections, rms eps 1e-6)

BASELINE.json names Llama-3-8B (TP=1) and Llama-3-70B (TP=8) as the configs.
There are no checkpoints offline, so weights are random-initialised with the
exact architecture, or loaded from a local HF safetensors directory whose
``config.json`` then defines the architecture (``config_from_hf``).
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace

ARCHS = ("llama", "mistral", "qwen2")


@dataclass(frozen=True)
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden: int = 4096
    intermediate: int = 14336
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    rope_scaling: dict | None = field(default=None, hash=False, compare=False)
    bos_id: int = 128000
    eos_ids: tuple[int, ...] = (128001, 128009)
    arch: str = "llama"
    qkv_bias: bool = False      # qwen2: q/k/v projections carry a bias
    add_bos: bool = True        # prepend bos_id to prompts (qwen2 tokenizers do not)

    @property
    def qkv_width(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def param_count(self) -> int:
        h, i, v = self.hidden, self.intermediate, self.vocab_size
        per = h * self.qkv_width + self.heads * self.head_dim * h + 2 * h * i + i * h + 2 * h
        per += self.qkv_width if self.qkv_bias else 0
        return self.layers * per + v * h * (1 if self.tie_embeddings else 2) + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.layers * 2 * self.kv_heads * self.head_dim * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)


_LLAMA31_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                    "original_max_position_embeddings": 8192}

PRESETS: dict[str, LlamaConfig] = {
    "llama3-8b": LlamaConfig(),
    "llama3.1-8b": LlamaConfig(name="llama3.1-8b", max_position=131072, rope_scaling=_LLAMA31_SCALING),
    "llama3-70b": LlamaConfig(name="llama3-70b", hidden=8192, intermediate=28672, layers=80, heads=64, kv_heads=8),
    "llama3.1-70b": LlamaConfig(name="llama3.1-70b", hidden=8192, intermediate=28672, layers=80, heads=64,
                                kv_heads=8, max_position=131072, rope_scaling=_LLAMA31_SCALING),
    "llama3.2-3b": LlamaConfig(name="llama3.2-3b", hidden=3072, intermediate=8192, layers=28, heads=24, kv_heads=8,
                               max_position=131072, tie_embeddings=True,
                               rope_scaling={**_LLAMA31_SCALING, "factor": 32.0}),
    "mistral-7b": LlamaConfig(name="mistral-7b", arch="mistral", vocab_size=32768, hidden=4096, intermediate=14336,
                              layers=32, heads=32, kv_heads=8, rope_theta=1e6, max_position=32768, bos_id=1,
                              eos_ids=(2,)),
    "qwen2.5-7b": LlamaConfig(name="qwen2.5-7b", arch="qwen2", vocab_size=152064, hidden=3584, intermediate=18944,
                              layers=28, heads=28, kv_heads=4, rope_theta=1e6, rms_eps=1e-6, max_position=32768,
                              qkv_bias=True, add_bos=False, bos_id=151643, eos_ids=(151645, 151643)),
    "qwen2.5-3b": LlamaConfig(name="qwen2.5-3b", arch="qwen2", vocab_size=151936, hidden=2048, intermediate=11008,
                              layers=36, heads=16, kv_heads=2, rope_theta=1e6, rms_eps=1e-6, max_position=32768,
                              tie_embeddings=True, qkv_bias=True, add_bos=False, bos_id=151643,
                              eos_ids=(151645, 151643)),
    # small configs with the same kernels (head_dim 128, GQA) for tests / quick runs
    "llama-1b-hd128": LlamaConfig(name="llama-1b-hd128", hidden=2048, intermediate=8192, layers=16, heads=16,
                                  kv_heads=4),
    "tiny": LlamaConfig(name="tiny", vocab_size=1024, hidden=256, intermediate=512, layers=2, heads=2, kv_heads=1,
                        max_position=4096, bos_id=1000, eos_ids=(1001,)),
    "tiny-gqa4": LlamaConfig(name="tiny-gqa4", vocab_size=2048, hidden=1024, intermediate=1024, layers=2, heads=8,
                             kv_heads=2, max_position=4096, bos_id=2000, eos_ids=(2001,)),
    # 70B-shaped head layout (GQA 8: 64/8 heads at 70B) that every TP degree up to 8 divides:
    # heads, kv heads, FFN width (64-feature SwiGLU blocks per rank) and vocab
    "tiny-tp8": LlamaConfig(name="tiny-tp8", vocab_size=2048, hidden=512, intermediate=1024, layers=2, heads=16,
                            kv_heads=8, max_position=4096, bos_id=2000, eos_ids=(2001,)),
    # qwen2-shaped: q/k/v bias and a GQA group of 7 (Qwen2.5-7B's 28/4)
    "tiny-qwen": LlamaConfig(name="tiny-qwen", arch="qwen2", vocab_size=2048, hidden=896, intermediate=1024, layers=2,
                             heads=7, kv_heads=1, rope_theta=1e6, rms_eps=1e-6, max_position=4096, qkv_bias=True,
                             add_bos=False, bos_id=2000, eos_ids=(2001,)),
}


def get_config(name: str, **overrides) -> LlamaConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    c = PRESETS[name]
    return replace(c, **overrides) if overrides else c


def _ids(v) -> tuple[int, ...]:
    if v is None:
        return ()
    return tuple(int(x) for x in (v if isinstance(v, (list, tuple)) else [v]))


def config_from_hf(path: str, name: str | None = None) -> LlamaConfig:
    """LlamaConfig from a HuggingFace checkpoint directory's ``config.json`` (plus the
    eos ids of ``generation_config.json`` when present). Raises ValueError for an
    architecture or shape the gfx950 kernels do not serve."""
    with open(os.path.join(path, "config.json")) as f:
        hc = json.load(f)
    mt = hc.get("model_type", "llama")
    if mt not in ARCHS:
        raise ValueError(f"{path}: model_type {mt!r} not supported (supported: {', '.join(ARCHS)})")
    heads = int(hc["num_attention_heads"])
    hidden = int(hc["hidden_size"])
    head_dim = int(hc.get("head_dim") or hidden // heads)
    if head_dim != 128:
        raise ValueError(f"{path}: head_dim {head_dim}; the attention kernels are built for head_dim 128")
    kv_heads = int(hc.get("num_key_value_heads") or heads)
    if heads % kv_heads or heads // kv_heads > 8:
        raise ValueError(f"{path}: GQA group {heads}/{kv_heads} not supported (1..8 query heads per kv head)")
    max_pos = int(hc.get("max_position_embeddings", 8192))
    sw = hc.get("sliding_window")
    if sw and (mt != "qwen2" or hc.get("use_sliding_window")):
        # full attention equals sliding-window attention while contexts stay inside the window
        max_pos = min(max_pos, int(sw))
    eos = _ids(hc.get("eos_token_id"))
    gen = os.path.join(path, "generation_config.json")
    if os.path.exists(gen):
        with open(gen) as f:
            eos = tuple(dict.fromkeys(eos + _ids(json.load(f).get("eos_token_id"))))
    rs = hc.get("rope_scaling")
    if rs is not None:
        rs = dict(rs)
        rs.setdefault("rope_type", rs.get("type"))
        if rs["rope_type"] not in ("llama3", "default", None):
            raise ValueError(f"{path}: rope_scaling type {rs['rope_type']!r} not supported")
        if rs["rope_type"] != "llama3":
            rs = None
    bos = hc.get("bos_token_id")
    return LlamaConfig(
        name=name or os.path.basename(os.path.normpath(path)), arch=mt, vocab_size=int(hc["vocab_size"]),
        hidden=hidden, intermediate=int(hc["intermediate_size"]), layers=int(hc["num_hidden_layers"]), heads=heads,
        kv_heads=kv_heads, head_dim=head_dim, rope_theta=float(hc.get("rope_theta", 10000.0)),
        rms_eps=float(hc.get("rms_norm_eps", 1e-5)), max_position=max_pos,
        tie_embeddings=bool(hc.get("tie_word_embeddings", False)), rope_scaling=rs,
        bos_id=int(bos) if bos is not None else -1, eos_ids=eos or (-1,),
        qkv_bias=bool(hc.get("attention_bias", mt == "qwen2")),
        add_bos=mt != "qwen2" and bos is not None)
