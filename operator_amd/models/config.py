"""Explanation-model configurations (Llama family, head_dim 128).

The reference delegates explanation to an external LLM via its ai-interface
service (J/service/AIInterfaceClient.java:45-59; AIProvider.spec.modelId).
Here the model runs on-node; BASELINE.json names Llama-3-8B (TP=1) and
Llama-3-70B (TP=8) as the configs. There are no checkpoints offline, so
weights are random-initialised with the exact architecture (or loaded from a
local safetensors directory when one exists).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace


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

    @property
    def qkv_width(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def param_count(self) -> int:
        h, i, v = self.hidden, self.intermediate, self.vocab_size
        per = h * self.qkv_width + self.heads * self.head_dim * h + 2 * h * i + i * h + 2 * h
        return self.layers * per + v * h * (1 if self.tie_embeddings else 2) + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.layers * 2 * self.kv_heads * self.head_dim * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)


PRESETS: dict[str, LlamaConfig] = {
    "llama3-8b": LlamaConfig(),
    "llama3.1-8b": LlamaConfig(name="llama3.1-8b", max_position=131072,
                               rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                             "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
    "llama3-70b": LlamaConfig(name="llama3-70b", hidden=8192, intermediate=28672, layers=80, heads=64, kv_heads=8),
    # small configs with the same kernels (head_dim 128, GQA) for tests / quick runs
    "llama-1b-hd128": LlamaConfig(name="llama-1b-hd128", hidden=2048, intermediate=8192, layers=16, heads=16,
                                  kv_heads=4),
    "tiny": LlamaConfig(name="tiny", vocab_size=1024, hidden=256, intermediate=512, layers=2, heads=2, kv_heads=1,
                        max_position=4096, bos_id=1000, eos_ids=(1001,)),
    "tiny-gqa4": LlamaConfig(name="tiny-gqa4", vocab_size=2048, hidden=1024, intermediate=1024, layers=2, heads=8,
                             kv_heads=2, max_position=4096, bos_id=2000, eos_ids=(2001,)),
}


def get_config(name: str, **overrides) -> LlamaConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; known: {sorted(PRESETS)}")
    c = PRESETS[name]
    return replace(c, **overrides) if overrides else c
