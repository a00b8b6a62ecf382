"""Llama-architecture explanation model on the gfx950 kernels.

This is the on-node replacement for the reference's external LLM hop
(ai-interface -> provider, J/service/AIInterfaceClient.java:45-59 and
AIInterfaceRestClient.java:37-39). Per layer:

    x   = rmsnorm(h)                          HIP  (fused residual add)
    qkv = x @ Wqkv^T                          GEMM (fused QKV projection)
    q,k,v = rope_kv(qkv) -> paged KV write    HIP  (fused RoPE + cache scatter)
    o   = attn(q, K, V)                       HIP  (MFMA flash prefill | split-KV paged decode)
    a   = o @ Wo^T                            GEMM
    x   = rmsnorm(allreduce(a) + h)           HIP  (TP: one fused one-shot AR + norm kernel)
    gu  = x @ Wgu^T                           GEMM (fused gate|up)
    m   = silu(g) * u                         HIP (fused into the gate|up GEMM at decode)
    d   = m @ Wd^T        [TP: fused AR+norm] GEMM
logits = rmsnorm(h) @ Wlm^T (vocab-parallel under TP); tokens = Gumbel-max
sampler on each vocab shard + a max over shards.

Tensor parallelism is Megatron-style: QKV and gate|up column-parallel (whole
heads / whole FFN columns per rank), O and down row-parallel followed by one
all-reduce each (2 per layer), embeddings replicated (2.1 GB at 70B, fits the
288 GB HBM trivially), lm_head vocab-parallel.
Decode-bucket GEMMs go to the gfx950 gemm_skinny / gemm_decode kernels, prefill GEMMs
and the lm_head to the 256x256-tile gemm_tile kernel (fused bias / SwiGLU epilogues);
everything else is a hand-written HIP kernel too (operator_amd.ops).
"""
from __future__ import annotations

import hashlib
import json
import math
import os
from dataclasses import dataclass, field

import torch

from operator_amd import ops
from operator_amd.ops import reference as ref
from operator_amd.parallel.comm import Group

from .config import LlamaConfig
from .kv_cache import PagedKVCache


@dataclass
class ForwardBatch:
    """Flattened tokens of one engine step (prefill or decode, never mixed)."""
    input_ids: torch.Tensor            # [T] int64
    positions: torch.Tensor            # [T] int64
    slots: torch.Tensor                # [T] int64 (cache slot, -1 = do not write)
    is_prefill: bool
    logits_index: torch.Tensor | None  # [n_out] int64 rows to produce logits for (None = all)
    # prefill
    seq_lens: list[int] = field(default_factory=list)
    prefill_work: tuple | None = None
    # shared prompt prefix (LLMEngine prefix sharing): (pk, pv, seq_pfx, pfx_lens), pk / pv the
    # cached post-RoPE K/V [layers, P, Hkv, D]; sequence s's tokens follow pfx_lens[s] of them
    prefix: tuple | None = None
    kv_sink: object = None   # called (layer, k, v) with each prefill layer's K/V (prefix capture)
    # decode
    block_tables: torch.Tensor | None = None   # [B, max_pages] int32
    context_lens: torch.Tensor | None = None   # [B] int32 (including the new token)
    num_splits: int = 1


@dataclass
class LayerWeights:
    wqkv: torch.Tensor
    wo: torch.Tensor
    wgu: torch.Tensor
    wd: torch.Tensor
    attn_norm: torch.Tensor
    mlp_norm: torch.Tensor
    # fp8 (e4m3fn) weights: per-output-row scales; None = bf16 weights
    sqkv: torch.Tensor | None = None
    so: torch.Tensor | None = None
    sgu: torch.Tensor | None = None
    sd: torch.Tensor | None = None
    bqkv: torch.Tensor | None = None   # q|k|v projection bias (Qwen2), bf16 [(hq + 2 hkv) D]


def _seed_for(seed: int, name: str) -> int:
    return int.from_bytes(hashlib.sha256(f"{seed}:{name}".encode()).digest()[:8], "little") & ((1 << 63) - 1)


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, device: str | torch.device = "cuda", tp: Group | None = None,
                 dtype: torch.dtype = torch.bfloat16, weight_dtype: str = "bfloat16"):
        self.cfg = cfg
        if weight_dtype not in ("bfloat16", "fp8"):
            raise ValueError(f"weight_dtype must be bfloat16 or fp8, not {weight_dtype}")
        # fp8: the four projection GEMMs run W8A8 e4m3fn (per-channel weight scales,
        # per-token activation scales); embeddings, norms and lm_head stay bf16
        self.fp8 = weight_dtype == "fp8"
        self.device = torch.device(device)
        self.tp = tp or Group.single()
        self.dtype = dtype
        W = self.tp.world
        if cfg.heads % W or cfg.kv_heads % W or cfg.intermediate % W or cfg.vocab_size % W:
            raise ValueError(f"{cfg.name}: heads/kv_heads/intermediate/vocab must divide by tp={W}")
        self.hq = cfg.heads // W
        self.hkv = cfg.kv_heads // W
        # gate|up rows interleaved in 64-feature blocks (fused SwiGLU GEMM epilogue)
        self.gu_block = ops.GU_BLOCK if (cfg.intermediate // W) % ops.GU_BLOCK == 0 else None
        self.inter = cfg.intermediate // W
        self.vocab_local = cfg.vocab_size // W
        self.vocab_offset = self.tp.rank * self.vocab_local
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        cos, sin = ref.rope_tables(cfg.max_position, cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.cos, self.sin = cos.to(self.device), sin.to(self.device)
        self.layers: list[LayerWeights] = []
        self.embed = self.final_norm = self.lm_head = None

    # ------------------------------------------------------------------ weights
    def _randn(self, seed: int, name: str, shape, std: float) -> torch.Tensor:
        g = torch.Generator(device=self.device)
        g.manual_seed(_seed_for(seed, name))
        t = torch.randn(shape, generator=g, device=self.device, dtype=self.dtype)
        return t.mul_(std)

    def init_random(self, seed: int = 0) -> "LlamaModel":
        """Random weights of the exact architecture. Each full tensor is generated from a
        name-derived seed and then sharded, so every TP degree sees the same global model."""
        c, r = self.cfg, self.tp.rank
        D, H = c.head_dim, c.hidden
        std_in = 1.0 / math.sqrt(H)
        self.embed = self._randn(seed, "embed", (c.vocab_size, H), 1.0)
        self.layers = []
        for i in range(c.layers):
            wq = self._randn(seed, f"l{i}.wq", (c.heads * D, H), std_in)
            wk = self._randn(seed, f"l{i}.wk", (c.kv_heads * D, H), std_in)
            wv = self._randn(seed, f"l{i}.wv", (c.kv_heads * D, H), std_in)
            wo = self._randn(seed, f"l{i}.wo", (H, c.heads * D), 1.0 / math.sqrt(c.heads * D))
            wg = self._randn(seed, f"l{i}.wg", (c.intermediate, H), std_in)
            wu = self._randn(seed, f"l{i}.wu", (c.intermediate, H), std_in)
            wd = self._randn(seed, f"l{i}.wd", (H, c.intermediate), 1.0 / math.sqrt(c.intermediate))
            bias = None
            if c.qkv_bias:  # Qwen2-style q/k/v bias (random, O(1) like trained ones)
                bias = tuple(self._randn(seed, f"l{i}.b{n}", (rows * D,), 0.5)
                             for n, rows in (("q", c.heads), ("k", c.kv_heads), ("v", c.kv_heads)))
            self.layers.append(self._shard_layer(wq, wk, wv, wo, wg, wu, wd,
                                                 torch.ones(H, dtype=self.dtype, device=self.device),
                                                 torch.ones(H, dtype=self.dtype, device=self.device), bias))
            del wq, wk, wv, wo, wg, wu, wd
        self.final_norm = torch.ones(H, dtype=self.dtype, device=self.device)
        lm = self.embed if c.tie_embeddings else self._randn(seed, "lm_head", (c.vocab_size, H), std_in)
        self.lm_head = lm[r * self.vocab_local:(r + 1) * self.vocab_local].contiguous()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return self

    def _quantize_layer(self, lw: LayerWeights) -> LayerWeights:
        if not self.fp8:
            return lw
        for name in ("wqkv", "wo", "wgu", "wd"):
            q, sc = ops.quantize_fp8(getattr(lw, name))
            setattr(lw, name, q)
            setattr(lw, {"wqkv": "sqkv", "wo": "so", "wgu": "sgu", "wd": "sd"}[name], sc)
        return lw

    def _lin(self, x: torch.Tensor, w: torch.Tensor, sc: torch.Tensor | None, defer: bool = False):
        """Projection; ``defer`` lets a split-K decode GEMM hand its fp32 slabs to the
        following rmsnorm (only when no TP all-reduce sits in between)."""
        if sc is not None:   # every fp8 consumer (rope_kv, the AR + norm, SwiGLU) sums slabs
            return ops.linear_fp8(x, w, sc, defer_reduce=defer)
        return ops.linear(x, w, defer_reduce=defer and self.tp.world == 1)

    def _shard_layer(self, wq, wk, wv, wo, wg, wu, wd, an, mn, bias=None) -> LayerWeights:
        """One layer's weights, sharded for this TP rank; ``bias`` = (bq, bk, bv) or None."""
        r, D = self.tp.rank, self.cfg.head_dim
        q = wq[r * self.hq * D:(r + 1) * self.hq * D]
        k = wk[r * self.hkv * D:(r + 1) * self.hkv * D]
        v = wv[r * self.hkv * D:(r + 1) * self.hkv * D]
        g = wg[r * self.inter:(r + 1) * self.inter]
        u = wu[r * self.inter:(r + 1) * self.inter]
        bqkv = None
        if bias is not None:
            bq, bk, bv = bias
            bqkv = torch.cat([bq[r * self.hq * D:(r + 1) * self.hq * D], bk[r * self.hkv * D:(r + 1) * self.hkv * D],
                              bv[r * self.hkv * D:(r + 1) * self.hkv * D]]).to(self.dtype).contiguous()
        return self._quantize_layer(LayerWeights(
            bqkv=bqkv,
            wqkv=torch.cat([q, k, v], 0).contiguous(),
            wo=wo[:, r * self.hq * D:(r + 1) * self.hq * D].contiguous(),
            wgu=(ops.interleave_gate_up(g, u, self.gu_block) if self.gu_block else torch.cat([g, u], 0).contiguous()),
            wd=wd[:, r * self.inter:(r + 1) * self.inter].contiguous(),
            attn_norm=an.contiguous(), mlp_norm=mn.contiguous()))

    def split_gate_up(self, wgu: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """(gate, up) rows of a layer's fused gate|up weight (undoes the interleave)."""
        inter = wgu.shape[0] // 2
        if not self.gu_block:
            return wgu[:inter], wgu[inter:]
        v = wgu.reshape(inter // self.gu_block, 2, self.gu_block, wgu.shape[1])
        return v[:, 0].reshape(inter, -1), v[:, 1].reshape(inter, -1)

    def load_hf(self, path: str) -> "LlamaModel":
        """Load a HuggingFace checkpoint directory (safetensors; llama / mistral / qwen2
        tensor names) and shard it. ``self.cfg`` must describe it (``config_from_hf``)."""
        from safetensors import safe_open

        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {path}")
        tensors: dict[str, str] = {}
        for f in files:
            with safe_open(os.path.join(path, f), framework="pt") as sf:
                for k in sf.keys():
                    tensors[k] = f

        def get(name):
            with safe_open(os.path.join(path, tensors[name]), framework="pt", device="cpu") as sf:
                return sf.get_tensor(name).to(self.device, self.dtype)

        c, r = self.cfg, self.tp.rank
        self.embed = get("model.embed_tokens.weight")
        self.layers = []
        for i in range(c.layers):
            p = f"model.layers.{i}."
            bias = None
            if c.qkv_bias:
                bias = tuple(get(p + f"self_attn.{n}_proj.bias") for n in "qkv")
            self.layers.append(self._shard_layer(
                get(p + "self_attn.q_proj.weight"), get(p + "self_attn.k_proj.weight"),
                get(p + "self_attn.v_proj.weight"), get(p + "self_attn.o_proj.weight"),
                get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight"), get(p + "mlp.down_proj.weight"),
                get(p + "input_layernorm.weight"), get(p + "post_attention_layernorm.weight"), bias))
        self.final_norm = get("model.norm.weight")
        lm = get("lm_head.weight") if "lm_head.weight" in tensors else self.embed
        self.lm_head = lm[r * self.vocab_local:(r + 1) * self.vocab_local].contiguous()
        return self

    def weight_bytes(self) -> int:
        n = sum(t.numel() * t.element_size() for t in (self.embed, self.final_norm, self.lm_head))
        for lw in self.layers:
            n += sum(t.numel() * t.element_size() for t in (lw.wqkv, lw.wo, lw.wgu, lw.wd, lw.attn_norm, lw.mlp_norm,
                                                            lw.sqkv, lw.so, lw.sgu, lw.sd, lw.bqkv) if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def forward(self, fb: ForwardBatch, kv: PagedKVCache) -> torch.Tensor:
        """Run all layers; returns logits [n_out, vocab_local] for fb.logits_index rows."""
        c = self.cfg
        h = ops.embedding(fb.input_ids, self.embed)          # residual stream [T, H]
        x = ops.rmsnorm(h, self.layers[0].attn_norm, c.rms_eps)
        T = h.shape[0]
        q8 = self.fp8 and h.is_cuda   # block epilogues emit e4m3fn rows for the next fp8 GEMM
        ws = None
        if not fb.is_prefill and h.is_cuda:  # split-KV partials, shared by every layer
            ws = ops.decode_workspace(T, self.hq, fb.num_splits, h.device)
        for i, lw in enumerate(self.layers):
            kc, vc = kv.layer(i)
            # a split-K decode QKV projection hands its fp32 slabs to rope_kv, which sums
            # them per element (no separate reduce kernel) and adds a Qwen2 bias before
            # rounding; a prefill bias rides the tile GEMM's epilogue
            bias = lw.bqkv
            if bias is not None and fb.is_prefill and lw.sqkv is None:
                qkv, bias = ops.linear(x, lw.wqkv, bias=bias), None
            else:
                qkv = self._lin(x, lw.wqkv, lw.sqkv, defer=True)
            if fb.is_prefill:
                q, k, v = ops.rope_kv(qkv, fb.positions, self.cos, self.sin, self.hq, self.hkv, kc, vc, fb.slots,
                                      want_kv=True, bias=bias, k_scale=kv.k_scale, v_scale=kv.v_scale)
                if fb.kv_sink is not None:
                    fb.kv_sink(i, k, v)
                pre = None
                if fb.prefix is not None:
                    pre = (fb.prefix[0][i], fb.prefix[1][i], fb.prefix[2], fb.prefix[3])
                o = ops.attn_prefill(q, k, v, fb.seq_lens, self.scale, work=fb.prefill_work, prefix=pre)
            else:
                # RoPE + the decode token's KV write run inside the attention kernel
                o = ops.attn_decode_rope(qkv, fb.positions, self.cos, self.sin, self.hq, kc, vc, fb.slots,
                                         fb.block_tables, fb.context_lens, self.scale, fb.num_splits, workspace=ws,
                                         bias=bias, k_scale=kv.k_scale, v_scale=kv.v_scale, quant=q8)
            a = self._lin(o if isinstance(o, tuple) else o.view(T, self.hq * c.head_dim), lw.wo, lw.so, defer=True)
            x = self.tp.all_reduce_rmsnorm(a, lw.mlp_norm, c.rms_eps, residual=h, quant=q8)   # fused under TP
            if lw.sgu is None:
                m = ops.gate_up_silu(x, lw.wgu, self.gu_block)
            elif q8:   # SwiGLU (+ the split-K sum) fused into the down GEMM's input quantization
                m = ops.silu_quantize_fp8(ops.linear_fp8(x, lw.wgu, lw.sgu, defer_reduce=True), self.gu_block)
            else:
                m = ops.silu_mul(ops.linear_fp8(x, lw.wgu, lw.sgu), block=self.gu_block)
            d = self._lin(m, lw.wd, lw.sd, defer=True)
            last = i + 1 == len(self.layers)
            nw = self.final_norm if last else self.layers[i + 1].attn_norm
            x = self.tp.all_reduce_rmsnorm(d, nw, c.rms_eps, residual=h, quant=q8 and not last)
        if fb.logits_index is not None:
            x = x.index_select(0, fb.logits_index)
        return ops.linear(x, self.lm_head)

    def sample(self, logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
               positions: torch.Tensor) -> torch.Tensor:
        """Sample one token per row; under TP each rank samples its vocab shard and the
        global winner is the max perturbed value (ties -> smaller token id)."""
        if self.tp.world == 1:
            return ops.sample(logits, temperature, seeds, positions)
        n = logits.shape[0]
        val = torch.empty(n, dtype=torch.float32, device=logits.device)
        tok = ops.sample(logits, temperature, seeds, positions, col_offset=self.vocab_offset, out_val=val)
        pair = torch.stack([val, tok.to(torch.float32)], 1)             # exact for ids < 2^24
        allp = self.tp.all_gather_into(pair)                             # [W, n, 2]
        vals, toks = allp[..., 0], allp[..., 1]
        best = vals.max(0).values
        cand = torch.where(vals == best.unsqueeze(0), toks, torch.full_like(toks, float("inf")))
        return cand.min(0).values.to(torch.long)
