"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

These define the numerics each gfx950 kernel is tested against (tests/test_kernels_gpu.py)
and are what runs when a model is executed on CPU (the CPU test tier, gloo
multi-process TP tests). They are intentionally simple and unfused.
"""
from __future__ import annotations

import math

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None):
    """y = rmsnorm(x [+ residual]); returns (y, new_residual). HF Llama numerics."""
    if residual is not None:
        x = (x.float() + residual.float()).to(x.dtype)
        new_res = x
    else:
        new_res = None
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    y = (xf * torch.rsqrt(var + eps)).to(x.dtype)
    return (y.float() * w.float()).to(x.dtype), new_res


def silu_mul(gu: torch.Tensor, block: int | None = None) -> torch.Tensor:
    """silu(gate) * up; gate|up columns interleaved in blocks of ``block`` features
    (None: the plain [gate | up] concatenation)."""
    inter = gu.shape[-1] // 2
    if block and block != inter:
        v = gu.reshape(*gu.shape[:-1], inter // block, 2, block)
        g, u = v[..., 0, :].reshape(*gu.shape[:-1], inter), v[..., 1, :].reshape(*gu.shape[:-1], inter)
    else:
        g, u = gu[..., :inter], gu[..., inter:]
    s = torch.nn.functional.silu(g.float()).to(gu.dtype)
    return (s.float() * u.float()).to(gu.dtype)


def embedding(ids: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    return table[ids.clamp(0, table.shape[0] - 1)]


def rope_tables(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """fp32 cos/sin tables [max_pos, head_dim/2]; supports Llama-3.1 'llama3' scaling."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x: [T, H, D] -> rotate-half RoPE at positions pos [T]."""
    half = x.shape[-1] // 2
    c = cos[pos].unsqueeze(1)
    s = sin[pos].unsqueeze(1)
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


K_TILE = 16  # tokens per K-cache tile


def k_tile_index(D: int = 128) -> torch.Tensor:
    """Physical offset inside a [16 tokens x D] K-cache tile of logical element (t, d).

    K is stored so that each MFMA fragment load of the decode-attention kernel is
    one contiguous 1 KB wave access: a tile is [ks 4][lg 4][token 16][8 dims]
    with d = 32*lg + 8*ks + j (lg = lane >> 4 group, ks = k-step) — instead of
    16 token rows x 64 B per instruction. V keeps the row layout."""
    t = torch.arange(K_TILE)[:, None]
    d = torch.arange(D)[None, :]
    lg, ks, j = d // 32, (d % 32) // 8, d % 8
    return ((ks * 4 + lg) * K_TILE + t) * 8 + j


def k_cache_logical(k_cache: torch.Tensor) -> torch.Tensor:
    """[pages, Hkv, P, D] tiled K cache -> logical (token-row) copy."""
    pages, Hkv, P, D = k_cache.shape
    idx = k_tile_index(D).flatten().to(k_cache.device)
    return k_cache.reshape(pages, Hkv, P // K_TILE, K_TILE * D)[..., idx].reshape(pages, Hkv, P, D)


def k_cache_write(k_cache: torch.Tensor, page: int, off: int, k: torch.Tensor) -> None:
    """k_cache[page, :, off] = k ([Hkv, D]) in the tiled K layout."""
    pages, Hkv, P, D = k_cache.shape
    idx = k_tile_index(D)[off % K_TILE].to(k_cache.device)
    k_cache.view(pages, Hkv, P // K_TILE, K_TILE * D)[page, :, off // K_TILE, idx] = k


FP8_KV_MAX = 448.0  # OCP e4m3fn


def kv_store(x: torch.Tensor, cache_dtype: torch.dtype, scale: float) -> torch.Tensor:
    """Value as held by a cache of ``cache_dtype``: as is, or e4m3fn(x / scale) saturated."""
    if cache_dtype == torch.float8_e4m3fn:
        return (x.float() / scale).clamp(-FP8_KV_MAX, FP8_KV_MAX).to(torch.float8_e4m3fn)
    return x.to(cache_dtype)


def kv_load(c: torch.Tensor, scale: float) -> torch.Tensor:
    """fp32 view of cache contents (fp8 caches dequantised by their scale)."""
    return c.float() * scale if c.dtype == torch.float8_e4m3fn else c.float()


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, Hq: int, Hkv: int,
            k_cache: torch.Tensor | None = None, v_cache: torch.Tensor | None = None,
            slots: torch.Tensor | None = None, k_scale: float = 1.0, v_scale: float = 1.0):
    """Split packed qkv, rotate q/k, optionally scatter k/v into the paged cache.

    Cache layout [pages, Hkv, page, D] (K tiled, see k_tile_index; V row-major);
    slot = page*page_size + offset; slot < 0 skips.
    Returns (q [T,Hq,D], k [T,Hkv,D], v [T,Hkv,D]).
    """
    T = qkv.shape[0]
    D = cos.shape[1] * 2
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    k = qkv[:, Hq * D: (Hq + Hkv) * D].reshape(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].reshape(T, Hkv, D)
    q = apply_rope(q, pos, cos, sin)
    k = apply_rope(k, pos, cos, sin)
    if k_cache is not None:
        P = k_cache.shape[2]
        for t in range(T):
            s = int(slots[t])
            if s < 0:
                continue
            k_cache_write(k_cache, s // P, s % P, kv_store(k[t], k_cache.dtype, k_scale))
            v_cache[s // P, :, s % P] = kv_store(v[t], v_cache.dtype, v_scale)
    return q, k.contiguous(), v.contiguous()


def attn_prefill(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens: list[int] | torch.Tensor,
                 scale: float, prefix: tuple | None = None) -> torch.Tensor:
    """Causal GQA attention over packed variable-length sequences. q [T,Hq,D], k/v [T,Hkv,D].
    ``prefix`` = (pk, pv, lens): sequence i's keys start with the rows pk[:lens[i]] /
    pv[:lens[i]] (a cached shared prompt prefix), visible to all of its query rows."""
    cu = [int(x) for x in cu_seqlens]
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    out = torch.empty_like(q)
    for i in range(len(cu) - 1):
        a, b = cu[i], cu[i + 1]
        if b == a:
            continue
        pl = int(prefix[2][i]) if prefix is not None else 0
        kk, vv = k[a:b], v[a:b]
        if pl:
            kk, vv = torch.cat([prefix[0][:pl].to(k.dtype), kk]), torch.cat([prefix[1][:pl].to(v.dtype), vv])
        qs = q[a:b].float().transpose(0, 1)                      # [Hq, L, D]
        ks = kk.float().transpose(0, 1).repeat_interleave(G, 0)
        vs = vv.float().transpose(0, 1).repeat_interleave(G, 0)
        s = torch.matmul(qs, ks.transpose(1, 2)) * scale
        L = b - a
        mask = torch.ones(L, L, dtype=torch.bool, device=q.device).triu(1)
        if pl:
            mask = torch.cat([torch.zeros(L, pl, dtype=torch.bool, device=q.device), mask], 1)
        s.masked_fill_(mask, float("-inf"))
        p = torch.softmax(s, -1)
        out[a:b] = torch.matmul(p, vs).transpose(0, 1).to(q.dtype)
    return out


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                seq_lens: torch.Tensor, scale: float, k_scale: float = 1.0, v_scale: float = 1.0) -> torch.Tensor:
    """One query token per sequence over a paged cache [pages, Hkv, page, D] (K tiled;
    bf16, or e4m3fn holding x / scale)."""
    B, Hq, D = q.shape
    Hkv, P = k_cache.shape[1], k_cache.shape[2]
    k_cache = k_cache_logical(k_cache)
    G = Hq // Hkv
    out = torch.zeros_like(q)
    for b in range(B):
        L = int(seq_lens[b])
        if L == 0:
            continue
        npg = (L + P - 1) // P
        pages = block_tables[b, :npg].long()
        ks = kv_load(k_cache[pages].permute(1, 0, 2, 3).reshape(Hkv, npg * P, D)[:, :L], k_scale)
        vs = kv_load(v_cache[pages].permute(1, 0, 2, 3).reshape(Hkv, npg * P, D)[:, :L], v_scale)
        ks = ks.repeat_interleave(G, 0)
        vs = vs.repeat_interleave(G, 0)
        s = torch.einsum("hd,hld->hl", q[b].float(), ks) * scale
        p = torch.softmax(s, -1)
        out[b] = torch.einsum("hl,hld->hd", p, vs).to(q.dtype)
    return out


def gumbel_noise_ref(seed: int, position: int, vocab: int, col_offset: int = 0) -> torch.Tensor:
    """Host mirror of the device counter hash (common.h mix64 / hash_col / uniform01), vectorised."""
    import numpy as np

    M = (1 << 64) - 1
    k = ((seed * 0x9E3779B97F4A7C15) & M) ^ ((position << 32) & M)
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M
    k ^= k >> 33
    k1, k2 = np.uint32(k & 0xFFFFFFFF), np.uint32(k >> 32)
    with np.errstate(over="ignore"):
        h = (np.arange(vocab, dtype=np.uint64) + np.uint64(col_offset & 0xFFFFFFFF)).astype(np.uint32) ^ k1
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x7FEB352D)
        h ^= h >> np.uint32(15)
        h ^= k2
        h *= np.uint32(0x846CA68B)
        h ^= h >> np.uint32(16)
    u = (h >> np.uint32(9)).astype(np.float64) + 0.5
    u = torch.from_numpy(u / 8388608.0)
    return -torch.log(-torch.log(u))


def sample_shard(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor, positions: torch.Tensor,
                 col_offset: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """Greedy when T<=0 else Gumbel-max with the same counter hash as the kernel.

    Returns (global token ids, winning perturbed values) for a vocab shard.
    """
    out = torch.empty(logits.shape[0], dtype=torch.long)
    val = torch.empty(logits.shape[0], dtype=torch.float32)
    for r in range(logits.shape[0]):
        x = logits[r].double().cpu()
        t = float(temperature[r])
        if t > 0:
            x = x / t + gumbel_noise_ref(int(seeds[r]), int(positions[r]), x.numel(), col_offset)
        i = int(torch.argmax(x))
        out[r] = i + col_offset
        val[r] = float(x[i])
    return out.to(logits.device), val.to(logits.device)


def sample(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
           positions: torch.Tensor) -> torch.Tensor:
    return sample_shard(logits, temperature, seeds, positions)[0]
