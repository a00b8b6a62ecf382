"""Device ops of the explanation model and the log scanner.

GPU tensors always go to the hand-written gfx950 kernels in ``operator_amd._C``
(loading fails loudly if the extension is missing); CPU tensors use the fp32
reference implementations in :mod:`operator_amd.ops.reference`.
"""
from __future__ import annotations

import json
import os

import torch
import torch.nn.functional as F

from . import reference
from ._native import kernels, native_available, patterns

__all__ = [
    "rmsnorm", "silu_mul", "embedding", "rope_kv", "attn_prefill", "attn_decode", "attn_decode_rope", "sample",
    "kernels", "patterns", "native_available", "reference", "prefill_work_list", "prefill_block_q", "prefill_variant", "decode_splits",
    "decode_workspace", "linear", "gemm_splits", "gemm_plan", "gate_up_silu", "interleave_gate_up",
    "quantize_fp8", "silu_quantize_fp8", "linear_fp8", "fp8_plan", "SplitK", "linear_tile", "tile_ok", "BLAS_CALLS",
]

# never split a sequence into pieces shorter than this / split only while B x Hkv
# decode-attention workgroups < this (env overrides for tuning runs)
DECODE_MIN_SPLIT_TOKENS = int(os.environ.get("OAMD_DECODE_MIN_SPLIT", "256"))
# one workgroup per CU: the best split count at every measured (B, group, ctx) of
# profiles/attn_decode_splits_sweep_r5.jsonl lands at B x Hkv x splits ~ 256
DECODE_TARGET_BLOCKS = int(os.environ.get("OAMD_DECODE_TARGET_BLOCKS", "256"))
# attn_decode schedule bits (csrc/kernels/attn_decode.hip): 2 = NT 2 (two 16-token tiles per wave),
# 4 = one kv-head across all sequences first (else a sequence's kv-heads back to back)
DECODE_ATTN_VARIANT = int(os.environ.get("OAMD_DECODE_ATTN_VARIANT", "0"))


class SplitK:
    """A decode GEMM's output left as S fp32 split-K slabs [S, M, N]; the consumer
    (rmsnorm) sums them, so the GEMM's separate reduction pass disappears."""

    __slots__ = ("p", "S", "shape", "device", "dtype", "is_cuda")

    def __init__(self, p: torch.Tensor, S: int, M: int, N: int):
        self.p, self.S, self.shape = p, S, (M, N)
        self.device, self.dtype, self.is_cuda = p.device, torch.bfloat16, True

    def materialize(self) -> torch.Tensor:
        M, N = self.shape
        return self.p[: self.S * M * N].view(self.S, M, N).sum(0).to(torch.bfloat16)


def rmsnorm(x, w: torch.Tensor, eps: float, residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """RMSNorm; if ``residual`` is given it is updated in place to x + residual first.
    ``x`` may be a :class:`SplitK` (slabs summed inside the kernel)."""
    if isinstance(x, SplitK):
        M, N = x.shape
        y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=x.device)
        kernels().rmsnorm(y, residual, w, y, eps, x.p, x.S)  # y doubles as the shape carrier
        return y
    if not x.is_cuda:
        y, r = reference.rmsnorm(x, w, eps, residual)
        if residual is not None:
            residual.copy_(r)
        if out is not None:
            out.copy_(y)
            return out
        return y
    y = out if out is not None else torch.empty_like(x)
    kernels().rmsnorm(x, residual, w, y, eps)
    return y


def silu_mul(gu: torch.Tensor, out: torch.Tensor | None = None, block: int | None = None) -> torch.Tensor:
    """silu(gate) * up for gate|up interleaved in ``block``-feature blocks (None: [gate | up])."""
    if not gu.is_cuda:
        r = reference.silu_mul(gu, block)
        if out is not None:
            out.copy_(r)
            return out
        return r
    inter = gu.shape[1] // 2
    o = out if out is not None else torch.empty(gu.shape[0], inter, dtype=gu.dtype, device=gu.device)
    kernels().silu_mul(gu, o, block or 0)
    return o


GU_BLOCK = 64  # gate|up weight rows interleaved in 64-feature blocks (fused SwiGLU epilogue)


def interleave_gate_up(g: torch.Tensor, u: torch.Tensor, block: int = GU_BLOCK) -> torch.Tensor:
    """[g; u] rows -> blocks of ``block`` gate rows followed by the same features' up rows."""
    inter, H = g.shape
    return torch.stack([g.reshape(inter // block, block, H), u.reshape(inter // block, block, H)], 1).reshape(
        2 * inter, H).contiguous()


def gate_up_silu(x: torch.Tensor, wgu: torch.Tensor, block: int | None) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) from the interleaved gate|up weight. Decode buckets run
    one fused gfx950 kernel (GEMM + SwiGLU epilogue, no [M, 2I] intermediate);
    other shapes run the GEMM then the silu_mul kernel."""
    M, K = x.shape
    N = wgu.shape[0]
    if (x.is_cuda and block == 64 and x.dtype == torch.bfloat16 and M <= SKINNY_MAX_M and N % 128 == 0
            and K % 128 == 0 and x.is_contiguous() and wgu.is_contiguous()
            and skinny_plan(M, N, K) is not None and _gemm_table_get().get(("silu", M, N, K)) != "blas"):
        y = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
        kernels().gemm_skinny(x, wgu, y, None, 1, True)
        return y
    if (x.is_cuda and block == 64 and x.dtype == torch.bfloat16 and M % 64 == 0 and M <= 256 and N % 128 == 0
            and K % 64 == 0 and x.is_contiguous() and wgu.is_contiguous()):
        t = _gemm_table_get().get(("silu", M, N, K))
        if isinstance(t, str) and t.startswith("pp"):   # ping-pong kernel, nt weight loads (bm 128 / 256)
            y = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
            bm = int(t[2:])
            ws, fl = _pp_sk_workspace(x.device, N // 128) if (bm == 256 and PP_STREAM_K) else (None, None)
            kernels().gemm_pp(x, wgu, y, None, 1, bm, True, True, False, ws, fl)
            return y
        if t != "blas":
            bm = t[0] if t else row_tile(M)
            ns = t[1] if t and len(t) > 1 else 3
            y = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
            kernels().gemm_decode(x, wgu, y, None, 1, 128, bm, True, False, ns)
            return y
    if block == 64 and tile_ok(x, wgu) and N % 128 == 0:
        return linear_tile(x, wgu, silu_gu=True)   # prefill: SwiGLU fused into the tile epilogue
    return silu_mul(linear(x, wgu), block=block)


# Stream-K form of the 256-row gate|up+SwiGLU decode GEMM (csrc/kernels/gemm_pp.hip SK): one block per
# CU over the flattened (tile, K-step) stream instead of one block per 128-feature tile (224 of 256 CUs
# busy at the 8B shape). OAMD_PP_STREAM_K=1 turns it on (A/B runs).
PP_STREAM_K = os.environ.get("OAMD_PP_STREAM_K", "0") == "1"
_PP_SK_WS: dict = {}


def _pp_sk_workspace(device, tiles: int):
    """(fp32 partials, zeroed int flags) for the stream-K gate|up kernel, one pair per (device,
    tile count), kept for the life of the process: captured decode graphs hold the pointers, and the
    kernel leaves the flags zero. A stream runs one such GEMM at a time (the engine's decode stream)."""
    key = (str(device), tiles)
    ws = _PP_SK_WS.get(key)
    if ws is None:
        ws = (torch.empty(tiles * 32768, dtype=torch.float32, device=device),
              torch.zeros(tiles, dtype=torch.int32, device=device))
        _PP_SK_WS[key] = ws
    return ws


def embedding(ids: torch.Tensor, table: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    if not ids.is_cuda:
        r = reference.embedding(ids, table)
        if out is not None:
            out.copy_(r)
            return out
        return r
    o = out if out is not None else torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=ids.device)
    kernels().embedding(ids, table, o)
    return o


def rope_kv(qkv: torch.Tensor, pos: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, Hq: int, Hkv: int,
            k_cache: torch.Tensor | None = None, v_cache: torch.Tensor | None = None,
            slots: torch.Tensor | None = None, want_kv: bool = True,
            q_out: torch.Tensor | None = None, bias: torch.Tensor | None = None,
            k_scale: float = 1.0, v_scale: float = 1.0):
    """Rotate q/k of the packed qkv rows and scatter k/v into the paged cache.
    ``bias`` [(Hq + 2 Hkv) D] is added to the projection first (Qwen2); with split-K
    slabs it is added before the single bf16 rounding. An e4m3fn cache stores
    x / k_scale, x / v_scale.

    Returns (q [T,Hq,D], k [T,Hkv,D] | None, v [T,Hkv,D] | None).
    """
    if isinstance(qkv, SplitK):
        T = qkv.shape[0]
        D = cos.shape[1] * 2
        dev = qkv.device
        q = q_out if q_out is not None else torch.empty(T, Hq, D, dtype=torch.bfloat16, device=dev)
        k = torch.empty(T, Hkv, D, dtype=torch.bfloat16, device=dev) if want_kv else None
        v = torch.empty(T, Hkv, D, dtype=torch.bfloat16, device=dev) if want_kv else None
        kernels().rope_kv(q, pos, cos, sin, Hq, Hkv, q, k, v, k_cache, v_cache, slots, qkv.p, qkv.S, bias,
                          k_scale, v_scale)
        return q, k, v
    if not qkv.is_cuda:
        if bias is not None:
            qkv = (qkv.float() + bias.float()).to(qkv.dtype)
        q, k, v = reference.rope_kv(qkv, pos, cos, sin, Hq, Hkv, k_cache, v_cache, slots, k_scale, v_scale)
        if q_out is not None:
            q_out.copy_(q.reshape(q_out.shape))
            q = q_out
        return q, (k if want_kv else None), (v if want_kv else None)
    T = qkv.shape[0]
    D = cos.shape[1] * 2
    q = q_out if q_out is not None else torch.empty(T, Hq, D, dtype=qkv.dtype, device=qkv.device)
    k = torch.empty(T, Hkv, D, dtype=qkv.dtype, device=qkv.device) if want_kv else None
    v = torch.empty(T, Hkv, D, dtype=qkv.dtype, device=qkv.device) if want_kv else None
    kernels().rope_kv(qkv, pos, cos, sin, Hq, Hkv, q, k, v, k_cache, v_cache, slots, None, 1, bias, k_scale, v_scale)
    return q, k, v


# v3 schedule options (csrc/kernels/attn_prefill.hip OPT bits): l = K/V loads after the
# S MFMAs, r = deferred rescale, d = two LDS tile buffers (one barrier per tile)
_PREFILL_VARIANTS = {"v1": 1, "v2": 2, "v3": 3, "v4": 4}


def prefill_variant(Hq: int, Hkv: int) -> int:
    """attn_prefill kernel variant: 1 = per-query-head (any G), 2 = GQA-grouped 16-row waves
    (G = Hq / Hkv in 1, 2, 4, 8), 3 = GQA-grouped swapped-operand 32x32 MFMA waves in 8-wave
    workgroups (G <= 8), 4 = the same waves in 4-wave workgroups, two per CU (G <= 4;
    profiles/prefill_attn_v3_vs_v4.jsonl: 6-9 % faster at 16x1024 and mixed lengths, equal at
    4x4096). Default: v4 where G <= 4, else v3. OAMD_PREFILL_ATTN=v1|v2|v3|v4 overrides it; a
    grouped variant that cannot take G falls back to v3, then v1."""
    G = Hq // Hkv if Hkv and Hq % Hkv == 0 else 0
    want = _PREFILL_VARIANTS.get(os.environ.get("OAMD_PREFILL_ATTN", ""), 4 if 1 <= G <= 4 else 3)
    if want == 2 and G not in (1, 2, 4, 8):
        want = 3
    if want == 4 and G > 4:
        want = 3
    return want if 1 <= G <= 8 else 1


def prefill_block_q(Hq: int, Hkv: int, variant: int | None = None) -> int:
    """Query rows per attn_prefill work item: 64 (v1), 16 x (8 / G) (v2), 32 x (8 / G) (v3),
    32 x (4 / G) (v4)."""
    v = prefill_variant(Hq, Hkv) if variant is None else variant
    if v == 1:
        return 64
    G = Hq // Hkv
    return (16 if v == 2 else 32) * ((4 if v == 4 else 8) // G)


def prefill_work_list(seq_lens: list[int], block_q: int = 64) -> tuple[list[int], list[int]]:
    """(work_seq, work_q0) for attn_prefill: one item per ``block_q``-row query block; longest first."""
    items = []
    for s, L in enumerate(seq_lens):
        for q0 in range(0, L, block_q):
            items.append((q0, s))
    items.sort(key=lambda t: -t[0])  # heavy (late, long-causal) blocks first
    return [s for _, s in items], [q0 for q0, _ in items]


def attn_prefill(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, seq_lens: list[int], scale: float,
                 out: torch.Tensor | None = None, work: tuple[torch.Tensor, torch.Tensor, torch.Tensor] | None = None,
                 prefix: tuple | None = None):
    """Causal attention over packed sequences (q [T,Hq,D], k/v [T,Hkv,D]).

    ``prefix`` = (pk, pv, seq_pfx, pfx_lens): a shared prompt prefix (LLMEngine prefix
    sharing) whose cached K/V rows pk / pv [P, Hkv, D] come before sequence s's own keys
    for its first pfx_lens[s] keys (<= P); the own query rows sit at
    positions pfx_lens[s] + row and see every prefix key. seq_pfx: the same lengths as an
    int32 device tensor (GPU), pfx_lens: as a host list (CPU reference; may be None on
    the GPU)."""
    cu = [0]
    for L in seq_lens:
        cu.append(cu[-1] + int(L))
    if not q.is_cuda:
        r = reference.attn_prefill(q, k, v, cu, scale,
                                   prefix=None if prefix is None else (prefix[0], prefix[1], prefix[3]))
        if out is not None:
            out.copy_(r)
            return out
        return r
    o = out if out is not None else torch.empty_like(q)
    if work is None:
        var = prefill_variant(q.shape[1], k.shape[1])
        ws, wq = prefill_work_list([int(x) for x in seq_lens], prefill_block_q(q.shape[1], k.shape[1], var))
        dev = q.device
        work = (torch.tensor(cu, dtype=torch.int32, device=dev), torch.tensor(ws, dtype=torch.int32, device=dev),
                torch.tensor(wq, dtype=torch.int32, device=dev), var)
    # work = (cu_seqlens, work_seq, work_q0, variant); the work list must be cut at that variant's block_q
    var = work[3] if len(work) > 3 else 1
    if prefix is not None:
        if var not in (3, 4):
            raise ValueError("a shared prefix needs attn_prefill variant 3 or 4")
        kernels().attn_prefill(q, k, v, o, work[0], work[1], work[2], scale, var, prefix[0], prefix[1], prefix[2])
    else:
        kernels().attn_prefill(q, k, v, o, work[0], work[1], work[2], scale, var)
    return o


GEMM_DECODE_M = (64, 128, 256)  # decode buckets the gfx950 gemm_decode kernel is tuned for
_GEMM_TABLE_PATH = os.environ.get("OAMD_GEMM_TABLE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "gemm_tuned.json")
_gemm_table: dict | None = None


def _gemm_table_get() -> dict:
    """Measured best (bm, bn, splits) per decode GEMM shape on MI355X, written by
    ``tools/bench_gemm.py --write-table`` ("blas" = hipBLASLt wins that shape)."""
    global _gemm_table
    if _gemm_table is None:
        try:
            with open(_GEMM_TABLE_PATH) as f:
                _gemm_table = {tuple(x if x in ("silu", "skinny") else int(x) for x in k.split(",")): v
                               for k, v in json.load(f).items()}
        except (OSError, ValueError):
            _gemm_table = {}
    return _gemm_table


def row_tile(M: int) -> int:
    """Largest gemm_decode row tile (256, 128, 64) dividing M (M % 64 == 0): a bucket of
    192 rows runs three 64-row tiles, not one 192-row tile the kernel has no variant for."""
    return next(b for b in (256, 128, 64) if M % b == 0)


LM_HEAD_MIN_N = 32768


def _measured_blas(M: int, N: int, K: int) -> bool:
    """The tuned table measured hipBLASLt fastest for this decode-bucket shape (small-M
    GEMMs that neither the decode kernels nor the 256-row tile kernel win)."""
    if N >= LM_HEAD_MIN_N:   # vocab projections always run on gemm_tile (weight-streaming bound there)
        return False
    t = _gemm_table_get()
    return t.get(("skinny", M, N, K) if M <= SKINNY_MAX_M else (M, N, K)) == "blas"


def gemm_splits(M: int, N: int, K: int) -> int:
    """Heuristic split-K ways for gemm_decode (shapes not in the tuned table): the
    smallest S | 8 whose (N/64) x S blocks reach one block per CU (256)."""
    tiles = N // 64
    best = 1
    for S in (1, 2, 4, 8):
        if K % (64 * S):
            break
        best = S
        if tiles * S >= 256:
            return S
    return best


def gemm_plan(M: int, N: int, K: int):
    """(bm, bn, splits) for the gfx950 gemm_decode kernel, or None for hipBLASLt."""
    if M % 64 or N % 64 or K % 64 or M > 256:
        return None
    t = _gemm_table_get().get((M, N, K))
    if t in ("blas", "tile"):   # hipBLASLt / the 256x256-tile kernel (linear decides which)
        return None
    if t is not None:
        return tuple(t)   # (bm, bn, S[, stages]) for gemm_decode
    return (row_tile(M), 64, gemm_splits(M, N, K))


SKINNY_MAX_M = 32


def skinny_plan(M: int, N: int, K: int) -> int | None:
    """Split-K count for the gfx950 gemm_skinny kernel (M <= 32 decode buckets), or None
    for hipBLASLt: tuned table entry ``skinny,M,N,K`` if present, else split K until
    the 16-row tiles give >= 512 blocks (K permitting)."""
    if M > SKINNY_MAX_M or N % 16 or K % 128 or os.environ.get("OAMD_SKINNY", "1") == "0":
        return None
    t = _gemm_table_get().get(("skinny", M, N, K))
    if t == "blas":
        return None
    if t is not None:
        return int(t)
    S = 1
    while (N // 16) * S < 512 and S < 8 and K % (128 * S * 2) == 0:
        S *= 2
    return S


# Every GPU GEMM of the model runs on the hand-written gfx950 kernels: prefill projections (M > 256
# rows) on gemm_tile's persistent p5 schedule (csrc/kernels/gemm_tile.hip), decode buckets on
# gemm_pp / gemm_tn / gemm_skinny, the lm_head on gemm_tile, fp8 on gemm_fp8. hipBLASLt is reached
# only by shapes none of them takes (K % 64 != 0, N % 16 != 0, non-bf16), counted in BLAS_CALLS.
# OAMD_PREFILL_BLAS=1 routes the plain prefill projections (QKV, O, down) to hipBLASLt instead, for
# A/B runs against the vendor library (profiles/gemm_tile_p5_vs_hipblaslt_r6.jsonl).
PREFILL_BLAS = os.environ.get("OAMD_PREFILL_BLAS", "0") == "1"
BLAS_CALLS = {"n": 0}   # GPU GEMMs that FELL BACK to hipBLASLt (tests assert it stays 0 on model shapes)
BLAS_PLANNED = {"n": 0}   # plain prefill projections run on hipBLASLt by design (PREFILL_BLAS)


def _blas(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None, bias: torch.Tensor | None,
          planned: bool = False):
    if x.is_cuda and planned:
        BLAS_PLANNED["n"] += 1
    elif x.is_cuda:
        BLAS_CALLS["n"] += 1
        if os.environ.get("OAMD_FORBID_BLAS") == "1":
            raise RuntimeError(f"hipBLASLt fallback for x {tuple(x.shape)} {x.dtype}, w {tuple(w.shape)} "
                               "(OAMD_FORBID_BLAS=1)")
    if out is not None:
        return F.linear(x, w, bias, out=out) if bias is None else out.copy_(F.linear(x, w, bias))
    return F.linear(x, w, bias)


def tile_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the 256x256-tile gfx950 GEMM (gemm_tile) takes: bf16, K % 64, N % 16."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 2
            and x.is_contiguous() and w.is_contiguous() and x.shape[1] % 64 == 0 and w.shape[0] % 16 == 0
            and x.shape[0] >= 1)


def tile_out_ok(out: torch.Tensor | None) -> bool:
    """An explicit output gemm_tile can write: unit column stride, a row stride that is a
    multiple of 4 elements and an 8-byte-aligned base (its epilogue stores 4 bf16 at once);
    anything else falls back instead of tripping the binding's TORCH_CHECK."""
    return out is None or (out.dim() == 2 and out.stride(1) == 1 and out.stride(0) % 4 == 0
                           and out.data_ptr() % 8 == 0 and out.dtype == torch.bfloat16)


def linear_tile(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None,
                bias: torch.Tensor | None = None, silu_gu: bool = False) -> torch.Tensor:
    """Prefill / lm_head GEMM on the compute-bound gfx950 tile kernel (256 x 256 tiles,
    LDS-DMA ping-pong pipeline; fused bias or SwiGLU epilogue)."""
    M = x.shape[0]
    N = w.shape[0]
    y = out if out is not None else torch.empty(M, N // 2 if silu_gu else N, dtype=x.dtype, device=x.device)
    kernels().gemm_tile(x, w, y, bias, silu_gu)
    return y


def linear(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None, splits: int | None = None,
           partial: torch.Tensor | None = None, bn: int | None = None, bm: int | None = None,
           defer_reduce: bool = False, stages: int | None = None, bias: torch.Tensor | None = None):
    """y = x @ w^T (+ bias) in bf16 on the gfx950 kernels: M <= 32 decode buckets on the
    weight-streaming gemm_skinny, M in {64, 128, 256} on the LDS-staged split-K
    gemm_decode (tuned tables), everything else (prefill, the lm_head, biased
    projections) on the 256x256-tile gemm_tile (persistent p5 past 256 rows). hipBLASLt only
    for shapes none of them takes (K % 64 != 0, N % 16 != 0, non-bf16), for decode shapes the
    tuned table measured it fastest on, or under OAMD_PREFILL_BLAS=1 (A/B); CPU tensors on torch."""
    M, K = x.shape
    N = w.shape[0]
    plan = None
    if bias is not None:
        if tile_ok(x, w) and tile_out_ok(out):
            return linear_tile(x, w, out, bias)
        return _blas(x, w, out, bias)
    if x.is_cuda and bm is None and bn is None and splits is None and _measured_blas(M, N, K):
        return _blas(x, w, out, None)
    if PREFILL_BLAS and x.is_cuda and M > 256 and N < LM_HEAD_MIN_N and splits is None and x.dtype == torch.bfloat16:
        return _blas(x, w, out, None, planned=True)
    if (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous() and M <= SKINNY_MAX_M
            and bm is None and bn is None):
        S = splits or skinny_plan(M, N, K)
        if S is not None:
            if S > 1 and (partial is None or partial.numel() < S * M * N):
                partial = torch.empty(S * M * N, dtype=torch.float32, device=x.device)
            if defer_reduce and S > 1 and out is None:
                kernels().gemm_skinny(x, w, None, partial, S, False)
                return SplitK(partial, S, M, N)
            y = out if out is not None else torch.empty(M, N, dtype=x.dtype, device=x.device)
            kernels().gemm_skinny(x, w, y, partial if S > 1 else None, S, False)
            return y
    if x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous():
        plan = gemm_plan(M, N, K)
        if plan is None and (splits or bn or bm) and M % 64 == 0 and M <= 256 and N % 64 == 0 and K % 64 == 0:
            plan = (row_tile(M), 64, 1)  # explicit request (tests / tuning)
    if plan is None:
        if tile_ok(x, w) and tile_out_ok(out):
            return linear_tile(x, w, out)
        return _blas(x, w, out, None)
    bm, bn, S = bm or plan[0], bn or plan[1], splits or plan[2]
    ns = stages or (plan[3] if len(plan) > 3 else 3)
    if S > 1 and (partial is None or partial.numel() < S * M * N):
        partial = torch.empty(S * M * N, dtype=torch.float32, device=x.device)
    if defer_reduce and S > 1 and out is None:
        kernels().gemm_decode(x, w, None, partial, S, bn, bm, False, False, ns)
        return SplitK(partial, S, M, N)
    y = out if out is not None else torch.empty(M, N, dtype=x.dtype, device=x.device)
    kernels().gemm_decode(x, w, y, partial if S > 1 else None, S, bn, bm, False, False, ns)
    return y


FP8_MAX = 448.0  # OCP e4m3fn


def quantize_fp8(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Per-row e4m3fn quantization: (q [M, K] float8_e4m3fn, s [M] fp32), x ~= q * s."""
    M, K = x.shape
    if x.is_cuda and x.dtype == torch.bfloat16 and K % 8 == 0:
        q = torch.empty(M, K, dtype=torch.float8_e4m3fn, device=x.device)
        sx = torch.empty(M, dtype=torch.float32, device=x.device)
        kernels().quantize_fp8(x.contiguous(), q, sx)
        return q, sx
    xf = x.float()
    amax = xf.abs().amax(1)
    sx = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    return (xf / sx[:, None]).to(torch.float8_e4m3fn), sx


def silu_quantize_fp8(gu, block: int | None = GU_BLOCK) -> tuple[torch.Tensor, torch.Tensor]:
    """quantize_fp8(silu_mul(gu, block)) — on the GPU one kernel for 64-feature
    interleaved gate|up rows (the SwiGLU never round-trips HBM as bf16). ``gu`` may be
    the gate|up GEMM's split-K slabs (:class:`SplitK`), summed inside the kernel."""
    M, N2 = gu.shape
    inter = N2 // 2
    if gu.is_cuda and block == GU_BLOCK and inter <= 16384 and N2 % 128 == 0:
        q = torch.empty(M, inter, dtype=torch.float8_e4m3fn, device=gu.device)
        sx = torch.empty(M, dtype=torch.float32, device=gu.device)
        if isinstance(gu, SplitK):
            kernels().silu_quantize_fp8(torch.empty(M, N2, dtype=torch.bfloat16, device=gu.device), q, sx,
                                        gu.p, gu.S)
            return q, sx
        if gu.stride(1) == 1:
            kernels().silu_quantize_fp8(gu, q, sx)
            return q, sx
    if isinstance(gu, SplitK):
        gu = gu.materialize()
    return quantize_fp8(silu_mul(gu, block=block))


def _fp8_overrides() -> dict:
    """OAMD_FP8_PLANS="NxK=bm,bn,S;..." (A/B of fp8 decode plans): (N, K) -> (bm, bn, S)."""
    out = {}
    for item in filter(None, os.environ.get("OAMD_FP8_PLANS", "").split(";")):
        shape, plan = item.split("=")
        n, k = (int(v) for v in shape.split("x"))
        out[(n, k)] = tuple(int(v) for v in plan.split(","))
    return out


_FP8_OVERRIDES = _fp8_overrides()


def fp8_plan(M: int, N: int, K: int) -> tuple[int, int, int]:
    """(bm, bn, splits) for gemm_fp8: row tile by M, 128-column tiles for wide N, and
    split-K until the blocks reach one per CU (K permitting)."""
    if (N, K) in _FP8_OVERRIDES:
        return _FP8_OVERRIDES[(N, K)]
    bm = 64 if M <= 64 else 128 if M <= 128 else 256
    bn = 128 if N % 128 == 0 and N // 128 >= 192 else 64
    mt = -(-M // bm)
    S = 1
    for s in (1, 2, 4, 8):
        if K % (128 * s):
            break
        S = s
        if (N // bn) * s * mt >= 256:
            break
    return bm, bn, S


def linear_fp8(x: torch.Tensor | tuple[torch.Tensor, torch.Tensor], w8: torch.Tensor, sw: torch.Tensor,
               out: torch.Tensor | None = None, plan: tuple[int, int, int] | None = None,
               defer_reduce: bool = False):
    """y = x @ (w8 * sw)^T with x quantized per token to e4m3fn (W8A8, fp32 accumulate).
    ``x`` may already be quantized: a (q, sx) pair from quantize_fp8 / silu_quantize_fp8.
    ``defer_reduce``: a split-K plan returns its fp32 slabs (:class:`SplitK`) for a
    consumer that sums them (rope_kv, rmsnorm, the fused all-reduce + norm, SwiGLU)."""
    q, sx = x if isinstance(x, tuple) else quantize_fp8(x)
    M, K = q.shape
    N = w8.shape[0]
    if not q.is_cuda:
        y = (q.float() * sx[:, None]) @ (w8.float() * sw[:, None]).t()
        return out.copy_(y) if out is not None else y.to(torch.bfloat16 if isinstance(x, tuple) else x.dtype)
    bm, bn, S = plan or fp8_plan(M, N, K)
    y = out if out is not None else torch.empty(M, N, dtype=torch.bfloat16, device=q.device)
    part = torch.empty(S * M * N, dtype=torch.float32, device=q.device) if S > 1 else None
    if defer_reduce and S > 1 and out is None:
        kernels().gemm_fp8(q, w8, sx, sw, y, part, S, bn, bm, False)
        return SplitK(part, S, M, N)
    kernels().gemm_fp8(q, w8, sx, sw, y, part, S, bn, bm)
    return y


def decode_splits(max_context: int, batch: int = 1, kv_heads: int = 8) -> int:
    """Workgroups per (sequence, kv-head) for decode attention: split only while
    ``batch * kv_heads`` workgroups cannot fill the GPU, never into pieces shorter
    than 256 tokens (measured on MI355X, B=16 ctx=1024: 1 split 25.9 us, 4 splits
    23.7 us, 16 splits 47.8 us). Powers of two, so a graph captured per value
    covers every context length with few captures."""
    want = -(-DECODE_TARGET_BLOCKS // max(1, batch * kv_heads))
    cap = -(-max(1, int(max_context)) // DECODE_MIN_SPLIT_TOKENS)
    ns = max(1, min(want, cap, 256))
    # the power of two at or BELOW: splits of 256-512 tokens, not 128-256 (B = 64, one kv-head,
    # ctx 1100: 4 splits 15.2 us vs 8 splits 19.9 us with the combine, profiles/attn_decode_tp8_splits_r5.jsonl)
    return 1 << (ns.bit_length() - 1)


def decode_workspace(B: int, Hq: int, num_splits: int, device, D: int = 128):
    """(o_part fp32, ml_part fp32) partial buffers for attn_decode (unused when num_splits == 1)."""
    n = max(1, B * Hq * num_splits) if num_splits > 1 else 1
    return (torch.empty(n * D, dtype=torch.float32, device=device),
            torch.empty(n * 2, dtype=torch.float32, device=device))


def attn_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                seq_lens: torch.Tensor, scale: float, num_splits: int, out: torch.Tensor | None = None,
                workspace: tuple[torch.Tensor, torch.Tensor] | None = None, variant: int | None = None,
                k_scale: float = 1.0, v_scale: float = 1.0, quant: bool = False):
    """Paged decode attention; ``num_splits`` workgroups per (sequence, kv-head)
    (``decode_splits``). Any value >= 1 is correct; it only changes the schedule.
    The cache is bf16, or e4m3fn holding x / k_scale and x / v_scale.
    ``quant``: return the [B, Hq*D] output rows as per-token e4m3fn ``(q, sx)`` for an
    fp8 o-projection, produced by the split-combine kernel itself (== quantize_fp8)."""
    if not q.is_cuda:
        r = reference.attn_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, k_scale, v_scale)
        if out is not None:
            out.copy_(r)
            r = out
        return quantize_fp8(r.reshape(r.shape[0], -1)) if quant else r
    B, Hq, D = q.shape
    variant = DECODE_ATTN_VARIANT if variant is None else variant
    o = out if out is not None else torch.empty_like(q)
    if workspace is None:
        workspace = decode_workspace(B, Hq, num_splits, q.device)
    q8 = sx = None
    if quant:
        q8 = torch.empty(B, Hq * D, dtype=torch.float8_e4m3fn, device=q.device)
        sx = torch.empty(B, dtype=torch.float32, device=q.device)
    kernels().attn_decode(q, k_cache, v_cache, block_tables, seq_lens, o, workspace[0], workspace[1],
                          num_splits, scale, variant, k_scale, v_scale, q8, sx)
    return (q8, sx) if quant else o


# decode RoPE + KV-cache write folded into decode attention (OAMD_FUSED_ROPE=0: rope_kv, then attn_decode),
# for batches of at most FUSED_ROPE_MAX_SEQ_HEADS (sequence, kv-head) pairs: there attention is
# latency-bound and the fold removes a launch (TP=8 70B fp8 B=64: 6.85 -> 6.64 ms/step); at the
# 8B flagship's 256 x 8 pairs attention streams HBM and every workgroup would pay the fold's
# slab reads and store drain up front (-1.3 % analyses/s, profiles/fused_decode_rope_ab_r5.jsonl)
FUSED_DECODE_ROPE = os.environ.get("OAMD_FUSED_ROPE", "1") != "0"
FUSED_ROPE_MAX_SEQ_HEADS = int(os.environ.get("OAMD_FUSED_ROPE_MAX", "256"))


def attn_decode_rope(qkv, pos: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, Hq: int, k_cache: torch.Tensor,
                     v_cache: torch.Tensor, slots: torch.Tensor, block_tables: torch.Tensor, seq_lens: torch.Tensor,
                     scale: float, num_splits: int, workspace: tuple[torch.Tensor, torch.Tensor] | None = None,
                     bias: torch.Tensor | None = None, k_scale: float = 1.0, v_scale: float = 1.0,
                     quant: bool = False, variant: int | None = None):
    """One decode step's ``rope_kv`` (want_kv=False) + ``attn_decode`` as ONE kernel: every
    attention workgroup rotates its q from the QKV projection (``qkv``: bf16 rows or the
    GEMM's :class:`SplitK` slabs, + the Qwen2 bias), and the workgroup holding each
    sequence's last token writes that token's rotated K and its V into the cache before
    reading it (csrc/kernels/attn_decode.hip, ``DecRope``). Same numerics as the two
    kernels; one launch and the q round trip fewer per layer."""
    Hkv = k_cache.shape[1]
    if not (qkv.is_cuda and FUSED_DECODE_ROPE and qkv.shape[0] * Hkv <= FUSED_ROPE_MAX_SEQ_HEADS):
        q, _, _ = rope_kv(qkv, pos, cos, sin, Hq, Hkv, k_cache, v_cache, slots, want_kv=False, bias=bias,
                          k_scale=k_scale, v_scale=v_scale)
        return attn_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, num_splits, workspace=workspace,
                           variant=variant, k_scale=k_scale, v_scale=v_scale, quant=quant)
    B = qkv.shape[0]
    D = cos.shape[1] * 2
    variant = DECODE_ATTN_VARIANT if variant is None else variant
    o = torch.empty(B, Hq, D, dtype=torch.bfloat16, device=qkv.device)
    if workspace is None:
        workspace = decode_workspace(B, Hq, num_splits, qkv.device)
    q8 = sx = None
    if quant:
        q8 = torch.empty(B, Hq * D, dtype=torch.float8_e4m3fn, device=qkv.device)
        sx = torch.empty(B, dtype=torch.float32, device=qkv.device)
    rx, S = (qkv.p, qkv.S) if isinstance(qkv, SplitK) else (qkv, 1)
    kernels().attn_decode(o, k_cache, v_cache, block_tables, seq_lens, o, workspace[0], workspace[1], num_splits,
                          scale, variant, k_scale, v_scale, q8, sx, rx, S, pos, cos, sin, slots, bias)
    return (q8, sx) if quant else o


def sample(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor, positions: torch.Tensor,
           out: torch.Tensor | None = None, col_offset: int = 0, out_val: torch.Tensor | None = None) -> torch.Tensor:
    """Temperature / Gumbel-max sampling (greedy rows where temperature <= 0).

    For a vocab shard pass ``col_offset`` (global id of column 0) and ``out_val``
    (receives each row's winning perturbed value) and take the max over shards.
    """
    if not logits.is_cuda:
        tok, val = reference.sample_shard(logits, temperature, seeds, positions, col_offset)
        if out_val is not None:
            out_val.copy_(val)
        if out is not None:
            out.copy_(tok)
            return out
        return tok
    o = out if out is not None else torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    kernels().sample(logits, temperature, seeds, positions, o, col_offset, out_val)
    return o
