"""Paged KV cache (SURVEY.md §2.4 N10/N12, §7.1 runtime/kvcache).

Layout per layer: K and V tensors [pages, Hkv_local, page_size, D] (bf16) —
a kv-head's tokens of one page are contiguous, which is what the decode
attention kernel streams (4 tokens = 1 KiB per wave load). All layers live in
two big allocations [L, pages, Hkv, P, D] sized up front from the HBM budget
(288 GB/GPU: for Llama-3-8B at 128 KiB/token, ~1.5M tokens fit beside the weights).

Page bookkeeping (free list, per-sequence page tables) is host-side and
O(pages) per request; block tables are uploaded as int32 rows.

``dtype=torch.float8_e4m3fn`` keeps K and V as OCP e4m3 with per-tensor scales
(``k_scale`` / ``v_scale``, stored value = x / scale): half the bytes per token,
so twice the tokens per GB and half the HBM traffic of decode attention, at
fp8 precision for the cached keys and values (queries and all compute stay
bf16 / fp32). Not the default.
"""
from __future__ import annotations

import threading

import torch


class PageAllocator:
    """LIFO free list of page ids (recently freed pages are reused first: warm in L2/MALL)."""

    def __init__(self, num_pages: int):
        self.num_pages = num_pages
        self._free = list(range(num_pages - 1, -1, -1))
        self._lock = threading.Lock()

    @property
    def free(self) -> int:
        return len(self._free)

    def alloc(self, n: int) -> list[int]:
        with self._lock:
            if n > len(self._free):
                raise MemoryError(f"KV cache exhausted: need {n} pages, {len(self._free)} free")
            out = self._free[-n:][::-1] if n else []
            del self._free[len(self._free) - n:]
            return out

    def release(self, pages: list[int]) -> None:
        with self._lock:
            self._free.extend(reversed(pages))


class PagedKVCache:
    def __init__(self, layers: int, num_pages: int, kv_heads: int, head_dim: int, page_size: int = 64,
                 device: str | torch.device = "cuda", dtype: torch.dtype = torch.bfloat16,
                 k_scale: float = 1.0, v_scale: float = 1.0):
        if page_size & (page_size - 1):
            raise ValueError("page_size must be a power of two")
        if k_scale <= 0 or v_scale <= 0:
            raise ValueError("KV scales must be positive")
        self.dtype, self.k_scale, self.v_scale = dtype, float(k_scale), float(v_scale)
        self.layers, self.num_pages, self.kv_heads, self.head_dim, self.page_size = (
            layers, num_pages, kv_heads, head_dim, page_size)
        shape = (layers, num_pages, kv_heads, page_size, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        self.allocator = PageAllocator(num_pages)

    @staticmethod
    def pages_for_budget(budget_bytes: int, layers: int, kv_heads: int, head_dim: int, page_size: int,
                         dtype_bytes: int = 2) -> int:
        per_page = 2 * layers * kv_heads * page_size * head_dim * dtype_bytes
        return max(1, int(budget_bytes // per_page))

    def pages_needed(self, tokens: int) -> int:
        return (tokens + self.page_size - 1) // self.page_size

    def layer(self, i: int) -> tuple[torch.Tensor, torch.Tensor]:
        return self.k[i], self.v[i]

    def slots_for(self, pages: list[int], start: int, n: int) -> list[int]:
        P = self.page_size
        return [pages[(start + j) // P] * P + (start + j) % P for j in range(n)]
