"""One-shot / two-shot all-reduce over peer-mapped HBM for tensor-parallel decode
(kernel: csrc/kernels/allreduce.hip).

RCCL's ring all-reduce over xGMI takes 2(n-1) dependent link hops; a TP decode
all-reduce is only M x hidden x 2 B (16 KB per token at 70B), so those hops,
not bandwidth, set its cost. Two protocols over the same fine-grained buffers,
both one kernel with no host involvement per call (device-side round counters),
so they are capturable in the decode hipGraph:

* one-shot: each rank pushes its whole input into a slot of every peer's receive
  buffer over the direct link to that peer and reduces the n slots locally: one
  fabric hop, (n-1) x S bytes out of each rank;
* two-shot: reduce-scatter (piece q of the input to rank q) then all-gather of the
  reduced pieces: two hops, 2(n-1)/n x S bytes out of each rank (at the 70B B=256
  decode all-reduce, 4 MB at world 8: 7 MB instead of 28 MB over the 7 links).

Size-aware dispatch: messages up to ``oneshot_max_bytes`` (config key
``engine.oneshot_max_kb``, default 512 KB as SURVEY §5.8 sizes it) go one-shot,
larger ones two-shot, up to ``max_bytes`` (``engine.oneshot_allreduce_mb``); above
that ``Group.all_reduce_`` keeps using RCCL. The one-shot/two-shot crossover is
UNMEASURED until an 8-GPU node is available (docs/PARITY.md); OAMD_CAR_PROTOCOL =
oneshot / twoshot / fence forces one protocol (fence: the original system-fence
one-shot hand-off, for A/B).

Set-up exchanges the 64-byte hipIpc handles over the process group (any
backend: gloo in tests, RCCL in production).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from operator_amd import ops


class CollectiveTimeout(RuntimeError):
    """A device-side collective gave up waiting for a peer: this replica's state is
    no longer consistent across ranks and it must be restarted as a whole."""


DEFAULT_MAX_BYTES = 8 << 20   # 256 tokens x 8192 x 2 B (70B hidden) = 4 MB, with room
DEFAULT_ONESHOT_MAX_BYTES = 512 << 10   # one-shot up to here, two-shot above (crossover unmeasured)
PROTO_ONESHOT, PROTO_TWOSHOT, PROTO_FENCE = 0, 1, 2   # csrc/kernels/kernels.h kCar*
_FORCED = {"oneshot": PROTO_ONESHOT, "twoshot": PROTO_TWOSHOT, "fence": PROTO_FENCE}
# workgroups of every one-shot call (fixed per group: each block keeps its own round
# counter and data-slot parity, so every call of a group must use the same count)
DEFAULT_BLOCKS = int(os.environ.get("OAMD_CAR_BLOCKS", "64"))   # 64 vs 32: 7.15 vs 7.63 ms TP8-sim step (profiles/tp8_car_blocks_r5.jsonl)


class OneShotAllReduce:
    """The IPC all-reduce of one TP group (one-shot and two-shot, size-dispatched)."""

    def __init__(self, group, device: torch.device | str, max_bytes: int = DEFAULT_MAX_BYTES,
                 blocks: int = DEFAULT_BLOCKS, timeout_s: float = 2.0,
                 oneshot_max_bytes: int = DEFAULT_ONESHOT_MAX_BYTES, protocol: str | None = None):
        self.group = group
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("OneShotAllReduce needs a GPU device")
        self.world, self.rank = group.world, group.rank
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks (one xGMI-connected node)")
        self.max_bytes = (int(max_bytes) + 15) // 16 * 16
        self.oneshot_max_bytes = int(oneshot_max_bytes)
        protocol = protocol or os.environ.get("OAMD_CAR_PROTOCOL", "auto")
        if protocol != "auto" and protocol not in _FORCED:
            raise ValueError(f"all-reduce protocol {protocol!r}: auto, oneshot, twoshot or fence")
        self.forced = _FORCED.get(protocol)
        self.by_proto = {PROTO_ONESHOT: 0, PROTO_TWOSHOT: 0, PROTO_FENCE: 0}
        self.ext = ops.kernels().CustomAllReduce(self.max_bytes, self.rank, self.world, int(blocks),
                                                 self.device.index or 0, float(timeout_s))
        handles = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(handles, self.ext.handle(), group=group.pg)
        else:
            handles = [self.ext.handle()]
        self.ext.open([bytes(h) for h in handles])
        self.calls = 0

    def fits(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32)
                and nbytes % 16 == 0 and nbytes <= self.max_bytes)

    def proto_for(self, nbytes: int) -> int:
        """One-shot up to ``oneshot_max_bytes``, two-shot above (or the forced protocol)."""
        p = self.forced if self.forced is not None else (
            PROTO_ONESHOT if nbytes <= self.oneshot_max_bytes else PROTO_TWOSHOT)
        self.by_proto[p] += 1
        self.calls += 1
        return p

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        self.ext.all_reduce(t, t, self.proto_for(t.numel() * t.element_size()))
        return t

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty_like(t)
        self.ext.all_reduce(t, out, self.proto_for(t.numel() * t.element_size()))
        return out

    def fits_rows(self, t) -> bool:
        """The fused all-reduce + RMSNorm takes bf16 [rows, hidden] (or the fp32 split-K
        slabs of such rows, ``ops.SplitK``) within capacity."""
        if isinstance(t, ops.SplitK):
            rows, hidden = t.shape
            return (t.p.is_cuda and t.p.is_contiguous() and hidden % 8 == 0 and hidden <= 16384
                    and rows * hidden * 2 <= self.max_bytes)
        return (self.fits(t) and t.dtype == torch.bfloat16 and t.dim() == 2 and t.shape[1] % 8 == 0
                and t.shape[1] <= 16384)

    def all_reduce_rmsnorm_(self, t, residual: torch.Tensor, w: torch.Tensor, eps: float,
                            out: torch.Tensor | None = None, quant: bool = False):
        """residual += sum over ranks of t (bf16-rounded); returns rmsnorm(residual) * w.
        One launch: the row-partitioned one-shot push, then each block normalises whole
        rows straight from its receive slots. ``t`` may be split-K slabs (summed in the
        kernel); ``quant`` returns the rows as per-row e4m3fn ``(q, sx)`` instead, for
        the next fp8 GEMM (== ``ops.quantize_fp8(y)``)."""
        rows, hidden = residual.shape
        y = out if out is not None else torch.empty_like(residual)
        q8 = sx = None
        if quant:
            q8 = torch.empty(rows, hidden, dtype=torch.float8_e4m3fn, device=residual.device)
            sx = torch.empty(rows, dtype=torch.float32, device=residual.device)
        proto = self.proto_for(rows * hidden * 2)
        if isinstance(t, ops.SplitK):
            self.ext.all_reduce_rmsnorm(None, residual, w, y, float(eps), t.p, t.S, q8, sx, proto)
        else:
            self.ext.all_reduce_rmsnorm(t, residual, w, y, float(eps), None, 1, q8, sx, proto)
        return (q8, sx) if quant else y

    @property
    def failed(self) -> bool:
        """A call timed out waiting for a peer. Sticky: every later call returns NaN
        without touching a peer until ``reset()``. A host read, no device sync."""
        return bool(self.ext.error())

    def check(self) -> None:
        """Raise if any call so far timed out waiting for a peer (its output, and that of
        every later call, is NaN: never a partial sum)."""
        if self.ext.error():
            raise CollectiveTimeout("one-shot all-reduce: a peer did not arrive in time; the TP replica must restart")

    def reset(self) -> None:
        """Collective re-arm (every rank, between barriers, nothing in flight)."""
        self.ext.reset()

    def close(self) -> None:
        self.ext.close()
