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

Size-aware dispatch, measured on the node: ``calibrate()`` (run by the engine factory when
the TP group is created, before any graph is captured) times one-shot, two-shot and the
group's own backend (RCCL in production) on the TP group's real decode message sizes (decode
bucket rows x hidden x 2 B), takes the MAX over ranks so every rank holds the same numbers,
and builds a dispatch table ``[(up_to_bytes, protocol)]`` with ``choose_protocols`` -- the
same table on every rank, which the protocol choice must be (a rank on RCCL while its peer
waits in a one-shot kernel is a deadlock). Without calibration (``engine.oneshot_max_kb`` > 0
as an override, or a forced protocol) messages up to ``oneshot_max_bytes`` go one-shot,
larger ones two-shot, up to ``max_bytes`` (``engine.oneshot_allreduce_mb``); above that
``Group.all_reduce_`` keeps using RCCL. OAMD_CAR_PROTOCOL = oneshot / twoshot / fence / ll forces
one protocol (fence: the original system-fence one-shot hand-off, for A/B).

* LL (flag-in-data one-shot): each 16-B vector travels as two packets that carry the call's
  round in their flag words, so the consumer polls the data itself -- no store-completion
  wait, barrier, flag store and flag poll between push and reduce; twice the bytes on the
  link, so it competes for the small decode messages (up to half the buffer capacity).

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
DEFAULT_ONESHOT_MAX_BYTES = 512 << 10   # uncalibrated: one-shot up to here, two-shot above
PROTO_ONESHOT, PROTO_TWOSHOT, PROTO_FENCE, PROTO_LL = 0, 1, 2, 3   # csrc/kernels/kernels.h kCar*
PROTO_BACKEND = -1   # the group's own all-reduce (RCCL): the IPC kernels step aside
PROTO_NAMES = {PROTO_ONESHOT: "oneshot", PROTO_TWOSHOT: "twoshot", PROTO_FENCE: "fence", PROTO_LL: "ll",
               PROTO_BACKEND: "backend"}


def choose_protocols(sizes: list[int], times: dict[int, list[float]], margin: float = 0.03) -> list[tuple[int, int]]:
    """Dispatch table from per-size timings: ``sizes`` ascending message bytes, ``times``
    {protocol: seconds per call at each size} (missing / non-finite = unavailable).
    The fastest protocol wins each size; the group backend (RCCL) must beat the best IPC
    protocol by ``margin`` to take a size (it also costs host launch work the IPC kernels
    do not). Runs of one protocol merge; the result is ``[(up_to_bytes, protocol)]`` with
    strictly increasing bounds, the last bound = the largest size. A pure function of its
    inputs, so ranks holding the same (max-reduced) timings build the same table."""
    if not sizes:
        return []
    table: list[tuple[int, int]] = []
    for k, size in enumerate(sizes):
        best, best_t = None, float("inf")
        for p in (PROTO_LL, PROTO_ONESHOT, PROTO_TWOSHOT):
            t = times.get(p, [float("inf")] * len(sizes))[k]
            if t == t and t < best_t:   # skips NaN
                best, best_t = p, t
        tb = times.get(PROTO_BACKEND, [float("inf")] * len(sizes))[k]
        if tb == tb and tb < best_t * (1.0 - margin):
            best = PROTO_BACKEND
        if best is None:
            best = PROTO_BACKEND
        if table and table[-1][1] == best:
            table[-1] = (size, best)
        else:
            table.append((size, best))
    return table


def lookup_protocol(table: list[tuple[int, int]], nbytes: int) -> int:
    """The protocol the table assigns to a message of ``nbytes`` (past its last bound:
    the last entry's protocol)."""
    for bound, p in table:
        if nbytes <= bound:
            return p
    return table[-1][1]
_FORCED = {"oneshot": PROTO_ONESHOT, "twoshot": PROTO_TWOSHOT, "fence": PROTO_FENCE, "ll": PROTO_LL}
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
        self.table: list[tuple[int, int]] | None = None   # calibrate(): measured dispatch table
        self.calibration: dict | None = None

    def route(self, nbytes: int) -> int:
        """Protocol for a message of ``nbytes``: the forced one, the calibrated table's, or
        one-shot up to ``oneshot_max_bytes`` and two-shot above. PROTO_BACKEND = RCCL."""
        if self.forced is not None:
            p = self.forced
        elif self.table:
            p = lookup_protocol(self.table, nbytes)
        else:
            p = PROTO_ONESHOT if nbytes <= self.oneshot_max_bytes else PROTO_TWOSHOT
        if p == PROTO_LL and 2 * nbytes > self.max_bytes:   # LL packets carry half their bytes as flags
            p = PROTO_ONESHOT
        return p

    def fits(self, t: torch.Tensor) -> bool:
        nbytes = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32)
                and nbytes % 16 == 0 and nbytes <= self.max_bytes and self.route(nbytes) != PROTO_BACKEND)

    def proto_for(self, nbytes: int) -> int:
        p = self.route(nbytes)
        self.by_proto[p] = self.by_proto.get(p, 0) + 1
        self.calls += 1
        return p

    def calibrate(self, sizes: list[int], iters: int = 20, warmup: int = 3, backend: bool = True) -> dict:
        """Time one-shot, two-shot and (``backend``) the group's own all-reduce on bf16
        messages of each size in ``sizes`` (bytes; capped at the IPC capacity), max over
        ranks, and install the resulting dispatch table. Collective over the group; call
        it before capturing graphs (they bake the protocol in). Returns the report that
        bench JSON lines carry: sizes, per-protocol microseconds and the table."""
        import time

        sizes = sorted({int(b) // 16 * 16 for b in sizes if 16 <= int(b) <= self.max_bytes})
        if not sizes:
            return {}
        forced, self.forced = self.forced, None
        protos = [PROTO_LL, PROTO_ONESHOT, PROTO_TWOSHOT] + ([PROTO_BACKEND] if backend and self.world > 1 else [])
        res = torch.full((len(protos), len(sizes)), float("nan"), dtype=torch.float64)
        buf = torch.zeros(sizes[-1] // 2, dtype=torch.bfloat16, device=self.device)

        def barrier():
            if self.world > 1:
                dist.barrier(group=self.group.pg)

        for k, size in enumerate(sizes):
            t = buf[: size // 2]
            for pi, p in enumerate(protos):
                if p == PROTO_LL and 2 * size > self.max_bytes:
                    continue   # beyond LL capacity: stays NaN (unavailable)
                if p == PROTO_BACKEND:
                    call = (lambda t=t: dist.all_reduce(t, group=self.group.pg))
                else:
                    call = (lambda t=t, p=p: self.ext.all_reduce(t, t, p))
                barrier()
                for _ in range(warmup):
                    call()
                torch.cuda.synchronize(self.device)
                barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    call()
                torch.cuda.synchronize(self.device)
                res[pi, k] = (time.perf_counter() - t0) / iters
        self.check()   # a peer that never arrived poisons the buffers: fail before dispatching on them
        if self.world > 1:   # every rank decides on the same (slowest-rank) numbers
            dev = self.device if dist.get_backend(self.group.pg) == "nccl" else torch.device("cpu")
            r = res.to(dev)
            dist.all_reduce(r, op=dist.ReduceOp.MAX, group=self.group.pg)
            res = r.cpu()
        times = {p: [float(x) for x in res[pi]] for pi, p in enumerate(protos)}
        self.forced = forced
        self.table = choose_protocols(sizes, times)
        self.calibration = {
            "world": self.world, "sizes": sizes,
            "us": {PROTO_NAMES[p]: [round(x * 1e6, 2) for x in v] for p, v in times.items()},
            "table": [[b, PROTO_NAMES[p]] for b, p in self.table],
            "backend": dist.get_backend(self.group.pg) if self.world > 1 else None,
        }
        return self.calibration

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
                    and rows * hidden * 2 <= self.max_bytes and self.route(rows * hidden * 2) != PROTO_BACKEND)
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
