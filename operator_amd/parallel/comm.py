"""Collective layer over torch.distributed (backend "nccl" == RCCL on ROCm,
"gloo" for the CPU test tier). SURVEY.md §2.4 X1 / §5.8.

* ``init_from_env()`` — torchrun-style env:// rendezvous (RANK, WORLD_SIZE,
  LOCAL_RANK, MASTER_ADDR=127.0.0.1), one process per GPU.
* ``Group`` — a thin handle used by the model: rank/world, in-place
  all-reduce, all-gather, broadcast; a world-1 group is a no-op so the same
  model code runs TP=1 without any communication.
* ``split_groups(tp)`` — carve the world into DP replicas of TP groups
  (TP ranks are consecutive = same xGMI-fully-connected node).

Sizing notes for MI355X xGMI (7 point-to-point links / GPU, ~153 GB/s each):
TP decode all-reduces are tiny (M x hidden x 2 B, e.g. 16 KB/token at 70B),
i.e. latency-bound: they run on the IPC kernels of ``parallel/custom_ar.py``
(one-shot / two-shot, fused with residual + RMSNorm), whose size crossovers are
measured on the node at engine start (``CustomAllReduce.calibrate``); RCCL takes
what the IPC buffers cannot hold and every other collective (barriers, the DFA
broadcast, timing maxima). DP needs no collective on the hot path (per-rank
engines, host-side result gathering).
"""
from __future__ import annotations

import datetime
import threading
import time
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"


def init_from_env(backend: str | None = None, timeout_s: int = 600) -> DistInfo:
    """Initialise the default process group from torchrun env vars (no-op when WORLD_SIZE<=1)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return DistInfo(0, 1, 0, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return DistInfo(rank, world, local, backend)


class _CollectiveStats:
    """Process-wide collective counters for the metrics endpoint (SURVEY.md §5.5 "RCCL
    time"): calls and bytes per (op, impl); wall time only where the host waits on
    the call (an RCCL / gloo collective issued eagerly: the launch-to-return time as
    seen by the host; calls recorded into a hipGraph are counted at capture only)."""

    def __init__(self):
        self._d: dict[tuple[str, str], list[float]] = {}
        self._lock = threading.Lock()

    def add(self, op: str, impl: str, nbytes: int, seconds: float = 0.0) -> None:
        with self._lock:
            st = self._d.setdefault((op, impl), [0, 0, 0.0])
            st[0] += 1
            st[1] += nbytes
            st[2] += seconds

    def snapshot(self) -> dict:
        with self._lock:
            return {k: tuple(v) for k, v in self._d.items()}


COLLECTIVES = _CollectiveStats()


def _nbytes(t) -> int:
    return t.numel() * t.element_size() if isinstance(t, torch.Tensor) else 0


class Group:
    """Process-group handle; world==1 makes every collective a no-op."""

    def __init__(self, pg=None, ranks: list[int] | None = None):
        self.pg = pg
        if pg is None and not (dist.is_available() and dist.is_initialized()):
            self.rank, self.world, self.ranks = 0, 1, [0]
        else:
            self.rank = dist.get_rank(pg)
            self.world = dist.get_world_size(pg)
            self.ranks = ranks if ranks is not None else list(range(self.world))

    @staticmethod
    def single() -> "Group":
        g = Group.__new__(Group)
        g.pg, g.rank, g.world, g.ranks = None, 0, 1, [0]
        return g

    def enable_oneshot(self, device, max_bytes: int | None = None, oneshot_max_bytes: int | None = None) -> bool:
        """Route GPU all-reduces up to ``max_bytes`` through the IPC kernels (custom_ar.py):
        one-shot up to ``oneshot_max_bytes``, two-shot above. Collective over the group;
        returns False (RCCL stays in use) on world 1 or CPU."""
        if self.world <= 1 or torch.device(device).type != "cuda":
            return False
        from .custom_ar import DEFAULT_MAX_BYTES, DEFAULT_ONESHOT_MAX_BYTES, OneShotAllReduce

        self.oneshot = OneShotAllReduce(self, device, max_bytes or DEFAULT_MAX_BYTES,
                                        oneshot_max_bytes=oneshot_max_bytes or DEFAULT_ONESHOT_MAX_BYTES)
        return True

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            car = getattr(self, "oneshot", None)
            if car is not None and car.fits(t):
                COLLECTIVES.add("all_reduce", "ipc", _nbytes(t))
                return car.all_reduce_(t)
            t0 = time.perf_counter()
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg)
            COLLECTIVES.add("all_reduce", dist.get_backend(self.pg), _nbytes(t), time.perf_counter() - t0)
        return t

    def all_reduce_rmsnorm(self, t, w: torch.Tensor, eps: float, residual: torch.Tensor, quant: bool = False):
        """The TP block epilogue: residual += all_reduce(t); return rmsnorm(residual) * w.
        With the one-shot IPC all-reduce enabled this is ONE fused gfx950 kernel (the
        reduced rows are normalised by the block that summed them; ``t`` may be the
        producing GEMM's split-K slabs, summed on the way in); otherwise the all-reduce
        (RCCL / gloo) then the rmsnorm kernel. World 1: just the rmsnorm (which also sums
        slabs). ``quant``: return per-row e4m3fn ``(q, sx)`` of the result (fused into the
        one-shot kernel) for an fp8 GEMM."""
        from operator_amd import ops

        if self.world > 1:
            car = getattr(self, "oneshot", None)
            if car is not None and car.fits_rows(t) and residual.is_contiguous():
                COLLECTIVES.add("all_reduce_rmsnorm", "ipc", 2 * t.shape[0] * t.shape[1])
                return car.all_reduce_rmsnorm_(t, residual, w, eps, quant=quant)
            if isinstance(t, ops.SplitK):
                t = t.materialize()
            self.all_reduce_(t)
        y = ops.rmsnorm(t, w, eps, residual=residual)
        return ops.quantize_fp8(y) if quant else y

    def all_gather(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        if self.world == 1:
            return t
        out = [torch.empty_like(t) for _ in range(self.world)]
        t0 = time.perf_counter()
        dist.all_gather(out, t.contiguous(), group=self.pg)
        COLLECTIVES.add("all_gather", dist.get_backend(self.pg), _nbytes(t) * self.world, time.perf_counter() - t0)
        return torch.cat(out, dim=dim)

    def all_gather_into(self, t: torch.Tensor) -> torch.Tensor:
        """Gather equal-shaped tensors along a new leading dim: [world, *t.shape]."""
        if self.world == 1:
            return t.unsqueeze(0)
        t = t.contiguous()
        out = torch.empty((self.world * t.shape[0], *t.shape[1:]), dtype=t.dtype, device=t.device)
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(out, t, group=self.pg)
        COLLECTIVES.add("all_gather", dist.get_backend(self.pg), _nbytes(out), time.perf_counter() - t0)
        return out.view(self.world, *t.shape)

    def broadcast_(self, t: torch.Tensor, src_local: int = 0) -> torch.Tensor:
        if self.world > 1:
            dist.broadcast(t, src=self.ranks[src_local], group=self.pg)
        return t

    def barrier(self) -> None:
        if self.world > 1:
            dist.barrier(group=self.pg)


class SimulatedTPGroup(Group):
    """Rank 0's shard of a TP=``world`` replica on ONE device, for per-rank performance
    (tools/bench_tp.py --simulate-tp): the model is sharded exactly as at TP=world and
    every collective launches the world-1 one-shot kernels (the same push / flag /
    reduce code path and fused RMSNorm, with no peer to wait for), so a step costs what
    one rank's step costs minus the xGMI transfer time. Gathers replicate the local
    shard. Without a GPU the collectives are no-ops."""

    def __init__(self, world: int, device):
        self.pg, self.rank, self.world, self.ranks = None, 0, int(world), list(range(int(world)))
        self.car = None
        if torch.device(device).type == "cuda":
            from .custom_ar import DEFAULT_MAX_BYTES, OneShotAllReduce

            self.car = OneShotAllReduce(Group.single(), device, DEFAULT_MAX_BYTES)

    def enable_oneshot(self, device, max_bytes: int | None = None) -> bool:
        return self.car is not None

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.car is not None and self.car.fits(t):
            COLLECTIVES.add("all_reduce", "oneshot-sim", _nbytes(t))
            return self.car.all_reduce_(t)
        return t

    def all_reduce_rmsnorm(self, t, w: torch.Tensor, eps: float, residual: torch.Tensor, quant: bool = False):
        from operator_amd import ops

        if self.car is not None and self.car.fits_rows(t) and residual.is_contiguous():
            COLLECTIVES.add("all_reduce_rmsnorm", "oneshot-sim", 2 * t.shape[0] * t.shape[1])
            return self.car.all_reduce_rmsnorm_(t, residual, w, eps, quant=quant)
        y = ops.rmsnorm(t, w, eps, residual=residual)
        return ops.quantize_fp8(y) if quant else y

    def all_gather(self, t: torch.Tensor, dim: int = 0) -> torch.Tensor:
        return torch.cat([t] * self.world, dim=dim)

    def all_gather_into(self, t: torch.Tensor) -> torch.Tensor:
        return t.unsqueeze(0).expand(self.world, *t.shape).contiguous()

    def broadcast_(self, t: torch.Tensor, src_local: int = 0) -> torch.Tensor:
        return t

    def barrier(self) -> None:
        pass


def split_groups(tp: int) -> tuple[Group, Group]:
    """Return (tp_group, dp_group) for this rank. World must be a multiple of tp."""
    if not (dist.is_available() and dist.is_initialized()):
        return Group.single(), Group.single()
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % tp:
        raise ValueError(f"world {world} not divisible by tp {tp}")
    tp_g = dp_g = None
    tp_ranks = dp_ranks = None
    for i in range(world // tp):
        ranks = list(range(i * tp, (i + 1) * tp))
        g = dist.new_group(ranks)
        if rank in ranks:
            tp_g, tp_ranks = g, ranks
    for j in range(tp):
        ranks = list(range(j, world, tp))
        g = dist.new_group(ranks)
        if rank in ranks:
            dp_g, dp_ranks = g, ranks
    return Group(tp_g, tp_ranks), Group(dp_g, dp_ranks)
