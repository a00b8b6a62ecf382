"""Data parallelism over failures.

Analyses are independent, so DP needs no collective on the hot path: each
rank owns a deterministic shard of the work (stable hash of the pod key, so
the same failure always lands on the same GPU — its cached DFA/KV state stays
warm and retries do not duplicate), runs the full match + explain pipeline
locally, and only small results move (object all-gather to the leader).
"""
from __future__ import annotations

import hashlib
from typing import Any, Callable, Sequence

import torch.distributed as dist


def stable_rank(key: str, world: int) -> int:
    return int.from_bytes(hashlib.blake2b(key.encode(), digest_size=8).digest(), "little") % world


class DPRouter:
    def __init__(self, group=None):
        self.group = group
        init = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank(group) if init else 0
        self.world = dist.get_world_size(group) if init else 1

    def owner(self, key: str) -> int:
        return stable_rank(key, self.world)

    def shard(self, items: Sequence[Any], key: Callable[[Any], str] = str) -> list[Any]:
        """This rank's items (hash-partitioned)."""
        return [x for x in items if self.owner(key(x)) == self.rank]

    def gather(self, local: list[Any], dst: int = 0) -> list[Any] | None:
        """Concatenate every rank's list on ``dst`` (None elsewhere)."""
        if self.world == 1:
            return list(local)
        out: list[Any] = [None] * self.world
        dist.all_gather_object(out, local, group=self.group)
        if self.rank != dst:
            return None
        return [x for part in out for x in part]
