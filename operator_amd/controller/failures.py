"""Pod-failure detection and de-duplication.

Reference semantics: a pod has failed iff any ``containerStatuses[].state.terminated``
has ``exitCode != 0`` (J/service/PodFailureWatcher.java:147-159); the dedupe
key is ``ns/name`` -> the FIRST terminated container's ``finishedAt``
(:180-194, :208-220). Differences, all opt-in or safety fixes:

* null-safe everywhere (the reconciler's copy NPEs: Q13);
* ``include_last_state`` also treats ``lastState.terminated`` (CrashLoopBackOff
  while the container is ``waiting``) as a failure, and ``include_init``
  checks initContainerStatuses — both off by default for parity;
* the processed-failure map is a bounded LRU with TTL (Q4: unbounded upstream).
"""
from __future__ import annotations

import threading
import time
import zlib
from collections import OrderedDict
from typing import Any


def _statuses(pod: dict, include_init: bool) -> list[dict]:
    st = (pod or {}).get("status") or {}
    out = list(st.get("containerStatuses") or [])
    if include_init:
        out += list(st.get("initContainerStatuses") or [])
    return [c for c in out if c]


def _exit_code(term: dict) -> int:
    try:
        return int(term.get("exitCode", 0) or 0)
    except (TypeError, ValueError):
        return 0


def has_pod_failed(pod: dict, include_last_state: bool = False, include_init: bool = False) -> bool:
    for cs in _statuses(pod, include_init):
        term = ((cs.get("state") or {}).get("terminated"))
        if term and _exit_code(term) != 0:
            return True
        if include_last_state:
            lt = (cs.get("lastState") or {}).get("terminated")
            if lt and _exit_code(lt) != 0:
                return True
    return False


def in_shard(pod: dict, index: int, count: int) -> bool:
    """Operator sharding: pod ns/name -> shard crc32 % count (stable across processes
    and restarts); every pod belongs to exactly one of ``count`` shards."""
    if count <= 1:
        return True
    md = pod.get("metadata") or {}
    return zlib.crc32(f"{md.get('namespace') or ''}/{md.get('name') or ''}".encode()) % count == index


def failure_time(pod: dict, include_last_state: bool = False) -> str | None:
    for cs in _statuses(pod, False):
        term = (cs.get("state") or {}).get("terminated")
        if term and term.get("finishedAt"):
            return str(term["finishedAt"])
    if include_last_state:
        for cs in _statuses(pod, False):
            lt = (cs.get("lastState") or {}).get("terminated")
            if lt and lt.get("finishedAt"):
                return str(lt["finishedAt"])
    return None


def failed_containers(pod: dict) -> list[str]:
    out = []
    for cs in _statuses(pod, True):
        term = (cs.get("state") or {}).get("terminated")
        if term and _exit_code(term) != 0:
            out.append(cs.get("name", ""))
    return out


class FailureDeduper:
    """processedFailures with bounded size and TTL; thread-safe."""

    def __init__(self, max_entries: int = 100_000, ttl_s: float = 7 * 24 * 3600, clock=time.monotonic):
        self.max_entries, self.ttl_s, self.clock = max_entries, ttl_s, clock
        self._d: OrderedDict[str, tuple[str, float]] = OrderedDict()
        self._lock = threading.Lock()

    @staticmethod
    def key(pod: dict) -> str:
        md = (pod or {}).get("metadata") or {}
        return f"{md.get('namespace')}/{md.get('name')}"

    def seen(self, pod: dict, ftime: str | None) -> bool:
        """True if this exact failure (same finishedAt) was already processed."""
        if ftime is None:
            return False
        k = self.key(pod)
        with self._lock:
            v = self._d.get(k)
            if v is None:
                return False
            if self.clock() - v[1] > self.ttl_s:
                del self._d[k]
                return False
            return v[0] == ftime

    def mark(self, pod: dict, ftime: str | None) -> None:
        if ftime is None:
            return
        k = self.key(pod)
        with self._lock:
            self._d[k] = (ftime, self.clock())
            self._d.move_to_end(k)
            while len(self._d) > self.max_entries:
                self._d.popitem(last=False)

    def check_and_mark(self, pod: dict, ftime: str | None) -> bool:
        """Atomically: return True (and record) if new; False if already processed."""
        with self._lock:
            k = self.key(pod)
            if ftime is not None:
                v = self._d.get(k)
                if v is not None and v[0] == ftime and self.clock() - v[1] <= self.ttl_s:
                    self._d.move_to_end(k)   # LRU: a repeat event keeps the entry recent (TTL unchanged)
                    return False
                self._d[k] = (ftime, self.clock())
                self._d.move_to_end(k)
                while len(self._d) > self.max_entries:
                    self._d.popitem(last=False)
            return True

    def __len__(self) -> int:
        return len(self._d)


def matches_monitor(pod: dict, monitor: dict) -> bool:
    """Podmortem selects pod? matchLabels AND matchExpressions; a selector with neither
    matches NOTHING (J/service/PodFailureWatcher.java:247-265)."""
    from operator_amd.kube.resources import match_selector, selector_is_empty

    spec: dict[str, Any] = (monitor or {}).get("spec") or {}
    sel = spec.get("podSelector")
    if selector_is_empty(sel):
        return False
    labels = ((pod or {}).get("metadata") or {}).get("labels")
    if labels is None:
        return False
    return match_selector(sel, labels)
