"""Minimal controller runtime (the role JOSDK plays for the reference:
J/reconcile/*Reconciler.java implement io.javaoperatorsdk Reconciler<T>).

* list + watch a custom resource, with watch restart on error (exponential
  backoff, resourceVersion resume) and an optional periodic resync;
* generation-aware: a MODIFIED event whose metadata.generation was already
  reconciled (i.e. a status-only write) does not trigger a reconcile
  (JOSDK's default generationAwareEventProcessing);
* per-object serialisation: one reconcile per object at a time; events that
  arrive meanwhile coalesce into one follow-up run;
* ``UpdateControl``: status merge-patch, reschedule-after, or no update;
* failed reconciles retry with backoff (2 s initial, x1.5, 5 attempts).
"""
from __future__ import annotations

import heapq
import itertools
import logging
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable

from operator_amd.kube.informer import WatchLoop
from operator_amd.kube.resources import Resource

log = logging.getLogger(__name__)


@dataclass
class UpdateControl:
    status: dict | None = None          # merge-patch for the status subresource
    reschedule_after: float | None = None

    @staticmethod
    def no_update(reschedule_after: float | None = None) -> "UpdateControl":
        return UpdateControl(None, reschedule_after)

    @staticmethod
    def patch_status(status: dict, reschedule_after: float | None = None) -> "UpdateControl":
        return UpdateControl(status, reschedule_after)


class _DelayQueue:
    def __init__(self):
        self._h: list[tuple[float, int, tuple]] = []
        self._cv = threading.Condition()
        self._n = itertools.count()
        self._closed = False

    def put(self, key: tuple, delay: float = 0.0) -> None:
        with self._cv:
            heapq.heappush(self._h, (time.monotonic() + delay, next(self._n), key))
            self._cv.notify()

    def get(self, timeout: float = 0.5) -> tuple | None:
        with self._cv:
            end = time.monotonic() + timeout
            while not self._closed:
                now = time.monotonic()
                if self._h and self._h[0][0] <= now:
                    return heapq.heappop(self._h)[2]
                wait = min(end - now, (self._h[0][0] - now) if self._h else end - now)
                if wait <= 0:
                    return None
                self._cv.wait(wait)
            return None

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()


class Controller:
    def __init__(self, kube, res: Resource, reconcile: Callable[[dict], UpdateControl | None], name: str = "",
                 workers: int = 2, resync_s: float | None = None, retry_initial_s: float = 2.0,
                 retry_multiplier: float = 1.5, max_attempts: int = 5, watch_restart_s: float = 5.0,
                 generation_aware: bool = True):
        self.kube, self.res, self.reconcile_fn = kube, res, reconcile
        self.name = name or res.kind
        self.workers = workers
        self.resync_s = resync_s
        self.retry_initial_s, self.retry_multiplier, self.max_attempts = retry_initial_s, retry_multiplier, max_attempts
        self.watch_restart_s = watch_restart_s
        self.generation_aware = generation_aware
        self.queue = _DelayQueue()
        self._inflight: set[tuple] = set()
        self._dirty: set[tuple] = set()
        self._queued: set[tuple] = set()
        self._attempts: dict[tuple, int] = {}
        self._gen: dict[tuple, int] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self._loop = WatchLoop(kube, res, None, self._on_event, relist=self._enqueue_all, name=f"{self.name}-watch",
                               restart_delay_s=watch_restart_s, stop=self._stop)
        self.reconciles = 0
        self.errors = 0

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self._stop.clear()
        self._initial_list()
        t = threading.Thread(target=self._loop.run, name=f"{self.name}-watch", daemon=True)
        t.start()
        self._threads.append(t)
        for i in range(self.workers):
            w = threading.Thread(target=self._work_loop, name=f"{self.name}-worker-{i}", daemon=True)
            w.start()
            self._threads.append(w)
        if self.resync_s:
            r = threading.Thread(target=self._resync_loop, name=f"{self.name}-resync", daemon=True)
            r.start()
            self._threads.append(r)

    def stop(self) -> None:
        self._stop.set()
        self.queue.close()
        self._loop.stop()
        for t in self._threads:
            t.join(timeout=2)
        self._threads.clear()

    # ------------------------------------------------------------------ event sources
    @staticmethod
    def _key(obj: dict) -> tuple:
        md = obj.get("metadata") or {}
        return (md.get("namespace") or "", md.get("name"))

    def enqueue(self, key: tuple, delay: float = 0.0) -> None:
        with self._lock:
            if key in self._inflight:
                self._dirty.add(key)
                return
            if key in self._queued and delay == 0.0:
                return
            self._queued.add(key)
        self.queue.put(key, delay)

    def _initial_list(self) -> None:
        self._enqueue_all(self._loop.list_now())

    def _enqueue_all(self, items: list[dict]) -> None:
        for o in items:
            self.enqueue(self._key(o))

    def _on_event(self, typ: str, obj: dict) -> None:
        key = self._key(obj)
        md = obj.get("metadata") or {}
        if typ == "DELETED":
            with self._lock:
                self._gen.pop(key, None)
            return
        gen = md.get("generation")
        if self.generation_aware and typ == "MODIFIED" and gen is not None and self._gen.get(key) == gen:
            return  # status-only change
        self.enqueue(key)

    def _resync_loop(self) -> None:
        while not self._stop.wait(self.resync_s):
            try:
                for o in self.kube.list(self.res):
                    self.enqueue(self._key(o))
            except Exception as e:  # noqa: BLE001
                log.warning("%s resync failed: %s", self.name, e)

    # ------------------------------------------------------------------ workers
    def _work_loop(self) -> None:
        while not self._stop.is_set():
            key = self.queue.get(timeout=0.25)
            if key is None:
                continue
            with self._lock:
                self._queued.discard(key)
                if key in self._inflight:
                    self._dirty.add(key)
                    continue
                self._inflight.add(key)
            try:
                self._reconcile_key(key)
            finally:
                with self._lock:
                    self._inflight.discard(key)
                    again = key in self._dirty
                    self._dirty.discard(key)
                if again:
                    self.enqueue(key)

    def reconcile_now(self, key: tuple) -> UpdateControl | None:
        """Synchronous reconcile of one object (tests / CLI)."""
        return self._reconcile_key(key)

    def _reconcile_key(self, key: tuple) -> UpdateControl | None:
        ns, name = key
        try:
            obj = self.kube.get(self.res, name, ns or None)
        except ApiError as e:
            log.warning("%s get %s failed: %s", self.name, key, e)
            self.enqueue(key, self.retry_initial_s)
            return None
        if obj is None:
            return None
        try:
            uc = self.reconcile_fn(obj)
            self.reconciles += 1
            if uc is not None and uc.status is not None:
                self.kube.patch_status(self.res, name, ns or None, uc.status)
            with self._lock:
                self._attempts.pop(key, None)
                gen = (obj.get("metadata") or {}).get("generation")
                if gen is not None:
                    self._gen[key] = gen
            if uc is not None and uc.reschedule_after is not None and not self._stop.is_set():
                self.queue.put(key, uc.reschedule_after)
            return uc
        except Exception as e:  # noqa: BLE001
            self.errors += 1
            with self._lock:
                n = self._attempts.get(key, 0) + 1
                self._attempts[key] = n
            if n < self.max_attempts:
                delay = self.retry_initial_s * (self.retry_multiplier ** (n - 1))
                log.warning("%s reconcile %s failed (%s), retry %d in %.1fs", self.name, key, e, n, delay)
                self.queue.put(key, delay)
            else:
                log.error("%s reconcile %s failed permanently: %s", self.name, key, e)
            return None
