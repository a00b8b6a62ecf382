"""Real-time pod failure watcher (J/service/PodFailureWatcher.java, the
reference's hot path).

* one watch on all namespaces, or one per namespace listed in
  ``podmortem.watch.namespaces`` (comma separated, trimmed, empties dropped:
  :52-53, :68-79, :89-100);
* only MODIFIED events are considered (Q1, replicated: avoids re-analysing
  every old failure when the operator restarts);
* a failed pod (any container terminated with exit != 0) is matched against
  every Podmortem (cached by an informer instead of a LIST per event) and
  de-duplicated on ns/name -> first terminated finishedAt (:169-200);
* each (pod, Podmortem) pair goes to the shared AnalysisPipeline on the
  worker pool, so the watch thread never blocks on apiserver or GPU work;
* when a watch closes with an error it is restarted after ``restart_delay_s``
  (5 s, :562-583) — resuming from the last resourceVersion seen instead of
  losing the events of the gap (fix), with backoff growth; a stream the
  apiserver ends on its own is reopened at once, and an expired (410)
  resourceVersion triggers a relist whose failed pods go through the same
  dedupe (kube/informer.WatchLoop).
"""
from __future__ import annotations

import logging
import threading

from operator_amd.kube.informer import WatchLoop
from operator_amd.kube.resources import PODMORTEMS, PODS, ApiError, WatchClosed

from .failures import FailureDeduper, failure_time, has_pod_failed, in_shard, matches_monitor
from .pipeline import AnalysisPipeline

log = logging.getLogger(__name__)


def parse_namespaces(value: str | None) -> list[str]:
    if not value or not value.strip():
        return []
    return sorted({s.strip() for s in value.split(",") if s.strip()})


class MonitorCache:
    """Informer-style cache of Podmortem objects (list + watch, kube/informer.WatchLoop);
    with ``res`` = AIPROVIDERS the same cache serves the analysis pipeline's AIProvider
    lookups (one API GET per analysis saved; a miss still falls back to a GET)."""

    def __init__(self, kube, restart_delay_s: float = 1.0, res=PODMORTEMS):
        self.kube = kube
        self.res = res
        self._objs: dict[tuple, dict] = {}
        self._lock = threading.Lock()
        self._loop = WatchLoop(kube, res, None, self._on_event, relist=self._replace_all,
                               name=f"{res.plural}-cache", restart_delay_s=restart_delay_s, max_delay_s=30.0)
        self._thread: threading.Thread | None = None
        self.synced = threading.Event()

    @staticmethod
    def _k(o: dict) -> tuple:
        return ((o["metadata"].get("namespace") or ""), o["metadata"]["name"])

    def start(self) -> None:
        self._replace_all(self._loop.list_now())
        self._thread = threading.Thread(target=self._loop.run, name=f"{self.res.plural}-cache", daemon=True)
        self._thread.start()

    def _replace_all(self, items: list[dict]) -> None:
        with self._lock:
            self._objs = {self._k(o): o for o in items}
        self.synced.set()

    def _on_event(self, typ: str, o: dict) -> None:
        with self._lock:
            if typ == "DELETED":
                self._objs.pop(self._k(o), None)
            else:
                self._objs[self._k(o)] = o

    def stop(self) -> None:
        self._loop.stop()

    def list(self) -> list[dict]:
        with self._lock:
            return list(self._objs.values())

    def get(self, name: str, namespace: str | None) -> dict | None:
        with self._lock:
            return self._objs.get((namespace or "", name))


class PodFailureWatcher:
    def __init__(self, kube, pipeline: AnalysisPipeline, deduper: FailureDeduper, namespaces: str | None = None,
                 monitors: MonitorCache | None = None, restart_delay_s: float = 5.0, include_last_state: bool = False,
                 include_init: bool = False, shard: tuple[int, int] = (0, 1)):
        self.kube, self.pipeline, self.deduper = kube, pipeline, deduper
        self.shard_index, self.shard_count = shard
        self.allowed = parse_namespaces(namespaces)
        self.monitors = monitors
        self.restart_delay_s = restart_delay_s
        self.include_last_state, self.include_init = include_last_state, include_init
        self._loops: list[WatchLoop] = []
        self._threads: list[threading.Thread] = []
        self._stop = threading.Event()
        self.events_seen = 0

    @property
    def restarts(self) -> int:
        return sum(lp.restarts for lp in self._loops)

    @property
    def reconnects(self) -> int:
        return sum(lp.reconnects for lp in self._loops)

    @property
    def relists(self) -> int:
        return sum(lp.relists for lp in self._loops)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self._stop.clear()
        targets: list[str | None] = list(self.allowed) if self.allowed else [None]
        self._loops = []
        for ns in targets:
            lp = WatchLoop(self.kube, PODS, ns, self.on_event, relist=self._catch_up,
                           name=f"pod-watch-{ns or 'all'}", restart_delay_s=self.restart_delay_s, stop=self._stop)
            self._loops.append(lp)
            # open the first watch here, not in the thread: once start() returns, no pod update is missed
            # (a new leader's reconcile pass covers failures that happened before it)
            first = None
            try:
                first = lp.open()
            except (ApiError, WatchClosed, OSError) as e:
                log.error("Pod watcher could not start: %s", e)
            t = threading.Thread(target=lp.run, args=(first,), name=f"pod-watch-{ns or 'all'}", daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        for lp in self._loops:
            lp.stop()

    def _catch_up(self, pods: list[dict]) -> None:
        """After 410 Gone the events of the gap are lost: the relisted pods stand in for
        them. Failed ones go through the same dedupe, so a failure already analysed is
        not analysed again and one that happened during the gap is."""
        for pod in pods:
            self.on_event("MODIFIED", pod)

    # ------------------------------------------------------------------ handling
    def on_event(self, action: str, pod: dict) -> None:
        self.events_seen += 1
        try:
            if action != "MODIFIED":
                return
            ns = (pod.get("metadata") or {}).get("namespace")
            if self.allowed and ns not in self.allowed:
                return
            if not in_shard(pod, self.shard_index, self.shard_count):   # another operator shard's pod
                return
            if has_pod_failed(pod, self.include_last_state, self.include_init):
                self.handle_failure(pod)
        except Exception as e:  # noqa: BLE001 (PodFailureWatcher.java:117-123)
            log.error("Error processing pod event for %s: %s", (pod.get("metadata") or {}).get("name"), e)

    def matching_monitors(self, pod: dict) -> list[dict]:
        items = self.monitors.list() if self.monitors is not None else self.kube.list(PODMORTEMS)
        return [m for m in items if matches_monitor(pod, m)]

    def handle_failure(self, pod: dict) -> list:
        key = FailureDeduper.key(pod)
        monitors = self.matching_monitors(pod)
        if not monitors:
            log.debug("Ignoring failure for unmonitored pod: %s", key)
            return []
        ft = failure_time(pod, self.include_last_state)
        if not self.deduper.check_and_mark(pod, ft):
            log.debug("Already processed failure for pod: %s", key)
            return []
        log.info("Pod failure detected: %s (%d monitors)", key, len(monitors))
        return [self.pipeline.submit(m, pod) for m in monitors]
