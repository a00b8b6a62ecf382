"""Result sinks: pod annotations and the Podmortem status (recentFailures ring).

Mirrors J/service/AnalysisStorageService.java:
* annotations ``podmortem.io/{analysis,severity,analyzed-at,monitor}`` on the pod
  (:42-46), full AI text or a pattern-only one-line summary (:145-155);
* ``status.recentFailures`` — newest first, capped at 10 (:48, :329-333), each
  entry {podName, podNamespace, failureTime, analysisStatus="Completed",
  explanation} with a multi-line pattern-only fallback (:295-326);
* every write is GET-latest -> modify -> PATCH with the fresh resourceVersion,
  retried on 409 up to 5 times with 100 ms doubling backoff (:75-76, :179-187);
  403 on the pod gives up immediately (:188-193).

Race fix: all status writes for one Podmortem go through
one ``StatusWriter`` lock, and the phase/message update is a merge patch of
just those two fields on a fresh object, so it can never clobber
``recentFailures`` (the reference patches the whole status from a stale list).

Group commit: a burst of failures for one monitor (hundreds of analyses
finishing in the same decode window) would otherwise be hundreds of serialized
GET+PATCH round trips on one object. Writers enqueue; whichever thread finds
no flush in progress becomes the flusher and commits everything queued in ONE
GET -> prepend-all -> PATCH (retried on 409 exactly as before), looping until
the queue is empty; the others wait for the commit that carried their entry.
The resulting ring is identical to one-at-a-time prepends in completion order.
Phase/message updates coalesce the same way: each overwrites the previous, so
only the latest queued one is written.
"""
from __future__ import annotations

import logging
import threading
import time
from collections import defaultdict
from concurrent.futures import Executor

from operator_amd.api.models import AnalysisResult
from operator_amd.kube.resources import PODMORTEMS, PODS, ApiError
from operator_amd.utils.javafmt import fmt2, is_blank, jstr
from operator_amd.utils.timefmt import instant_str

log = logging.getLogger(__name__)

ANNOTATION_PREFIX = "podmortem.io/"
ANALYSIS_ANNOTATION = ANNOTATION_PREFIX + "analysis"
SEVERITY_ANNOTATION = ANNOTATION_PREFIX + "severity"
TIMESTAMP_ANNOTATION = ANNOTATION_PREFIX + "analyzed-at"
MONITOR_ANNOTATION = ANNOTATION_PREFIX + "monitor"
MAX_RECENT_FAILURES = 10


def pattern_annotation(result: AnalysisResult) -> str:
    s = result.summary
    return "Pattern Analysis: Severity=%s, SignificantEvents=%d, TotalMatches=%d" % (
        jstr(s.highest_severity) if s is not None else "UNKNOWN",
        s.significant_events if s is not None else 0,
        len(result.events) if result.events is not None else 0)


def pattern_explanation(result: AnalysisResult) -> str:
    out = ["Pattern Analysis Results:\n", "========================\n"]
    s = result.summary
    if s is not None:
        out.append(f"Highest Severity: {jstr(s.highest_severity)}\n")
        out.append(f"Significant Events: {s.significant_events}\n")
    if result.events:
        out.append("\nTop Matches:\n")
        for e in result.events[:5]:
            if e.matched_pattern is not None:
                out.append(f"- {jstr(e.matched_pattern.name)} (Severity: {jstr(e.matched_pattern.severity)}, "
                           f"Score: {fmt2(e.score)})\n")
    return "".join(out)


class Retrier:
    """409 retry schedule: ``max_retries`` retries, delays doubling from ``initial_delay_s``
    (AnalysisStorageService.java:75-76: 5 x 100 ms). With several operator shards writing
    one Podmortem's status, every shard's retry would land on the same doubling ticks
    and collide again: ``jitter`` spreads each delay uniformly over ±jitter of its value,
    and delays stop doubling at ``max_delay_s``."""

    def __init__(self, max_retries: int = 5, initial_delay_s: float = 0.1, sleep=time.sleep, jitter: float = 0.0,
                 max_delay_s: float = 1.6, rng=None):
        self.max_retries, self.initial_delay_s, self.sleep = max_retries, initial_delay_s, sleep
        self.jitter, self.max_delay_s = jitter, max_delay_s
        import random

        self.rng = rng or random.Random()

    def delay(self, nominal: float) -> float:
        return nominal * (1.0 + self.jitter * (2.0 * self.rng.random() - 1.0)) if self.jitter else nominal


class _Commit:
    """Outcome of one queued write, filled in by whichever thread flushed it."""
    __slots__ = ("done", "ok")

    def __init__(self):
        self.done, self.ok = False, False


class _Queue:
    """Per-Podmortem write queue + flusher flag (group commit)."""

    def __init__(self):
        self.cv = threading.Condition()
        self.items: list = []
        self.flushing = False


class StatusWriter:
    """Single writer per Podmortem (per-key lock), with group commit of bursts."""

    def __init__(self, kube, retrier: Retrier | None = None, use_finished_at: bool = False):
        self.kube = kube
        self.retrier = retrier or Retrier()
        self.use_finished_at = use_finished_at
        self._locks: dict[tuple[str, str], threading.Lock] = defaultdict(threading.Lock)
        self._queues: dict[tuple[str, str, str], _Queue] = defaultdict(_Queue)
        self._guard = threading.Lock()
        self.commits = 0   # PATCHes actually issued (observability / tests)

    def _key(self, monitor: dict) -> tuple[str, str]:
        md = monitor.get("metadata") or {}
        return (md.get("namespace") or "", md.get("name") or "")

    def _lock(self, monitor: dict) -> threading.Lock:
        with self._guard:
            return self._locks[self._key(monitor)]

    def _group_commit(self, kind: str, monitor: dict, item, flush) -> bool:
        """Queue ``item``; flush the queue (``flush(items) -> bool``) unless another
        thread is already flushing it, and return the outcome of the commit that
        carried ``item``."""
        with self._guard:
            q = self._queues[(kind, *self._key(monitor))]
        mine = _Commit()
        with q.cv:
            q.items.append((item, mine))
            if q.flushing:
                while not mine.done:
                    q.cv.wait()
                return mine.ok
            q.flushing = True
        while True:
            with q.cv:
                batch, q.items = q.items, []
                if not batch:
                    q.flushing = False
                    q.cv.notify_all()
                    return mine.ok
            try:
                with self._lock(monitor):
                    ok = bool(flush([it for it, _ in batch]))
            except Exception as e:  # noqa: BLE001 - never leave waiters hanging
                log.warning("status commit failed: %s", e)
                ok = False
            self.commits += 1
            with q.cv:
                for _, c in batch:
                    c.ok, c.done = ok, True
                q.cv.notify_all()

    def _with_retry(self, what: str, fn) -> bool:
        delay = self.retrier.initial_delay_s
        for attempt in range(self.retrier.max_retries + 1):
            if attempt:
                self.retrier.sleep(self.retrier.delay(delay))
                delay = min(delay * 2, self.retrier.max_delay_s)
            try:
                return fn()
            except ApiError as e:
                if e.code == 409 and attempt < self.retrier.max_retries:
                    log.debug("conflict on %s, retry %d/%d", what, attempt + 1, self.retrier.max_retries)
                    continue
                if e.code == 403:
                    log.warning("Forbidden to update %s - check RBAC permissions: %s", what, e)
                else:
                    log.warning("Failed to store %s after %d attempts: %s", what, attempt + 1, e)
                return False
            except Exception as e:  # noqa: BLE001
                log.warning("Unexpected error storing %s: %s", what, e)
                return False
        return False

    # ------------------------------------------------------------------ phase/message
    def set_phase(self, monitor: dict, phase: str, message: str, observed_generation: bool = False) -> bool:
        md = monitor.get("metadata") or {}

        def flush(items):
            # each update overwrites the previous one: only the latest queued is written
            ph, msg, og = items[-1]
            patch = {"phase": ph, "message": msg, "lastUpdate": instant_str()}
            if any(x[2] for x in items) and md.get("generation") is not None:
                patch["observedGeneration"] = md.get("generation")

            def do():
                self.kube.patch_status(PODMORTEMS, md["name"], md.get("namespace"), patch)
                return True

            return self._with_retry(f"Podmortem {md.get('name')} status", do)

        return self._group_commit("phase", monitor, (phase, message, observed_generation), flush)

    def update_pod_failure(self, monitor: dict, pod: dict, message: str) -> bool:
        """PodFailureWatcher.updatePodFailureStatusAsync (:452-502): phase Processing,
        message "<msg> (Pod: <name>)"."""
        return self.set_phase(monitor, "Processing", f"{message} (Pod: {(pod.get('metadata') or {}).get('name')})")

    # ------------------------------------------------------------------ recentFailures ring
    def append_failure(self, pod: dict, monitor: dict, result: AnalysisResult, ai_analysis: str | None) -> bool:
        md = monitor.get("metadata") or {}
        pmd = pod.get("metadata") or {}
        when = instant_str()
        if self.use_finished_at:
            for cs in (pod.get("status") or {}).get("containerStatuses") or []:
                t = ((cs or {}).get("state") or {}).get("terminated") or {}
                if t.get("finishedAt"):
                    when = t["finishedAt"]
                    break
        entry = {"podName": pmd.get("name"), "podNamespace": pmd.get("namespace"), "failureTime": when,
                 "analysisStatus": "Completed",
                 "explanation": ai_analysis if not is_blank(ai_analysis) else pattern_explanation(result)}

        def flush(entries):
            def do():
                latest = self.kube.get(PODMORTEMS, md["name"], md.get("namespace"))
                if latest is None:
                    log.warning("Podmortem not found: %s", md.get("name"))
                    return False
                recent = list((latest.get("status") or {}).get("recentFailures") or [])
                # newest first: the same ring as prepending each entry in completion order
                recent = (entries[::-1] + recent)[:MAX_RECENT_FAILURES]
                self.kube.patch_status(PODMORTEMS, md["name"], md.get("namespace"),
                                       {"recentFailures": recent, "lastUpdate": instant_str()},
                                       resource_version=latest["metadata"]["resourceVersion"])
                return True

            return self._with_retry(f"Podmortem {md.get('name')} status", do)

        return self._group_commit("ring", monitor, entry, flush)


class AnalysisStorage:
    """storeAnalysisResults: annotations + status ring, both on the worker pool."""

    def __init__(self, kube, status: StatusWriter, executor: Executor | None = None, retrier: Retrier | None = None):
        self.kube, self.status, self.executor = kube, status, executor
        self.retrier = retrier or status.retrier

    def store(self, pod: dict, monitor: dict, result: AnalysisResult, ai_analysis: str | None):
        futs = []
        for fn in (self.store_annotations, self.status.append_failure):
            if self.executor is None:
                fn(pod, monitor, result, ai_analysis)
            else:
                futs.append(self.executor.submit(fn, pod, monitor, result, ai_analysis))
        return futs

    def store_annotations(self, pod: dict, monitor: dict, result: AnalysisResult, ai_analysis: str | None) -> bool:
        pmd = pod.get("metadata") or {}
        name, ns = pmd.get("name"), pmd.get("namespace")

        # The reference GETs the latest pod, merges its annotations and PATCHes with that
        # resourceVersion (409 -> retry). A JSON merge patch of just these keys without a
        # resourceVersion is applied atomically by the API server: the other annotations
        # survive, there is nothing to conflict on, and it is one request instead of two
        # (the operator's hot path is ~10 API calls per analysis).
        def do():
            ann = {ANALYSIS_ANNOTATION: ai_analysis if not is_blank(ai_analysis) else pattern_annotation(result)}
            if result.summary is not None and result.summary.highest_severity is not None:
                ann[SEVERITY_ANNOTATION] = result.summary.highest_severity
            ann[TIMESTAMP_ANNOTATION] = instant_str()
            ann[MONITOR_ANNOTATION] = (monitor.get("metadata") or {}).get("name")
            try:
                self.kube.patch(PODS, name, ns, {"metadata": {"annotations": ann}})
            except ApiError as e:
                if e.code == 404:
                    log.warning("Pod not found: %s", name)
                    return False
                raise
            return True

        return self.status._with_retry(f"pod annotations for {name}", do)
