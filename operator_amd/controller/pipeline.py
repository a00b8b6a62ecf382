"""The per-failure analysis pipeline, shared by the pod watcher and the
Podmortem reconciler (Q3 "fix": one code path, one dedupe).

    emitFailureDetected -> collect(log, core events) -> match -> [AI] -> store -> status -> Events

Branching and strings follow J/service/PodFailureWatcher.java:276-443:
  * collect / match failure      -> status "Processing failed: …" / "Analysis failed: …" + error Event
  * AI disabled / no providerRef -> store(pattern-only) + "Pattern analysis completed (AI disabled)"
  * provider missing             -> store(pattern-only) + "Analysis completed, AI provider not found"
  * AI ok                        -> store(ai text)      + "Analysis completed with AI analysis"
  * AI failed                    -> NO store (Q6, replicated) + "Pattern analysis completed, AI failed: …"
                                    + complete("AI failed: …") + error("AI analysis failed: …")

The remote hops are replaced by in-process services (operator_amd.engine.service):
MatchService.analyze(PodFailureData) and ExplainService.explain(AnalysisResult,
AIProviderConfig). Per-stage timings feed the Prometheus histograms.
"""
from __future__ import annotations

import contextlib
import logging
import threading
import time
from concurrent.futures import Executor, Future

from operator_amd.api.models import AnalysisResult, PodFailureData
from operator_amd.kube.resources import CORE_EVENTS

from operator_amd.utils.tracing import trace_range

from . import ai_client
from .events import EventEmitter
from .storage import AnalysisStorage, StatusWriter

log = logging.getLogger(__name__)


def _msg(e: BaseException) -> str:
    s = str(e)
    return s if s else "null"  # Java getMessage() of a message-less exception is null


class AnalysisPipeline:
    def __init__(self, kube, matcher, explainer, events: EventEmitter, storage: AnalysisStorage,
                 status: StatusWriter, executor: Executor | None = None, metrics=None,
                 log_container: str | None = None, log_previous: bool = False, log_limit_bytes: int | None = None,
                 sink_concurrency: int = 0):
        self.provider_cache = None   # Operator sets its AIProvider informer cache (MonitorCache)
        self.kube, self.matcher, self.explainer = kube, matcher, explainer
        self._sinks = threading.BoundedSemaphore(sink_concurrency) if sink_concurrency > 0 else None
        self.events, self.storage, self.status = events, storage, status
        self.executor, self.metrics = executor, metrics
        self.log_container, self.log_previous, self.log_limit_bytes = log_container, log_previous, log_limit_bytes
        self.completed = 0
        self.failed = 0
        self.listeners: list = []  # callables (monitor, pod, outcome) after each finished analysis

    # ------------------------------------------------------------------ entry points
    def submit(self, monitor: dict, pod: dict) -> Future | None:
        with trace_range("detected"):
            self.events.emit_failure_detected(pod, monitor)
        if self.metrics:
            self.metrics.failures_detected.inc()
        if self.executor is None:
            self.process(monitor, pod)
            return None
        return self.executor.submit(self.process, monitor, pod)

    def collect(self, pod: dict) -> PodFailureData:
        md = pod.get("metadata") or {}
        logs = self.kube.pod_log(md.get("name"), md.get("namespace"), container=self.log_container,
                                 previous=self.log_previous, limit_bytes=self.log_limit_bytes)
        evs = self.kube.list(CORE_EVENTS, md.get("namespace"), field_selector=f"involvedObject.name={md.get('name')}")
        return PodFailureData(pod=pod, logs=logs, events=evs)

    def process(self, monitor: dict, pod: dict) -> str:
        t0 = time.perf_counter()
        try:
            with trace_range("collect"):
                data = self.collect(pod)
        except Exception as e:  # noqa: BLE001
            log.error("Error processing pod failure for pod %s: %s", (pod.get("metadata") or {}).get("name"), e)
            self._fail(monitor, pod, "Processing failed: " + _msg(e))
            return "collect-failed"
        t1 = time.perf_counter()
        try:
            result = self.matcher.analyze(data)
        except Exception as e:  # noqa: BLE001
            log.error("Log analysis failed for pod %s: %s", (pod.get("metadata") or {}).get("name"), e)
            self._fail(monitor, pod, "Analysis failed: " + _msg(e))
            return "match-failed"
        t2 = time.perf_counter()
        if self.metrics:
            self.metrics.stage_seconds.labels(stage="collect").observe(t1 - t0)
            self.metrics.stage_seconds.labels(stage="match").observe(t2 - t1)
        out = self.handle_result(monitor, pod, result)
        if self.metrics:
            self.metrics.stage_seconds.labels(stage="total").observe(time.perf_counter() - t0)
            self.metrics.analyses.labels(outcome=out).inc()
        self.completed += 1
        self._notify(monitor, pod, out)
        return out

    def _sink_slot(self):
        """One of ``sink_concurrency`` result-writing slots (annotations, status ring,
        Events), or no bound."""
        return self._sinks if self._sinks is not None else contextlib.nullcontext()

    def _notify(self, monitor: dict, pod: dict, outcome: str) -> None:
        for fn in self.listeners:
            try:
                fn(monitor, pod, outcome)
            except Exception as e:  # noqa: BLE001
                log.warning("pipeline listener failed: %s", e)

    def _fail(self, monitor: dict, pod: dict, message: str) -> None:
        self.failed += 1
        self.status.update_pod_failure(monitor, pod, message)
        self.events.emit_analysis_error(pod, monitor, message)
        if self.metrics:
            self.metrics.analyses.labels(outcome="error").inc()
        self._notify(monitor, pod, "error")

    # ------------------------------------------------------------------ branching (PodFailureWatcher.java:347-443)
    def handle_result(self, monitor: dict, pod: dict, result: AnalysisResult) -> str:
        if not ai_client.ai_enabled(monitor):
            with self._sink_slot():
                self.storage.store(pod, monitor, result, None)
                self.status.update_pod_failure(monitor, pod, "Pattern analysis completed (AI disabled)")
                self.events.emit_analysis_complete(pod, monitor, result, "AI disabled")
            return "pattern-only"
        try:
            provider = ai_client.get_provider(self.kube, monitor, self.provider_cache)
        except Exception as e:  # noqa: BLE001 (executor-level failure)
            md = pod.get("metadata") or {}
            log.warning("AI provider lookup for pod %s/%s failed: %s", md.get("namespace"), md.get("name"), e)
            with self._sink_slot():
                self.status.update_pod_failure(monitor, pod, "Analysis completed, AI provider lookup failed")
                self.events.emit_analysis_complete(pod, monitor, result, "AI provider lookup failed")
            return "provider-lookup-failed"
        if provider is None:
            with self._sink_slot():
                self.storage.store(pod, monitor, result, None)
                self.status.update_pod_failure(monitor, pod, "Analysis completed, AI provider not found")
                self.events.emit_analysis_complete(pod, monitor, result, "AI provider not found")
            return "provider-not-found"
        t0 = time.perf_counter()
        try:
            cfg = ai_client.to_provider_config(self.kube, provider)
            resp = self.explainer.explain(result, cfg)
            text = resp.explanation
        except Exception as e:  # noqa: BLE001
            m = _msg(e)
            log.error("AI analysis failed for pod %s: %s", (pod.get("metadata") or {}).get("name"), m)
            with self._sink_slot():
                self.status.update_pod_failure(monitor, pod, "Pattern analysis completed, AI failed: " + m)
                self.events.emit_analysis_complete(pod, monitor, result, "AI failed: " + m)
                self.events.emit_analysis_error(pod, monitor, "AI analysis failed: " + m)
            return "ai-failed"
        if self.metrics:
            self.metrics.stage_seconds.labels(stage="explain").observe(time.perf_counter() - t0)
        with self._sink_slot(), trace_range("sinks"):
            self.storage.store(pod, monitor, result, text)
            self.status.update_pod_failure(monitor, pod, "Analysis completed with AI analysis")
            self.events.emit_analysis_complete(pod, monitor, result, text)
        return "ai-complete"
