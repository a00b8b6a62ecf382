"""Operator assembly: the process that replaces the reference's Quarkus app
(SURVEY.md §3.1 "init").

    kube client (HTTPS or FakeKube)
      -> Podmortem cache (informer) + PodFailureWatcher      (hot path)
      -> controllers: Podmortem, PatternLibrary, AIProvider   (reconcile loops)
      -> AnalysisPipeline -> MatchService (GPU scan) / ExplainService (GPU LLM)
      -> sinks: pod annotations, Podmortem status ring, Events
      -> HTTP: /q/health/{live,ready}, /metrics

Patterns: the synced libraries under ``patterns.cache_dir/<PatternLibrary>``
(filtered by each CR's ``enabledLibraries``, Q8) plus the built-in catalog;
recompiled and hot-swapped after every successful PatternLibrary sync.
"""
from __future__ import annotations

import logging
import threading
from pathlib import Path

from operator_amd.config import Settings
from operator_amd.kube.resources import AIPROVIDERS, PATTERNLIBRARIES, PODMORTEMS
from operator_amd.patterns.schema import PatternSet
from operator_amd.patterns.synth import catalog_library
from operator_amd.utils.executors import TrackedExecutor
from operator_amd.utils.metrics import Metrics

from .aiprovider import AIProviderReconciler
from .events import EventEmitter
from .failures import FailureDeduper
from .health import HealthServer, PatternLibraryReadiness
from .patternlibrary import PatternLibraryReconciler
from .pipeline import AnalysisPipeline
from .podmortem import PodmortemReconciler
from .runtime import Controller
from .storage import AnalysisStorage, Retrier, StatusWriter
from .sync import PatternSync
from .watcher import MonitorCache, PodFailureWatcher

log = logging.getLogger(__name__)


def load_patterns(settings: Settings, kube) -> PatternSet:
    ps = catalog_library() if settings.patterns.builtin_catalog else PatternSet([], [])
    root = Path(settings.patterns.cache_dir)
    try:
        libs = kube.list(PATTERNLIBRARIES)
    except Exception as e:  # noqa: BLE001
        log.warning("cannot list PatternLibraries: %s", e)
        libs = []
    for lib in libs:
        name = lib["metadata"]["name"]
        enabled = (lib.get("spec") or {}).get("enabledLibraries") or None
        try:
            ps = ps.merged(PatternSet.load_dir(root / name, enabled))
        except Exception as e:  # noqa: BLE001
            log.error("failed to load patterns of library %s: %s", name, e)
    return ps


class Operator:
    @staticmethod
    def pipeline_workers(s: Settings) -> int:
        """operator.workers, or (0 = auto) enough threads for two engine batches per GPU in
        flight: the one being explained and the previous one whose results are being
        stored (a pipeline task holds its thread from detection to its last Event)."""
        if s.operator.workers > 0:
            return s.operator.workers
        return 2 * s.engine.max_batch * max(1, s.engine.gpus) + 16

    def __init__(self, kube, settings: Settings, match_service=None, explain_service=None, metrics: Metrics | None = None,
                 match_engine_factory=None):
        s = self.settings = settings
        self.kube = kube
        self.metrics = metrics or Metrics()
        self.io_pool = TrackedExecutor(s.operator.io_workers, thread_name_prefix="kube-io")
        self.pool = TrackedExecutor(self.pipeline_workers(s), thread_name_prefix="analysis")
        retrier = Retrier(s.storage.max_retries, s.storage.initial_backoff_s)
        # the status ring is the one object every operator shard writes: a larger 409 budget
        # with jittered delays there (pod annotations are per pod: one writer, no change)
        status_retrier = retrier if s.operator.shard_count <= 1 else Retrier(
            max(s.storage.max_retries, s.storage.sharded_max_retries), s.storage.initial_backoff_s,
            jitter=s.storage.sharded_jitter)
        self.status = StatusWriter(kube, status_retrier, s.storage.failure_time_from_pod)
        self.storage = AnalysisStorage(kube, self.status, self.io_pool, retrier)
        self.events = EventEmitter(kube, self.io_pool, self.metrics)
        self.match_engine_factory = match_engine_factory
        self.matcher = match_service
        # providerId routing: on-node engine by default, external OpenAI / Ollama APIs for
        # AIProviders that name them (engine/providers.py)
        from operator_amd.engine.providers import ProviderRouter

        self.explainer = ProviderRouter(explain_service, enabled=s.services.external_providers)
        self.pipeline = AnalysisPipeline(kube, self.matcher, self.explainer, self.events, self.storage, self.status,
                                         self.pool, self.metrics, log_container=s.watch.log_container,
                                         log_previous=s.watch.log_previous, log_limit_bytes=s.watch.log_limit_bytes,
                                         sink_concurrency=s.operator.sink_concurrency)
        self.deduper = FailureDeduper(s.watch.dedupe_max_entries, s.watch.dedupe_ttl_s)
        self.sync = PatternSync(s.patterns.cache_dir)
        self._make_workers()
        self.elector = None
        self._workers_running = False
        self._workers_lock = threading.Lock()
        self.readiness = PatternLibraryReadiness(kube, s.patterns.cache_dir, s.health.grace_s)
        self.health: HealthServer | None = None
        self._reload_lock = threading.Lock()
        self.pattern_count = 0

    def _make_workers(self) -> None:
        """Watcher, informer and reconcilers: what only the leader runs."""
        s, kube = self.settings, self.kube
        self.monitors = MonitorCache(kube)
        self.providers = MonitorCache(kube, res=AIPROVIDERS)   # AIProvider lookups of the analysis pipeline
        self.pipeline.provider_cache = self.providers
        shard = (s.operator.shard_index, s.operator.shard_count)
        if not 0 <= shard[0] < max(1, shard[1]):
            raise ValueError(f"operator.shard_index {shard[0]} outside 0..{shard[1] - 1}")
        self.watcher = PodFailureWatcher(kube, self.pipeline, self.deduper, s.watch.namespaces, self.monitors,
                                         s.watch.restart_delay_s, s.watch.include_last_state,
                                         s.watch.include_init_containers, shard=shard)
        self.pm_reconciler = PodmortemReconciler(kube, self.pipeline, self.deduper, s.watch.include_last_state,
                                                 shard=shard)
        self.pl_reconciler = PatternLibraryReconciler(kube, self.sync, on_synced=lambda lib: self.reload_patterns())
        self.aip_reconciler = AIProviderReconciler(kube, self.explainer, s.engine.model)
        self.controllers = [
            Controller(kube, PODMORTEMS, self.pm_reconciler.reconcile, name="podmortem"),
            Controller(kube, PATTERNLIBRARIES, self.pl_reconciler.reconcile, name="patternlibrary"),
            Controller(kube, AIPROVIDERS, self.aip_reconciler.reconcile, name="aiprovider"),
        ]

    def _start_workers(self) -> None:
        with self._workers_lock:
            if self._workers_running:
                return
            if getattr(self, "_workers_used", False):  # re-elected after a loss: fresh watch state
                self._make_workers()
            self._workers_used = True
            # watch before the controllers' first reconcile pass, so a failure is seen by one or the other
            self.monitors.start()
            self.providers.start()
            self.watcher.start()
            for c in self.controllers:
                c.start()
            self._workers_running = True

    def _stop_workers(self) -> None:
        with self._workers_lock:
            if not self._workers_running:
                return
            self.watcher.stop()
            for c in self.controllers:
                c.stop()
            self.monitors.stop()
            self.providers.stop()
            self._workers_running = False

    @property
    def is_leader(self) -> bool:
        return self._workers_running and (self.elector is None or self.elector.leading)

    # ------------------------------------------------------------------ patterns
    def reload_patterns(self) -> int:
        with self._reload_lock:
            ps = load_patterns(self.settings, self.kube)
            self.pattern_count = len(ps)
            if self.match_engine_factory is not None and hasattr(self.matcher, "swap_engine"):
                self.matcher.swap_engine(self.match_engine_factory(ps))
            log.info("pattern set reloaded: %d patterns from %s", len(ps), ps.libraries)
            return len(ps)

    def _engine_ready(self) -> tuple[str, bool]:
        ok = self.matcher is not None and self.explainer.ready()
        return "analysis-engine", bool(ok)

    # ------------------------------------------------------------------ lifecycle
    def start(self, http: bool | None = None) -> "Operator":
        if self.matcher is None and self.match_engine_factory is not None:
            from operator_amd.engine.service import LocalMatchService

            self.matcher = LocalMatchService(self.match_engine_factory(load_patterns(self.settings, self.kube)),
                                             self.settings.services.match_max_batch,
                                             self.settings.services.match_batch_wait_ms, self.metrics)
            self.pipeline.matcher = self.matcher
        o = self.settings.operator
        if o.leader_election:
            from operator_amd.controller.leader import LeaderElector

            lease = o.lease_name if o.shard_count <= 1 else f"{o.lease_name}-shard{o.shard_index}"
            self.elector = LeaderElector(self.kube, lease, o.lease_namespace,
                                         lease_duration_s=o.lease_duration_s,
                                         renew_deadline_s=o.lease_renew_deadline_s,
                                         retry_period_s=o.lease_retry_period_s,
                                         on_started_leading=self._start_workers,
                                         on_stopped_leading=self._stop_workers).start()
        else:
            self._start_workers()
        if http if http is not None else self.settings.health.enabled:
            self.health = HealthServer(self.settings.health.host, self.settings.health.port,
                                       readiness=[self.readiness, self._engine_ready],
                                       liveness=[lambda: ("liveness", True)], metrics=self.metrics)
            self.health.start()
        log.info("operator started")
        return self

    def stop(self) -> None:
        if self.elector is not None:
            self.elector.stop()
        self._stop_workers()
        if self.health is not None:
            self.health.stop()
        self.pool.shutdown(wait=False, cancel_futures=True)
        self.io_pool.shutdown(wait=False, cancel_futures=True)
        for svc in (self.matcher, self.explainer):
            close = getattr(svc, "close", None)
            if close:
                close()

    def drain(self, timeout: float = 30.0) -> bool:
        """Wait until queued analyses and their kube writes have finished (tests / bench)."""
        import time

        end = time.monotonic() + timeout
        while time.monotonic() < end:
            ok = self.pool.wait_idle(max(0.0, end - time.monotonic()))
            ok = self.io_pool.wait_idle(max(0.0, end - time.monotonic())) and ok
            if ok and self.pool.pending == 0 and self.io_pool.pending == 0:
                return True
        return False
