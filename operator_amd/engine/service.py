"""Service fronts used by the controller pipeline (the two REST hops of the
reference, pulled in-process).

* ``LocalMatchService``  — micro-batching front of a MatchEngine: every
  ``analyze()`` call made within ``max_wait_ms`` of another is scanned in ONE
  GPU batch (the log-parser replacement). Patterns are hot-swappable after a
  PatternLibrary sync.
* ``LocalExplainService`` — ExplainEngine front (the ai-interface replacement).
* ``EchoExplainService`` — deterministic stub (plumbing benchmark, tests).
* ``RemoteLogParser`` / ``RemoteAIInterface`` — optional compatibility shims
  that speak the reference's wire contracts (POST /parse,
  POST /api/v1/analysis/analyze) with its timeouts, for mixed deployments.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
from concurrent.futures import Future

from operator_amd.api.models import (AIProviderConfig, AIResponse, AnalysisRequest, AnalysisResult,
                                     PodFailureData)

log = logging.getLogger(__name__)


def _pod_id(pod: dict) -> tuple[str | None, str | None]:
    md = (pod or {}).get("metadata") or {}
    return md.get("name"), md.get("namespace")


class LocalMatchService:
    def __init__(self, engine, max_batch: int = 1024, max_wait_ms: float = 2.0, metrics=None):
        self.engine = engine
        self.max_batch, self.max_wait_s = max_batch, max_wait_ms / 1e3
        self.metrics = metrics
        self._q: queue.Queue = queue.Queue()
        self._lock = threading.Lock()
        self._stop = False
        self._t = threading.Thread(target=self._loop, name="match-batcher", daemon=True)
        self._t.start()
        self.batches = 0

    def swap_engine(self, engine) -> None:
        with self._lock:
            self.engine = engine

    def close(self) -> None:
        self._stop = True
        self._q.put(None)

    def analyze(self, data: PodFailureData) -> AnalysisResult:
        return self.submit(data).result()

    def submit(self, data: PodFailureData, log_bytes: bytes | None = None) -> Future:
        """``log_bytes``: the pod log already as bytes (the engine pool's shared-memory
        transfer), used instead of ``data.logs``."""
        f: Future = Future()
        self._q.put((data, f, log_bytes))
        return f

    def analyze_many(self, datas: list[PodFailureData]) -> list[AnalysisResult]:
        fs = [self.submit(d) for d in datas]
        return [f.result() for f in fs]

    def _loop(self) -> None:
        import torch

        dev = getattr(self.engine, "device", None)
        if dev is not None and getattr(dev, "type", "") == "cuda":
            torch.cuda.set_device(dev)
        while not self._stop:
            item = self._q.get()
            if item is None:
                break
            batch = [item]
            deadline = time.perf_counter() + self.max_wait_s
            while len(batch) < self.max_batch:
                left = deadline - time.perf_counter()
                if left <= 0:
                    break
                try:
                    nxt = self._q.get(timeout=left)
                except queue.Empty:
                    break
                if nxt is None:
                    self._stop = True
                    break
                batch.append(nxt)
            self._run(batch)

    def _run(self, batch) -> None:
        from operator_amd.utils.tracing import trace_range

        with trace_range(f"match.batch[{len(batch)}]"):
            self._run_batch(batch)

    def _run_batch(self, batch) -> None:
        docs = [raw if raw is not None else (d.logs or "").encode("utf-8", "replace") for d, _, raw in batch]
        pods = [_pod_id(d.pod) for d, _, _ in batch]
        try:
            with self._lock:
                eng = self.engine
            t0 = time.perf_counter()
            res = eng.analyze(docs, pods, lazy=True)
            self.batches += 1
            if self.metrics:
                self.metrics.observe_scan(sum(map(len, docs)), time.perf_counter() - t0)
            for i, (_, f, _) in enumerate(batch):   # each waiter wakes as soon as ITS result is built
                f.set_result(res[i])
        except Exception as e:  # noqa: BLE001
            log.error("match batch of %d failed: %s", len(batch), e)
            for _, f, _ in batch:
                if not f.done():
                    f.set_exception(e)


class StubMatchService:
    """The stub log-parser of BASELINE config 1 (``services.match=stub``): one fixed
    CRITICAL out-of-memory event per pod, no scan — for benchmarking the operator's and
    the engine pool's plumbing on its own."""

    def analyze(self, data: PodFailureData) -> AnalysisResult:
        return self.submit(data).result()

    def submit(self, data: PodFailureData, log_bytes: bytes | None = None) -> Future:
        from operator_amd.api.models import AnalysisEvent, AnalysisSummary, MatchedPattern

        name, ns = _pod_id(data.pod)
        ev = AnalysisEvent(line_number=91, score=0.9, matched_line="java.lang.OutOfMemoryError: Java heap space",
                           matched_pattern=MatchedPattern(id="oom", name="Java heap exhausted", severity="CRITICAL"))
        f: Future = Future()
        f.set_result(AnalysisResult(pod_name=name, pod_namespace=ns, events=[ev],
                                    summary=AnalysisSummary(highest_severity="CRITICAL", significant_events=1,
                                                            total_events=1),
                                    metadata={"bytes": len(log_bytes) if log_bytes is not None
                                              else len((data.logs or "").encode())}))
        return f

    def swap_engine(self, engine) -> None:
        pass

    def close(self) -> None:
        pass


class LocalExplainService:
    def __init__(self, explain_engine, metrics=None):
        self.ee = explain_engine
        self.metrics = metrics

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        t0 = time.perf_counter()
        r = self.ee.explain(result, cfg)
        if self.metrics:
            self.metrics.explain_seconds.observe(time.perf_counter() - t0)
            self.metrics.tokens_generated.inc(r.tokens_generated or 0)
            if r.queue_ms is not None and not r.cached:
                self.metrics.stage_seconds.labels(stage="explain_queue_prefill").observe(r.queue_ms / 1e3)
                self.metrics.stage_seconds.labels(stage="explain_decode").observe((r.decode_ms or 0) / 1e3)
        return r

    def explain_many(self, items):
        return self.ee.explain_many(items)

    def complete(self, prompt=None, messages=None, model: str | None = None, **kw) -> dict:
        """Raw completion (``prompt`` text) or chat (``messages``) on this engine."""
        tok = self.ee.tok
        ids = tok.encode_chat(messages) if messages is not None else tok.encode_text(prompt or "")
        out = self.ee.complete(ids, **kw)
        out["model"] = self.ee.model_id
        if self.metrics:
            self.metrics.tokens_generated.inc(out["completion_tokens"])
        return out

    @property
    def models(self) -> list[str]:
        return [self.ee.model_id]

    def ready(self) -> bool:
        return self.ee.loop.is_alive() and self.ee.loop.error is None


class MultiModelExplainService:
    """Several on-node models behind one explain service (``engine.extra_models``): a
    request goes to the engine serving ``AIProviderConfig.model_id`` (case-insensitive),
    anything else to the default model — the reference forwards ``spec.modelId`` to its
    ai-interface, which picks the model (J/service/AIInterfaceClient.java:76-84)."""

    def __init__(self, services: dict, default: str):
        if default not in services:
            raise ValueError(f"default model {default!r} is not served")
        self.services, self.default = dict(services), default
        self._by_lower = {k.lower(): v for k, v in services.items()}
        self.ee = services[default].ee      # the default model's engine (stats, health)

    @property
    def models(self) -> list[str]:
        return list(self.services)

    def pick(self, cfg: AIProviderConfig):
        return self._by_lower.get((cfg.model_id or "").lower(), self.services[self.default])

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        return self.pick(cfg).explain(result, cfg)

    def explain_many(self, items):
        out = [None] * len(items)
        groups: dict[int, tuple] = {}
        for i, (r, c) in enumerate(items):
            svc = self.pick(c)
            groups.setdefault(id(svc), (svc, []))[1].append(i)
        gl = list(groups.values())
        if len(gl) == 1:
            svc, idx = gl[0]
            return svc.explain_many(items)

        def run(svc, idx):   # one continuous batch per model, all models at once
            try:
                for i, res in zip(idx, svc.explain_many([items[i] for i in idx])):
                    out[i] = res
            except Exception as e:  # noqa: BLE001 - reported per item, like the engines do
                for i in idx:
                    out[i] = e

        ts = [threading.Thread(target=run, args=g, name="explain-group", daemon=True) for g in gl]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        return out

    def complete(self, prompt=None, messages=None, model: str | None = None, **kw) -> dict:
        svc = self._by_lower.get((model or "").lower(), self.services[self.default])
        return svc.complete(prompt=prompt, messages=messages, model=model, **kw)

    def ready(self) -> bool:
        return all(getattr(v, "ready", lambda: True)() for v in self.services.values())

    def close(self) -> None:
        for v in self.services.values():
            v.ee.close()


class EchoExplainService:
    """Deterministic stand-in for the ai-interface (no model): renders a short
    Root Cause / Evidence / Fix text from the pattern result."""

    def __init__(self, fail_with: str | None = None, delay_s: float = 0.0):
        self.fail_with, self.delay_s = fail_with, delay_s
        self.calls = 0

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        self.calls += 1
        if self.delay_s:
            time.sleep(self.delay_s)
        if self.fail_with:
            raise RuntimeError(self.fail_with)
        top = (result.events or [None])[0]
        name = top.matched_pattern.name if top and top.matched_pattern else "unknown failure"
        line = top.matched_line if top else ""
        sev = result.summary.highest_severity if result.summary else None
        text = (f"Root Cause: {name} (severity {sev}).\nEvidence: {line}\n"
                f"Fix: address the {name.lower()} reported by the pod.")
        return AIResponse(explanation=text, provider_id=cfg.provider_id, model_id=cfg.model_id or "echo",
                          tokens_generated=len(text.split()), cached=False)

    def ready(self) -> bool:
        return True


class RemoteLogParser:
    """POST {url}/parse with PodFailureData (J/service/LogParserRestClient.java:37-39)."""

    def __init__(self, url: str, read_timeout_s: float = 30.0, connect_timeout_s: float = 10.0):
        import httpx

        self.url = url.rstrip("/")
        self.client = httpx.Client(timeout=httpx.Timeout(read_timeout_s, connect=connect_timeout_s))

    def analyze(self, data: PodFailureData) -> AnalysisResult:
        r = self.client.post(self.url + "/parse", json=data.to_obj())
        r.raise_for_status()
        return AnalysisResult.model_validate(r.json())


class RemoteAIInterface:
    """POST {url}/api/v1/analysis/analyze with AnalysisRequest (J/service/AIInterfaceRestClient.java:23-39)."""

    def __init__(self, url: str, read_timeout_s: float = 180.0, connect_timeout_s: float = 120.0):
        import httpx

        self.url = url.rstrip("/")
        self.client = httpx.Client(timeout=httpx.Timeout(read_timeout_s, connect=connect_timeout_s))

    def explain(self, result: AnalysisResult, cfg: AIProviderConfig) -> AIResponse:
        req = AnalysisRequest(analysis_result=result, provider_config=cfg)
        r = self.client.post(self.url + "/api/v1/analysis/analyze", json=req.to_obj())
        r.raise_for_status()
        return AIResponse.model_validate(r.json())

    def ready(self) -> bool:
        return True
