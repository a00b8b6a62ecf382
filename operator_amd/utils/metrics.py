"""Prometheus metrics (SURVEY.md §5.5 — the reference exposes none): analyses/s,
stage latency histograms, scan GB/s, tokens/s, per-GPU HBM, collective (RCCL /
one-shot all-reduce) calls, bytes and time.

A private registry per Operator so several operators (tests) can coexist.
"""
from __future__ import annotations

import threading
import time

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest


class _Rate:
    """Rate of a monotonically increasing count over a sliding window (host clock)."""

    def __init__(self, window_s: float = 10.0):
        self.window_s = window_s
        self._pts: list[tuple[float, float]] = []
        self._lock = threading.Lock()

    def add(self, total: float) -> float:
        now = time.monotonic()
        with self._lock:
            self._pts.append((now, float(total)))
            while len(self._pts) > 2 and now - self._pts[1][0] > self.window_s:
                self._pts.pop(0)
            (t0, v0), (t1, v1) = self._pts[0], self._pts[-1]
        return (v1 - v0) / (t1 - t0) if t1 > t0 else 0.0

_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 180)


class Metrics:
    def __init__(self):
        r = self.registry = CollectorRegistry()
        self.failures_detected = Counter("podmortem_failures_detected_total", "Pod failures queued for analysis",
                                         registry=r)
        self.analyses = Counter("podmortem_analyses_total", "Completed analyses by outcome", ["outcome"], registry=r)
        self.stage_seconds = Histogram("podmortem_stage_seconds", "Pipeline stage latency", ["stage"],
                                       buckets=_BUCKETS, registry=r)
        self.events_emitted = Counter("podmortem_events_emitted_total", "Kubernetes Events created", ["reason"],
                                      registry=r)
        self.scan_bytes = Counter("podmortem_scan_bytes_total", "Log bytes scanned", registry=r)
        self.scan_batches = Counter("podmortem_scan_batches_total", "GPU scan batches", registry=r)
        self.tokens_generated = Counter("podmortem_tokens_generated_total", "Explanation tokens generated",
                                        registry=r)
        self.explain_seconds = Histogram("podmortem_explain_seconds", "Explanation latency", buckets=_BUCKETS,
                                         registry=r)
        self.gpu_mem_bytes = Gauge("podmortem_gpu_memory_allocated_bytes", "GPU memory allocated", ["device"],
                                   registry=r)
        self.kv_pages_free = Gauge("podmortem_kv_pages_free", "Free KV-cache pages", registry=r)
        self.scan_seconds = Histogram("podmortem_scan_batch_seconds", "Match (scan + verify + score) batch latency",
                                      buckets=_BUCKETS, registry=r)
        self.scan_gbps = Gauge("podmortem_scan_gigabytes_per_second",
                               "Log bytes analysed per second by the last match batch", registry=r)
        self.tokens_per_s = Gauge("podmortem_tokens_per_second", "Explanation tokens generated per second "
                                  "(10 s window)", registry=r)
        self.analyses_per_s = Gauge("podmortem_analyses_per_second", "Completed analyses per second (10 s window)",
                                    registry=r)
        self.gpu_mem_reserved = Gauge("podmortem_gpu_memory_reserved_bytes", "GPU memory held by the caching "
                                      "allocator", ["device"], registry=r)
        self.gpu_mem_total = Gauge("podmortem_gpu_memory_total_bytes", "GPU HBM capacity", ["device"], registry=r)
        self.gpu_mem_free = Gauge("podmortem_gpu_memory_free_bytes", "GPU HBM free (device view)", ["device"],
                                  registry=r)
        self.collective_calls = Gauge("podmortem_collective_calls_total", "Collectives issued by this process",
                                      ["op", "impl"], registry=r)
        self.collective_bytes = Gauge("podmortem_collective_bytes_total", "Bytes reduced / gathered by collectives",
                                      ["op", "impl"], registry=r)
        self.collective_seconds = Gauge("podmortem_collective_seconds_total",
                                        "Host-observed time in collectives outside captured graphs (RCCL / gloo "
                                        "calls; captured one-shot all-reduces run inside the decode graph)",
                                        ["op", "impl"], registry=r)
        self._tok_rate, self._ana_rate = _Rate(), _Rate()

    def observe_scan(self, nbytes: int, seconds: float) -> None:
        self.scan_batches.inc()
        self.scan_bytes.inc(nbytes)
        self.scan_seconds.observe(seconds)
        if seconds > 0:
            self.scan_gbps.set(nbytes / seconds / 1e9)

    def _total(self, counter) -> float:
        return sum(s.value for m in counter.collect() for s in m.samples if s.name.endswith("_total"))

    def render(self) -> bytes:
        self.tokens_per_s.set(self._tok_rate.add(self._total(self.tokens_generated)))
        self.analyses_per_s.set(self._ana_rate.add(self._total(self.analyses)))
        from operator_amd.parallel.comm import COLLECTIVES

        for (op, impl), st in COLLECTIVES.snapshot().items():
            self.collective_calls.labels(op=op, impl=impl).set(st[0])
            self.collective_bytes.labels(op=op, impl=impl).set(st[1])
            self.collective_seconds.labels(op=op, impl=impl).set(st[2])
        try:
            import torch

            if torch.cuda.is_available():
                for i in range(torch.cuda.device_count()):
                    d = str(i)
                    self.gpu_mem_bytes.labels(device=d).set(torch.cuda.memory_allocated(i))
                    self.gpu_mem_reserved.labels(device=d).set(torch.cuda.memory_reserved(i))
                    free, total = torch.cuda.mem_get_info(i)
                    self.gpu_mem_free.labels(device=d).set(free)
                    self.gpu_mem_total.labels(device=d).set(total)
        except Exception:  # noqa: BLE001
            pass
        return generate_latest(self.registry)
