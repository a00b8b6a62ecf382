"""Prometheus metrics (SURVEY.md §5.5 — the reference exposes none).

A private registry per Operator so several operators (tests) can coexist.
"""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

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

    def render(self) -> bytes:
        try:
            import torch

            if torch.cuda.is_available():
                for i in range(torch.cuda.device_count()):
                    self.gpu_mem_bytes.labels(device=str(i)).set(torch.cuda.memory_allocated(i))
        except Exception:  # noqa: BLE001
            pass
        return generate_latest(self.registry)
