"""Podmortem reconciler (J/reconcile/PodmortemReconciler.java:72-97).

On every reconcile: list pods in ANY namespace that match spec.podSelector
(full LabelSelector), route each failed one through the SAME dedupe +
pipeline as the watcher (SURVEY.md Q3 fix: the reference re-analysed every
failed pod on every reconcile and never stored results), then set status
phase Ready / "Monitoring pods for failures" (:88), or Error /
"Failed to reconcile: <msg>" (:92-96). ``observedGeneration`` is now set.
The null-unsafe ``hasPodFailed`` of the reference (Q13) is replaced by the
watcher's null-safe one. An empty selector selects nothing (Q2).
"""
from __future__ import annotations

import logging

from operator_amd.kube.resources import PODS, selector_is_empty

from .failures import FailureDeduper, failure_time, has_pod_failed, in_shard
from .pipeline import AnalysisPipeline
from .runtime import UpdateControl

log = logging.getLogger(__name__)


class PodmortemReconciler:
    def __init__(self, kube, pipeline: AnalysisPipeline, deduper: FailureDeduper, include_last_state: bool = False,
                 shard: tuple[int, int] = (0, 1)):
        self.kube, self.pipeline, self.deduper = kube, pipeline, deduper
        self.include_last_state = include_last_state
        self.shard_index, self.shard_count = shard

    def find_matching_pods(self, monitor: dict) -> list[dict]:
        sel = (monitor.get("spec") or {}).get("podSelector")
        if selector_is_empty(sel):
            return []
        return self.kube.list(PODS, None, label_selector=sel)

    def reconcile(self, monitor: dict) -> UpdateControl:
        name = (monitor.get("metadata") or {}).get("name")
        log.info("Reconciling Podmortem: %s", name)
        try:
            for pod in self.find_matching_pods(monitor):
                if not in_shard(pod, self.shard_index, self.shard_count):
                    continue
                if has_pod_failed(pod, self.include_last_state):
                    if self.deduper.check_and_mark(pod, failure_time(pod, self.include_last_state)):
                        self.pipeline.submit(monitor, pod)
            phase, msg = "Ready", "Monitoring pods for failures"
        except Exception as e:  # noqa: BLE001
            log.error("Error reconciling Podmortem: %s: %s", name, e)
            phase, msg = "Error", f"Failed to reconcile: {e}"
        # through the single status writer (same lock as the pipeline's writes: R1/R3)
        self.pipeline.status.set_phase(monitor, phase, msg, observed_generation=True)
        return UpdateControl.no_update()
