"""Kubernetes Event emission (events.k8s.io/v1).

Behaviour of the reference's EventService (J/service/EventService.java):
reasons, types, message formats and size caps are identical; every Event goes
to the failed pod and to the Podmortem CR, and to the owning Deployment when
the pod -> ReplicaSet -> Deployment owner chain resolves.

Deliberate fixes: owner resolution runs on the worker pool
instead of the caller's thread and a 403/404 there is swallowed (the
reference's RBAC grants no ``apps`` access: K/operator-rbac.yaml:6-17; our
generated ClusterRole adds get on replicasets/deployments).
"""
from __future__ import annotations

import logging
import uuid
from concurrent.futures import Executor
from typing import Any

from operator_amd.api.models import AnalysisResult
from operator_amd.kube.resources import DEPLOYMENTS, EVENTS, REPLICASETS, ApiError
from operator_amd.utils.javafmt import is_blank, jstr, jtrim
from operator_amd.utils.timefmt import epoch_millis, now

log = logging.getLogger(__name__)

REPORTING_CONTROLLER = "podmortem.operator"          # EventService.java:32
REPORTING_INSTANCE = REPORTING_CONTROLLER + ".instance"
REASON_DETECTED = "PodFailureDetected"
REASON_COMPLETE = "PodmortemAnalysisComplete"
REASON_ERROR = "PodmortemAnalysisError"
MSG_DETECTED = "Pod failure detected and queued for analysis"
DETAIL_BUDGET = 850                                   # EventService.java:87
ERROR_CAP = 900                                       # EventService.java:117


def truncate(text: str | None, max_len: int) -> str | None:
    """EventService.truncate (EventService.java:278-305), including the path that keeps
    both the "Root Cause" and "Fix" sections. Where the Java code would throw
    (a "Fix" before "Root Cause" with no "Evidence") we fall back to plain truncation."""
    if text is None:
        return None
    if len(text) <= max_len:
        return text
    if "Root Cause" in text and "Fix" in text:
        rc = text.index("Root Cause")
        fx = text.index("Fix")
        rce = text.find("Evidence", rc)
        if rce < 0:
            rce = fx
        end1 = min(rce, rc + max_len // 2)
        if end1 >= rc:
            root = text[rc:end1]
            fix = text[fx:min(len(text), fx + max_len // 2)]
            combined = jtrim(root) + " ... " + jtrim(fix)
            if len(combined) > max_len:
                return combined[: max(0, max_len - 3)] + "..."
            return combined
    return text[: max(0, max_len - 3)] + "..."


def complete_message(result: AnalysisResult, detail: str | None) -> str:
    s = result.summary
    base = f"Analysis complete. Severity={jstr(s.highest_severity if s else None)}, " \
           f"Events={s.significant_events if s else 0}"
    if not is_blank(detail):
        return base + " | " + truncate(detail, DETAIL_BUDGET - len(base))
    return base


def _ref(obj: dict) -> dict:
    md = obj.get("metadata") or {}
    return {"apiVersion": obj.get("apiVersion"), "kind": obj.get("kind"), "name": md.get("name"),
            "namespace": md.get("namespace"), "uid": md.get("uid")}


def micro_time() -> str:
    t = now()
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond:06d}Z"


class EventEmitter:
    def __init__(self, kube, executor: Executor | None = None, metrics=None):
        self.kube = kube
        self.executor = executor
        self.metrics = metrics

    # ------------------------------------------------------------------ public API (EventService.java:45-128)
    def emit_failure_detected(self, pod: dict, monitor: dict) -> None:
        self._emit_all(pod, monitor, REASON_DETECTED, MSG_DETECTED, "Warning")

    def emit_analysis_complete(self, pod: dict, monitor: dict, result: AnalysisResult, detail: str | None) -> None:
        self._emit_all(pod, monitor, REASON_COMPLETE, complete_message(result, detail), "Normal")

    def emit_analysis_error(self, pod: dict, monitor: dict, error_message: str | None) -> None:
        self._emit_all(pod, monitor, REASON_ERROR, truncate(error_message, ERROR_CAP), "Warning")

    # ------------------------------------------------------------------ internals
    def _submit(self, fn, *a) -> None:
        if self.executor is None:
            fn(*a)
        else:
            self.executor.submit(fn, *a)

    def _emit_all(self, pod: dict, monitor: dict, reason: str, message: str | None, typ: str) -> None:
        pod_ns = (pod.get("metadata") or {}).get("namespace")
        self._submit(self._emit, pod, pod_ns, reason, message, typ)
        self._submit(self._emit, monitor, (monitor.get("metadata") or {}).get("namespace"), reason, message, typ)
        owners = (pod.get("metadata") or {}).get("ownerReferences") or []
        if any((o or {}).get("kind") == "ReplicaSet" for o in owners):   # else no Deployment to find
            self._submit(self._emit_to_deployment, pod, pod_ns, reason, message, typ)

    def _emit_to_deployment(self, pod: dict, ns: str, reason: str, message: str, typ: str) -> None:
        dep = self.find_owning_deployment(pod)
        if dep is not None:
            self._emit(dep, ns, reason, message, typ)

    def find_owning_deployment(self, pod: dict) -> dict | None:
        """pod -> ReplicaSet -> Deployment via ownerReferences (EventService.java:224-256)."""
        md = pod.get("metadata") or {}
        owners = md.get("ownerReferences")
        if not owners:
            return None
        rs_ref = next((o for o in owners if o.get("kind") == "ReplicaSet"), None)
        if rs_ref is None:
            return None
        try:
            rs = self.kube.get(REPLICASETS, rs_ref.get("name"), md.get("namespace"))
            if rs is None or not rs.get("metadata"):
                return None
            dep_ref = next((o for o in (rs["metadata"].get("ownerReferences") or []) if o.get("kind") == "Deployment"),
                           None)
            if dep_ref is None:
                return None
            return self.kube.get(DEPLOYMENTS, dep_ref.get("name"), md.get("namespace"))
        except ApiError as e:
            log.debug("owner lookup for %s failed: %s", md.get("name"), e)
            return None

    def build_event(self, target: dict, namespace: str, reason: str, message: str | None, typ: str) -> dict[str, Any]:
        name = (target.get("metadata") or {}).get("name")
        return {
            "apiVersion": "events.k8s.io/v1", "kind": "Event",
            "metadata": {"name": f"{name}.{str(uuid.uuid4())[:8]}.{epoch_millis()}", "namespace": namespace},
            "reason": reason, "type": typ, "action": "Report", "note": message,
            "reportingController": REPORTING_CONTROLLER, "reportingInstance": REPORTING_INSTANCE,
            "eventTime": micro_time(), "regarding": _ref(target),
        }

    def _emit(self, target: dict, namespace: str, reason: str, message: str | None, typ: str) -> None:
        try:
            self.kube.create(EVENTS, self.build_event(target, namespace, reason, message, typ), namespace)
            if self.metrics:
                self.metrics.events_emitted.labels(reason=reason).inc()
        except Exception as e:  # EventService.java:192-195: failures are logged, never raised
            log.debug("Failed to emit event '%s': %s", reason, e)
