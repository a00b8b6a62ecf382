"""Lease-based leader election (coordination.k8s.io/v1).

The reference runs a single replica with no lease (SURVEY.md §5.3 "Elastic
recovery / leader election: none"; K/operator-deployment.yaml:11). Here
several operator replicas may run: only the Lease holder starts the watcher
and the reconcilers, and a standby takes over when the holder stops renewing
(crash, partition) — so pod-failure handling survives the loss of a node.

Protocol (the client-go leaderelection algorithm, re-implemented): read the
Lease; if it is free, expired (renewTime + leaseDurationSeconds < now) or ours,
write it with our identity under the read resourceVersion. The write is an
optimistic compare-and-swap: of two contenders only one update succeeds (409
for the other). The holder renews every ``retry_period_s``; if it cannot renew
within ``renew_deadline_s`` it stops leading before anyone else can take over.
"""
from __future__ import annotations

import logging
import os
import socket
import threading
import time
import uuid
from datetime import datetime, timezone

from operator_amd.kube.resources import LEASES, ApiError

log = logging.getLogger(__name__)


def _now_micro() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse_micro(s: str | None) -> float:
    if not s:
        return 0.0
    for fmt in ("%Y-%m-%dT%H:%M:%S.%fZ", "%Y-%m-%dT%H:%M:%SZ"):
        try:
            return datetime.strptime(s, fmt).replace(tzinfo=timezone.utc).timestamp()
        except ValueError:
            continue
    return 0.0


class LeaderElector:
    def __init__(self, kube, name: str = "podmortem-operator-leader", namespace: str = "podmortem-system",
                 identity: str | None = None, lease_duration_s: float = 15.0, renew_deadline_s: float = 10.0,
                 retry_period_s: float = 2.0, on_started_leading=None, on_stopped_leading=None):
        if not (lease_duration_s > renew_deadline_s > retry_period_s > 0):
            raise ValueError("need lease_duration > renew_deadline > retry_period > 0")
        self.kube, self.name, self.namespace = kube, name, namespace
        self.identity = identity or f"{socket.gethostname()}_{os.getpid()}_{uuid.uuid4().hex[:6]}"
        self.lease_duration_s, self.renew_deadline_s, self.retry_period_s = (
            lease_duration_s, renew_deadline_s, retry_period_s)
        self.on_started_leading, self.on_stopped_leading = on_started_leading, on_stopped_leading
        self.leading = False
        self.transitions = 0
        self._stop = threading.Event()
        self._t: threading.Thread | None = None
        self._last_renew = 0.0

    # ------------------------------------------------------------------ one attempt
    def try_acquire_or_renew(self) -> bool:
        now = time.time()
        spec = {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_duration_s),
                "renewTime": _now_micro()}
        try:
            cur = self.kube.get(LEASES, self.name, self.namespace)
        except ApiError as e:
            log.warning("lease get failed: %s", e)
            return False
        try:
            if cur is None:
                spec.update(acquireTime=spec["renewTime"], leaseTransitions=0)
                self.kube.create(LEASES, {"metadata": {"name": self.name, "namespace": self.namespace},
                                          "spec": spec}, self.namespace)
                return True
            old = cur.get("spec") or {}
            holder = old.get("holderIdentity")
            expired = _parse_micro(old.get("renewTime")) + float(old.get("leaseDurationSeconds") or 0) < now
            if holder and holder != self.identity and not expired:
                return False
            if holder != self.identity:
                spec["acquireTime"] = spec["renewTime"]
                spec["leaseTransitions"] = int(old.get("leaseTransitions") or 0) + 1
            else:
                spec["acquireTime"] = old.get("acquireTime") or spec["renewTime"]
                spec["leaseTransitions"] = int(old.get("leaseTransitions") or 0)
            cur["spec"] = spec
            self.kube.replace(LEASES, cur, self.namespace)  # CAS on metadata.resourceVersion
            return True
        except ApiError as e:
            if e.code not in (409, 404):
                log.warning("lease update failed: %s", e)
            return False

    def release(self) -> None:
        """Give the lease up on clean shutdown so a standby need not wait for expiry."""
        try:
            cur = self.kube.get(LEASES, self.name, self.namespace)
            if cur and (cur.get("spec") or {}).get("holderIdentity") == self.identity:
                cur["spec"]["holderIdentity"] = ""
                cur["spec"]["renewTime"] = None
                self.kube.replace(LEASES, cur, self.namespace)
        except ApiError:
            pass

    # ------------------------------------------------------------------ loop
    def run(self) -> None:
        while not self._stop.is_set():
            ok = self.try_acquire_or_renew()
            now = time.monotonic()
            if ok:
                self._last_renew = now
                if not self.leading:
                    self.leading = True
                    self.transitions += 1
                    log.info("%s: became leader", self.identity)
                    if self.on_started_leading:
                        self.on_started_leading()
            elif self.leading and now - self._last_renew > self.renew_deadline_s:
                self.leading = False
                log.warning("%s: lost leadership (no renewal for %.1fs)", self.identity, now - self._last_renew)
                if self.on_stopped_leading:
                    self.on_stopped_leading()
            self._stop.wait(self.retry_period_s)
        if self.leading:
            self.leading = False
            self.release()
            if self.on_stopped_leading:
                self.on_stopped_leading()

    def start(self) -> "LeaderElector":
        self._t = threading.Thread(target=self.run, name="leader-elector", daemon=True)
        self._t.start()
        return self

    def stop(self, timeout: float = 10.0) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout)
