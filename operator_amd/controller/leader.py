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
        self._pending: threading.Event | None = None

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
    def _bounded_attempt(self, timeout: float) -> bool:
        """One acquire/renew, but never waited on past ``timeout``: a get/replace that
        stalls (a slow apiserver; the client's own HTTP timeout is 30 s, longer than the
        lease) must not keep this replica leading after a standby may have taken the
        lease over. A stalled attempt is abandoned (its result ignored) and no second
        one is started while it is still blocked."""
        if self._pending is not None and not self._pending.is_set():
            self._pending.wait(max(0.0, timeout))
            if not self._pending.is_set():
                return False
        done, box = threading.Event(), [False]

        def attempt():
            try:
                box[0] = self.try_acquire_or_renew()
            except Exception as e:  # noqa: BLE001
                log.warning("lease attempt failed: %s", e)
            finally:
                done.set()

        self._pending = done
        threading.Thread(target=attempt, name="lease-attempt", daemon=True).start()
        if not done.wait(max(0.0, timeout)):
            log.warning("%s: lease request still blocked after %.1fs; treating it as failed", self.identity,
                        timeout)
            return False
        return box[0]

    def _callback(self, fn, what: str) -> bool:
        if fn is None:
            return True
        try:
            fn()
            return True
        except Exception as e:  # noqa: BLE001 - the elector thread must survive its callbacks
            log.exception("%s: %s callback failed: %s", self.identity, what, e)
            return False

    def _step_down(self, release: bool) -> None:
        self.leading = False
        if release:
            self.release()
        self._callback(self.on_stopped_leading, "on_stopped_leading")

    def run(self) -> None:
        while not self._stop.is_set():
            start = time.monotonic()
            budget = (self.renew_deadline_s - (start - self._last_renew)) if self.leading else self.retry_period_s
            ok = self._bounded_attempt(budget)
            now = time.monotonic()
            if ok:
                self._last_renew = start   # the lease counts from the renewTime stamped at the attempt's start
                if not self.leading:
                    self.leading = True
                    self.transitions += 1
                    log.info("%s: became leader", self.identity)
                    if not self._callback(self.on_started_leading, "on_started_leading"):
                        # could not start leading (e.g. the first list failed): hand the lease
                        # back at once and compete again after a retry period
                        self._step_down(release=True)
            elif self.leading and now - self._last_renew >= self.renew_deadline_s:
                log.warning("%s: lost leadership (no renewal for %.1fs)", self.identity, now - self._last_renew)
                self._step_down(release=False)
            self._stop.wait(max(0.0, self.retry_period_s - (time.monotonic() - start)) if ok else self.retry_period_s)
        if self.leading:
            self._step_down(release=True)

    def start(self) -> "LeaderElector":
        self._t = threading.Thread(target=self.run, name="leader-elector", daemon=True)
        self._t.start()
        return self

    def stop(self, timeout: float = 10.0) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout)
