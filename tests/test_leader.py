"""Lease-based leader election: one of several operator replicas leads (runs the
watcher and reconcilers); a standby takes over when the leader stops renewing,
and a cleanly stopped leader hands the lease over at once."""
import time

from operator_amd.config import load_settings
from operator_amd.controller.leader import LeaderElector
from operator_amd.controller.operator import Operator
from operator_amd.engine.match import MatchEngine
from operator_amd.engine.service import EchoExplainService, LocalMatchService
from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
from operator_amd.kube.resources import LEASES, PODMORTEMS, PODS
from operator_amd.patterns.synth import catalog_library


def wait_for(fn, timeout=20.0):
    end = time.time() + timeout
    while time.time() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.02)
    raise AssertionError("timed out")


def test_elector_cas_and_expiry():
    fk = FakeKube()
    a = LeaderElector(fk, "l", "ns", identity="a", lease_duration_s=1.0, renew_deadline_s=0.6, retry_period_s=0.1)
    b = LeaderElector(fk, "l", "ns", identity="b", lease_duration_s=1.0, renew_deadline_s=0.6, retry_period_s=0.1)
    assert a.try_acquire_or_renew() and not b.try_acquire_or_renew()
    assert a.try_acquire_or_renew()  # renew keeps acquireTime, no transition
    lease = fk.get(LEASES, "l", "ns")
    assert lease["spec"]["holderIdentity"] == "a" and lease["spec"]["leaseTransitions"] == 0
    time.sleep(1.2)  # a stops renewing -> expired
    assert b.try_acquire_or_renew()
    lease = fk.get(LEASES, "l", "ns")
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    assert not a.try_acquire_or_renew()


def _operator(fk, tmp_path, ident):
    s = load_settings(env={}, overrides={
        "patterns.cache_dir": str(tmp_path / "patterns"), "health.enabled": False, "watch.restart_delay_s": 0.05,
        "operator.leader_election": True, "operator.lease_duration_s": 1.0, "operator.lease_renew_deadline_s": 0.6,
        "operator.lease_retry_period_s": 0.1})
    op = Operator(fk, s, match_service=LocalMatchService(MatchEngine(catalog_library(), device="cpu"), max_wait_ms=1),
                  explain_service=EchoExplainService())
    return op.start(http=False)


def _fail(fk, name):
    fk.create(PODS, running_pod(name, labels={"app": "demo"}))
    fk.set_log("default", name, b"boot\nOOMKilled: container exceeded memory limit\n")
    cur = fk.get(PODS, name, "default")
    cur["status"] = failed_pod(name, finished_at="2025-08-29T10:00:00Z")["status"]
    fk.replace(PODS, cur)


def _analyzed(fk, name):
    p = fk.get(PODS, name, "default")
    return p and "podmortem.io/analysis" in (p["metadata"].get("annotations") or {})


def test_one_leader_and_failover(tmp_path):
    fk = FakeKube()
    fk.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"},
                           "spec": {"podSelector": {"matchLabels": {"app": "demo"}}, "aiAnalysisEnabled": False}})
    a, b = _operator(fk, tmp_path, "a"), _operator(fk, tmp_path, "b")
    try:
        wait_for(lambda: a.is_leader or b.is_leader)
        time.sleep(0.3)
        assert a.is_leader != b.is_leader
        leader, standby = (a, b) if a.is_leader else (b, a)
        wait_for(lambda: leader.monitors.list())
        _fail(fk, "p1")
        wait_for(lambda: _analyzed(fk, "p1"))
        # only the leader's pipeline ran
        assert leader.metrics.failures_detected._value.get() >= 1
        assert standby.metrics.failures_detected._value.get() == 0
        # the leader "crashes": its elector stops renewing without releasing the lease
        leader.elector._stop.set()
        leader.elector.leading = False
        leader._stop_workers()
        wait_for(lambda: standby.is_leader, timeout=10)
        wait_for(lambda: standby.monitors.list())
        _fail(fk, "p2")
        wait_for(lambda: _analyzed(fk, "p2"))
        assert standby.metrics.failures_detected._value.get() >= 1
        # clean stop hands over immediately (lease released)
        standby.stop()
        lease = fk.get(LEASES, "podmortem-operator-leader", "podmortem-system")
        assert lease["spec"]["holderIdentity"] == ""
    finally:
        a.stop()
        b.stop()


class _StallingKube:
    """FakeKube whose lease writes can be made to block (a stalled apiserver)."""

    def __init__(self, fk):
        self.fk = fk
        self.stall_s = 0.0

    def __getattr__(self, name):
        return getattr(self.fk, name)

    def replace(self, res, obj, namespace=None):
        if self.stall_s and res == LEASES:
            time.sleep(self.stall_s)
        return self.fk.replace(res, obj, namespace)


def test_stalled_renewal_stops_leading_within_deadline():
    fk = FakeKube()
    slow = _StallingKube(fk)
    events = []
    a = LeaderElector(slow, "l", "ns", identity="a", lease_duration_s=1.5, renew_deadline_s=0.8, retry_period_s=0.1,
                      on_started_leading=lambda: events.append(("a", "start", time.monotonic())),
                      on_stopped_leading=lambda: events.append(("a", "stop", time.monotonic()))).start()
    b = None
    try:
        wait_for(lambda: a.leading)
        # the standby starts once a holds the lease: started together, b could win the
        # first acquisition and a would never lead (a race, not the behaviour under test)
        b = LeaderElector(fk, "l", "ns", identity="b", lease_duration_s=1.5, renew_deadline_s=0.8,
                          retry_period_s=0.1,
                          on_started_leading=lambda: events.append(("b", "start", time.monotonic()))).start()
        time.sleep(0.3)
        assert not b.leading
        t_stall = time.monotonic()
        slow.stall_s = 30.0   # every renewal now blocks far longer than the lease
        wait_for(lambda: not a.leading, timeout=15)
        stop_t = next(t for who, what, t in events if who == "a" and what == "stop")
        # stopped within renew_deadline (+ one retry period, + scheduling slack when the
        # test runs beside a loaded suite), long before the stalled call (30 s) returns
        assert stop_t - t_stall < 0.8 + 0.1 + 1.0
        wait_for(lambda: b.leading, timeout=15)
        start_b = next(t for who, what, t in events if who == "b" and what == "start")
        assert start_b > stop_t    # never two leaders at once
    finally:
        slow.stall_s = 0.0
        if b is not None:
            b.stop()
        a.stop(timeout=1)


def test_failing_start_callback_releases_lease_and_retries():
    fk = FakeKube()
    calls = {"n": 0}

    def flaky_start():
        calls["n"] += 1
        if calls["n"] < 3:
            raise RuntimeError("initial list failed")

    a = LeaderElector(fk, "l", "ns", identity="a", lease_duration_s=1.0, renew_deadline_s=0.6, retry_period_s=0.05,
                      on_started_leading=flaky_start).start()
    try:
        wait_for(lambda: a.leading and calls["n"] >= 3, timeout=5)
        assert a._t.is_alive()
        assert fk.get(LEASES, "l", "ns")["spec"]["holderIdentity"] == "a"
    finally:
        a.stop()
