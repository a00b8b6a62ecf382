"""Controller behaviour against FakeKube (CPU tier): the reference's watch ->
collect -> match -> explain -> store/status/Events flow, with its exact strings."""
import base64
import subprocess
import time

import pytest

from operator_amd.api.models import AnalysisEvent, AnalysisResult, AnalysisSummary, MatchedPattern
from operator_amd.config import load_settings
from operator_amd.controller import events as ev
from operator_amd.controller import storage as st
from operator_amd.controller.failures import FailureDeduper, has_pod_failed, matches_monitor
from operator_amd.controller.health import PatternLibraryReadiness
from operator_amd.controller.operator import Operator
from operator_amd.controller.patternlibrary import needs_sync, parse_refresh_interval
from operator_amd.engine.match import MatchEngine
from operator_amd.engine.service import EchoExplainService, LocalMatchService
from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
from operator_amd.kube.resources import (AIPROVIDERS, DEPLOYMENTS, EVENTS, PATTERNLIBRARIES, PODMORTEMS, PODS,
                                         REPLICASETS, SECRETS)
from operator_amd.patterns.synth import catalog_library, library_yaml


def wait_for(pred, timeout=10.0, step=0.02):
    end = time.time() + timeout
    while time.time() < end:
        v = pred()
        if v:
            return v
        time.sleep(step)
    raise AssertionError("condition not met in time")


# ---------------------------------------------------------------- golden strings
def test_truncate_semantics():
    assert ev.truncate(None, 10) is None
    assert ev.truncate("short", 10) == "short"
    assert ev.truncate("x" * 20, 10) == "xxxxxxx..."
    text = "Intro " + "a" * 50 + " Root Cause: db down. Evidence: logs " + "b" * 40 + " Fix: restart db " + "c" * 60
    out = ev.truncate(text, 60)
    assert out.startswith("Root Cause: db down.") and " ... Fix: restart db" in out and len(out) <= 60
    # Fix before Root Cause and no Evidence: Java would throw; we fall back to plain truncation
    weird = "Fix it. " + "z" * 40 + " Root Cause: q" + "y" * 40
    assert ev.truncate(weird, 30) == weird[:27] + "..."


def _result(sev="HIGH", sig=2, events=None):
    events = events if events is not None else [
        AnalysisEvent(line_number=3, matched_pattern=MatchedPattern(name="OOM", severity="CRITICAL"), score=0.125),
        AnalysisEvent(line_number=9, matched_pattern=MatchedPattern(name="Conn", severity="HIGH"), score=0.675)]
    return AnalysisResult(summary=AnalysisSummary(highest_severity=sev, significant_events=sig), events=events)


def test_messages_and_annotations():
    r = _result()
    assert ev.complete_message(r, None) == "Analysis complete. Severity=HIGH, Events=2"
    assert ev.complete_message(r, "AI disabled") == "Analysis complete. Severity=HIGH, Events=2 | AI disabled"
    assert ev.complete_message(_result(sev=None), "  ") == "Analysis complete. Severity=null, Events=2"
    long = ev.complete_message(r, "d" * 2000)
    assert len(long) <= 850 + 3
    assert st.pattern_annotation(r) == "Pattern Analysis: Severity=HIGH, SignificantEvents=2, TotalMatches=2"
    assert st.pattern_annotation(AnalysisResult()) == \
        "Pattern Analysis: Severity=UNKNOWN, SignificantEvents=0, TotalMatches=0"
    # Java %.2f rounds HALF_UP from the shortest decimal: 0.125 -> 0.13, 0.675 -> 0.68
    assert st.pattern_explanation(r) == (
        "Pattern Analysis Results:\n========================\nHighest Severity: HIGH\nSignificant Events: 2\n"
        "\nTop Matches:\n- OOM (Severity: CRITICAL, Score: 0.13)\n- Conn (Severity: HIGH, Score: 0.68)\n")


def test_refresh_interval_parser():
    P = parse_refresh_interval
    assert P("30s").total_seconds() == 30
    assert P("5m").total_seconds() == 300
    assert P(" 2H ").total_seconds() == 7200
    assert P("2d").total_seconds() == 172800
    assert P("1h30m").total_seconds() == 5400
    assert P("garbage").total_seconds() == 3600
    assert P(None).total_seconds() == 3600
    assert needs_sync({"status": {}})
    assert not needs_sync({"status": {"lastSyncTime": "2099-01-01T00:00:00Z"}, "spec": {"refreshInterval": "1h"}})


def test_failure_detection_and_selector():
    p = failed_pod("a", labels={"app": "x"})
    assert has_pod_failed(p)
    assert not has_pod_failed(running_pod("b"))
    assert not has_pod_failed({"status": {"containerStatuses": [{"state": None}]}})
    assert not has_pod_failed(failed_pod("c", exit_code=0))
    crash = {"status": {"containerStatuses": [{"state": {"waiting": {}}, "lastState": {"terminated": {"exitCode": 2}}}]}}
    assert not has_pod_failed(crash) and has_pod_failed(crash, include_last_state=True)
    pm = {"spec": {"podSelector": {"matchLabels": {"app": "x"}}}}
    assert matches_monitor(p, pm)
    assert not matches_monitor(p, {"spec": {"podSelector": {}}})
    assert not matches_monitor(p, {"spec": {}})
    assert matches_monitor(p, {"spec": {"podSelector": {"matchExpressions": [{"key": "app", "operator": "In",
                                                                            "values": ["x", "y"]}]}}})
    d = FailureDeduper(max_entries=2)
    assert d.check_and_mark(p, "t1") and not d.check_and_mark(p, "t1") and d.check_and_mark(p, "t2")
    assert d.check_and_mark(p, None) and d.check_and_mark(p, None)


# ---------------------------------------------------------------- operator integration
@pytest.fixture
def env(tmp_path):
    fk = FakeKube()
    s = load_settings(env={}, overrides={"patterns.cache_dir": str(tmp_path / "patterns"), "health.enabled": False,
                                         "watch.restart_delay_s": 0.05, "storage.initial_backoff_s": 0.001})
    eng = MatchEngine(catalog_library(), device="cpu")
    match = LocalMatchService(eng, max_wait_ms=1)
    echo = EchoExplainService()
    op = Operator(fk, s, match_service=match, explain_service=echo)
    op.start(http=False)
    yield fk, op, echo
    op.stop()


def _pm(fk, name="demo-monitor", ns="default", ai=False, provider=None, labels=None):
    spec = {"podSelector": {"matchLabels": labels or {"app": "demo"}}, "aiAnalysisEnabled": ai}
    if provider:
        spec["aiProviderRef"] = {"name": provider}
    return fk.create(PODMORTEMS, {"apiVersion": "podmortem.redhat.com/v1alpha1", "kind": "Podmortem",
                                  "metadata": {"name": name, "namespace": ns}, "spec": spec})


def _fail(fk, name, log=b"starting\nOOMKilled: container exceeded memory limit\n", finished="2025-08-29T10:00:00Z",
          labels=None, owner_rs=None):
    fk.create(PODS, running_pod(name, labels=labels or {"app": "demo"}))
    fk.set_log("default", name, log)
    cur = fk.get(PODS, name, "default")
    bad = failed_pod(name, labels=labels or {"app": "demo"}, finished_at=finished, owner_rs=owner_rs)
    cur["status"] = bad["status"]
    if owner_rs:
        cur["metadata"]["ownerReferences"] = bad["metadata"]["ownerReferences"]
    fk.replace(PODS, cur)  # MODIFIED event


def _events(fk, reason=None):
    return [e for e in fk.list(EVENTS) if reason is None or e["reason"] == reason]


def test_watch_flow_ai_disabled(env):
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: (fk.get(PODMORTEMS, "demo-monitor", "default").get("status") or {}).get("phase") == "Ready")
    _fail(fk, "web-1")
    pod = wait_for(lambda: (lambda p: p if "podmortem.io/analysis" in (p["metadata"].get("annotations") or {})
                            else None)(fk.get(PODS, "web-1", "default")))
    ann = pod["metadata"]["annotations"]
    assert ann["podmortem.io/analysis"].startswith("Pattern Analysis: Severity=CRITICAL, SignificantEvents=")
    assert ann["podmortem.io/severity"] == "CRITICAL"
    assert ann["podmortem.io/monitor"] == "demo-monitor"
    assert ann["podmortem.io/analyzed-at"].endswith("Z")
    pm = wait_for(lambda: (lambda o: o if (o.get("status") or {}).get("recentFailures") else None)(
        fk.get(PODMORTEMS, "demo-monitor", "default")))
    rf = pm["status"]["recentFailures"][0]
    assert rf["podName"] == "web-1" and rf["analysisStatus"] == "Completed"
    assert rf["explanation"].startswith("Pattern Analysis Results:\n========================\n")
    op.drain()
    pm = fk.get(PODMORTEMS, "demo-monitor", "default")
    assert pm["status"]["message"] == "Pattern analysis completed (AI disabled) (Pod: web-1)"
    assert pm["status"]["phase"] == "Processing"
    det = _events(fk, "PodFailureDetected")
    assert {e["regarding"]["kind"] for e in det} == {"Pod", "Podmortem"}
    assert det[0]["note"] == "Pod failure detected and queued for analysis" and det[0]["type"] == "Warning"
    comp = _events(fk, "PodmortemAnalysisComplete")
    assert len(comp) == 2 and comp[0]["note"].endswith(" | AI disabled") and comp[0]["type"] == "Normal"
    assert comp[0]["reportingController"] == "podmortem.operator" and comp[0]["action"] == "Report"
    assert comp[0]["metadata"]["name"].startswith("web-1.") or comp[0]["metadata"]["name"].startswith("demo-monitor.")


def test_dedupe_and_added_ignored(env):
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    # the Podmortem's first reconcile (which analyses failed pods that already exist, §3.3)
    # must be over before the ADDED-only pod appears, or it rightly analyses that pod too
    wait_for(lambda: ((fk.get(PODMORTEMS, "demo-monitor", "default") or {}).get("status") or {}).get("phase") == "Ready")
    fk.create(PODS, failed_pod("added-only", labels={"app": "demo"}))  # ADDED: ignored by the watcher
    _fail(fk, "w2", finished="2025-08-29T10:00:00Z")
    wait_for(lambda: len(_events(fk, "PodmortemAnalysisComplete")) >= 2)
    op.drain()
    n = len(_events(fk, "PodFailureDetected"))
    cur = fk.get(PODS, "w2", "default")
    cur["metadata"].setdefault("labels", {})["touched"] = "1"
    fk.replace(PODS, cur)  # same finishedAt -> deduped
    time.sleep(0.2)
    op.drain()
    assert len(_events(fk, "PodFailureDetected")) == n
    cur = fk.get(PODS, "w2", "default")
    cur["status"]["containerStatuses"][0]["state"]["terminated"]["finishedAt"] = "2025-08-29T11:00:00Z"
    fk.replace(PODS, cur)  # a new failure of the same pod
    wait_for(lambda: len(_events(fk, "PodFailureDetected")) > n)
    assert not any(e["regarding"]["name"] == "added-only" for e in _events(fk))


def test_ai_enabled_success_with_secret(env):
    fk, op, echo = env
    fk.create(SECRETS, {"metadata": {"name": "creds", "namespace": "default"},
                        "data": {"api-key": base64.b64encode(b"sk-123").decode()}})
    fk.create(AIPROVIDERS, {"metadata": {"name": "local", "namespace": "default"},
                            "spec": {"providerId": "local", "modelId": "llama3-8b",
                                     "authenticationRef": {"secretName": "creds", "secretKey": "api-key"}}})
    _pm(fk, ai=True, provider="local")
    wait_for(lambda: op.monitors.list())
    _fail(fk, "api-1")
    pod = wait_for(lambda: (lambda p: p if "podmortem.io/analysis" in (p["metadata"].get("annotations") or {})
                            else None)(fk.get(PODS, "api-1", "default")))
    assert pod["metadata"]["annotations"]["podmortem.io/analysis"].startswith("Root Cause: Container OOMKilled")
    op.drain()
    assert fk.get(PODMORTEMS, "demo-monitor", "default")["status"]["message"] == \
        "Analysis completed with AI analysis (Pod: api-1)"
    comp = _events(fk, "PodmortemAnalysisComplete")
    assert comp and "| Root Cause: Container OOMKilled" in comp[0]["note"]
    aip = wait_for(lambda: (lambda o: o if (o.get("status") or {}).get("phase") else None)(
        fk.get(AIPROVIDERS, "local", "default")))
    assert aip["status"]["phase"] == "Ready"


def test_ai_failure_does_not_store(env):
    fk, op, echo = env
    echo.fail_with = "model exploded"
    fk.create(AIPROVIDERS, {"metadata": {"name": "p", "namespace": "default"}, "spec": {"providerId": "x"}})
    _pm(fk, ai=True, provider="p")
    wait_for(lambda: op.monitors.list())
    _fail(fk, "f-1")
    wait_for(lambda: _events(fk, "PodmortemAnalysisError"))
    op.drain()
    assert "podmortem.io/analysis" not in (fk.get(PODS, "f-1", "default")["metadata"].get("annotations") or {})
    errs = _events(fk, "PodmortemAnalysisError")
    assert errs[0]["note"] == "AI analysis failed: model exploded"
    assert fk.get(PODMORTEMS, "demo-monitor", "default")["status"]["message"] == \
        "Pattern analysis completed, AI failed: model exploded (Pod: f-1)"


def test_provider_not_found_stores_pattern_result(env):
    fk, op, _ = env
    _pm(fk, ai=True, provider="missing")
    wait_for(lambda: op.monitors.list())
    _fail(fk, "nf-1")
    wait_for(lambda: "podmortem.io/analysis" in (fk.get(PODS, "nf-1", "default")["metadata"].get("annotations") or {}))
    op.drain()
    assert fk.get(PODMORTEMS, "demo-monitor", "default")["status"]["message"] == \
        "Analysis completed, AI provider not found (Pod: nf-1)"


def test_conflicts_retried_and_forbidden_gives_up(env):
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    fk.inject("patch", "pods", 409, times=3)
    _fail(fk, "c-1")
    wait_for(lambda: "podmortem.io/analysis" in (fk.get(PODS, "c-1", "default")["metadata"].get("annotations") or {}))
    op.drain()
    fk.inject("patch", "pods", 403, times=1)
    _fail(fk, "c-2")
    wait_for(lambda: len([e for e in _events(fk, "PodmortemAnalysisComplete") if e["regarding"]["name"] == "c-2"]))
    op.drain()
    assert "podmortem.io/analysis" not in (fk.get(PODS, "c-2", "default")["metadata"].get("annotations") or {})


def test_recent_failures_ring_is_capped(env):
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    for i in range(13):
        _fail(fk, f"r-{i}")
    wait_for(lambda: len(_events(fk, "PodmortemAnalysisComplete")) >= 26, timeout=20)
    op.drain()
    rf = fk.get(PODMORTEMS, "demo-monitor", "default")["status"]["recentFailures"]
    assert len(rf) == 10
    assert len({r["podName"] for r in rf}) == 10


def test_watch_restart_after_error(env):
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    wait_for(lambda: fk.open_watches(PODS) == 1)
    fk.fail_watches(res=PODS)
    wait_for(lambda: op.watcher.restarts >= 1)
    wait_for(lambda: fk.open_watches(PODS) == 1)
    _fail(fk, "after-restart")
    wait_for(lambda: "podmortem.io/analysis" in
             (fk.get(PODS, "after-restart", "default")["metadata"].get("annotations") or {}))


def test_owner_deployment_gets_events(env):
    fk, op, _ = env
    fk.create(DEPLOYMENTS, {"metadata": {"name": "web", "namespace": "default"}, "spec": {}})
    fk.create(REPLICASETS, {"metadata": {"name": "web-abc", "namespace": "default", "ownerReferences": [
        {"kind": "Deployment", "name": "web", "apiVersion": "apps/v1"}]}})
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    _fail(fk, "web-abc-1", owner_rs="web-abc")
    wait_for(lambda: any(e["regarding"]["kind"] == "Deployment" for e in _events(fk, "PodmortemAnalysisComplete")))


def test_reconciler_analyses_existing_failures_once(env):
    fk, op, _ = env
    fk.create(PODS, failed_pod("old-1", labels={"app": "demo"}, finished_at="2025-08-01T00:00:00Z"))
    fk.set_log("default", "old-1", "panic: boom\ngoroutine 1 [running]:\n")
    _pm(fk)
    wait_for(lambda: "podmortem.io/analysis" in (fk.get(PODS, "old-1", "default")["metadata"].get("annotations") or {}))
    op.drain()
    pm = fk.get(PODMORTEMS, "demo-monitor", "default")
    assert pm["status"]["observedGeneration"] == 1
    n = len(_events(fk, "PodFailureDetected"))
    pm["spec"]["podSelector"]["matchLabels"]["tier"] = None  # no-op spec edit still bumps generation
    del pm["spec"]["podSelector"]["matchLabels"]["tier"]
    pm["spec"]["aiAnalysisEnabled"] = False
    pm["spec"]["extra"] = "x"
    fk.replace(PODMORTEMS, pm)
    wait_for(lambda: fk.get(PODMORTEMS, "demo-monitor", "default")["status"].get("observedGeneration") == 2)
    op.drain()
    assert len(_events(fk, "PodFailureDetected")) == n  # shared dedupe: not re-analysed


def _bare_repo(tmp_path, files):
    src = tmp_path / "src"
    src.mkdir()
    for name, text in files.items():
        (src / name).write_text(text)
    run = lambda *a, cwd=src: subprocess.run(["git", *a], cwd=cwd, check=True, capture_output=True)  # noqa: E731
    run("init", "-q", "-b", "main")
    run("-c", "user.email=a@b", "-c", "user.name=t", "add", ".")
    run("-c", "user.email=a@b", "-c", "user.name=t", "commit", "-q", "-m", "init")
    bare = tmp_path / "patterns.git"
    subprocess.run(["git", "clone", "-q", "--bare", str(src), str(bare)], check=True, capture_output=True)
    return bare


def test_pattern_library_sync_and_reload(env, tmp_path):
    fk, op, _ = env
    bare = _bare_repo(tmp_path, {"java.yaml": library_yaml(5, library_id="java"),
                                 "net.yml": library_yaml(3, seed=2, library_id="net")})
    fk.create(PATTERNLIBRARIES, {"metadata": {"name": "core", "namespace": "default"},
                                 "spec": {"repositories": [{"name": "r1", "url": f"file://{bare}"},
                                                           {"name": "bad", "url": f"file://{tmp_path}/nope.git"}],
                                          "refreshInterval": "1h", "enabledLibraries": ["java"]}})
    pl = wait_for(lambda: (lambda o: o if (o.get("status") or {}).get("phase") == "Ready" else None)(
        fk.get(PATTERNLIBRARIES, "core", "default")), timeout=20)
    s = pl["status"]
    assert s["message"] == "Sync completed: 2 repositories, 2 libraries available"
    assert sorted(s["availableLibraries"]) == ["java", "net"]
    by = {r["name"]: r for r in s["syncedRepositories"]}
    assert by["r1"]["status"] == "Success" and len(by["r1"]["lastCommit"]) == 40
    assert by["bad"]["status"] == "Failed" and by["bad"]["error"]
    assert op.pattern_count == len(catalog_library()) + 5  # enabledLibraries filter: only java
    r = op.readiness()
    assert r == ("pattern-library-sync", True)


def test_readiness_check(tmp_path):
    fk = FakeKube()
    t = [0.0]
    chk = PatternLibraryReadiness(fk, str(tmp_path / "cache"), grace_s=300, clock=lambda: t[0])
    assert chk()[1] is True  # no PatternLibrary CRs
    fk.create(PATTERNLIBRARIES, {"metadata": {"name": "x", "namespace": "default"}, "spec": {}})
    assert chk()[1] is False  # no cache dir yet
    (tmp_path / "cache").mkdir()
    assert chk()[1] is False
    (tmp_path / "cache" / "a.yaml").write_text("patterns: []")
    assert chk()[1] is True
    (tmp_path / "cache" / "a.yaml").unlink()
    t[0] = 301
    assert chk()[1] is True  # grace period exceeded


def test_status_group_commit_coalesces_bursts():
    """Concurrent ring appends for one Podmortem are committed in batches: fewer
    PATCHes than entries, and the ring equals one-by-one prepends in commit order."""
    import threading

    fk = FakeKube()
    fk.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"}, "spec": {}})
    order = []
    real_patch = fk.patch_status

    def slow_patch(res, name, ns, patch, **kw):
        time.sleep(0.01)
        if "recentFailures" in patch:
            order.append([e["podName"] for e in patch["recentFailures"]])
        return real_patch(res, name, ns, patch, **kw)

    fk.patch_status = slow_patch
    w = st.StatusWriter(fk)
    mon = fk.get(PODMORTEMS, "m", "default")
    res = AnalysisResult(summary=AnalysisSummary(highest_severity="HIGH", significant_events=1), events=[])
    oks = []
    th = [threading.Thread(target=lambda i=i: oks.append(w.append_failure(failed_pod(f"p{i}"), mon, res, f"x{i}")))
          for i in range(40)]
    th += [threading.Thread(target=lambda i=i: w.update_pod_failure(mon, failed_pod(f"p{i}"), "done")) for i in range(40)]
    for t in th:
        t.start()
    for t in th:
        t.join(30)
    assert oks == [True] * 40
    assert w.commits < 80   # both queues coalesced
    rf = fk.get(PODMORTEMS, "m", "default")["status"]["recentFailures"]
    assert len(rf) == 10 and [e["podName"] for e in rf] == order[-1]
    assert len(order) < 40   # ring PATCHes: one per flushed batch, not one per entry
    assert fk.get(PODMORTEMS, "m", "default")["status"]["message"].startswith("done (Pod: p")


# ---------------------------------------------------------------- watch lifecycle
def test_watch_reconnects_after_clean_server_close(env):
    """The apiserver ends every watch after its min-request-timeout with no error:
    the pod watcher must reopen it (fabric8 does), not stop for good."""
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    wait_for(lambda: fk.open_watches(PODS) == 1)
    for _ in range(3):   # several server-side timeouts in a row
        n = op.watcher.reconnects
        assert fk.end_watches(PODS) == 1
        wait_for(lambda: op.watcher.reconnects > n)
        wait_for(lambda: fk.open_watches(PODS) == 1)
    assert op.watcher.restarts == 0
    _fail(fk, "after-timeout")
    wait_for(lambda: "podmortem.io/analysis" in
             (fk.get(PODS, "after-timeout", "default")["metadata"].get("annotations") or {}))
    # the Podmortem cache reconnects too: a monitor created after its stream ended is seen
    fk.end_watches(PODMORTEMS)
    _pm(fk, name="second", labels={"app": "two"})
    wait_for(lambda: len(op.monitors.list()) == 2)


def test_watch_relists_after_410_and_catches_up(env):
    """A watch resumed from a compacted resourceVersion fails with 410 Gone: the watcher
    must not retry that resourceVersion forever but relist, and a failure that happened
    while it was disconnected is still analysed (once)."""
    fk, op, _ = env
    _pm(fk)
    wait_for(lambda: op.monitors.list())
    _fail(fk, "before-gap")
    wait_for(lambda: "podmortem.io/analysis" in
             (fk.get(PODS, "before-gap", "default")["metadata"].get("annotations") or {}))
    op.drain()
    detected = len(_events(fk, "PodFailureDetected"))
    # the watch errors out; while it waits to restart a pod fails and the history is compacted
    fk.inject("watch", "pods", 503, times=10_000)   # hold the watcher off until the gap is set up
    fk.fail_watches("connection reset", res=PODS)
    wait_for(lambda: fk.open_watches(PODS) == 0)
    _fail(fk, "during-gap")
    fk.compact()
    fk.clear_faults()
    wait_for(lambda: op.watcher.relists >= 1)
    wait_for(lambda: "podmortem.io/analysis" in
             (fk.get(PODS, "during-gap", "default")["metadata"].get("annotations") or {}))
    op.drain()
    names = [e["regarding"]["name"] for e in _events(fk, "PodFailureDetected") if e["regarding"]["kind"] == "Pod"]
    assert names.count("before-gap") == 1 and names.count("during-gap") == 1   # dedupe across the relist
    assert len(_events(fk, "PodFailureDetected")) == detected + 2
    wait_for(lambda: fk.open_watches(PODS) == 1)
    _fail(fk, "after-relist")
    wait_for(lambda: "podmortem.io/analysis" in
             (fk.get(PODS, "after-relist", "default")["metadata"].get("annotations") or {}))


def test_bookmarks_advance_the_resume_point():
    from operator_amd.kube.informer import WatchLoop

    fk = FakeKube()
    seen = []
    lp = WatchLoop(fk, PODS, None, lambda t, o: seen.append((t, o["metadata"]["name"])), restart_delay_s=0.01)
    lp.list_now()
    import threading

    th = threading.Thread(target=lp.run, daemon=True)
    th.start()
    wait_for(lambda: fk.open_watches(PODS) == 1)
    fk.create(PODS, running_pod("a"))
    wait_for(lambda: seen == [("ADDED", "a")])
    for i in range(5):   # unrelated churn elsewhere moves the store's resourceVersion
        fk.create(PODMORTEMS, {"metadata": {"name": f"pm{i}", "namespace": "default"}, "spec": {}})
    rv_before = lp.rv
    fk.bookmark(PODS)
    wait_for(lambda: lp.rv != rv_before)
    assert lp.rv == fk.current_resource_version() and seen == [("ADDED", "a")]   # bookmarks are not events
    # compaction up to the bookmark: resuming from it still works (no 410, no relist)
    fk.compact()
    fk.end_watches(PODS)
    wait_for(lambda: lp.reconnects == 1 and fk.open_watches(PODS) == 1)
    fk.create(PODS, running_pod("b"))
    wait_for(lambda: seen[-1] == ("ADDED", "b"))
    assert lp.relists == 0 and lp.restarts == 0
    lp.stop()
    th.join(5)
    assert not th.is_alive()


def test_list_resource_version_is_the_lists_own():
    """The resume point after a LIST is the list's metadata.resourceVersion, not the
    maximum of the items' (which misses deletions and can be long compacted)."""
    fk = FakeKube()
    fk.create(PODS, running_pod("a"))
    fk.create(PODS, running_pod("b"))
    fk.delete(PODS, "b", "default")
    items, rv = fk.list_rv(PODS)
    assert [o["metadata"]["name"] for o in items] == ["a"]
    assert int(rv) > max(int(o["metadata"]["resourceVersion"]) for o in items)
    w = fk.watch(PODS, None, resource_version=rv)   # nothing to replay: the DELETE is before rv
    fk.create(PODS, running_pod("c"))
    assert next(iter(w))[1]["metadata"]["name"] == "c"
    w.close()


def test_operator_shards_split_failures_exactly_once(tmp_path):
    """Two operator shards on one API server (operator.shard_count=2): every failed pod
    is analysed by exactly one of them, both take part, and both keep the CR status."""
    from operator_amd.controller.failures import in_shard

    fk = FakeKube()
    ops_, echos = [], []
    for i in range(2):
        s = load_settings(env={}, overrides={"patterns.cache_dir": str(tmp_path / f"p{i}"), "health.enabled": False,
                                             "operator.shard_count": 2, "operator.shard_index": i})
        echo = EchoExplainService()
        op = Operator(fk, s, match_service=LocalMatchService(MatchEngine(catalog_library(), device="cpu"),
                                                             max_wait_ms=1), explain_service=echo)
        ops_.append(op.start(http=False))
        echos.append(echo)
    try:
        _pm(fk, ai=False)
        wait_for(lambda: all(o.monitors.list() for o in ops_))
        names = [f"sh-{i}" for i in range(24)]
        for n in names:
            _fail(fk, n)
        wait_for(lambda: all("podmortem.io/analysis" in (fk.get(PODS, n, "default")["metadata"].get("annotations")
                                                         or {}) for n in names), timeout=30)
        for o in ops_:
            o.drain()
        per = [sum(1 for n in names if in_shard(fk.get(PODS, n, "default"), i, 2)) for i in range(2)]
        assert per[0] > 0 and per[1] > 0 and sum(per) == len(names)
        det = [e for e in _events(fk, "PodFailureDetected") if e["regarding"]["kind"] == "Pod"]
        assert sorted(e["regarding"]["name"] for e in det) == sorted(names)   # exactly once each
        assert len(fk.get(PODMORTEMS, "demo-monitor", "default")["status"]["recentFailures"]) == 10
    finally:
        for o in ops_:
            o.stop()


def test_sink_concurrency_bounds_result_writers(monkeypatch):
    """operator.sink_concurrency: at most N analyses write their results at once; every
    analysis still stores its result."""
    import threading
    import time as _time

    from operator_amd.api.models import AIProviderConfig, AIResponse, AnalysisResult
    from operator_amd.controller import ai_client
    from operator_amd.controller.pipeline import AnalysisPipeline

    monkeypatch.setattr(ai_client, "get_provider", lambda kube, m, cache=None: {"spec": {}})
    monkeypatch.setattr(ai_client, "to_provider_config", lambda kube, p: AIProviderConfig())
    state = {"now": 0, "max": 0, "stored": 0}
    lock = threading.Lock()

    class Storage:
        def store(self, pod, monitor, result, text):
            with lock:
                state["now"] += 1
                state["max"] = max(state["max"], state["now"])
            _time.sleep(0.02)
            with lock:
                state["now"] -= 1
                state["stored"] += 1

    class Nop:
        def __getattr__(self, name):
            return lambda *a, **k: None

    class Explainer:
        def explain(self, result, cfg):
            return AIResponse(explanation="x")

    p = AnalysisPipeline(None, None, Explainer(), Nop(), Storage(), Nop(), sink_concurrency=3)
    ai = {"metadata": {"name": "m", "namespace": "default"}, "spec": {"aiProviderRef": {"name": "p"}}}
    off = {"metadata": {"name": "m", "namespace": "default"}, "spec": {"aiAnalysisEnabled": False}}
    ts = [threading.Thread(target=p.handle_result,
                           args=(ai if i % 2 else off, {"metadata": {"name": f"p{i}"}}, AnalysisResult()))
          for i in range(12)]   # AI-explained and pattern-only results share the bound
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert state["stored"] == 12 and 1 <= state["max"] <= 3


def test_metrics_rates_and_collectives():
    """SURVEY.md §5.5 gauges: scan GB/s of the last batch, tokens/s and analyses/s over
    a window, and the process-wide collective counters."""
    from operator_amd.parallel.comm import COLLECTIVES
    from operator_amd.utils.metrics import Metrics

    m = Metrics()
    m.observe_scan(2 * 10**9, 0.5)
    COLLECTIVES.add("all_reduce", "gloo", 4096, 0.002)
    m.tokens_generated.inc(10)
    m.render()
    m.tokens_generated.inc(500)
    import time as _t

    _t.sleep(0.05)
    txt = m.render().decode()
    vals = {ln.split(" ")[0]: float(ln.split(" ")[-1]) for ln in txt.splitlines() if ln and not ln.startswith("#")}
    assert vals["podmortem_scan_gigabytes_per_second"] == 4.0
    assert vals["podmortem_tokens_per_second"] > 0
    assert vals['podmortem_collective_calls_total{impl="gloo",op="all_reduce"}'] >= 1
