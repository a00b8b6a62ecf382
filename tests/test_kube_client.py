"""The HTTPS kube client against the FakeKube REST server (wire level), the
operator running over it end to end, the compat REST server, and the CLI."""
import json
import os
import subprocess
import sys
import threading
import time

import httpx
import pytest

from operator_amd.config import load_settings
from operator_amd.controller.operator import Operator
from operator_amd.engine.match import MatchEngine
from operator_amd.engine.server import CompatServer
from operator_amd.engine.service import EchoExplainService, LocalMatchService
from operator_amd.kube.client import KubeClient, KubeConfig
from operator_amd.kube.fake import FakeKube, failed_pod, running_pod
from operator_amd.kube.fake_aserver import AsyncFakeKubeServer
from operator_amd.kube.fake_server import FakeKubeServer
from operator_amd.kube.resources import EVENTS, PODMORTEMS, PODS, ApiError, WatchClosed
from operator_amd.patterns.synth import catalog_library


def wait_for(fn, timeout=20.0):
    end = time.time() + timeout
    while time.time() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.02)
    raise AssertionError("timed out")


@pytest.fixture(params=["threaded", "asyncio"])
def server(request):
    """The REST FakeKube in both process models: a thread per connection (in-process
    tests) and one asyncio loop (the standalone API server of shard-per-GPU runs)."""
    fk = FakeKube()
    srv = (FakeKubeServer(fk) if request.param == "threaded" else AsyncFakeKubeServer(fk)).start()
    kc = KubeClient(KubeConfig(srv.url, token="test-token"), timeout_s=10)
    yield fk, srv, kc
    srv.stop()


def test_verbs_over_http(server):
    fk, srv, kc = server
    p = kc.create(PODS, running_pod("web-1", labels={"app": "x", "tier": "a"}))
    assert p["metadata"]["name"] == "web-1" and p["metadata"]["resourceVersion"]
    kc.create(PODS, running_pod("web-2", labels={"app": "y"}))
    assert kc.get(PODS, "web-1", "default")["kind"] == "Pod"
    assert kc.get(PODS, "nope", "default") is None
    assert [o["metadata"]["name"] for o in kc.list(PODS, "default", label_selector={"app": "x"})] == ["web-1"]
    assert [o["metadata"]["name"] for o in kc.list(PODS, "default", label_selector="app in (x,y)")] == \
        ["web-1", "web-2"]
    # optimistic concurrency: a stale resourceVersion gets 409
    stale = kc.get(PODS, "web-1", "default")
    fresh = kc.get(PODS, "web-1", "default")
    fresh["metadata"].setdefault("annotations", {})["a"] = "1"
    kc.replace(PODS, fresh)
    stale["metadata"].setdefault("annotations", {})["a"] = "2"
    with pytest.raises(ApiError) as e:
        kc.replace(PODS, stale)
    assert e.value.code == 409
    kc.patch(PODS, "web-1", "default", {"metadata": {"annotations": {"b": "2"}}})
    ann = kc.get(PODS, "web-1", "default")["metadata"]["annotations"]
    assert ann == {"a": "1", "b": "2"}
    pm = kc.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"},
                                "spec": {"podSelector": {"matchLabels": {"app": "x"}}}})
    kc.patch_status(PODMORTEMS, "m", "default", {"phase": "Ready"})
    assert kc.get(PODMORTEMS, "m", "default")["status"]["phase"] == "Ready"
    assert pm["kind"] == "Podmortem"
    fk.set_log("default", "web-1", b"line1\nline2\n")
    assert kc.pod_log("web-1", "default") == "line1\nline2\n"
    assert kc.delete(PODS, "web-2", "default")
    assert kc.get(PODS, "web-2", "default") is None


def test_watch_stream_and_close(server):
    fk, srv, kc = server
    w = kc.watch(PODS, "default")
    got = []

    def reader():
        try:
            for typ, obj in w:
                got.append((typ, obj["metadata"]["name"]))
        except WatchClosed:
            got.append(("CLOSED", ""))

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    time.sleep(0.2)
    fk.create(PODS, running_pod("a"))
    cur = fk.get(PODS, "a", "default")
    cur["status"] = failed_pod("a")["status"]
    fk.replace(PODS, cur)
    fk.delete(PODS, "a", "default")
    wait_for(lambda: len(got) >= 3)
    assert [g[0] for g in got[:3]] == ["ADDED", "MODIFIED", "DELETED"]
    fk.fail_watches("boom")
    wait_for(lambda: got and got[-1][0] == "CLOSED")


def test_operator_end_to_end_over_http(server, tmp_path):
    fk, srv, kc = server
    s = load_settings(env={}, overrides={"patterns.cache_dir": str(tmp_path / "p"), "health.enabled": False,
                                         "watch.restart_delay_s": 0.05})
    op = Operator(kc, s, match_service=LocalMatchService(MatchEngine(catalog_library(), device="cpu"), max_wait_ms=1),
                  explain_service=EchoExplainService()).start(http=False)
    try:
        kc.create(PODMORTEMS, {"metadata": {"name": "mon", "namespace": "default"},
                               "spec": {"podSelector": {"matchLabels": {"app": "demo"}}, "aiAnalysisEnabled": False}})
        wait_for(lambda: op.monitors.list())
        kc.create(PODS, running_pod("api-1", labels={"app": "demo"}))
        fk.set_log("default", "api-1", b"boot\njava.lang.OutOfMemoryError: Java heap space\n")
        cur = kc.get(PODS, "api-1", "default")
        cur["status"] = failed_pod("api-1", finished_at="2025-08-29T10:00:00Z")["status"]
        kc.replace(PODS, cur)
        pod = wait_for(lambda: (lambda p: p if "podmortem.io/analysis" in (p["metadata"].get("annotations") or {})
                                else None)(kc.get(PODS, "api-1", "default")))
        assert pod["metadata"]["annotations"]["podmortem.io/severity"] in ("CRITICAL", "HIGH")
        wait_for(lambda: any(e["reason"] == "PodmortemAnalysisComplete" for e in kc.list(EVENTS, "default")))
    finally:
        op.stop()


def test_compat_server_contracts():
    matcher = LocalMatchService(MatchEngine(catalog_library(), device="cpu"), max_wait_ms=1)
    srv = CompatServer(matcher, EchoExplainService(), "127.0.0.1", 0).start()
    try:
        base = f"http://127.0.0.1:{srv.port}"
        body = {"pod": failed_pod("p"), "logs": "start\nOOMKilled: container exceeded memory limit\n", "events": []}
        r = httpx.post(base + "/parse", json=body, timeout=30)
        assert r.status_code == 200
        res = r.json()
        assert res["summary"]["highestSeverity"] in ("CRITICAL", "HIGH") and res["events"]
        r2 = httpx.post(base + "/api/v1/analysis/analyze",
                        json={"analysisResult": res, "providerConfig": {"providerId": "echo", "maxTokens": 50}},
                        timeout=30)
        assert r2.status_code == 200 and r2.json()["explanation"]
        assert httpx.get(base + "/q/health/ready").json()["status"] == "UP"
        assert httpx.post(base + "/nope", json={}).status_code == 404
    finally:
        srv.stop()


def test_cli_manifests_and_scan(tmp_path):
    r = subprocess.run([sys.executable, "-m", "operator_amd", "manifests", "--replicas", "2"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "kind: CustomResourceDefinition" in r.stdout
    assert "PODMORTEM_OPERATOR__LEADER_ELECTION" in r.stdout
    log = tmp_path / "pod.log"
    log.write_text("hello\njava.lang.OutOfMemoryError: Java heap space\nbye\n")
    r = subprocess.run([sys.executable, "-m", "operator_amd", "scan", str(log), "--device", "cpu"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout)
    assert out[0]["summary"]["highestSeverity"] in ("CRITICAL", "HIGH")


def test_watch_bookmark_410_and_list_rv_over_http(server):
    """Wire level: BOOKMARK events reach the caller, an expired resourceVersion surfaces
    as WatchClosed(code=410), and list_rv returns the list's metadata.resourceVersion."""
    fk, srv, kc = server
    kc.create(PODS, running_pod("a"))
    items, rv = kc.list_rv(PODS, "default")
    assert [o["metadata"]["name"] for o in items] == ["a"] and rv == fk.current_resource_version()
    w = kc.watch(PODS, "default", resource_version=rv)
    got = []

    def reader():
        try:
            for typ, obj in w:
                got.append((typ, obj["metadata"].get("resourceVersion")))
        except WatchClosed as e:
            got.append(("CLOSED", e.code))

    t = threading.Thread(target=reader, daemon=True)
    t.start()
    wait_for(lambda: fk.open_watches(PODS) == 1)
    fk.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"}, "spec": {}})
    fk.bookmark(PODS)
    wait_for(lambda: got)
    assert got[0] == ("BOOKMARK", fk.current_resource_version())
    fk.end_watches(PODS)          # clean server-side end: the iterator just stops
    t.join(5)
    assert not t.is_alive() and got[-1][0] == "BOOKMARK"
    fk.compact()
    w2 = kc.watch(PODS, "default", resource_version=rv)   # rv is now older than the compaction point
    with pytest.raises(WatchClosed) as e:
        next(iter(w2))
    assert e.value.code == 410 and e.value.expired


def test_cli_run_with_two_shards_starts_and_stops_both(tmp_path):
    """`run --shards 2`: a second operator process (shard 1, health port + 1) comes up
    beside the first, is started again when it dies, and goes away when the first is
    stopped."""
    import signal
    import socket
    import time as _t
    import urllib.request

    import random

    # two consecutive free ports below the ephemeral range (port + 1 of an ephemeral port
    # can be any outgoing connection's, and shard 1 then never binds)
    rng = random.Random()
    for _ in range(200):
        port = rng.randrange(20000, 32000)
        try:
            with socket.socket() as a, socket.socket() as b:
                a.bind(("127.0.0.1", port))
                b.bind(("127.0.0.1", port + 1))
            break
        except OSError:
            continue
    env = dict(os.environ, PODMORTEM_LOG_LEVEL="WARNING")
    p = subprocess.Popen([sys.executable, "-m", "operator_amd", "run", "--fake", "--shards", "2",
                          "--set", f"health.port={port}", "--set", "health.host=127.0.0.1",
                          "--set", "services.explain=echo", "--set", "services.match=cpu",
                          "--set", f"patterns.cache_dir={tmp_path}"], env=env)
    try:
        def up(pt):
            try:
                return urllib.request.urlopen(f"http://127.0.0.1:{pt}/q/health/live", timeout=1).status == 200
            except OSError:
                return False
        end = _t.time() + 90
        while _t.time() < end and not (up(port) and up(port + 1)):
            _t.sleep(0.2)
        assert up(port) and up(port + 1)
        # the shard process dies: the first one starts it again
        import psutil

        kids = psutil.Process(p.pid).children()
        assert len(kids) == 1
        kids[0].kill()
        kids[0].wait(30)
        end = _t.time() + 90
        while _t.time() < end and not (up(port + 1) and psutil.Process(p.pid).children()):
            _t.sleep(0.2)
        again = psutil.Process(p.pid).children()
        assert up(port + 1) and len(again) == 1 and again[0].pid != kids[0].pid
    finally:
        p.send_signal(signal.SIGTERM)
        assert p.wait(60) == 0
    _t.sleep(0.5)
    assert not up(port + 1)


def test_shard_env_and_sizing():
    from operator_amd.cli import apply_shard_env, shard_env, shard_sizing
    from operator_amd.config import load_settings

    env = shard_env({"X": "1"}, 1, 2, 8080)
    s = load_settings(env={}, overrides={"health.port": 9999})
    apply_shard_env(s, env)
    assert (s.operator.shard_index, s.operator.shard_count, s.health.port) == (1, 2, 8081) and env["X"] == "1"
    shard_sizing(s, 2)
    assert s.engine.max_batch == 128 and s.engine.kv_cache_gb == 32.0


def test_shard_supervisor_restarts_then_gives_up(monkeypatch):
    """A shard that exits is started again; more than max_restarts exits within the
    window make poll() False (the pod fails and is restarted by Kubernetes)."""
    from operator_amd import cli

    class Dead:
        def poll(self):
            return 1

    started = []
    monkeypatch.setattr(cli.ShardSupervisor, "_start", lambda self, i: started.append(i) or Dead())
    now = [0.0]
    sup = cli.ShardSupervisor(["run"], 3, 8080, max_restarts=3, window_s=100.0, clock=lambda: now[0])
    assert started == [1, 2]
    assert sup.poll()              # restarts 1 and 2 (two restarts)
    now[0] = 200.0                 # the earlier restarts leave the window
    assert sup.poll()              # two more, two within the window
    assert sup.poll() is False     # the fifth exit is the fourth within the window


def test_shard_per_gpu_topology_analyses_each_failure_exactly_once(tmp_path):
    """The multi-GPU production topology on the CPU: `run --shard-per-gpu --gpus 8` (eight
    operator shard processes with stub engines) against ONE REST API server process;
    2000 pods fail at once and every one is analysed exactly once (one
    PodmortemAnalysisComplete Event per pod: no double, no miss), with the shared
    Podmortem status ring written by all eight."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from bench_plumbing import run_sharded

    r = run_sharded(8, 2000, str(tmp_path), timeout_s=400)
    assert r["analysed"] == 2000, r
    assert r["complete_events_per_pod"] == {1: 2000}, r


def test_shard_groups_on_two_apiservers_analyse_each_failure_exactly_once(tmp_path):
    """bench.py's N = 8 layout (--ranks-per-apiserver 4): two API server processes, each
    with its own 4-shard operator; 2000 failures split over them are each analysed exactly
    once, and the two servers' CPU per analysis gives the node >= 2x the ~260 analyses/s
    eight MI355X ranks ask of it (each server carries half the load)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from bench_plumbing import run_sharded

    r = run_sharded(8, 2000, str(tmp_path), timeout_s=400, apiservers=2)
    assert r["analysed"] == 2000, r
    assert r["complete_events_per_pod"] == {1: 2000}, r
    assert len(r["apiserver_cpu_ms_per_analysis"]) == 2
    # capacity from the servers' own CPU time: each analysis costs one server a few ms
    assert r["apiserver_capacity_analyses_per_s"] >= 520, r


def test_shard_per_gpu_env_and_jittered_retrier():
    """--shard-per-gpu: shard i gets cuda:i (cpu stays cpu) and no engine pool; the
    shared status ring's 409 schedule is jittered and its delays stop doubling."""
    import random

    from operator_amd.cli import apply_shard_env, shard_device, shard_env
    from operator_amd.config import load_settings
    from operator_amd.controller.storage import Retrier

    s = load_settings(env={})
    s.engine.gpus = 8
    apply_shard_env(s, shard_env({}, 3, 8, 9000, shard_device("cuda", 3)))
    assert (s.operator.shard_index, s.operator.shard_count, s.health.port) == (3, 8, 9003)
    assert s.engine.device == "cuda:3" and s.engine.gpus == 1
    assert shard_device("cpu", 5) == "cpu"
    r = Retrier(12, 0.1, jitter=0.5, rng=random.Random(0))
    ds = [r.delay(0.1) for _ in range(200)]
    assert 0.05 <= min(ds) < 0.07 and 0.13 < max(ds) <= 0.15
    assert Retrier(5, 0.1).delay(0.4) == 0.4


def _drop_second_request_server():
    """HTTP/1.1 server: answers the first request of every connection (keep-alive) and
    drops the connection after READING the second one, unanswered -- the server may have
    acted on it. Returns (port, seen list of methods, stop)."""
    import socket
    import threading

    seen: list[str] = []
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("127.0.0.1", 0))
    srv.listen(8)
    stop = threading.Event()

    def read_req(f):
        line = f.readline()
        if not line:
            return None
        n = 0
        while True:
            h = f.readline()
            if h in (b"\r\n", b"\n", b""):
                break
            k, _, v = h.decode().partition(":")
            if k.strip().lower() == "content-length":
                n = int(v)
        if n:
            f.read(n)
        return line.split()[0].decode()

    def conn_loop(c):
        with c, c.makefile("rb") as f:
            m = read_req(f)
            if m is None:
                return
            seen.append(m)
            c.sendall(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: 2\r\n\r\n{}")
            m = read_req(f)
            if m is not None:
                seen.append(m)   # processed, then the reply is lost

    def accept_loop():
        srv.settimeout(0.2)
        while not stop.is_set():
            try:
                c, _ = srv.accept()
            except OSError:
                continue
            threading.Thread(target=conn_loop, args=(c,), daemon=True).start()

    threading.Thread(target=accept_loop, daemon=True).start()
    return srv.getsockname()[1], seen, lambda: (stop.set(), srv.close())


def test_pool_resends_only_idempotent_requests_after_a_lost_reply():
    """A request sent on a reused connection whose reply is lost is resent once for GET
    (idempotent), never for POST (the server may already have created the object)."""
    import http.client

    from operator_amd.kube.client import _Pool

    port, seen, stop = _drop_second_request_server()
    try:
        p = _Pool(f"http://127.0.0.1:{port}", {}, 5.0)
        assert p.request("GET", "/a")[0] == 200
        assert p.request("GET", "/a")[0] == 200          # lost reply on the reused conn -> resent
        assert seen == ["GET", "GET", "GET"]
        p.close()
        seen.clear()
        p = _Pool(f"http://127.0.0.1:{port}", {}, 5.0)
        assert p.request("POST", "/e", b"{}")[0] == 200
        with pytest.raises((http.client.RemoteDisconnected, ConnectionResetError)):
            p.request("POST", "/e", b"{}")
        assert seen == ["POST", "POST"]                  # not sent a third time
        p.close()
    finally:
        stop()
