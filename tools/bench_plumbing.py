"""BASELINE.json config 1, "plumbing": the controller with stub engines, on the CPU.

The reference's config 1 is one Podmortem CR reconciled in Quarkus dev mode with stub
log-parser / ai-interface endpoints. Here: FakeKube (in-memory API server) + the
operator (watcher, reconcilers, pipeline, sinks) with the CPU pattern matcher (Python
oracle semantics, catalog library) and the echo explainer (no model). Reports

* reconcile latency: Podmortem CR created -> status.phase Ready, over --crs CRs;
* --match stub (default): a fixed pattern result, as the reference's stub log-parser —
  the controller alone; --match cpu: the CPU pattern matcher over the pod log;
* analyses/s: --failures pods fail at once (MODIFIED events) -> every analysis stored
  (four pod annotations, recentFailures ring, Events), p50 / p99 per failure.

One JSON line on stdout.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from operator_amd.api.models import AnalysisEvent, AnalysisResult, AnalysisSummary, MatchedPattern  # noqa: E402
from operator_amd.config import load_settings  # noqa: E402
from operator_amd.controller.operator import Operator  # noqa: E402
from operator_amd.engine.match import MatchEngine  # noqa: E402
from operator_amd.engine.service import EchoExplainService, LocalMatchService  # noqa: E402
from operator_amd.kube.fake import FakeKube, failed_pod, running_pod  # noqa: E402
from operator_amd.kube.resources import AIPROVIDERS, PODMORTEMS, PODS  # noqa: E402
from operator_amd.patterns.synth import catalog_library  # noqa: E402

LOG = ("\n".join(["starting app", "loading config", "connected to db"] * 30 +
                 ["java.lang.OutOfMemoryError: Java heap space", "\tat com.example.Cache.grow(Cache.java:42)"] +
                 ["shutting down"] * 5)).encode()


class StubMatch:
    """The stub log-parser: one fixed CRITICAL OOM event for every pod."""

    def analyze(self, data):
        meta = data.pod.get("metadata") or {}
        ev = AnalysisEvent(line_number=91, score=0.9, matched_line="java.lang.OutOfMemoryError: Java heap space",
                           matched_pattern=MatchedPattern(id="oom", name="Java heap exhausted", severity="CRITICAL"))
        return AnalysisResult(pod_name=meta.get("name"), pod_namespace=meta.get("namespace"), events=[ev],
                              summary=AnalysisSummary(highest_severity="CRITICAL", significant_events=1,
                                                      total_events=1))


def wait(pred, timeout):
    end = time.perf_counter() + timeout
    while time.perf_counter() < end:
        if pred():
            return True
        time.sleep(0.001)
    return False


def free_port_block(n: int) -> int:
    """First of ``n`` consecutive free TCP ports (shard i serves health on base + i), taken
    below the kernel's ephemeral range so the shards' and harness's outgoing connections
    cannot occupy one between this check and the shard binding it."""
    import random
    import socket

    rng = random.Random()
    for _ in range(200):
        base = rng.randrange(20000, 32000 - n)
        socks = []
        try:
            for i in range(n):
                sk = socket.socket()
                socks.append(sk)
                sk.bind(("127.0.0.1", base + i))
            return base
        except OSError:
            continue
        finally:
            for sk in socks:
                sk.close()
    raise RuntimeError(f"no block of {n} free ports")


def run_sharded(shards: int, failures: int, workdir: str, timeout_s: float = 600.0, log_kb: int = 0,
                apiservers: int = 1) -> dict:
    """The production multi-GPU topology on the CPU: ``apiservers`` API server processes (the
    REST FakeKube), each with its own ``run --shard-per-gpu --gpus shards/apiservers`` operator
    (the operator shard processes, each with its own stub log-parser + echo explainer,
    splitting that server's pods by hash) -- bench.py's N-rank layout (``--ranks-per-apiserver``).
    Fails ``failures`` pods at once (pod i on server i % apiservers) and waits until every one
    carries its analysis annotation; returns the rate, each server's CPU time per analysis (its
    capacity = 1000 / ms analyses/s) and, per pod, how many PodmortemAnalysisComplete Events it
    got (exactly one each = no double, no miss)."""
    import signal
    import subprocess
    from collections import Counter
    from concurrent.futures import ThreadPoolExecutor

    from operator_amd.kube.client import KubeClient, KubeConfig
    from operator_amd.kube.fake_server import spawn, write_kubeconfig
    from operator_amd.kube.resources import EVENTS

    if shards % apiservers:
        raise ValueError("shards must split evenly over the API servers")
    per = shards // apiservers
    env = dict(os.environ, PODMORTEM_LOG_LEVEL="WARNING")
    srvs, kubes, ops = [], [], []
    names = [f"p{i}" for i in range(failures)]
    try:
        for g in range(apiservers):
            srv, url = spawn(os.path.join(workdir, f"apiserver{g}.url"))
            srvs.append(srv)
            kc = write_kubeconfig(url, os.path.join(workdir, f"kubeconfig{g}"))
            kube = KubeClient(KubeConfig(url), 30.0)
            kubes.append(kube)
            kube.create(AIPROVIDERS, {"metadata": {"name": "stub", "namespace": "default"},
                                      "spec": {"providerId": "stub", "modelId": "echo"}})
            kube.create(PODMORTEMS, {"metadata": {"name": "m0", "namespace": "default"},
                                     "spec": {"podSelector": {"matchLabels": {"app": "demo"}},
                                              "aiAnalysisEnabled": True, "aiProviderRef": {"name": "stub"}}})
            log = LOG
            if log_kb:
                filler = b"INFO request served in 3 ms from cache shard 7\n"
                log = filler * max(0, (log_kb * 1024 - len(LOG)) // len(filler)) + LOG
            import httpx

            with httpx.Client(base_url=url, timeout=30) as h:
                for n in names[g::apiservers]:
                    kube.create(PODS, running_pod(n, labels={"app": "demo"}))
                    h.put(f"/api/v1/namespaces/default/pods/{n}/log", content=log).raise_for_status()
            port = free_port_block(per)
            ops.append((subprocess.Popen([sys.executable, "-m", "operator_amd", "run", "--shard-per-gpu", "--gpus", str(per),
                                          "--set", "engine.device=cpu", "--set", "services.match=stub",
                                          "--set", "services.explain=echo", "--set", "kube.mode=kubeconfig",
                                          "--set", f"kube.kubeconfig={kc}", "--set", f"health.port={port}",
                                          "--set", "health.host=127.0.0.1",
                                          "--set", f"patterns.cache_dir={workdir}/patterns{g}",
                                          "--set", "operator.workers=64"], env=env), port))
        import urllib.request

        def up(pt):
            try:
                return urllib.request.urlopen(f"http://127.0.0.1:{pt}/q/health/ready", timeout=1).status == 200
            except OSError:
                return False
        assert wait(lambda: all(up(pt + i) for _, pt in ops for i in range(per)), 180), "shards did not come up"
        # the failures arrive as they would from many kubelets: concurrent status merge patches
        st = failed_pod("x", finished_at="2025-08-29T10:00:00Z")["status"]

        def cpu_s(pid):   # user + system CPU seconds of a process (Linux /proc)
            try:
                f = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
                return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")
            except OSError:
                return float("nan")
        c0 = [cpu_s(p.pid) for p in srvs]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(16) as ex:
            list(ex.map(lambda i: kubes[i % apiservers].patch_status(PODS, names[i], "default", st), range(failures)))
        t_inj = time.perf_counter() - t0

        def analysed():
            return sum(1 for k in kubes for p in k.list(PODS, "default")
                       if "podmortem.io/analysis" in ((p.get("metadata") or {}).get("annotations") or {}))
        end = time.perf_counter() + timeout_s
        n_done = 0
        while time.perf_counter() < end:
            # a LIST of every pod is the API server's most expensive request: poll it sparingly
            # (the servers are shared with the shards under test)
            time.sleep(0.5)
            n_done = analysed()
            if n_done >= failures:
                break
        elapsed = time.perf_counter() - t0
        srv_cpu = [cpu_s(p.pid) - c for p, c in zip(srvs, c0)]
        time.sleep(2.0)   # let the last Events land before counting them
        per_pod = Counter(e.get("regarding", {}).get("name") for k in kubes for e in k.list(EVENTS, "default")
                          if e.get("reason") == "PodmortemAnalysisComplete"
                          and e.get("regarding", {}).get("kind") == "Pod")
        ms = [1e3 * c / (failures / apiservers) for c in srv_cpu]
        return {"topology": f"{apiservers} REST API server(s) x shard-per-gpu {per} (stub log-parser + echo explainer)",
                "failures": failures, "analysed": n_done, "analyses_per_s": round(failures / elapsed, 1),
                "inject_s": round(t_inj, 2), "elapsed_s": round(elapsed, 2),
                # each API server's CPU time over the run: its ms per analysis bound the rate one
                # server process can sustain (1000 / ms analyses/s); the servers add up
                "apiserver_cpu_s": [round(c, 2) for c in srv_cpu],
                "apiserver_cpu_ms_per_analysis": [round(m, 2) for m in ms],
                "apiserver_capacity_analyses_per_s": round(sum(1e3 / m for m in ms if m > 0), 1),
                "complete_events_per_pod": dict(Counter(per_pod.get(n, 0) for n in names))}
    finally:
        for op, _ in ops:
            op.send_signal(signal.SIGTERM)
        for op, _ in ops:
            try:
                op.wait(60)
            except subprocess.TimeoutExpired:
                op.kill()
        for k in kubes:
            k.close() if hasattr(k, "close") else None
        for p in srvs:
            p.terminate()
            p.wait(30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--failures", type=int, default=2000)
    ap.add_argument("--crs", type=int, default=20)
    ap.add_argument("--workers", type=int, default=64)
    ap.add_argument("--match", choices=["stub", "cpu"], default="stub")
    ap.add_argument("--pool", type=int, default=0,
                    help="engines in N worker processes behind the EnginePool (the `run --gpus N` topology: "
                         "CPU matcher + echo explainer per worker) instead of in this process")
    ap.add_argument("--log-kb", type=int, default=0, help="pad every pod log to this size (KiB)")
    ap.add_argument("--shard-per-gpu", type=int, default=0,
                    help="N operator shard processes (`run --shard-per-gpu`, CPU stub engines) on REST API server "
                         "processes (--apiservers), instead of everything in this process")
    ap.add_argument("--apiservers", type=int, default=1, help="API server processes the shards split over")
    a = ap.parse_args()
    if a.shard_per_gpu:
        import tempfile

        with tempfile.TemporaryDirectory() as d:
            print(json.dumps({"bench": "plumbing (BASELINE config 1)", **run_sharded(a.shard_per_gpu, a.failures, d,
                                                                                      log_kb=a.log_kb,
                                                                                      apiservers=a.apiservers)}))
        return
    s = load_settings(env={}, overrides={"patterns.cache_dir": "/tmp/oamd-plumbing", "health.enabled": False,
                                         "operator.workers": a.workers})
    fk = FakeKube()
    done = {}
    pool = None
    if a.pool:
        from operator_amd.engine.pool import EnginePool, PoolExplainService, PoolMatchService

        s.services.explain = "echo"
        s.services.match = "stub" if a.match == "stub" else "cpu"
        pool = EnginePool(s, catalog_library(), ["cpu"] * a.pool)
        assert pool.wait_ready(300) == a.pool, pool.health()
        match, explain = PoolMatchService(pool), PoolExplainService(pool)
    else:
        match = StubMatch() if a.match == "stub" else LocalMatchService(MatchEngine(catalog_library(), device="cpu"),
                                                                       max_wait_ms=2.0)
        explain = EchoExplainService()
    op = Operator(fk, s, match_service=match, explain_service=explain)
    op.pipeline.listeners.append(lambda monitor, pod, outcome: done.setdefault(pod["metadata"]["name"],
                                                                                 time.perf_counter()))
    op.start(http=False)
    fk.create(AIPROVIDERS, {"metadata": {"name": "stub", "namespace": "default"},
                            "spec": {"providerId": "stub", "modelId": "echo"}})
    # reconcile latency of fresh Podmortem CRs (the first one is the monitor used below)
    rec = []
    for i in range(a.crs):
        t0 = time.perf_counter()
        fk.create(PODMORTEMS, {"metadata": {"name": f"m{i}", "namespace": "default"},
                               "spec": {"podSelector": {"matchLabels": {"app": "demo" if i == 0 else f"x{i}"}},
                                        "aiAnalysisEnabled": True, "aiProviderRef": {"name": "stub"}}})
        ok = wait(lambda: (fk.get(PODMORTEMS, f"m{i}", "default").get("status") or {}).get("phase") == "Ready", 30)
        assert ok, "reconcile timed out"
        rec.append(time.perf_counter() - t0)
    names = [f"p{i}" for i in range(a.failures)]
    log = LOG
    if a.log_kb:
        filler = b"INFO request served in 3 ms from cache shard 7\n"
        log = filler * max(0, (a.log_kb * 1024 - len(LOG)) // len(filler)) + LOG
    for n in names:
        fk.create(PODS, running_pod(n, labels={"app": "demo"}))
        fk.set_log("default", n, log)
    t_fail = {}
    t0 = time.perf_counter()
    for n in names:
        cur = fk.get(PODS, n, "default")
        cur["status"] = failed_pod(n, finished_at="2025-08-29T10:00:00Z")["status"]
        t_fail[n] = time.perf_counter()
        fk.replace(PODS, cur)
    assert wait(lambda: len(done) >= a.failures, 600), f"only {len(done)} of {a.failures} analysed"
    op.drain(120)
    elapsed = time.perf_counter() - t0
    lat = sorted(done[n] - t_fail[n] for n in names)
    op.stop()
    shm = None
    if pool is not None:
        h = pool.health()["workers"]
        shm = {"shm_logs": sum(w["shm_logs"] for w in h), "shm_fallbacks": sum(w["shm_fallbacks"] for w in h)}
        pool.close()
    print(json.dumps({"pool_log_transfer": shm, "bench": "plumbing (BASELINE config 1)", "failures": a.failures,
                      "topology": (f"EnginePool x{a.pool} ({'stub' if a.match == 'stub' else 'CPU'} matcher + echo)"
                                   if a.pool else "in-process"),
                      "log_bytes": len(log),
                      "analyses_per_s": round(a.failures / elapsed, 1),
                      "p50_ms": round(statistics.median(lat) * 1e3, 1), "p99_ms": round(lat[int(0.99 * len(lat))] * 1e3, 1),
                      "reconcile_p50_ms": round(statistics.median(rec) * 1e3, 2),
                      "reconcile_max_ms": round(max(rec) * 1e3, 2), "crs": a.crs,
                      "engines": ("stub log-parser" if a.match == "stub" else "CPU matcher (catalog)") +
                      " + echo explainer", "pipeline_workers": a.workers}))


if __name__ == "__main__":
    main()
