"""Engine pool (one engine process per device) on the CPU tier: routing, parity
with the in-process engines, pattern broadcast, and the §5.3 health loop —
a worker that crashes or hangs is drained, its in-flight requests finish on the
survivors, and it is respawned."""
import time

import pytest

from operator_amd.api.models import AIProviderConfig, PodFailureData
from operator_amd.config import load_settings
from operator_amd.engine.match import MatchEngine
from operator_amd.engine.pool import EnginePool, PoolExplainService, PoolMatchService, WorkerDied
from operator_amd.kube.fake import failed_pod
from operator_amd.patterns.schema import PatternSet
from operator_amd.patterns.synth import LogFactory, catalog_library

LOG_OOM = "\n".join(["starting app", "loading config"] * 20 + [
    "java.lang.OutOfMemoryError: Java heap space", "\tat com.example.Cache.grow(Cache.java:42)"] + ["tick"] * 10)


def _settings(**extra):
    ov = {"engine.model": "tiny", "engine.device": "cpu", "engine.kv_cache_gb": 0.02, "engine.use_graphs": False,
          "engine.max_context": 512, "engine.max_prompt_tokens": 256, "engine.max_batch": 8,
          "services.explain": "local", "services.match": "cpu", "operator.workers": 4,
          "services.match_batch_wait_ms": 1.0}
    ov.update(extra)
    return load_settings(env={}, overrides=ov)


@pytest.fixture(scope="module")
def pool():
    p = EnginePool(_settings(), catalog_library(), ["cpu", "cpu"], heartbeat_s=0.2, heartbeat_timeout_s=20.0,
                   max_restarts=2)
    try:
        assert p.wait_ready(600) == 2, p.health()
        yield p
    finally:
        p.close()


def _data(name, log=LOG_OOM):
    return PodFailureData(pod=failed_pod(name), logs=log, events=[])


def test_pool_match_matches_in_process_engine(pool):
    ms = PoolMatchService(pool)
    eng = MatchEngine(catalog_library(), device="cpu")
    fac = LogFactory(n_patterns=30, seed=3)
    docs, _ = fac.batch(6, 8 * 1024, n_failures=2, seed=5)
    for i, d in enumerate(docs):
        got = ms.analyze(_data(f"p{i}", d.decode()))
        want = eng.analyze([d], [(f"p{i}", "default")])[0]
        assert got.to_obj()["summary"] == want.to_obj()["summary"]
        assert [e["matchedPattern"]["id"] for e in got.to_obj()["events"]] == \
               [e["matchedPattern"]["id"] for e in want.to_obj()["events"]]
        assert [e["context"] for e in got.to_obj()["events"]] == [e["context"] for e in want.to_obj()["events"]]
    # the logs travelled through the workers' shared-memory rings, not the pickled queue
    assert sum(w["shm_logs"] for w in pool.health()["workers"]) >= len(docs)


def test_log_arena_ring_allocation():
    """The controller-side ring: in-order reclaim, wrap-around, fallback when full."""
    from operator_amd.engine.pool import _LogArena

    a = _LogArena(1000)
    try:
        assert a.put(1, b"a" * 250) == 0 and a.put(2, b"b" * 200) == 250
        assert a.put(3, b"c" * 260) is None                 # > size // 4: pickled instead
        assert a.put(3, b"c" * 250) == 450 and a.put(4, b"d" * 250) == 700
        assert a.put(5, b"e" * 100) is None                 # 950 + 100 > 1000 and the tail is 0
        a.release(2)                                        # out of order: 1 still holds the tail
        assert a.tail == 0 and a.put(5, b"e" * 100) is None
        a.release(1)                                        # reclaims 1 and 2: tail -> 450
        assert a.tail == 450
        assert a.put(5, b"e" * 100) == 0                    # wraps
        assert bytes(a.shm.buf[0:100]) == b"e" * 100 and bytes(a.shm.buf[450:700]) == b"c" * 250
        assert a.put(6, b"f" * 250) == 100                  # [100, 350) < tail 450
        assert a.put(7, b"g" * 100) is None                 # would reach the tail
        for r in (3, 4, 5, 6):
            a.release(r)
        assert a.head == a.tail == 0 and a.put(8, b"h" * 250) == 0
        assert a.copied == 7 and a.fallbacks == 4
    finally:
        a.close()


def test_pool_explain_and_routing(pool):
    ms, es = PoolMatchService(pool), PoolExplainService(pool)
    res = ms.analyze(_data("exp"))
    assert res.summary.highest_severity in ("CRITICAL", "HIGH")
    outs = es.explain_many([(res, AIProviderConfig(max_tokens=6, temperature=0.0))] * 4)
    assert all(o.explanation for o in outs)
    # greedy decoding is deterministic across workers
    assert len({o.explanation for o in outs}) == 1
    # both workers served traffic (least-outstanding routing under concurrency)
    futs = [pool.submit_match(_data(f"r{i}")) for i in range(16)]
    assert all(f.result(120).summary.highest_severity == res.summary.highest_severity for f in futs)


def test_pool_worker_stats(pool):
    es = PoolExplainService(pool)
    before = pool.worker_stats()
    assert len(before) == 2 and all("llm" in w for w in before)
    res = PoolMatchService(pool).analyze(_data("stats"))
    es.explain_many([(res, AIProviderConfig(max_tokens=4, temperature=0.0, caching_enabled=False))] * 3)
    after = pool.worker_stats()
    gen = sum(w["llm"]["decode_tokens"] for w in after) - sum(w["llm"]["decode_tokens"] for w in before)
    assert gen >= 3 * 3                       # 4 tokens each: 1 from the prefill + 3 decode steps
    assert all(len(w.inflight) == 0 for w in pool.workers)   # stats requests do not linger


def test_pool_pattern_broadcast(pool):
    ms = PoolMatchService(pool)
    custom = PatternSet.from_yaml_text("""
metadata: {library_id: custom}
patterns:
  - id: zz-custom
    name: Custom marker
    severity: CRITICAL
    primary_pattern: {regex: "ZZ_CUSTOM_FAILURE_[0-9]+"}
""")
    ms.swap_engine(custom)
    time.sleep(0.5)
    r = ms.analyze(_data("c", "ok\nZZ_CUSTOM_FAILURE_42\nbye"))
    assert [e.matched_pattern.id for e in r.events] == ["zz-custom"]
    ms.swap_engine(catalog_library())
    time.sleep(0.5)


def test_pool_crash_requeues_and_respawns(pool):
    before = pool.stats["deaths"]
    futs = [pool.submit_match(_data(f"c{i}")) for i in range(24)]
    pool.inject_crash(0)
    results = [f.result(300) for f in futs]
    assert all(r.summary.highest_severity for r in results)
    deadline = time.time() + 120
    while pool.stats["deaths"] == before and time.time() < deadline:
        time.sleep(0.1)
    assert pool.stats["deaths"] == before + 1
    assert pool.wait_ready(600) == 2, pool.health()
    assert pool.workers[0].restarts >= 1


def test_pool_hang_detected(pool):
    before = pool.stats["deaths"]
    pool.inject_hang(1)
    deadline = time.time() + 120
    while pool.stats["deaths"] == before and time.time() < deadline:
        time.sleep(0.2)
    assert pool.stats["deaths"] == before + 1
    assert pool.wait_ready(600) == 2, pool.health()
    assert PoolMatchService(pool).analyze(_data("after-hang")).summary.highest_severity


def test_pool_start_failure_is_fatal():
    p = EnginePool(_settings(**{"engine.model": "no-such-model"}), catalog_library(), ["cpu"], heartbeat_s=0.2,
                   max_restarts=3)
    try:
        assert p.wait_ready(300) == 0
        deadline = time.time() + 60
        while p.workers[0].alive and time.time() < deadline:
            time.sleep(0.1)
        assert not p.workers[0].alive and "fatal" in p.workers[0].info
        with pytest.raises(WorkerDied):
            p.submit_match(_data("x")).result(10)
    finally:
        p.close()


def test_pool_tp2_replica_matches_tp1_engine():
    """engine.tp=2: one explanation replica over two ranks (leader + follower,
    lock-stepped through the control group, gloo collectives on the CPU tier)
    gives the same tokens as the in-process TP=1 engine; a follower crash takes
    the whole replica down and it is respawned."""
    from operator_amd.engine import factory

    ov = {"engine.dtype": "float32", "engine.model": "tiny-gqa4", "engine.tp": 2}
    s1 = _settings(**{"engine.dtype": "float32", "engine.model": "tiny-gqa4"})
    res = MatchEngine(catalog_library(), device="cpu").analyze([LOG_OOM.encode()], [("tp", "default")])[0]
    cfgs = [AIProviderConfig(max_tokens=8, temperature=0.0), AIProviderConfig(max_tokens=8, temperature=0.3)]
    ref = factory.build_explain_service(s1)
    try:
        want = [ref.explain(res, c).explanation for c in cfgs]
    finally:
        ref.ee.close(join_s=10)
    p = EnginePool(_settings(**ov), catalog_library(), ["cpu", "cpu"], roles=("explain",), heartbeat_s=0.2,
                   heartbeat_timeout_s=20.0, max_restarts=1)
    try:
        assert len(p.workers) == 1 and p.workers[0].follower_devices == ["cpu"]
        assert p.wait_ready(600) == 1, p.health()
        es = PoolExplainService(p, timeout_s=300)
        got = [o.explanation for o in es.explain_many([(res, c) for c in cfgs])]
        assert got == want
        before = p.stats["deaths"]
        p.workers[0].followers[0].kill()
        deadline = time.time() + 120
        while p.stats["deaths"] == before and time.time() < deadline:
            time.sleep(0.1)
        assert p.stats["deaths"] == before + 1
        assert p.wait_ready(600) == 1, p.health()
        assert es.explain(res, cfgs[0]).explanation == want[0]
    finally:
        p.close()


def test_engine_loop_collective_timeout_is_fatal():
    """A timed-out TP collective makes the engine loop stop serving (fatal), fail every
    waiter, and exit its thread: the pool worker then dies and is respawned."""
    import threading

    from operator_amd.engine.explain import EngineLoop
    from operator_amd.parallel.custom_ar import CollectiveTimeout

    class _Req:
        def __init__(self):
            self.error, self.done, self.event = None, False, threading.Event()

    class _LLM:
        device = __import__("torch").device("cpu")

        def __init__(self):
            self.running, self.waiting = [_Req()], [_Req()]

        def has_work(self):
            return True

        def step(self):
            raise CollectiveTimeout("peer did not arrive")

    llm = _LLM()
    reqs = llm.running + llm.waiting
    loop = EngineLoop(llm)
    loop.start()
    loop.join(5)
    assert not loop.is_alive()
    assert isinstance(loop.fatal, CollectiveTimeout)
    assert all(r.done and r.event.is_set() and "engine failure" in r.error for r in reqs)
