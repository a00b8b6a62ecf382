"""GPU Aho-Corasick scan (ac_scan + scan_fixup) against the CPU oracle."""
import numpy as np
import pytest
import torch

from operator_amd.engine.match import MatchEngine
from operator_amd.patterns import oracle
from operator_amd.patterns.schema import PatternSet
from operator_amd.patterns.synth import LogFactory, catalog_library, synthetic_library

pytestmark = pytest.mark.gpu


def _rows(a):
    return sorted(map(tuple, np.asarray(a).tolist()))


@pytest.mark.parametrize("seg", [64, 256, 1024, 4096])
def test_raw_scan_equals_cpu_scan(seg):
    ps = PatternSet.from_dicts([
        {"id": "a", "primary_pattern": {"literal": "Connection refused"}},
        {"id": "b", "primary_pattern": {"literal": "refused"}},
        {"id": "c", "primary_pattern": {"literal": "x" * 64}},
        {"id": "d", "primary_pattern": {"literal": "ab"}},
    ])
    eng = MatchEngine(ps, device="cuda", seg_bytes=seg)
    docs = [
        b"",
        b"connection REFUSED\n" * 3,
        (b"y" * (seg - 9)) + b"Connection refused" + b"\n" + b"x" * 200,   # straddles a segment seam
        b"a" * (seg - 1) + b"b",                                             # doc exactly one segment long
        b"ab" * 700 + b"\n\n\nab",
        bytes(range(256)) * 3,
    ]
    gpu = eng.scan_gpu(docs)
    cpu = eng.scan_cpu(docs)
    assert _rows(gpu) == _rows(cpu)


def test_engine_matches_oracle_1k_patterns():
    ps = synthetic_library(1000, seed=0)
    fac = LogFactory(n_patterns=1000, seed=0)
    docs, truth = fac.batch(48, 40000, n_failures=5)
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024)
    evs, _ = eng.events(docs)
    ref = oracle.analyze_docs(eng.cp, docs)
    for a, b in zip(evs, ref):
        assert [(e.pattern, e.line) for e in a] == [(e.pattern, e.line) for e in b]
        assert np.allclose([e.score for e in a], [e.score for e in b])
    res = eng.analyze(docs)
    for r, t, d in zip(res, truth, docs):
        ids = {e.matched_pattern.id for e in r.events}
        assert set(t) <= ids
        assert r.metadata["totalLines"] == d.count(b"\n") + 1


@pytest.mark.parametrize("seg", [64, 1024])
def test_total_lines_from_gpu_newline_counts(seg):
    """AnalysisResult.metadata.totalLines comes from the scan's per-segment newline
    counts (no host re-read of the logs); it equals the host count for edge-case docs
    and for a batch large enough to use full-size segments."""
    eng = MatchEngine(catalog_library(), device="cuda", seg_bytes=seg)
    docs = [b"", b"\n", b"no newline at all", b"\n" * (3 * seg + 5), b"OOMKilled\n" * 999 + b"tail",
            (b"x" * (seg - 1) + b"\n") * 7, bytes(range(256)) * 9]
    for r, d in zip(eng.analyze(docs), docs):
        assert r.metadata["totalLines"] == d.count(b"\n") + 1
    big, _ = LogFactory(n_patterns=len(catalog_library()), seed=3, pool_lines=512).batch(600, 64 * 1024, n_failures=2)
    for r, d in zip(eng.analyze(big), big):
        assert r.metadata["totalLines"] == d.count(b"\n") + 1


def test_match_overflow_grows_and_rescans():
    ps = PatternSet.from_dicts([{"id": "e", "primary_pattern": {"literal": "e"}}])
    eng = MatchEngine(ps, device="cuda", seg_bytes=256, match_cap=64)
    docs = [b"eee\n" * 500]
    out = eng.scan_gpu(docs)
    assert out.shape[0] == 1500
    assert eng.match_cap >= 1500


def test_catalog_context_and_lines():
    eng = MatchEngine(catalog_library(), device="cuda", seg_bytes=256)
    doc = b"line one\nline two\nOOMKilled: container memory limit\nline four\n"
    r = eng.analyze([doc])[0]
    e = r.events[0]
    assert e.matched_pattern.id == "oom-killed"
    assert e.line_number == 3
    assert e.matched_line == "OOMKilled: container memory limit"
    assert e.context[0] == "line one" and e.context[-1] == "line four"
    assert r.summary.highest_severity == "CRITICAL"


def test_large_batch_throughput_smoke():
    """~64 MB through the scan; checks counts against a CPU count of one literal."""
    ps = synthetic_library(1000, seed=0)
    fac = LogFactory(n_patterns=1000, seed=1)
    docs, _ = fac.batch(512, 128 * 1024, n_failures=3)
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024)
    raw = eng.scan_gpu(docs)
    fid = eng.cp.factors.index(b"oomkilled")
    want = sum(d.lower().count(b"oomkilled") for d in docs)
    assert int((raw[:, 1] == fid).sum()) == want
    torch.cuda.synchronize()


def test_gpu_scorer_matches_host_scorer():
    """score.hip (score + rank + summary on the GPU) == the C++ host scorer."""
    from operator_amd.engine.match import MatchEngine
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    ps = synthetic_library(300, seed=2)
    fac = LogFactory(n_patterns=300, seed=4)
    docs, _ = fac.batch(24, 32 * 1024, n_failures=4, seed=9)
    docs.append(b"")  # empty doc
    g = MatchEngine(ps, device="cuda", gpu_scorer=True)
    h = MatchEngine(ps, device="cuda", gpu_scorer=False)
    eg, _ = g.events(docs)
    eh, _ = h.events(docs)
    assert len(eg) == len(eh)
    for a, b in zip(eg, eh):
        assert [(e.pattern, e.line) for e in a] == [(e.pattern, e.line) for e in b]
        assert all(abs(x.score - y.score) < 1e-9 for x, y in zip(a, b))
    ra = [r.to_obj()["summary"] for r in g.analyze(docs)]
    rb = [r.to_obj()["summary"] for r in h.analyze(docs)]
    assert ra == rb


def test_profiled_state_order_gives_identical_scan():
    """MatchEngine renumbers DFA states by visit count on the first scan
    (profile_bytes): the raw hits must equal the breadth-first-numbered DFA's."""
    ps = synthetic_library(1000, seed=0)
    docs, _ = LogFactory(n_patterns=1000, seed=4).batch(96, 32 * 1024, n_failures=3)
    a = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=0)
    b = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=1 << 20)
    ra, rb = a.scan_gpu(docs), b.scan_gpu(docs)
    assert b.hot_coverage is not None and b.hot_coverage[1] >= b.hot_coverage[0]
    assert len(ra) > 0 and _rows(ra) == _rows(rb)
    assert _rows(b.scan_gpu(docs[::-1])) == _rows(a.scan_gpu(docs[::-1]))


def test_scan_graph_replays_equal_eager_scans():
    """The captured scan tail (scan_graphs=True) returns what the eager launches return,
    across batches that share a graph bucket and batches that need a new one, and it
    falls back to the eager rescan on match overflow."""
    ps = synthetic_library(400, seed=1)
    fac = LogFactory(n_patterns=400, seed=6)
    batches = [fac.batch(n, kb * 1024, n_failures=3, seed=s)[0]
               for n, kb, s in ((32, 16, 1), (32, 16, 2), (30, 17, 3), (64, 64, 4), (5, 3, 5))]
    eager = MatchEngine(ps, device="cuda", seg_bytes=1024, scan_graphs=False, profile_bytes=0)
    graph = MatchEngine(ps, device="cuda", seg_bytes=1024, scan_graphs=True, profile_bytes=0)
    for docs in batches + batches[:2]:
        assert _rows(graph.scan_gpu(docs)) == _rows(eager.scan_gpu(docs))
        ra = [r.metadata["totalLines"] for r in graph.analyze(docs)]
        assert ra == [d.count(b"\n") + 1 for d in docs]
    assert graph.graph_replays >= 10 and eager.graph_replays == 0
    assert len(graph._graphs) < 2 * len(batches)
    small = MatchEngine(PatternSet.from_dicts([{"id": "e", "primary_pattern": {"literal": "e"}}]), device="cuda",
                        seg_bytes=256, match_cap=64, profile_bytes=0)
    assert small.scan_gpu([b"eee\n" * 500]).shape[0] == 1500 and small.match_cap >= 1500
    assert small.scan_gpu([b"eee\n" * 500]).shape[0] == 1500   # the grown cap: a graph again
