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


def test_line_prefix_equals_cumsum_and_replays():
    """line_prefix (decoupled look-back scan, line_index.hip) == an exclusive cumsum for
    tile-boundary lengths, twice on the same state buffer (the launcher's memset makes it
    replay-safe); doc_lines == per-doc differences."""
    from operator_amd.ops import kernels

    C = kernels()
    g = torch.Generator(device="cpu").manual_seed(7)
    for n in (1, 100, 4095, 4096, 4097, 262145, 1000003):
        cnt = torch.randint(0, 50, (n,), generator=g, dtype=torch.int32).cuda()
        ref = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(cnt.cpu().to(torch.int64), 0)])
        excl = torch.full((n + 1,), -1, dtype=torch.int64, device="cuda")
        st = torch.empty(C.line_prefix_state_words(n), dtype=torch.int64, device="cuda")
        for _ in range(2):
            C.line_prefix(cnt, excl, st)
            assert torch.equal(excl.cpu(), ref), n
            assert int(st[1]) == 0, n   # error word: no look-back gave up
        first = torch.tensor(sorted({0, n} | set(torch.randint(0, n + 1, (5,), generator=g).tolist())),
                             dtype=torch.int64)
        dn = torch.empty(len(first) - 1, dtype=torch.int64, device="cuda")
        C.doc_lines(excl, first.cuda(), dn)
        assert dn.cpu().tolist() == [int(ref[b] - ref[a]) for a, b in zip(first[:-1], first[1:])]


def test_context_spans_equal_host_contexts():
    """The +-k windows located on the GPU (context_spans + contexts_from_spans) equal the
    host's native `contexts` for every kind of edge: empty lines, lines longer than a
    64-byte step, a leading newline, no trailing newline, offsets at 0 / len / on a
    newline, k = 0..5 — and MatchEngine.analyze uses them for its results."""
    import random

    from operator_amd.ops import kernels, patterns

    rng = random.Random(11)

    def line():
        n = rng.choice([0, 0, 3, 20, 63, 64, 65, 130, 700])
        return bytes(rng.choice(b"abcdefgh \t\xc3\xa9") for _ in range(n))

    docs = []
    for i in range(40):
        ls = [line() for _ in range(rng.randrange(0, 30))]
        d = b"\n".join(ls)
        if i % 3 == 0:
            d = b"\n" + d
        if i % 4 == 1:
            d = d + b"\n"
        docs.append(d)
    docs[5] = b""
    docs[6] = b"\n\n\n"
    seg = 256
    P = patterns()
    total, first = P.plan_docs([len(d) for d in docs], seg)
    buf = bytearray(total)
    for d, f in zip(docs, first):
        buf[f * seg:f * seg + len(d)] = d
    text = torch.frombuffer(buf, dtype=torch.uint8).cuda()
    q_doc, q_off, q_k = [], [], []
    for di, d in enumerate(docs):
        offs = {0, len(d)} | {rng.randrange(0, len(d) + 1) for _ in range(6)} | \
               {i for i, c in enumerate(d) if c == 10 and rng.random() < 0.3}
        for o in sorted(offs):
            q_doc.append(di)
            q_off.append(o)
            q_k.append(rng.randrange(0, 6))
    q = torch.tensor(list(zip(q_doc, q_off, q_k)), dtype=torch.int64).cuda()
    out = torch.empty(len(q_doc), 4, dtype=torch.int64, device="cuda")
    base = torch.tensor(first[:-1], dtype=torch.int64).cuda() * seg
    lens = torch.tensor([len(d) for d in docs], dtype=torch.int64).cuda()
    kernels().context_spans(text, base, lens, q, out)
    got = P.contexts_from_spans(docs, q_doc, out.cpu().numpy())
    want = P.contexts(docs, q_doc, q_off, q_k)
    assert got == want
    # through the engine: eager analyze locates its windows on the GPU, same results as the host
    ps = synthetic_library(200, seed=3)
    fac = LogFactory(n_patterns=200, seed=9)
    bdocs = fac.batch(24, 8 * 1024, n_failures=3, seed=2)[0]
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=0)
    calls = {"n": 0}
    orig = eng._contexts_gpu

    def spy(*a):
        r = orig(*a)
        calls["n"] += r is not None
        return r
    eng._contexts_gpu = spy
    gpu = [r.to_obj() for r in eng.analyze(bdocs)]
    assert calls["n"] == 1
    host = MatchEngine(ps, device="cpu").analyze(bdocs)
    for a, b in zip(gpu, host):
        b = b.to_obj()
        assert [e["context"] for e in a["events"]] == [e["context"] for e in b["events"]]
        assert a["metadata"]["totalLines"] == b["metadata"]["totalLines"]


def test_context_windows_while_default_stream_is_busy():
    """The flagship runs the LLM's decode graphs on the default stream while the match
    engine scans on its own: the GPU context windows (lazy analyze) must not read their
    query / length buffers before those land (they are made on the scan stream)."""
    ps = synthetic_library(200, seed=3)
    bdocs = LogFactory(n_patterns=200, seed=9).batch(48, 8 * 1024, n_failures=3, seed=5)[0]
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=0)
    host = [r.to_obj() for r in MatchEngine(ps, device="cpu").analyze(bdocs)]
    for _ in range(3):
        torch.cuda._sleep(300_000_000)   # the default stream stays busy for ~0.1 s
        got = eng.analyze(bdocs, lazy=True)
        for i, b in enumerate(host):
            a = got[i].to_obj()
            assert [e["context"] for e in a["events"]] == [e["context"] for e in b["events"]]
    torch.cuda.synchronize()


def test_scan_match_overflow_regrows():
    small = MatchEngine(PatternSet.from_dicts([{"id": "e", "primary_pattern": {"literal": "e"}}]), device="cuda",
                        seg_bytes=256, match_cap=64, profile_bytes=0)
    assert small.scan_gpu([b"eee\n" * 500]).shape[0] == 1500 and small.match_cap >= 1500
    assert small.scan_gpu([b"eee\n" * 500]).shape[0] == 1500


def test_noisy_log_every_line_matches_equals_cpu_scan():
    """A pattern that hits every line of a noisy log (and one whose output set holds
    several patterns: "ERROR" ends both "ERROR" and "RROR"): the wave-aggregated match
    append (one counter atomic per wave and round) gives exactly the CPU scan's records."""
    ps = PatternSet.from_dicts([
        {"id": "err", "primary_pattern": {"literal": "ERROR"}},
        {"id": "rror", "primary_pattern": {"literal": "RROR"}},
        {"id": "ror", "primary_pattern": {"literal": "ROR"}},
        {"id": "id", "primary_pattern": {"literal": "req-"}},
    ])
    eng = MatchEngine(ps, device="cuda", seg_bytes=1024)
    docs = [b"".join(b"2025-08-29 ERROR req-%d failed\n" % i for i in range(40000)),
            b"ERRORERRORERROR\n" * 3000, b"", b"no match here\n" * 100]
    gpu = eng.scan_gpu(docs)
    cpu = eng.scan_cpu(docs)
    assert gpu.shape[0] == cpu.shape[0] > 4 * 40000
    assert _rows(gpu) == _rows(cpu)


@pytest.mark.parametrize("lazy", [False, True])
def test_pipelined_analyze_equals_one_batch(lazy):
    """A large batch is analysed in sub-batches (MatchEngine._analyze_pipelined: the next
    sub-batch's pack + H2D + scan on a worker thread in the other buffer set, while the
    host verifies, scores and builds the previous one): every result equals the
    one-batch analyze and the host path, and three back-to-back calls reuse both
    buffer sets."""
    ps = synthetic_library(300, seed=4)
    docs = LogFactory(n_patterns=300, seed=11).batch(61, 24 * 1024, n_failures=3, seed=3)[0]
    docs[7] = b""                      # an empty doc inside a sub-batch
    one = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=0)
    one.PIPE_SUB_BYTES = 0
    pipe = MatchEngine(ps, device="cuda", seg_bytes=1024, profile_bytes=0)
    pipe.PIPE_MIN_BYTES = 1
    pipe.PIPE_SUB_BYTES = 200 * 1024   # ~7 sub-batches
    subs = pipe._sub_batches(docs)
    assert subs is not None and len(subs) >= 5
    assert subs[0][0] == 0 and subs[-1][1] == len(docs) and all(a[1] == b[0] for a, b in zip(subs, subs[1:]))
    pods = [(f"pod-{i}", "ns") for i in range(len(docs))]

    def strip(o):
        o = dict(o)
        o.pop("analysisId", None)
        o.pop("analysis_id", None)
        m = dict(o.get("metadata", {}))
        m.pop("processingTimeMs", None)
        m.pop("engine", None)
        o["metadata"] = m
        return o

    want = [strip(r.to_obj()) for r in one.analyze(docs, pods)]
    host = [strip(r.to_obj()) for r in MatchEngine(ps, device="cpu").analyze(docs, pods)]
    assert want == host
    for _ in range(3):
        got = pipe.analyze(docs, pods, lazy=lazy)
        assert len(got) == len(docs)
        assert [strip(got[i].to_obj()) for i in range(len(docs))] == want
        assert pipe.last_timing["subs"] == len(subs)
    torch.cuda.synchronize()
