"""Pattern schema / compiler / DFA / scorer (CPU tier)."""
import re

import numpy as np
import pytest

from operator_amd.engine.match import MatchEngine
from operator_amd.ops import patterns as native_patterns
from operator_amd.patterns import oracle
from operator_amd.patterns.compiler import compile_patterns, required_cover
from operator_amd.patterns.schema import PatternError, PatternSet
from operator_amd.patterns.synth import LogFactory, catalog_library, library_yaml, synthetic_library


def _dfa_scan(d, text: bytes):
    """Python walk of the native DFA table (what ac_scan does on the device)."""
    C = 1 << d["log2_classes"]
    tab = np.frombuffer(d["table"], dtype=np.uint16).reshape(-1, C)
    cls = np.frombuffer(d["cls_map"], dtype=np.uint8)
    off = np.frombuffer(d["out_off"], dtype=np.uint32)
    ids = np.frombuffer(d["out_ids"], dtype=np.uint32)
    s = 0
    out = []
    for i, b in enumerate(text):
        e = int(tab[s, cls[b]])
        s = e & 0x7FFF
        if e & 0x8000:
            for k in range(off[s], off[s + 1]):
                out.append((i, int(ids[k])))
    return out


def test_dfa_matches_naive_find():
    facs = [b"he", b"she", b"his", b"hers", b"connection refused", b"refused", b"a"]
    d = native_patterns().compile_dfa(facs)
    text = b"ushers Connection REFUSED: a his"
    got = sorted(_dfa_scan(d, text))
    want = []
    low = text.lower()
    for fi, f in enumerate(facs):
        i = low.find(f)
        while i >= 0:
            want.append((i + len(f) - 1, fi))
            i = low.find(f, i + 1)
    assert got == sorted(want)
    # BFS numbering: depth is non-decreasing
    assert d["depth"] == sorted(d["depth"])


def test_dfa_rejects_bad_factors():
    P = native_patterns()
    with pytest.raises(ValueError):
        P.compile_dfa([b"a\nb"])
    with pytest.raises(ValueError):
        P.compile_dfa([b""])
    with pytest.raises(ValueError):
        P.compile_dfa([b"x" * 65])


def test_nul_resets_dfa():
    d = native_patterns().compile_dfa([b"abcd"])
    assert _dfa_scan(d, b"ab\0cd") == []
    assert _dfa_scan(d, b"ab\0abcd") == [(6, 0)]


def test_required_cover():
    assert required_cover(rb"java\.lang\.OutOfMemoryError: (a|b)") == [b"java.lang.OutOfMemoryError: "]
    assert sorted(required_cover(rb"foo bar|baz qux")) == [b"baz qux", b"foo bar"]
    assert required_cover(rb"a.b") is None
    assert required_cover(rb"(abc)+def") in ([b"abc"], [b"def"])


def test_schema_validation():
    with pytest.raises(PatternError):
        PatternSet.from_dicts([{"id": "x", "severity": "BAD", "primary_pattern": {"literal": "a"}}])
    with pytest.raises(PatternError):
        PatternSet.from_dicts([{"id": "x", "primary_pattern": {"literal": "a", "regex": "b"}}])
    with pytest.raises(PatternError):
        PatternSet.from_dicts([{"id": "x", "primary_pattern": {"regex": "("}}])
    ps = PatternSet.from_dicts([{"id": "x", "primaryPattern": {"literal": "boom", "confidence": 0.7},
                                 "secondaryPatterns": [{"literal": "bang", "weight": 0.2, "proximityWindow": 3}]}])
    assert ps.patterns[0].secondary[0].window == 3
    ys = PatternSet.from_yaml_text(library_yaml(20))
    assert len(ys) == 20 and ys.libraries == ["synthetic"]


def test_load_dir_enabled_filter(tmp_path):
    (tmp_path / "a").mkdir()
    (tmp_path / "a" / "one.yaml").write_text(library_yaml(3, library_id="one"))
    (tmp_path / "two.yml").write_text(library_yaml(4, seed=1, library_id="two"))
    assert len(PatternSet.load_dir(tmp_path)) == 7
    assert len(PatternSet.load_dir(tmp_path, enabled=["two"])) == 4


def _compare_engine_to_oracle(eng, docs):
    cp = eng.cp
    evs, _ = eng.events(docs)
    ref = oracle.analyze_docs(cp, docs)
    assert len(evs) == len(ref)
    for a, b in zip(evs, ref):
        assert [(e.pattern, e.line) for e in a] == [(e.pattern, e.line) for e in b]
        assert np.allclose([e.score for e in a], [e.score for e in b])


def test_cpu_engine_matches_oracle_catalog():
    ps = catalog_library()
    fac = LogFactory(n_patterns=len(ps), seed=3, pool_lines=256)
    docs, truth = fac.batch(6, 6000, n_failures=4)
    docs.append(b"")
    docs.append(b"no newline at end: Connection refused")
    eng = MatchEngine(ps, device="cpu")
    _compare_engine_to_oracle(eng, docs)
    res = eng.analyze(docs)
    for r, t in zip(res, truth):
        found = {e.matched_pattern.id for e in r.events}
        for pid in t:
            assert pid in found, (pid, found)
    assert res[-2].summary.highest_severity is None and res[-2].summary.total_events == 0
    assert res[-1].events[0].matched_pattern.id == "conn-refused"
    assert res[-1].events[0].line_number == 1


def test_native_scorer_equals_python_scorer():
    ps = synthetic_library(120, seed=5)
    fac = LogFactory(n_patterns=120, seed=5, pool_lines=256)
    docs, _ = fac.batch(5, 20000, n_failures=8)
    a = MatchEngine(ps, device="cpu", use_native_scorer=True)
    b = MatchEngine(ps, device="cpu", use_native_scorer=False)
    ea, _ = a.events(docs)
    eb, _ = b.events(docs)
    assert [[(e.pattern, e.line, round(e.score, 12)) for e in d] for d in ea] == \
           [[(e.pattern, e.line, round(e.score, 12)) for e in d] for d in eb]


def test_scoring_proximity():
    ps = PatternSet.from_dicts([{
        "id": "p", "severity": "HIGH", "primary_pattern": {"literal": "boom", "confidence": 0.8},
        "secondary_patterns": [{"literal": "bang", "weight": 1.0, "proximity_window": 3}]}])
    cp = compile_patterns(ps)
    doc = b"boom\nx\nbang\nx\nx\nx\nx\nx\nboom\n"
    ev = oracle.score_doc(cp, oracle.doc_hits(cp, doc))
    # line 0: bang at distance 2 -> bonus 1*(1-2/4)=0.5 -> 0.8*1.5/2 = 0.6 ; line 8: distance 6 > 3 -> 0.4
    assert [(e.line, round(e.score, 6)) for e in ev] == [(0, 0.6), (8, 0.4)]


def test_case_sensitive_literal_is_verified():
    ps = PatternSet.from_dicts([{"id": "cs", "primary_pattern": {"literal": "FATAL", "ignore_case": False}}])
    eng = MatchEngine(ps, device="cpu")
    evs, _ = eng.events([b"fatal\nFATAL\nFaTaL"])
    assert [e.line for e in evs[0]] == [1]


def test_reorder_dfa_preserves_matches_and_raises_hot_coverage():
    """Profile-guided renumbering (reorder_dfa) permutes states only: every match is
    unchanged, the root stays state 0, and the sampled visits move into the hot prefix."""
    ps = synthetic_library(200, seed=3)
    cp = compile_patterns(ps)
    d = cp.dfa
    fac = LogFactory(n_patterns=200, seed=5)
    sample = b"".join(fac.batch(4, 16 * 1024, n_failures=3)[0])
    hot = 64
    r = native_patterns().reorder_dfa(d["table"], d["out_off"], d["out_ids"], d["log2_classes"], d["num_states"],
                                      d["cls_map"], sample, hot)
    assert r["hot_after"] >= r["hot_before"]
    assert r["sampled"] == len(sample)
    d2 = dict(d, table=r["table"], out_off=r["out_off"], out_ids=r["out_ids"])
    text = b"".join(LogFactory(n_patterns=200, seed=9).batch(3, 8 * 1024, n_failures=3)[0])
    text += b" ".join(cp.factors[:50])  # every one of these must match
    assert _dfa_scan(d2, text) == _dfa_scan(d, text)
    # root row: transitions out of state 0 on the same byte class lead to the same factors
    C = 1 << d["log2_classes"]
    t1 = np.frombuffer(d["table"], np.uint16).reshape(-1, C)
    t2 = np.frombuffer(r["table"], np.uint16).reshape(-1, C)
    assert ((t1[0] & 0x8000) == (t2[0] & 0x8000)).all()


def _chain_scan(d, chain: bytes, text: bytes, hot: int):
    """The kernel's exact re-walk (csrc/kernels/scan.hip slow_sub): cold states follow
    the chain byte when its class matches, the table otherwise."""
    C = 1 << d["log2_classes"]
    tab = np.frombuffer(d["table"], dtype=np.uint16).reshape(-1, C)
    cls = np.frombuffer(d["cls_map"], dtype=np.uint8)
    ch = np.frombuffer(chain, dtype=np.uint8)
    s, out, hits = 0, [], 0
    for i, b in enumerate(text):
        c = int(cls[b])
        x = int(ch[s])
        if s >= hot and (x & 0x40) and (x & 0x3F) == c:
            e, hits = (s + 1) | ((x & 0x80) << 8), hits + 1
        else:
            e = int(tab[s, c])
        s = e & 0x7FFF
        if e & 0x8000:
            out.append((i, s))
    return out, hits


def test_reorder_dfa_chains_cold_states_along_pattern_literals():
    """Cold states are numbered along trie paths (a state's most-visited goto child is the
    next state), and dfa_chain's bytes name the class of that step exactly: a walk that
    follows them equals the table walk, and a failure line's excursion through cold states
    is mostly chain steps (no table read)."""
    ps = synthetic_library(200, seed=3)
    cp = compile_patterns(ps)
    d = cp.dfa
    S, l2c = d["num_states"], d["log2_classes"]
    fac = LogFactory(n_patterns=200, seed=5)
    sample = b"".join(fac.batch(4, 16 * 1024, n_failures=3)[0])
    hot = 64
    r = native_patterns().reorder_dfa(d["table"], d["out_off"], d["out_ids"], l2c, S, d["cls_map"], sample, hot)
    d2 = dict(d, table=r["table"], out_off=r["out_off"], out_ids=r["out_ids"])
    chain = native_patterns().dfa_chain(r["table"], l2c, S)
    assert len(chain) >= (S + 15) // 16 * 16 + 16 and len(chain) % 16 == 0
    C = 1 << l2c
    tab = np.frombuffer(r["table"], np.uint16).reshape(-1, C)
    ch = np.frombuffer(chain, np.uint8)[:S]
    v = np.nonzero(ch & 0x40)[0]
    assert len(v) > S // 2
    assert ((tab[v, ch[v] & 0x3F].astype(np.int64)) == ((v + 1) | ((ch[v].astype(np.int64) & 0x80) << 8))).all()
    text = b"".join(LogFactory(n_patterns=200, seed=9).batch(3, 8 * 1024, n_failures=3)[0])
    text += b" ".join(cp.factors[:50])
    got, hits = _chain_scan(d2, chain, text, hot)
    want = [(i, e & 0x7FFF) for i, e in ((i, int(x)) for i, x in enumerate(_table_entries(d2, text))) if e & 0x8000]
    assert got == want
    assert hits > 0
    # the unprofiled (BFS) numbering gets valid, if few, chain bytes too
    ch0 = np.frombuffer(native_patterns().dfa_chain(d["table"], l2c, S), np.uint8)[:S]
    t0 = np.frombuffer(d["table"], np.uint16).reshape(-1, C)
    v0 = np.nonzero(ch0 & 0x40)[0]
    assert ((t0[v0, ch0[v0] & 0x3F] & 0x7FFF).astype(np.int64) == v0 + 1).all()


def _table_entries(d, text: bytes):
    C = 1 << d["log2_classes"]
    tab = np.frombuffer(d["table"], dtype=np.uint16).reshape(-1, C)
    cls = np.frombuffer(d["cls_map"], dtype=np.uint8)
    s, out = 0, []
    for b in text:
        e = int(tab[s, cls[b]])
        out.append(e)
        s = e & 0x7FFF
    return out


def test_log_factory_injects_signatures_of_the_scanned_library_for_any_seed():
    """Benchmark workload invariance: whatever the factory's seed (bench.py seeds it per
    rank and shard), every injected failure is a signature of synthetic_library(n, 0),
    so each shard and rank analyses equally heavy failures."""
    from operator_amd.engine.match import MatchEngine
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    eng = MatchEngine(synthetic_library(1000, seed=0), device="cpu")
    for seed in (0, 1, 3, 101):
        docs, truth = LogFactory(n_patterns=1000, seed=seed, pool_lines=256).batch(3, 8 * 1024, n_failures=3,
                                                                                  seed=seed + 7)
        for r, t in zip(eng.analyze(docs), truth):
            assert set(t) <= {e.matched_pattern.id for e in r.events}, (seed, t)


def test_pipelined_analyze_sub_batches_cover_the_batch_in_order():
    """MatchEngine._sub_batches (the GPU analyze pipeline's split): doc-aligned, contiguous,
    non-empty, about PIPE_SUB_BYTES each, None below PIPE_MIN_BYTES or with the pipeline
    off (the split logic itself touches no GPU: the device is only compared)."""
    import torch

    eng = MatchEngine(catalog_library(), device="cpu")
    assert eng._sub_batches([b"x" * 10] * 4) is None            # CPU engine: never split
    eng.device = torch.device("cuda")
    eng.PIPE_MIN_BYTES, eng.PIPE_SUB_BYTES = 1000, 300
    docs = [b"a" * n for n in (100, 250, 40, 0, 600, 10, 10, 200, 90)]
    subs = eng._sub_batches(docs)
    assert subs[0][0] == 0 and subs[-1][1] == len(docs)
    assert all(lo < hi for lo, hi in subs) and all(a[1] == b[0] for a, b in zip(subs, subs[1:]))
    total = sum(map(len, docs))
    assert len(subs) <= -(-total // eng.PIPE_SUB_BYTES)
    assert eng._sub_batches(docs[:2]) is None                  # below PIPE_MIN_BYTES
    eng.PIPE_SUB_BYTES = 0
    assert eng._sub_batches(docs) is None                      # pipeline off
