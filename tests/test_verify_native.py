"""Native N3/N4 (csrc/patterns/verify.cpp + operator_amd/patterns/nfa.py) against
Python: the Pike-VM verifier must give exactly `re.search(line) is not None` for
every regex it accepts (anything else is left to `re`), and the native context
windows must equal the Python reference `_context`."""
import random
import re

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from operator_amd.engine.match import _context
from operator_amd.ops import patterns
from operator_amd.patterns.nfa import compile_nfa

FIXED = [
    rb"OutOfMemoryError", rb"exit code \d+", rb"(?i)connection (refused|reset)", rb"^FATAL\b", rb"timeout$",
    rb"[A-Z][a-z]+Exception: .*", rb"\bpanic: ", rb"fail(ed|ure)?", rb"a{2,4}b", rb"x*?y+?", rb"\d{3}-\d{4}",
    rb"[^\s]+@[^\s]+", rb"\Berror", rb"(ab|cd)*ef", rb"(?i:disk)\s+full", rb"\Aerror\Z", rb"[.]\w+", rb"colou?r",
    rb"(a|b|)c", rb"", rb"(?s)a.b", rb"[\d\-_]+", rb"\W+", rb"caf\xc3\xa9",
]
UNSUPPORTED = [rb"(a)\1", rb"foo(?=bar)", rb"(?<!x)y", rb"(?(1)a|b)"]


def _lines(rng: random.Random, n: int):
    alphabet = b"abcdefxyzABEF0123456789 _-.:@\t\xc3\xa9"
    out = [b"", b"OutOfMemoryError", b"FATAL boot", b"connection REFUSED", b"exit code 137", b"aaab", b"aab",
           b"xxyy", b"555-1234", b"user@host", b"abef", b"cdabef", b"disk   FULL", b"error", b"a\nb", b"color"]
    for _ in range(n):
        out.append(bytes(rng.choice(alphabet) for _ in range(rng.randint(0, 40))))
    return out


def _check(rx: bytes, flags: int, lines) -> None:
    prog = compile_nfa(rx, flags)
    assert prog is not None, rx
    rs = patterns().RegexSet([prog])
    py = re.compile(rx, flags)
    for ln in lines:
        assert rs.search(0, ln) == (py.search(ln) is not None), (rx, flags, ln)


@pytest.mark.parametrize("rx", FIXED)
@pytest.mark.parametrize("flags", [0, re.IGNORECASE])
def test_nfa_matches_python_re(rx, flags):
    _check(rx, flags, _lines(random.Random(hash(rx) & 0xffff), 200))


@pytest.mark.parametrize("rx", UNSUPPORTED)
def test_unsupported_constructs_fall_back_to_re(rx):
    assert compile_nfa(rx) is None


_atoms = st.sampled_from([b"a", b"b", b"x", b"0", b".", b"\\d", b"\\w", b"\\s", b"[a-c]", b"[^ab]", b"[0-9x]",
                          b"\\b", b"^", b"$", b"A", b"-"])
_quants = st.sampled_from([b"", b"*", b"+", b"?", b"{1,3}", b"*?", b"{2}"])


@st.composite
def _flat(draw):
    """1-3 unquantified atoms: the body of a quantified group."""
    return b"".join(draw(_atoms) for _ in range(draw(st.integers(1, 3))))


@st.composite
def _regex(draw, depth=0):
    """Random regex in the verifier's subset, shaped so Python ``re`` (the oracle, a
    backtracking matcher) stays polynomial: a quantified group holds only a flat run of
    atoms -- never a nested quantifier or an alternation, the shapes that backtrack
    exponentially (e.g. ``(.|[^ab])*A``) -- while unquantified groups may nest and
    alternate freely."""
    parts = []
    for _ in range(draw(st.integers(1, 4))):
        kind = draw(st.integers(0, 6 if depth < 2 else 2))
        q = b""
        if kind <= 2:
            a = draw(_atoms)
            if a not in (b"\\b", b"^", b"$"):
                q = draw(_quants)
        elif kind == 3:
            a = b"(" + draw(_regex(depth + 1)) + b"|" + draw(_regex(depth + 1)) + b")"
        elif kind == 4:
            a = b"(" + draw(_regex(depth + 1)) + b")"
        else:
            a = b"(" + draw(_flat()) + b")"
            q = draw(_quants)
        parts.append(a + q)
    return b"".join(parts)


# derandomize: the same 300 examples every run, so the CPU tier's runtime is fixed
@settings(max_examples=300, deadline=None, derandomize=True)
@given(_regex(), st.lists(st.binary(min_size=0, max_size=24).map(lambda b: bytes(x % 128 for x in b if x != 10)),
                          min_size=1, max_size=12), st.booleans())
def test_nfa_property_random_regexes(rx, lines, icase):
    flags = re.IGNORECASE if icase else 0
    try:
        re.compile(rx, flags)
    except re.error:
        return
    prog = compile_nfa(rx, flags)
    if prog is None:
        return
    _check(rx, flags, lines + [b"ab0 x-A", b"", b"bbb", b"A0A"])


def test_native_contexts_equal_python():
    rng = random.Random(5)
    docs = [b"", b"one line no newline", b"a\nb\nc\n", b"\n\n\nx\n", b"first\nsecond\nthird\nfourth\nfifth",
            "café\nnaïve\n\xff\xfe bad utf8\n".encode("utf-8") + b"\xff\xfe\n"]
    for _ in range(20):
        docs.append(b"\n".join(bytes(rng.choice(b"abc xyz") for _ in range(rng.randint(0, 12)))
                               for _ in range(rng.randint(1, 9))))
    q = []
    for di, d in enumerate(docs):
        for off in sorted({0, len(d) // 2, max(0, len(d) - 1), len(d)} | {rng.randint(0, len(d)) for _ in range(3)}):
            for k in (0, 1, 2, 5):
                q.append((di, off, k))
    got = patterns().contexts(docs, [x[0] for x in q], [x[1] for x in q], [x[2] for x in q])
    for (di, off, k), (ctx, line) in zip(q, got):
        ref_ctx, ref_line = _context(docs[di], off, k)
        assert (list(ctx), line) == (ref_ctx, ref_line), (docs[di], off, k)


def test_fast_construct_equals_model_construct():
    """KModel.fast (the match engine's result builder) builds what model_construct builds."""
    from operator_amd.api.models import AnalysisEvent, AnalysisResult, AnalysisSummary, MatchedPattern

    mp = MatchedPattern.fast(id="oom", name="OOM", severity="HIGH")
    assert mp == MatchedPattern.model_construct(id="oom", name="OOM", severity="HIGH")
    assert mp.model_fields_set == {"id", "name", "severity"}
    ev = AnalysisEvent.fast(line_number=3, matched_pattern=mp, score=0.5, matched_line="x")
    want = AnalysisEvent.model_construct(line_number=3, matched_pattern=mp, score=0.5, matched_line="x")
    assert ev == want and ev.context == [] and ev.to_obj() == want.to_obj()
    e2 = AnalysisEvent.fast()
    assert e2.context is not ev.context            # default factories are per instance
    sm = AnalysisSummary.fast(total_events=2)
    r = AnalysisResult.fast(analysis_id="a", events=[ev], summary=sm)
    r0 = AnalysisResult.model_construct(analysis_id="a", events=[ev], summary=sm)
    assert r == r0 and r.to_obj() == r0.to_obj() and list(r.__dict__) == list(r0.__dict__)
    assert r.model_dump_json() == r0.model_dump_json()


def test_uuid4_strs_are_version4_uuids():
    import uuid

    from operator_amd.engine.match import uuid4_strs

    ids = uuid4_strs(500)
    assert len(set(ids)) == 500
    for s in ids:
        u = uuid.UUID(s)
        assert u.version == 4 and u.variant == uuid.RFC_4122 and str(u) == s
    assert uuid4_strs(0) == []


def test_lazy_analyze_equals_eager():
    """analyze(lazy=True) builds, per doc on first access, what the eager batch builds."""
    from operator_amd.engine.match import LazyResults, MatchEngine
    from operator_amd.patterns.synth import LogFactory, synthetic_library

    docs, _ = LogFactory(n_patterns=120, seed=3).batch(12, 6 * 1024, n_failures=2)
    eng = MatchEngine(synthetic_library(120, seed=0), device="cpu")
    pods = [(f"p{i}", "ns") for i in range(len(docs))]
    eager = eng.analyze(docs, pods)
    lazy = eng.analyze(docs, pods, lazy=True)
    assert isinstance(lazy, LazyResults) and len(lazy) == len(eager)
    strip = lambda r: {k: v for k, v in r.to_obj().items() if k not in ("analysisId", "metadata")}  # noqa: E731
    assert sum(len(r.events or []) for r in eager) > 0
    for i in (3, 0, len(docs) - 1):            # any order
        assert strip(lazy[i]) == strip(eager[i])
    assert [strip(r) for r in lazy] == [strip(r) for r in eager]
    assert lazy[2] is lazy[2] and lazy[-1] is lazy[len(docs) - 1]
    assert len({r.analysis_id for r in lazy}) == len(docs)
