"""Property tests (hypothesis) for the pure pieces of the control and data planes
(SURVEY.md §4.2 "unit, CPU ... pytest plus hypothesis property tests").

Each property is checked against an independent, obviously-correct model:
  * DFA compile (N1) + walk == naive case-insensitive find, for random factor sets;
    profile-guided renumbering (reorder_dfa) never changes a match;
  * EventService.truncate: never longer than the cap, identity below it;
  * refresh-interval grammar (PatternLibraryReconciler.parseRefreshInterval);
  * LabelSelector semantics vs a direct set-based model;
  * the failure deduper (Q4 fix): bounded, and idempotent per (pod, finishedAt);
  * the status ring: newest first, capped at MAX_RECENT_FAILURES.
"""
import datetime as dt

import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from operator_amd.controller.events import truncate
from operator_amd.controller.failures import FailureDeduper
from operator_amd.controller.patternlibrary import parse_refresh_interval
from operator_amd.kube.resources import match_selector
from operator_amd.ops import patterns as native_patterns

SETTINGS = dict(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def _walk(d, text: bytes):
    C = 1 << d["log2_classes"]
    tab = np.frombuffer(d["table"], dtype=np.uint16).reshape(-1, C)
    cls = np.frombuffer(d["cls_map"], dtype=np.uint8)
    off = np.frombuffer(d["out_off"], dtype=np.uint32)
    ids = np.frombuffer(d["out_ids"], dtype=np.uint32)
    s, out = 0, []
    for i, b in enumerate(text):
        e = int(tab[s, cls[b]])
        s = e & 0x7FFF
        if e & 0x8000:
            out.extend((i, int(ids[k])) for k in range(off[s], off[s + 1]))
    return sorted(out)


def _naive(factors, text: bytes):
    low = text.lower()
    out = []
    for fi, f in enumerate(factors):
        f = f.lower()
        start = 0
        while True:
            i = low.find(f, start)
            if i < 0:
                break
            out.append((i + len(f) - 1, fi))
            start = i + 1
    return sorted(out)


# small alphabet (with case) so factors overlap and recur in the text
_alpha = st.sampled_from(list(b"abcAB .:-\n"))
_factor = st.lists(st.sampled_from(list(b"abcAB .:-")), min_size=1, max_size=6).map(bytes)


@settings(**SETTINGS)
@given(factors=st.lists(_factor, min_size=1, max_size=12, unique_by=lambda f: f.lower()),
       text=st.lists(_alpha, max_size=300).map(bytes))
def test_dfa_equals_naive_find(factors, text):
    d = native_patterns().compile_dfa(factors)
    assert _walk(d, text) == _naive(factors, text)


@settings(**SETTINGS)
@given(factors=st.lists(_factor, min_size=1, max_size=12, unique_by=lambda f: f.lower()),
       sample=st.lists(_alpha, max_size=400).map(bytes), text=st.lists(_alpha, max_size=300).map(bytes),
       hot=st.integers(1, 64))
def test_reorder_dfa_never_changes_matches(factors, sample, text, hot):
    d = native_patterns().compile_dfa(factors)
    r = native_patterns().reorder_dfa(d["table"], d["out_off"], d["out_ids"], d["log2_classes"], d["num_states"],
                                      d["cls_map"], sample, hot)
    assert r["hot_after"] >= r["hot_before"] - 1e-12
    assert _walk(dict(d, table=r["table"], out_off=r["out_off"], out_ids=r["out_ids"]), text) == _walk(d, text)


_words = st.sampled_from(["Root Cause", "Evidence", "Fix", "the pod", "OOMKilled", " ", "\n", "x" * 40, "é"])


@settings(**SETTINGS)
@given(text=st.one_of(st.none(), st.lists(_words, max_size=80).map("".join), st.text(max_size=2000)),
       cap=st.integers(3, 1200))
def test_truncate_never_exceeds_cap(text, cap):
    out = truncate(text, cap)
    if text is None:
        assert out is None
    elif len(text) <= cap:
        assert out == text
    else:
        assert len(out) <= cap
        if not ("Root Cause" in text and "Fix" in text):
            assert out == text[:cap - 3] + "..."


@settings(**SETTINGS)
@given(n=st.integers(0, 10 ** 6), unit=st.sampled_from("smhd"), upper=st.booleans(),
       pad=st.sampled_from(["", " ", "  "]))
def test_refresh_interval_units(n, unit, upper, pad):
    v = f"{pad}{n}{unit.upper() if upper else unit}{pad}"
    want = {"s": dt.timedelta(seconds=n), "m": dt.timedelta(minutes=n), "h": dt.timedelta(hours=n),
            "d": dt.timedelta(days=n)}[unit]
    assert parse_refresh_interval(v) == want


@settings(**SETTINGS)
@given(h=st.integers(0, 10 ** 4), m=st.integers(0, 10 ** 4))
def test_refresh_interval_hours_minutes(h, m):
    assert parse_refresh_interval(f"{h}h{m}m") == dt.timedelta(hours=h, minutes=m)


@settings(**SETTINGS)
@given(v=st.text(max_size=12).filter(lambda s: not any(ch.isdigit() for ch in s)))
def test_refresh_interval_garbage_is_one_hour(v):
    assert parse_refresh_interval(v) == dt.timedelta(hours=1)


_keys = st.sampled_from(["app", "tier", "team", "env"])
_vals = st.sampled_from(["a", "b", "c"])
_labels = st.dictionaries(_keys, _vals, max_size=4)
_expr = st.one_of(
    st.builds(lambda k, vs: {"key": k, "operator": "In", "values": vs}, _keys, st.lists(_vals, min_size=1, max_size=3)),
    st.builds(lambda k, vs: {"key": k, "operator": "NotIn", "values": vs}, _keys,
              st.lists(_vals, min_size=1, max_size=3)),
    st.builds(lambda k: {"key": k, "operator": "Exists"}, _keys),
    st.builds(lambda k: {"key": k, "operator": "DoesNotExist"}, _keys))


def _model_match(sel, labels):
    for k, v in (sel.get("matchLabels") or {}).items():
        if labels.get(k) != v:
            return False
    for e in sel.get("matchExpressions") or []:
        k, op, vs = e["key"], e["operator"], set(e.get("values") or [])
        ok = {"In": k in labels and labels[k] in vs, "NotIn": k not in labels or labels[k] not in vs,
              "Exists": k in labels, "DoesNotExist": k not in labels}[op]
        if not ok:
            return False
    return True


@settings(**SETTINGS)
@given(ml=_labels, exprs=st.lists(_expr, max_size=3), labels=_labels)
def test_label_selector_semantics(ml, exprs, labels):
    sel = {"matchLabels": ml, "matchExpressions": exprs}
    assert match_selector(sel, labels) == _model_match(sel, labels)


@settings(**SETTINGS)
@given(events=st.lists(st.tuples(st.integers(0, 30), st.sampled_from(["t1", "t2", None])), max_size=200),
       cap=st.integers(1, 16))
def test_deduper_bounded_and_idempotent(events, cap):
    dd = FailureDeduper(max_entries=cap)
    model: dict[str, str] = {}
    order: list[str] = []
    for pod_i, ft in events:
        pod = {"metadata": {"namespace": "ns", "name": f"p{pod_i}"}}
        k = f"ns/p{pod_i}"
        fresh = dd.check_and_mark(pod, ft)
        if ft is None:
            assert fresh            # no finishedAt: never deduped (reference behaviour)
            continue
        assert fresh == (model.get(k) != ft)
        model[k] = ft
        if k in order:
            order.remove(k)
        order.append(k)
        while len(order) > cap:      # LRU eviction
            model.pop(order.pop(0))
        assert len(dd) <= cap


@pytest.fixture(scope="module")
def _fk_status():
    from operator_amd.controller.storage import StatusWriter
    from operator_amd.kube.fake import FakeKube
    from operator_amd.kube.resources import PODMORTEMS

    fk = FakeKube()
    fk.create(PODMORTEMS, {"metadata": {"name": "m", "namespace": "default"}, "spec": {}})
    return fk, StatusWriter(fk), PODMORTEMS


@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(n=st.integers(1, 25))
def test_status_ring_newest_first_capped(_fk_status, n):
    from operator_amd.api.models import AnalysisResult, AnalysisSummary
    from operator_amd.controller.storage import MAX_RECENT_FAILURES

    fk, sw, kind = _fk_status
    names = [f"pod-{n}-{i}" for i in range(n)]
    for name in names:
        mon = fk.get(kind, "m", "default")
        res = AnalysisResult(pod_name=name, pod_namespace="default",
                             summary=AnalysisSummary(highest_severity="HIGH", significant_events=1, total_events=1))
        sw.append_failure({"metadata": {"name": name, "namespace": "default"}}, mon, res, None)
    ring = (fk.get(kind, "m", "default").get("status") or {}).get("recentFailures") or []
    assert len(ring) <= MAX_RECENT_FAILURES
    want = list(reversed(names))[:MAX_RECENT_FAILURES]
    assert [r["podName"] for r in ring][:len(want)] == want[:len(ring)]


@settings(max_examples=200, deadline=None)
@given(st.integers(1, 8).map(lambda m: 32 * m), st.sampled_from([128, 512, 1024, 6144, 14336, 28672]),
       st.sampled_from([512, 1024, 4096, 14336]))
def test_gemm_plans_are_launchable(M, N, K):
    """Every gemm_decode plan satisfies the binding's launch checks: the row tile is
    a kernel variant dividing M (a 192-row decode bucket included) and K splits into
    S slices of whole 64-column steps (uneven slices allowed, S <= 16)."""
    from operator_amd import ops

    p = ops.gemm_plan(M, N, K)
    if p is None:
        return
    bm, bn, S = p[0], p[1], p[2]
    assert bm in (64, 128, 256) and M % bm == 0
    assert bn in (64, 128) and N % bn == 0
    assert 1 <= S <= 16 and K % 64 == 0 and K // 64 >= S
