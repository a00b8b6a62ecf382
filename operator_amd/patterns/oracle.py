"""CPU reference matcher + scorer: the correctness oracle for the GPU scan.

Semantics (our design, SURVEY.md §2.2 "Decision"):
* a log is split into lines on ``\\n``; matcher m hits line L iff
  ``re.search(m.regex, line)`` (bytes regex; IGNORECASE = ASCII folding);
* every primary hit (doc, L) of pattern p is one event with
      score = conf_p * (1 + sum_j w_j * (1 - |dL_j| / (W_j + 1))) / (1 + sum_j w_j)
  where the sum runs over secondaries j whose nearest hit lies within W_j
  lines (|dL_j| <= W_j);
* events sort by (score desc, severity desc, line asc, pattern index asc).

This module is deliberately simple, unfused Python. The native scorer
(csrc/patterns/patterns.cpp::score_events) and the GPU scan must agree with it.
"""
from __future__ import annotations

import bisect
from dataclasses import dataclass

from .compiler import CompiledPatterns


@dataclass(frozen=True)
class Event:
    pattern: int      # index into patset.patterns
    line: int         # 0-based line
    score: float


def split_lines(doc: bytes) -> list[bytes]:
    return doc.split(b"\n")


def doc_hits(cp: CompiledPatterns, doc: bytes) -> set[tuple[int, int]]:
    """{(matcher, line)} for one doc (every matcher evaluated on every line)."""
    hits = set()
    for li, line in enumerate(split_lines(doc)):
        for mi, rx in enumerate(cp.regexes):
            if rx.search(line):
                hits.add((mi, li))
    return hits


def score_doc(cp: CompiledPatterns, hits: set[tuple[int, int]]) -> list[Event]:
    by_m: dict[int, list[int]] = {}
    for m, l in hits:
        by_m.setdefault(m, []).append(l)
    for v in by_m.values():
        v.sort()

    def nearest(m: int, line: int) -> int | None:
        v = by_m.get(m)
        if not v:
            return None
        i = bisect.bisect_left(v, line)
        best = None
        if i < len(v):
            best = v[i] - line
        if i > 0:
            d = line - v[i - 1]
            if best is None or d < best:
                best = d
        return best

    evs: list[Event] = []
    for pi, p in enumerate(cp.patset.patterns):
        prim = cp.pattern_primary[pi]
        for line in by_m.get(prim, []):
            bonus = wsum = 0.0
            for j, sm in enumerate(cp.pattern_secondary[pi]):
                w = p.secondary[j].weight
                win = p.secondary[j].window
                wsum += w
                d = nearest(sm, line)
                if d is not None and d <= win:
                    bonus += w * (1.0 - d / (win + 1))
            evs.append(Event(pi, line, p.primary.confidence * (1.0 + bonus) / (1.0 + wsum)))
    evs.sort(key=lambda e: (-e.score, -cp.patset.patterns[e.pattern].severity_rank, e.line, e.pattern))
    return evs


def analyze_docs(cp: CompiledPatterns, docs: list[bytes]) -> list[list[Event]]:
    return [score_doc(cp, doc_hits(cp, d)) for d in docs]
