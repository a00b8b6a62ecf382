"""Pattern set -> literal factors -> DFA (host compile step).

Every matcher (primary or secondary) is reduced to *factors*: literals, one of
which must occur (case-folded) on any line the matcher accepts.

* ``literal`` matchers: the literal itself. Exact when ``ignore_case`` (the
  DFA runs on folded bytes), otherwise verified.
* ``regex`` matchers: a *cover* — a set of literals at least one of which
  every match contains (literal runs, groups, alternations), found by walking
  the regex parse tree; always verified with ``re`` on the candidate line only. A regex with no required literal of >= 3 bytes is
  *unfiltered* and is evaluated on every line by the CPU (rare by design).

Factors longer than 64 bytes are cut to 64 (and verified). Identical folded
factors are shared; ``factor_matchers`` maps factor id -> matcher ids.
The DFA itself is built by the native compiler (csrc/patterns/patterns.cpp).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

try:  # py3.11+
    import re._parser as sre_parse  # type: ignore
    import re._constants as sre_c  # type: ignore
except ImportError:  # py3.10
    import sre_parse  # type: ignore
    import sre_constants as sre_c  # type: ignore

from .schema import Matcher, Pattern, PatternSet

MAX_FACTOR = 64
MIN_REGEX_FACTOR = 3


def _fold(b: bytes) -> bytes:
    return b.lower()  # bytes.lower() folds ASCII A-Z only == the kernel's class map


def required_cover(regex: bytes) -> list[bytes] | None:
    """A set of literals such that every match of ``regex`` contains at least one.

    Sequences contribute literal runs; groups / repeats with min >= 1 recurse;
    alternations contribute the union of each branch's best cover. Among the
    candidates the one whose SHORTEST literal is longest wins (fewest spurious
    candidate lines). Returns None if no cover has all literals >= 3 bytes.
    """
    try:
        tree = sre_parse.parse(regex.decode("latin-1"))
    except Exception:
        return None

    def quality(c):
        return min(len(x) for x in c) if c else -1

    def best_of(cands):
        best = None
        for c in cands:
            if c and (best is None or quality(c) > quality(best)):
                best = c
        return best

    def cover(seq):
        cands = []
        run = bytearray()
        for op, av in seq:
            if op is sre_c.LITERAL:
                run.append(av)
                continue
            if run:
                cands.append([bytes(run)])
            run = bytearray()
            if op is sre_c.SUBPATTERN:
                cands.append(cover(av[-1]))
            elif op in (sre_c.MAX_REPEAT, sre_c.MIN_REPEAT) and av[0] >= 1:
                cands.append(cover(av[2]))
            elif op is sre_c.BRANCH:
                parts = [cover(b) for b in av[1]]
                if all(parts):
                    cands.append(sorted({x for p_ in parts for x in p_}))
        if run:
            cands.append([bytes(run)])
        return best_of(cands)

    c = cover(tree)
    if not c or quality(c) < MIN_REGEX_FACTOR or any(b"\n" in x or b"\0" in x for x in c):
        return None
    return c


@dataclass
class CompiledPatterns:
    patset: PatternSet
    matchers: list[Matcher]
    pattern_primary: list[int]                 # pattern -> primary matcher id
    pattern_secondary: list[list[int]]         # pattern -> secondary matcher ids
    factors: list[bytes]                       # folded literals
    factor_matchers: list[list[int]]           # factor -> matcher ids
    matcher_verify: list[bool]                 # needs re verification on the candidate line
    unfiltered: list[int]                      # matchers with no factor: CPU line scan
    regexes: list[re.Pattern]                  # compiled per-matcher verifier (bytes)
    dfa: dict = field(default_factory=dict)    # native compile_dfa output

    @property
    def num_matchers(self) -> int:
        return len(self.matchers)


def compile_patterns(ps: PatternSet, build_dfa: bool = True) -> CompiledPatterns:
    matchers: list[Matcher] = []
    mid: dict[tuple, int] = {}

    def add(m: Matcher) -> int:
        k = m.key()
        if k not in mid:
            mid[k] = len(matchers)
            matchers.append(m)
        return mid[k]

    prim, secs = [], []
    for p in ps.patterns:
        prim.append(add(p.primary))
        secs.append([add(s) for s in p.secondary])

    factors: list[bytes] = []
    fid: dict[bytes, int] = {}
    fmat: list[list[int]] = []
    verify: list[bool] = []
    unfiltered: list[int] = []
    regexes: list[re.Pattern] = []
    for i, m in enumerate(matchers):
        flags = re.IGNORECASE if m.ignore_case else 0
        regexes.append(re.compile(m.regex_source(), flags))
        if m.literal is not None:
            f = _fold(m.literal)
            need = (not m.ignore_case and m.literal.lower() != m.literal.upper()) or len(f) > MAX_FACTOR
        else:
            lits = required_cover(m.regex)
            if lits is None:
                unfiltered.append(i)
                verify.append(True)
                continue
            verify.append(True)
            for lit in lits:
                f = _fold(lit)[:MAX_FACTOR]
                if f not in fid:
                    fid[f] = len(factors)
                    factors.append(f)
                    fmat.append([])
                if i not in fmat[fid[f]]:
                    fmat[fid[f]].append(i)
            continue
        f = f[:MAX_FACTOR]
        verify.append(bool(need))
        if f not in fid:
            fid[f] = len(factors)
            factors.append(f)
            fmat.append([])
        fmat[fid[f]].append(i)

    cp = CompiledPatterns(ps, matchers, prim, secs, factors, fmat, verify, unfiltered, regexes)
    if build_dfa and factors:
        cp.dfa = compile_dfa_cached(factors)
    return cp


def _cache_dir():
    import os
    from pathlib import Path

    return Path(os.environ.get("OAMD_CACHE_DIR", Path(__file__).resolve().parent.parent / ".cache")) / "dfa"


def compile_dfa_cached(factors: list[bytes]) -> dict:
    """Native DFA compile with an on-disk cache keyed by the factor set (restarts and
    PatternLibrary re-syncs with unchanged patterns skip the compile)."""
    import hashlib
    import json
    import os

    from operator_amd.ops._native import patterns as native

    h = hashlib.sha256(b"dfa-v1\0" + b"\0".join(factors)).hexdigest()[:24]
    f = _cache_dir() / f"{h}.npz"
    if f.exists():
        try:
            import numpy as np

            z = np.load(f, allow_pickle=False)
            d = json.loads(bytes(z["meta"]).decode())
            for k in ("cls_map", "table", "out_off", "out_ids"):
                d[k] = z[k].tobytes()
            return d
        except Exception:  # noqa: BLE001 - corrupt cache entry: recompile
            pass
    d = native().compile_dfa(factors)
    try:
        import numpy as np

        f.parent.mkdir(parents=True, exist_ok=True)
        meta = {k: v for k, v in d.items() if k not in ("cls_map", "table", "out_off", "out_ids")}
        tmp = f.with_suffix(f".{os.getpid()}.tmp.npz")
        np.savez(tmp, meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
                 **{k: np.frombuffer(d[k], dtype=np.uint8) for k in ("cls_map", "table", "out_off", "out_ids")})
        os.replace(tmp, f)
    except OSError:
        pass
    return d
