"""Pattern-library schema (OUR design — the reference's pattern format and
scoring live in external repos/services it never vendors: SURVEY.md §2.2,
README.md:43-47 of the reference).

A pattern library is a YAML file::

    metadata: {library_id: core, name: ..., version: "1.0"}
    patterns:
      - id: java-oom
        name: Java OutOfMemoryError
        severity: CRITICAL            # CRITICAL | HIGH | MEDIUM | LOW | INFO
        category: memory
        primary_pattern:              # camelCase keys are accepted too
          regex: 'java\\.lang\\.OutOfMemoryError'   # or  literal: "..."
          confidence: 0.95            # (0, 1]
          ignore_case: true           # default true
        secondary_patterns:
          - literal: "GC overhead limit exceeded"
            weight: 0.4               # >= 0
            proximity_window: 20      # lines, >= 0
        context_lines: 3
        remediation: {description: "...", commands: [...]}

Each primary/secondary entry is a *matcher*. Matching is per log line (lines
split on ``\\n``), with Python ``re`` byte-regex semantics (ASCII case folding).
"""
from __future__ import annotations

import hashlib
import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Iterable

import yaml

SEVERITIES = ("INFO", "LOW", "MEDIUM", "HIGH", "CRITICAL")
SEVERITY_RANK = {s: i for i, s in enumerate(SEVERITIES)}


class PatternError(ValueError):
    pass


@dataclass(frozen=True)
class Matcher:
    literal: bytes | None = None
    regex: bytes | None = None
    ignore_case: bool = True
    confidence: float = 1.0        # primaries only
    weight: float = 0.0            # secondaries only
    window: int = 0                # secondaries only (lines)

    def key(self) -> tuple:
        return (self.literal, self.regex, self.ignore_case)

    def regex_source(self) -> bytes:
        import re

        return re.escape(self.literal) if self.literal is not None else self.regex


@dataclass(frozen=True)
class Pattern:
    id: str
    name: str
    severity: str
    primary: Matcher
    secondary: tuple[Matcher, ...] = ()
    category: str = ""
    context_lines: int = 3
    remediation: dict = field(default_factory=dict, hash=False, compare=False)
    library: str = ""

    @property
    def severity_rank(self) -> int:
        return SEVERITY_RANK[self.severity]


def _get(d: dict, *names, default=None):
    for n in names:
        if n in d:
            return d[n]
    return default


def _matcher(d: Any, primary: bool, where: str) -> Matcher:
    if isinstance(d, str):
        d = {"literal": d}
    if not isinstance(d, dict):
        raise PatternError(f"{where}: matcher must be a mapping or string")
    lit, rx = d.get("literal"), d.get("regex")
    if (lit is None) == (rx is None):
        raise PatternError(f"{where}: exactly one of 'literal' / 'regex' is required")
    ic = bool(_get(d, "ignore_case", "ignoreCase", default=True))
    if lit is not None:
        lb = lit.encode() if isinstance(lit, str) else bytes(lit)
        if not lb or b"\n" in lb or b"\0" in lb:
            raise PatternError(f"{where}: literal must be non-empty and contain no newline/NUL")
        m = dict(literal=lb)
    else:
        rb = rx.encode() if isinstance(rx, str) else bytes(rx)
        import re

        try:
            re.compile(rb)
        except re.error as e:
            raise PatternError(f"{where}: bad regex: {e}") from e
        m = dict(regex=rb)
    conf = float(_get(d, "confidence", default=0.8)) if primary else 1.0
    if primary and not (0.0 < conf <= 1.0):
        raise PatternError(f"{where}: confidence must be in (0, 1]")
    w = float(_get(d, "weight", default=0.5)) if not primary else 0.0
    win = int(_get(d, "proximity_window", "proximityWindow", "window", default=10)) if not primary else 0
    if w < 0 or win < 0:
        raise PatternError(f"{where}: weight / proximity_window must be >= 0")
    return Matcher(ignore_case=ic, confidence=conf, weight=w, window=win, **m)


def parse_pattern(d: dict, library: str = "") -> Pattern:
    pid = str(_get(d, "id", default="") or "")
    if not pid:
        raise PatternError("pattern without id")
    sev = str(_get(d, "severity", default="MEDIUM")).upper()
    if sev not in SEVERITY_RANK:
        raise PatternError(f"{pid}: unknown severity {sev}")
    prim = _get(d, "primary_pattern", "primaryPattern", "primary")
    if prim is None:
        raise PatternError(f"{pid}: primary_pattern is required")
    secs = _get(d, "secondary_patterns", "secondaryPatterns", "secondary", default=[]) or []
    return Pattern(
        id=pid,
        name=str(_get(d, "name", default=pid)),
        severity=sev,
        primary=_matcher(prim, True, f"{pid}.primary"),
        secondary=tuple(_matcher(s, False, f"{pid}.secondary[{i}]") for i, s in enumerate(secs)),
        category=str(_get(d, "category", default="")),
        context_lines=int(_get(d, "context_lines", "contextLines", default=3)),
        remediation=dict(_get(d, "remediation", default={}) or {}),
        library=library,
    )


@dataclass
class PatternSet:
    patterns: list[Pattern]
    libraries: list[str] = field(default_factory=list)

    def __len__(self) -> int:
        return len(self.patterns)

    def digest(self) -> str:
        h = hashlib.sha256()
        for p in self.patterns:
            h.update(json.dumps([p.id, p.severity, repr(p.primary), [repr(s) for s in p.secondary]]).encode())
        return h.hexdigest()[:16]

    @staticmethod
    def from_dicts(items: Iterable[dict], library: str = "") -> "PatternSet":
        pats = [parse_pattern(d, library) for d in items]
        ids = [p.id for p in pats]
        if len(set(ids)) != len(ids):
            raise PatternError("duplicate pattern ids")
        return PatternSet(pats, [library] if library else [])

    @staticmethod
    def from_yaml_text(text: str, default_library: str = "") -> "PatternSet":
        doc = yaml.safe_load(text) or {}
        if isinstance(doc, list):
            items, lib = doc, default_library
        else:
            meta = doc.get("metadata", {}) or {}
            lib = str(meta.get("library_id", meta.get("libraryId", default_library)) or default_library)
            items = doc.get("patterns", []) or []
        return PatternSet.from_dicts(items, lib)

    @staticmethod
    def load_dir(root: str | Path, enabled: Iterable[str] | None = None) -> "PatternSet":
        """Load every *.yaml/*.yml under root (sorted). ``enabled`` filters by file stem
        or library_id (PatternLibrary.spec.enabledLibraries; SURVEY.md Q8 'fix')."""
        root = Path(root)
        en = set(enabled) if enabled else None
        pats: list[Pattern] = []
        libs: list[str] = []
        seen: set[str] = set()
        if not root.exists():
            return PatternSet([], [])
        for f in sorted(list(root.rglob("*.yaml")) + list(root.rglob("*.yml"))):
            if ".git" in f.parts or not f.is_file():
                continue
            ps = PatternSet.from_yaml_text(f.read_text(errors="replace"), f.stem)
            lib = ps.libraries[0] if ps.libraries else f.stem
            if en is not None and f.stem not in en and lib not in en:
                continue
            libs.append(lib)
            for p in ps.patterns:
                pid = p.id if p.id not in seen else f"{lib}/{p.id}"
                seen.add(pid)
                pats.append(Pattern(pid, p.name, p.severity, p.primary, p.secondary, p.category,
                                    p.context_lines, p.remediation, lib))
        return PatternSet(pats, libs)

    def merged(self, other: "PatternSet") -> "PatternSet":
        return PatternSet(self.patterns + other.patterns, self.libraries + other.libraries)
