"""Timestamps in the reference's wire format.

The reference writes ``java.time.Instant.toString()`` values (ISO-8601, UTC,
``Z`` suffix, fraction printed in groups of 3 digits and omitted when zero),
e.g. ``Instant.now().toString()`` in J/service/AnalysisStorageService.java:161
and J/service/EventService.java:187. Python datetimes carry microseconds, so
the fraction is 0, 3 or 6 digits.
"""
from __future__ import annotations

import datetime as _dt
import time as _time

UTC = _dt.timezone.utc


def now() -> _dt.datetime:
    return _dt.datetime.now(tz=UTC)


def instant_str(t: _dt.datetime | None = None) -> str:
    t = (t or now()).astimezone(UTC)
    base = t.strftime("%Y-%m-%dT%H:%M:%S")
    us = t.microsecond
    if us == 0:
        frac = ""
    elif us % 1000 == 0:
        frac = f".{us // 1000:03d}"
    else:
        frac = f".{us:06d}"
    return f"{base}{frac}Z"


def parse_instant(s: str | None) -> _dt.datetime | None:
    if not s:
        return None
    s = s.strip()
    if s.endswith("Z"):
        s = s[:-1] + "+00:00"
    # trim nanosecond fractions to microseconds
    if "." in s:
        head, rest = s.split(".", 1)
        digits = ""
        i = 0
        while i < len(rest) and rest[i].isdigit():
            digits += rest[i]
            i += 1
        s = f"{head}.{(digits + '000000')[:6]}{rest[i:]}"
    t = _dt.datetime.fromisoformat(s)
    if t.tzinfo is None:
        t = t.replace(tzinfo=UTC)
    return t


def epoch_millis(t: _dt.datetime | None = None) -> int:
    if t is None:
        return int(_time.time() * 1000)
    return int(t.timestamp() * 1000)
