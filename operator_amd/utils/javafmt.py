"""Tiny helpers that reproduce Java formatting semantics the reference's
user-visible strings depend on (so annotations / Events / status messages
are byte-identical for the same inputs)."""
from __future__ import annotations

from decimal import ROUND_HALF_UP, Decimal


def jstr(v) -> str:
    """String.format("%s") / string concatenation of a possibly-null value."""
    if v is None:
        return "null"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def fmt2(x: float) -> str:
    """String.format("%.2f", double). Java's Formatter rounds HALF_UP starting from the
    shortest round-trip decimal of the double (FormattedFloatingDecimal), so
    0.675 -> "0.68" and 0.125 -> "0.13" (C printf would give 0.67 / 0.12)."""
    return str(Decimal(repr(float(x))).quantize(Decimal("0.01"), rounding=ROUND_HALF_UP))


def jtrim(s: str) -> str:
    """java.lang.String.trim(): strips chars <= U+0020 at both ends."""
    i, j = 0, len(s)
    while i < j and ord(s[i]) <= 32:
        i += 1
    while j > i and ord(s[j - 1]) <= 32:
        j -= 1
    return s[i:j]


def is_blank(s: str | None) -> bool:
    """String.isBlank() (null-safe): empty or only whitespace."""
    return s is None or s.strip() == ""
