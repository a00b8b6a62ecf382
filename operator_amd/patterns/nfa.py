"""Regex -> Pike-VM bytecode for the native verifier (csrc/patterns/verify.cpp, SURVEY.md
§2.4 N4: "Confirms regex candidates flagged by N1 on the matched line only ...
bit-exact with the Python regex oracle").

A matcher's verification question is ``re.search(line) is not None``. For the regular
subset below that answer does not depend on backtracking order (greedy vs lazy,
alternation order), so a Thompson-NFA simulation computes exactly what ``re`` does:

  literals (IGNORECASE folded over ASCII, as ``re`` does for bytes patterns), ``.``
  (DOTALL), character classes with ranges / negation / ``\\d \\w \\s`` and their
  complements (ASCII, bytes semantics), groups (with scoped ``(?i:...)`` flags),
  alternation, ``* + ? {m,n}`` greedy or lazy, ``^ $ \\A \\Z \\b \\B`` on a single
  line (lines never contain ``\\n``).

Anything else (back-references, lookaround, conditionals, atomic / possessive, LOCALE,
or a program that would exceed ``MAX_INSTR`` after repeat expansion) returns None and
the matcher keeps using Python ``re`` — so results are exact by construction.

Bytecode (little-endian int32 triples) and 256-bit class bitmaps; opcodes mirror
verify.cpp: CHAR c | CLASS k | ANY | SPLIT x y | JMP x | ASSERT kind | MATCH.
"""
from __future__ import annotations

import re
import struct

try:  # py3.11+
    import re._constants as sre_c  # type: ignore
    import re._parser as sre_parse  # type: ignore
except ImportError:  # py3.10
    import sre_constants as sre_c  # type: ignore
    import sre_parse  # type: ignore

CHAR, CLASS, ANY, SPLIT, JMP, ASSERT, MATCH = range(7)
BOL, EOL, WORDB, NWORDB = range(4)
MAX_INSTR = 4096

_DIGIT = frozenset(range(0x30, 0x3A))
_SPACE = frozenset(b" \t\n\r\f\v")
_WORD = frozenset(b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789_")
_ALL = frozenset(range(256))
_CATS = {
    sre_c.CATEGORY_DIGIT: _DIGIT, sre_c.CATEGORY_NOT_DIGIT: _ALL - _DIGIT,
    sre_c.CATEGORY_SPACE: _SPACE, sre_c.CATEGORY_NOT_SPACE: _ALL - _SPACE,
    sre_c.CATEGORY_WORD: _WORD, sre_c.CATEGORY_NOT_WORD: _ALL - _WORD,
}
_UNSUPPORTED_FLAGS = re.LOCALE | re.UNICODE


class Unsupported(Exception):
    pass


def _swap(c: int) -> int:
    if 0x41 <= c <= 0x5A or 0x61 <= c <= 0x7A:
        return c ^ 0x20
    return c


class _Compiler:
    def __init__(self):
        self.ins: list[list[int]] = []
        self.classes: list[frozenset] = []
        self._cls_id: dict[frozenset, int] = {}

    def emit(self, op: int, a: int = 0, b: int = 0) -> int:
        if len(self.ins) >= MAX_INSTR:
            raise Unsupported("program too large")
        self.ins.append([op, a, b])
        return len(self.ins) - 1

    def cls(self, s: frozenset) -> int:
        if s not in self._cls_id:
            self._cls_id[s] = len(self.classes)
            self.classes.append(s)
        return self._cls_id[s]

    def charset(self, s: set, icase: bool) -> None:
        if icase:
            s = set(s) | {_swap(c) for c in s}
        s = frozenset(s)
        if len(s) == 1:
            self.emit(CHAR, next(iter(s)))
        else:
            self.emit(CLASS, self.cls(s))

    def seq(self, items, flags: int) -> None:
        for op, av in items:
            self.node(op, av, flags)

    def node(self, op, av, flags: int) -> None:
        icase = bool(flags & re.IGNORECASE)
        if op is sre_c.LITERAL:
            self.charset({av}, icase)
        elif op is sre_c.NOT_LITERAL:
            excl = {av, _swap(av)} if icase else {av}
            self.emit(CLASS, self.cls(frozenset(_ALL - excl)))
        elif op is sre_c.ANY:
            if flags & re.DOTALL:
                self.emit(CLASS, self.cls(_ALL))
            else:
                self.emit(ANY)
        elif op is sre_c.IN:
            self.emit(CLASS, self.cls(frozenset(self._in_set(av, icase))))
        elif op is sre_c.BRANCH:
            alts = av[1]
            jumps = []
            for i, alt in enumerate(alts):
                if i + 1 < len(alts):
                    sp = self.emit(SPLIT)
                    self.ins[sp][1] = len(self.ins)
                    self.seq(alt, flags)
                    jumps.append(self.emit(JMP))
                    self.ins[sp][2] = len(self.ins)
                else:
                    self.seq(alt, flags)
            for j in jumps:
                self.ins[j][1] = len(self.ins)
        elif op is sre_c.SUBPATTERN:
            _, add, dele, p = av
            f = (flags | add) & ~dele
            if f & _UNSUPPORTED_FLAGS:
                raise Unsupported("locale / unicode flags")
            self.seq(p, f)
        elif op in (sre_c.MAX_REPEAT, sre_c.MIN_REPEAT):
            lo, hi, p = av
            for _ in range(lo):
                self.seq(p, flags)
            if hi == sre_c.MAXREPEAT:
                sp = self.emit(SPLIT)          # L: split body, out
                self.ins[sp][1] = len(self.ins)
                self.seq(p, flags)
                self.emit(JMP, sp)
                self.ins[sp][2] = len(self.ins)
            else:
                outs = []
                for _ in range(hi - lo):       # nested optionals: (body (body (...)?)?)?
                    sp = self.emit(SPLIT)
                    self.ins[sp][1] = len(self.ins)
                    outs.append(sp)
                    self.seq(p, flags)
                for sp in outs:
                    self.ins[sp][2] = len(self.ins)
        elif op is sre_c.AT:
            kind = {sre_c.AT_BEGINNING: BOL, sre_c.AT_BEGINNING_STRING: BOL, sre_c.AT_END: EOL,
                    sre_c.AT_END_STRING: EOL, sre_c.AT_BOUNDARY: WORDB, sre_c.AT_NON_BOUNDARY: NWORDB}.get(av)
            if kind is None:
                raise Unsupported(f"anchor {av}")
            self.emit(ASSERT, kind)
        else:
            raise Unsupported(str(op))

    def _in_set(self, items, icase: bool) -> set:
        s: set[int] = set()
        neg = False
        for op, av in items:
            if op is sre_c.NEGATE:
                neg = True
            elif op is sre_c.LITERAL:
                s.add(av)
            elif op is sre_c.RANGE:
                s.update(range(av[0], av[1] + 1))
            elif op is sre_c.CATEGORY:
                if av not in _CATS:
                    raise Unsupported(f"category {av}")
                s.update(_CATS[av])
            else:
                raise Unsupported(f"class item {op}")
        if icase:
            s |= {_swap(c) for c in s}
        s = {c for c in s if c < 256}
        return (set(_ALL) - s) if neg else s


def compile_nfa(source: bytes | str, flags: int = 0) -> tuple[bytes, bytes] | None:
    """(instructions, class bitmaps) for the native verifier, or None if the regex is
    outside the exactly-simulated subset (then Python ``re`` verifies it)."""
    if isinstance(source, str):
        source = source.encode("latin-1")
    try:
        tree = sre_parse.parse(source, flags)
    except Exception:  # noqa: BLE001
        return None
    gflags = flags | tree.state.flags
    if gflags & _UNSUPPORTED_FLAGS & ~re.UNICODE or (gflags & re.LOCALE):
        return None
    c = _Compiler()
    try:
        c.seq(tree, gflags)
        c.emit(MATCH)
    except (Unsupported, RecursionError):
        return None
    ins = b"".join(struct.pack("<3i", *x) for x in c.ins)
    bm = bytearray()
    for s in c.classes:
        words = [0, 0, 0, 0]
        for b in s:
            words[b >> 6] |= 1 << (b & 63)
        bm += struct.pack("<4Q", *words)
    return ins, bytes(bm)
