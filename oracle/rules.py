"""TEST INFRASTRUCTURE ONLY -- restatement of hashcat's CPU rule processor for the ops dwpa's rule files use.

dwpa expands wordlists with `hashcat --stdout -r bestWPA.rule` (help_crack/help_crack.py:508,575) and runs
server rules with `-S -r` (:445-447,931-933): both use hashcat's host-side rule engine (third-party, not in
/root/reference, not installed here), so these semantics are PARITY UNPINNED by the reference: they restate
hashcat's documented rule behaviour (RP_PASSWORD_SIZE = 256; an op whose result would not fit is a no-op;
empty or > 256-byte inputs are rejected) and pin the GPU engine (dwpa_amd/csrc/rules_dev.hip) to it.
"""
from __future__ import annotations

RP = 256


def _pos(c: str):
    if "0" <= c <= "9":
        return ord(c) - 48
    if "A" <= c <= "Z":
        return ord(c) - 55
    return None


def parse(line: str):
    """Rule line -> list of (op, p1, p2) or None if unsupported/malformed (hashcat skips such lines)."""
    line = line.rstrip("\r\n")
    if not line or line.startswith("#"):
        return None
    ops, i = [], 0
    while i < len(line):
        op = line[i]
        i += 1
        if op == " ":
            continue
        if op in ":lucCtrdf{}[]q":
            ops.append((op, None, None))
        elif op in "TpD'zZ":
            if i >= len(line) or _pos(line[i]) is None:
                return None
            ops.append((op, _pos(line[i]), None))
            i += 1
        elif op in "$^@":
            if i >= len(line):
                return None
            ops.append((op, line[i].encode("latin-1")[0], None))
            i += 1
        elif op == "s":
            if i + 2 > len(line):
                return None
            ops.append((op, line[i].encode("latin-1")[0], line[i + 1].encode("latin-1")[0]))
            i += 2
        else:
            return None
    return ops or None


def _low(b):
    return bytes(c | 0x20 if 65 <= c <= 90 else c for c in b)


def _up(b):
    return bytes(c & ~0x20 if 97 <= c <= 122 else c for c in b)


def _tog(c):
    return c ^ 0x20 if (65 <= c <= 90 or 97 <= c <= 122) else c


def apply(ops, word: bytes):
    """Returns the candidate, or None if hashcat rejects the input word."""
    if len(word) < 1 or len(word) > RP:
        return None
    w = bytearray(word)
    for op, p1, p2 in ops:
        n = len(w)
        if op == ":":
            pass
        elif op == "l":
            w = bytearray(_low(w))
        elif op == "u":
            w = bytearray(_up(w))
        elif op == "c":
            w = bytearray(_low(w))
            if n:
                w[0:1] = _up(w[0:1])
        elif op == "C":
            w = bytearray(_up(w))
            if n:
                w[0:1] = _low(w[0:1])
        elif op == "t":
            w = bytearray(_tog(c) for c in w)
        elif op == "T":
            if p1 < n:
                w[p1] = _tog(w[p1])
        elif op == "r":
            w.reverse()
        elif op == "d":
            if 2 * n < RP:
                w = w + w
        elif op == "p":
            if n * p1 + n < RP:
                w = w * (p1 + 1)
        elif op == "f":
            if 2 * n < RP:
                w = w + w[::-1]
        elif op == "{":
            if n:
                w = w[1:] + w[:1]
        elif op == "}":
            if n:
                w = w[-1:] + w[:-1]
        elif op == "[":
            if n:
                w = w[1:]
        elif op == "]":
            if n:
                w = w[:-1]
        elif op == "q":
            if 2 * n < RP:
                w = bytearray(c for c in w for _ in (0, 1))
        elif op == "D":
            if p1 < n:
                del w[p1]
        elif op == "'":
            if p1 < n:
                w = w[:p1]
        elif op == "z":
            if n and n + p1 < RP:
                w = bytearray([w[0]]) * p1 + w
        elif op == "Z":
            if n and n + p1 < RP:
                w = w + bytearray([w[-1]]) * p1
        elif op == "$":
            if n + 1 < RP:
                w.append(p1)
        elif op == "^":
            if n + 1 < RP:
                w.insert(0, p1)
        elif op == "s":
            w = bytearray(p2 if c == p1 else c for c in w)
        elif op == "@":
            w = bytearray(c for c in w if c != p1)
    return bytes(w)


def expand(rule_lines, words):
    rules = [r for r in (parse(x) for x in rule_lines) if r]
    return [[apply(r, w) for r in rules] for w in words]
