"""TEST INFRASTRUCTURE ONLY -- restatement of hashcat's rule language (every function of hashcat >= 6.2.6's rule
engine), the oracle the GPU rule engine (dwpa_amd/csrc/rules_dev.hip) and the host re-application
(dwpa_amd/csrc/rules.cpp, RuleSet::apply_host) are pinned to.

Where rules reach the client:
  * `hashcat --stdout -r bestWPA.rule` expands wordlists (help_crack/help_crack.py:508,575);
  * the server's per-dictionary rules (`dicts.rules`, db/wpa.sql:48; "add rules depending on dictionary contents",
    INSTALL.md:110) are merged by get_work (web/content/get_work.php:86-92) and run with `-S -r`
    (help_crack/help_crack.py:445-447,931-933).
hashcat is third party (not in /root/reference, not installed here), so these semantics are PARITY UNPINNED by the
reference: they restate hashcat's documented rule functions (hashcat wiki "rule_based_attack") and its rule
processor's bounds.  Conventions:

  * Positions and lengths N, M, I are one character each: 0-9 then A-Z (10-35).
  * The work buffer is RP_PASSWORD_SIZE = 256 bytes.  An input word that is empty or longer than 256 bytes is
    rejected.  A function whose result would not fit (length >= 256) leaves the word unchanged, except the memory
    functions 4 / 6 / X, which reject the candidate (as hashcat's rule processor returns RULE_RC_REJECT_ERROR).
  * A position outside the word leaves it unchanged (T D ' o * L R + - . , x O i y Y), as the documentation says.
  * Reject functions drop the candidate (None), like a candidate outside the 8..63 m22000 filter.
  * Memory starts as the input word; M saves the current word.  X inserts mem[N:N+M] at I (M >= 1, N+M within
    the memory, I <= length, result <= 256 bytes, else reject).  Q rejects a word equal to the memory.
  * Byte arithmetic (L R + -) is on unsigned bytes, mod 256.
  * E / eX: lower-case the word, upper-case its first byte and every byte that follows a separator (' ' for E;
    separator positions taken in the lower-cased word).
  * 3NX toggles the case of the byte after the N-th (0-based) occurrence of X.
  * Spaces between functions are ignored; a line of spaces is the no-op rule.  Lines starting with '#' and empty
    lines are not rules.  Any other line that does not parse completely is skipped (hashcat: "Skipping invalid or
    unsupported rule"), and counted.
hashcat's own rule-file loader (-r) accepts only functions its GPU rule engine has -- not the reject functions
(< > _ ! / ( ) = % Q) nor the memory functions (M 4 6 X), which work only with -j/-k -- and skips such a line like
an invalid one: `hashcat_loads` below.  The library's rule files follow it by default (DWPA_RULES_HASHCAT); its
DWPA_RULES_FULL mode runs those lines too, a superset.
"""
from __future__ import annotations

RP = 256

NOARG = set(":lucCtrdf{}[]kKqEM46Q")
POS1 = set("TpDzZ'yYLR+-.,<>_")
CHR1 = set("$^@!/()e")
POS_CHR = set("io=%3")
CHR2 = set("s")
POS2 = set("xO*")
POS3 = set("X")
ALL_OPS = NOARG | POS1 | CHR1 | POS_CHR | CHR2 | POS2 | POS3


def _pos(c: str):
    if "0" <= c <= "9":
        return ord(c) - 48
    if "A" <= c <= "Z":
        return ord(c) - 55
    return None


def parse(line: str):
    """Rule line -> list of (op, p1, p2, p3), or None for a comment / empty line or a line that does not parse."""
    line = line.rstrip("\r\n")
    if not line or line.startswith("#"):
        return None
    ops, i, n = [], 0, len(line)

    def chr_at(j):
        return line[j].encode("latin-1")[0]

    while i < n:
        op = line[i]
        i += 1
        if op == " ":
            continue
        if op in NOARG:
            ops.append((op, 0, 0, 0))
        elif op in POS1:
            if i >= n or _pos(line[i]) is None:
                return None
            ops.append((op, _pos(line[i]), 0, 0))
            i += 1
        elif op in CHR1:
            if i >= n:
                return None
            ops.append((op, chr_at(i), 0, 0))
            i += 1
        elif op in POS_CHR:
            if i + 2 > n or _pos(line[i]) is None:
                return None
            ops.append((op, _pos(line[i]), chr_at(i + 1), 0))
            i += 2
        elif op in CHR2:
            if i + 2 > n:
                return None
            ops.append((op, chr_at(i), chr_at(i + 1), 0))
            i += 2
        elif op in POS2:
            if i + 2 > n or _pos(line[i]) is None or _pos(line[i + 1]) is None:
                return None
            ops.append((op, _pos(line[i]), _pos(line[i + 1]), 0))
            i += 2
        elif op in POS3:
            if i + 3 > n or any(_pos(line[i + k]) is None for k in range(3)):
                return None
            ops.append((op, _pos(line[i]), _pos(line[i + 1]), _pos(line[i + 2])))
            i += 3
        else:
            return None
    return ops or [(":", 0, 0, 0)]


REJECT_OPS = set("<>_!/()=%Q")
MEMORY_OPS = set("M46X")


def hashcat_loads(line: str) -> bool:
    """Whether hashcat's -r loader keeps this rule line: it parses and uses no reject or memory function."""
    ops = parse(line)
    return ops is not None and not any(op in REJECT_OPS | MEMORY_OPS for op, *_ in ops)


def count(lines):
    """(rules present, rules that parse): present = lines that are neither empty nor comments."""
    present = [l for l in (x.rstrip("\r\n") for x in lines) if l and not l.startswith("#")]
    return len(present), sum(1 for l in present if parse(l) is not None)


def _lower(c):
    return c | 0x20 if 65 <= c <= 90 else c


def _upper(c):
    return c & ~0x20 if 97 <= c <= 122 else c


def _tog(c):
    return c ^ 0x20 if (65 <= c <= 90 or 97 <= c <= 122) else c


def apply(ops, word: bytes):
    """Returns the candidate, or None if the input is rejected or a reject / memory function rejects it."""
    if len(word) < 1 or len(word) > RP:
        return None
    w = bytearray(word)
    mem = bytes(word)
    for op, p1, p2, p3 in ops:
        n = len(w)
        if op == ":":
            pass
        elif op == "l":
            w = bytearray(_lower(c) for c in w)
        elif op == "u":
            w = bytearray(_upper(c) for c in w)
        elif op == "c":
            w = bytearray(_lower(c) for c in w)
            if n:
                w[0] = _upper(w[0])
        elif op == "C":
            w = bytearray(_upper(c) for c in w)
            if n:
                w[0] = _lower(w[0])
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
        elif op == "x":
            if p1 < n and p1 + p2 <= n:
                w = w[p1:p1 + p2]
        elif op == "O":
            if p1 < n and p1 + p2 <= n:
                del w[p1:p1 + p2]
        elif op == "i":
            if p1 <= n and n + 1 < RP:
                w.insert(p1, p2)
        elif op == "o":
            if p1 < n:
                w[p1] = p2
        elif op == "*":
            if p1 < n and p2 < n:
                w[p1], w[p2] = w[p2], w[p1]
        elif op == "k":
            if n >= 2:
                w[0], w[1] = w[1], w[0]
        elif op == "K":
            if n >= 2:
                w[n - 1], w[n - 2] = w[n - 2], w[n - 1]
        elif op == "L":
            if p1 < n:
                w[p1] = (w[p1] << 1) & 0xFF
        elif op == "R":
            if p1 < n:
                w[p1] = w[p1] >> 1
        elif op == "+":
            if p1 < n:
                w[p1] = (w[p1] + 1) & 0xFF
        elif op == "-":
            if p1 < n:
                w[p1] = (w[p1] - 1) & 0xFF
        elif op == ".":
            if p1 + 1 < n:
                w[p1] = w[p1 + 1]
        elif op == ",":
            if 1 <= p1 < n:
                w[p1] = w[p1 - 1]
        elif op == "y":
            if p1 <= n and n + p1 < RP:
                w = w[:p1] + w
        elif op == "Y":
            if p1 <= n and n + p1 < RP:
                w = w + w[n - p1:]
        elif op in "Ee":
            sep = 0x20 if op == "E" else p1
            low = bytearray(_lower(c) for c in w)
            out = bytearray(low)
            if n:
                out[0] = _upper(out[0])
            for j in range(n - 1):
                if low[j] == sep:
                    out[j + 1] = _upper(out[j + 1])
            w = out
        elif op == "3":
            seen = 0
            for j in range(n):
                if w[j] == p2:
                    if seen == p1:
                        if j + 1 < n:
                            w[j + 1] = _tog(w[j + 1])
                        break
                    seen += 1
        elif op == "M":
            mem = bytes(w)
        elif op == "4":
            if n + len(mem) >= RP:
                return None
            w = w + mem
        elif op == "6":
            if n + len(mem) >= RP:
                return None
            w = bytearray(mem) + w
        elif op == "X":
            if p2 < 1 or p1 + p2 > len(mem) or p3 > n or n + p2 > RP:
                return None
            w = w[:p3] + mem[p1:p1 + p2] + w[p3:]
        elif op == "<":
            if n > p1:
                return None
        elif op == ">":
            if n < p1:
                return None
        elif op == "_":
            if n != p1:
                return None
        elif op == "!":
            if p1 in w:
                return None
        elif op == "/":
            if p1 not in w:
                return None
        elif op == "(":
            if not n or w[0] != p1:
                return None
        elif op == ")":
            if not n or w[-1] != p1:
                return None
        elif op == "=":
            if p1 >= n or w[p1] != p2:
                return None
        elif op == "%":
            if w.count(p2) < p1:
                return None
        elif op == "Q":
            if bytes(w) == mem:
                return None
        else:  # pragma: no cover - parse() admits only the ops above
            raise ValueError(op)
    return bytes(w)


def expand(rule_lines, words):
    rules = [r for r in (parse(x) for x in rule_lines) if r]
    return [[apply(r, w) for r in rules] for w in words]
