"""Test corpus for the hashcat rule language: every rule function at edge arguments, on edge words.

Used by tests/test_rules_language.py (host interpreter vs oracle/rules.py, CPU) and tests/test_gpu_parity.py
(GPU rule engine vs oracle/rules.py).  Positions are hashcat's 0-9A-Z characters; the words put them at 0, len-1,
len and beyond, and include the edge sizes of hashcat's 256-byte rule buffer.
"""
from __future__ import annotations

import random

POS = "0123456789ABCFKVZ"          # 0..35 (F=15, K=20, V=31, Z=35)
CHRS = ["a", "A", "s", "1", "-", " ", "$", "\x80", "\xff", "z", "@"]


def words():
    """Edge words: 1..256 bytes (257 is rejected by the engine, so is the empty word), cases, separators, bytes
    >= 0x80, repeated characters for the count / occurrence functions."""
    w = [b"a", b"ab", b"abc", b"password", b"Pass Word-1x", b"p@ssW0rd w0rld", b"aaaa-aaaa-aaaa", b"-a-b-c-",
         b"MiXeD cAsE wOrDs", b"\x80\xff\x7f\x01abc", b"  spaced  out  ", b"0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ",
         b"x" * 35, b"y" * 36, b"qwertyuiop" * 6 + b"abc", b"z" * 64, b"a-" * 64, b"Q" * 127, b"b" * 128,
         b"c" * 200, b"Ab" * 127 + b"X", b"e" * 255, b"f" * 256, b"", b"g" * 257]
    return w


def single_function_rules():
    """Every function of the language alone, at edge arguments."""
    r = list(":lucCtrdf{}[]kKqEM46Q")
    for op in "TpDzZ'yYLR+-.,<>_":
        r += [op + p for p in POS]
    for op in "$^@!/()e":
        r += [op + c for c in CHRS]
    for op in "io=%3":
        r += [op + p + c for p in "0123789AZ" for c in ("a", "-", "1", "\xff")]
    r += ["s" + a + b for a in ("a", "-", " ", "\xff") for b in ("A", "x", "\x00", " ")]
    for op in "xO*":
        r += [op + p + q for p in "0128AZ" for q in "0138AZ"]
    r += ["X" + n + m + i for n in "0138" for m in "0138Z" for i in "018Z"]
    return r


def memory_rules():
    """Memory functions after other functions (memory = the input word until M; Q against it)."""
    return ["M $1 4", "M ^x 6", "$1 M ]", "d M 4", "u 4", "l 6", "M r Q", "M Q", "Q", "r Q", "M c X012 Q",
            "M d X0A0", "X004", "X0Z0", "X100 X100", "M [ X031", "M ] ] 4 X021", "c M t 6 4", "p9 4", "d d d 4",
            "M p9 6", "f M 4", "$a M $b Q", ": Q", "M : Q", "M l Q", "6 6 6", "4 4 4 4", "M X018 4"]


def combo_rules(n: int = 400, seed: int = 11):
    """Random sequences of 2-6 functions over the whole language (seeded)."""
    rng = random.Random(seed)
    pool = single_function_rules() + memory_rules()
    return [" ".join(rng.choice(pool) for _ in range(rng.randint(2, 6))) for _ in range(n)]


def invalid_rules():
    """Lines hashcat skips ("Skipping invalid or unsupported rule"): unknown functions, missing or bad arguments."""
    return ["a", "I", "?", "T", "Ta", "$", "s", "sa", "x1", "x1a", "X01", "X0a1", "i1", "%", "=1", "3a-", "O0",
            "*1", "c T", "u $", "w", "h", "v12", "L", "Ra", "+", ": : J"]


def all_rules():
    return single_function_rules() + memory_rules() + combo_rules()


def fuzz_rules(n: int = 3000, seed: int = 17):
    """Random rule strings over the rule alphabet: function letters, position characters, arbitrary argument bytes
    and spaces, 1-12 characters -- valid and invalid lines alike (seeded)."""
    rng = random.Random(seed)
    ops = ":lucCtrdf{}[]kKqEM46QTpDzZ'yYLR+-.,<>_$^@e!/()io=%3sxO*X"
    args = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcz-$ @\x80\xff"
    out = []
    for _ in range(n):
        m = rng.randint(1, 12)
        out.append("".join(rng.choice(ops) if rng.random() < 0.45 else rng.choice(args) for _ in range(m)))
    return [r for r in out if not r.startswith("#") and r.strip("\r\n")]


def fuzz_words(seed: int = 19):
    rng = random.Random(seed)
    return [bytes(rng.randrange(256) if rng.random() < 0.1 else rng.choice(b"abcdEFGH0123-$ @z") for _ in
                  range(rng.choice([1, 2, 3, 5, 8, 12, 35, 36, 63, 100, 255, 256]))) for _ in range(12)]
