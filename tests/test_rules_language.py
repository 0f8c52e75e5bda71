"""CPU: hashcat's rule language.  The server's per-dictionary rules (db/wpa.sql:48,
INSTALL.md:110) reach the client merged (web/content/get_work.php:86-92) and run with `-S -r`
(help_crack/help_crack.py:931-933); bestWPA.rule runs through `--stdout -r` (:508,575).

* the library's host rule parser (dwpa_rules_count) accepts exactly the lines oracle/rules.py parses, and reports
  the ones it skips (counts, first line) -- nothing is dropped silently;
* the interpreter the GPU runs (rules_apply.hpp), compiled for the host (dwpa_rules_apply_host), equals the oracle
  on every function at edge arguments and edge words, on memory sequences and on random combinations.
The GPU side of the same corpus is tests/test_gpu_parity.py::test_rules_language_gpu_vs_oracle.
hashcat is third party: parity with hashcat itself is unpinned (oracle/rules.py states the semantics).
"""
import pytest

import dwpa_amd
from oracle import rules as R
from tests import rule_corpus as C


def test_every_function_parses():
    lines = C.single_function_rules() + C.memory_rules()
    assert all(R.parse(l) is not None for l in lines)
    ops = {op for l in lines for op, *_ in R.parse(l)}
    assert ops == R.ALL_OPS  # the corpus covers the whole language
    present, parsed, first = dwpa_amd.rules_count("\n".join(lines).encode("latin-1"))
    assert (present, parsed, first) == (len(lines), len(lines), 0)


def test_hashcat_loader_counts_vs_oracle():
    """dwpa_rules_count_ex reports both loaders -- the whole language (DWPA_RULES_FULL) and
    hashcat's -r loader (DWPA_RULES_HASHCAT, the default for rule files), which skips lines using reject or memory
    functions -- equal to oracle/rules.py's parse / hashcat_loads, line by line, on the fuzz corpus and in bulk."""
    rules = C.fuzz_rules() + C.single_function_rules() + C.memory_rules()
    for r in rules:
        c = dwpa_amd.rules_count_ex(r.encode("latin-1"))
        ok = R.parse(r) is not None
        assert (c["parsed"], c["loaded_hashcat"], c["rejmem"], c["invalid"]) == \
            (int(ok), int(R.hashcat_loads(r)), int(ok and not R.hashcat_loads(r)), int(not ok)), r
    text = "\n".join(rules).encode("latin-1")
    c = dwpa_amd.rules_count_ex(text)
    parsed = [r for r in rules if R.parse(r) is not None]
    loads = [r for r in rules if R.hashcat_loads(r)]
    assert c["present"] == R.count(rules)[0] and c["parsed"] == len(parsed) and c["loaded_hashcat"] == len(loads)
    assert c["rejmem"] == len(parsed) - len(loads) > 0 and c["invalid"] == len(rules) - len(parsed) > 0
    assert c["first_rejmem_line"] == 1 + next(i for i, r in enumerate(rules) if R.parse(r) and not R.hashcat_loads(r))
    assert dwpa_amd.rules_count(text)[:2] == (c["present"], c["parsed"])  # the interpreter's count is the full one
    # bestWPA.rule's ops (help_crack's --stdout expansion) use neither family: both loaders keep every line
    from dwpa_amd.rulesets import wpa_rules
    w = dwpa_amd.rules_count_ex("\n".join(wpa_rules()).encode())
    assert w["parsed"] == w["loaded_hashcat"] == len(wpa_rules()) and w["rejmem"] == 0


def test_invalid_rules_are_counted_not_dropped():
    bad = C.invalid_rules()
    assert all(R.parse(l) is None for l in bad), [l for l in bad if R.parse(l) is not None]
    good = ["c", "$1", "x12", "X012", "%2a", "30-"]
    lines = ["# comment", ""] + good[:3] + bad + good[3:] + ["   "]
    text = "\n".join(lines).encode("latin-1")
    present, parsed, first = dwpa_amd.rules_count(text)
    assert present == R.count(lines)[0] == len(good) + len(bad) + 1  # the line of spaces is the no-op rule
    assert parsed == R.count(lines)[1] == len(good) + 1
    assert first == 6  # 1-based: '# comment', '', c, $1, x12, then the first invalid line
    for line in bad:
        assert dwpa_amd.rules_count(line.encode("latin-1"))[:2] == (1, 0), line


@pytest.mark.parametrize("group", ["single", "memory", "combo"])
def test_host_interpreter_vs_oracle(group):
    rules = {"single": C.single_function_rules, "memory": C.memory_rules, "combo": C.combo_rules}[group]()
    words = C.words()
    bad = []
    for rule in rules:
        ops = R.parse(rule)
        for w in words:
            exp = R.apply(ops, w)
            got = dwpa_amd.m22000.rules_apply_host(rule.encode("latin-1"), 0, w)
            if got != exp:
                bad.append((rule, w[:20], len(w), got, exp))
    assert not bad, bad[:10]


def test_documented_examples():
    """The examples of hashcat's rule documentation (wiki rule_based_attack), on the host interpreter."""
    ex = [("c", b"p@ssW0rd", b"P@ssw0rd"), ("C", b"p@ssW0rd", b"p@SSW0RD"), ("t", b"p@ssW0rd", b"P@SSw0RD"),
          ("T3", b"p@ssW0rd", b"p@sSW0rd"), ("r", b"p@ssW0rd", b"dr0Wss@p"), ("d", b"p@ssW0rd", b"p@ssW0rdp@ssW0rd"),
          ("p2", b"p@ssW0rd", b"p@ssW0rdp@ssW0rdp@ssW0rd"), ("f", b"p@ssW0rd", b"p@ssW0rddr0Wss@p"),
          ("{", b"p@ssW0rd", b"@ssW0rdp"), ("}", b"p@ssW0rd", b"dp@ssW0r"), ("$1", b"p@ssW0rd", b"p@ssW0rd1"),
          ("^1", b"p@ssW0rd", b"1p@ssW0rd"), ("[", b"p@ssW0rd", b"@ssW0rd"), ("]", b"p@ssW0rd", b"p@ssW0r"),
          ("D3", b"p@ssW0rd", b"p@sW0rd"), ("x04", b"p@ssW0rd", b"p@ss"), ("O12", b"p@ssW0rd", b"psW0rd"),
          ("i4!", b"p@ssW0rd", b"p@ss!W0rd"), ("o3$", b"p@ssW0rd", b"p@s$W0rd"), ("'6", b"p@ssW0rd", b"p@ssW0"),
          ("ss$", b"p@ssW0rd", b"p@$$W0rd"), ("@s", b"p@ssW0rd", b"p@W0rd"), ("z2", b"p@ssW0rd", b"ppp@ssW0rd"),
          ("Z2", b"p@ssW0rd", b"p@ssW0rddd"), ("q", b"p@ssW0rd", b"pp@@ssssWW00rrdd"),
          ("k", b"p@ssW0rd", b"@pssW0rd"), ("K", b"p@ssW0rd", b"p@ssW0dr"), ("*34", b"p@ssW0rd", b"p@sWs0rd"),
          ("L2", b"p@ssW0rd", b"p@\xe6sW0rd"), ("R2", b"p@ssW0rd", b"p@9sW0rd"), ("+2", b"p@ssW0rd", b"p@tsW0rd"),
          ("-1", b"p@ssW0rd", b"p?ssW0rd"), (".1", b"p@ssW0rd", b"psssW0rd"), (",1", b"p@ssW0rd", b"ppssW0rd"),
          ("y2", b"p@ssW0rd", b"p@p@ssW0rd"), ("Y2", b"p@ssW0rd", b"p@ssW0rdrd"),
          ("E", b"p@ssW0rd w0rld", b"P@ssw0rd W0rld"), ("e-", b"p@ssW0rd-w0rld", b"P@ssw0rd-W0rld"),
          ("30-", b"pass-word", b"pass-Word"), ("X428", b"p@ssW0rd", b"p@ssW0rdW0"),
          ("M 4", b"p@ssW0rd", b"p@ssW0rdp@ssW0rd"), ("6", b"p@ssW0rd", b"p@ssW0rdp@ssW0rd"),
          ("<8", b"p@ssW0rd", b"p@ssW0rd"), ("<7", b"p@ssW0rd", None), (">8", b"p@ssW0rd", b"p@ssW0rd"),
          (">9", b"p@ssW0rd", None), ("_8", b"p@ssW0rd", b"p@ssW0rd"), ("_7", b"p@ssW0rd", None),
          ("!z", b"p@ssW0rd", b"p@ssW0rd"), ("!@", b"p@ssW0rd", None), ("/p", b"p@ssW0rd", b"p@ssW0rd"),
          ("/z", b"p@ssW0rd", None), ("(p", b"p@ssW0rd", b"p@ssW0rd"), ("(d", b"p@ssW0rd", None),
          (")d", b"p@ssW0rd", b"p@ssW0rd"), (")p", b"p@ssW0rd", None), ("=1@", b"p@ssW0rd", b"p@ssW0rd"),
          ("=1a", b"p@ssW0rd", None), ("%2s", b"p@ssW0rd", b"p@ssW0rd"), ("%3s", b"p@ssW0rd", None),
          ("rMr Q", b"racecar", None), ("rMr Q", b"p@ssW0rd", b"p@ssW0rd")]
    for rule, w, exp in ex:
        assert R.apply(R.parse(rule), w) == exp, rule
        assert dwpa_amd.m22000.rules_apply_host(rule.encode(), 0, w) == exp, rule


def test_fuzz_parse_and_apply_vs_oracle():
    """Random rule strings (valid and invalid) over the whole alphabet: the library parses exactly the lines the
    oracle parses, and the host interpreter equals the oracle on every parsed one."""
    rules = C.fuzz_rules()
    words = C.fuzz_words()
    lib_parsed = [dwpa_amd.rules_count(r.encode("latin-1"))[1] == 1 for r in rules]
    orc_parsed = [R.parse(r) is not None for r in rules]
    assert lib_parsed == orc_parsed, [r for r, a, b in zip(rules, lib_parsed, orc_parsed) if a != b][:10]
    assert 0.05 < sum(orc_parsed) / len(rules) < 0.95  # both kinds are exercised
    bad = []
    for r, ok in zip(rules, orc_parsed):
        if not ok:
            continue
        ops = R.parse(r)
        for w in words:
            got = dwpa_amd.m22000.rules_apply_host(r.encode("latin-1"), 0, w)
            if got != R.apply(ops, w):
                bad.append((r, w[:12], len(w)))
    assert not bad, bad[:10]


def test_interpreter_under_address_sanitizer():
    """tools/bin/rules_fuzz_asan (make tools): random rule lines (well-formed with out-of-range arguments, and
    garbage) applied to words of 0..300 bytes by the interpreter the GPU runs, compiled for the host with
    AddressSanitizer + UBSan, with the GPU's exact 256 + 4-byte buffers: no out-of-bounds access, no candidate
    longer than 256 bytes."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "bin", "rules_fuzz_asan")
    if not os.path.exists(exe):
        pytest.skip("tools/bin/rules_fuzz_asan not built (make tools)")
    r = subprocess.run([exe, "40000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    st = json.loads(r.stdout.strip().splitlines()[-1])
    assert st["rules_parsed"] > 20000 and st["candidates"] > 20000 and st["rejected"] > 20000
