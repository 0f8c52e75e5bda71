"""CPU: the reference's own rule file (help_crack/bestWPA.rule:1-145, what `hashcat --stdout -r bestWPA.rule`
expands at help_crack.py:508-509,575-576) is fully handled.

The file stays in the reference (it is read here when /root/reference is present, and the test is skipped
otherwise -- e.g. on the GPU box).  Two facts are pinned:

* every one of its 145 rules parses through the library's host rule parser (`dwpa_rules_expand` with
  out == NULL only parses, no device is touched), and through the rule oracle (oracle/rules.py);
* every (op, argument) pair the file uses occurs in `dwpa_amd.rulesets.wpa_rules()`, the rule set the GPU rule
  tests (tests/test_gpu_parity.py, tests/test_gpu_baseline_sizes.py) run against the oracle -- so the GPU rule
  engine is exercised on every operation bestWPA.rule can ask of it.
"""
import ctypes
import os

import pytest

from dwpa_amd import _lib as L
from dwpa_amd.rulesets import wpa_rules
from oracle import rules as R

BEST_WPA = "/root/reference/help_crack/bestWPA.rule"

pytestmark = pytest.mark.skipif(not os.path.exists(BEST_WPA), reason="reference rule file not present")


def _best_rules():
    with open(BEST_WPA, "rb") as f:
        txt = f.read().decode("latin-1")
    return txt, [l for l in txt.split("\n") if l.strip()]


def _nrules_host(text: str) -> int:
    raw = text.encode("latin-1")
    n = ctypes.c_uint32(0)
    rc = L.load().dwpa_rules_expand(0, raw, len(raw), None, 0, None, None, ctypes.byref(n))
    assert rc == 0
    return n.value


def test_best_wpa_all_rules_parse_host_and_oracle():
    txt, lines = _best_rules()
    assert len(lines) == 145
    assert _nrules_host(txt) == 145
    # rule by rule: each one parses on its own (none is silently merged or dropped)
    assert all(_nrules_host(l) == 1 for l in lines)
    assert all(R.parse(l) for l in lines)


def test_best_wpa_ops_covered_by_tested_rule_set():
    _, lines = _best_rules()
    best_ops = {op for l in lines for op in R.parse(l)}
    tested_ops = {op for l in wpa_rules() for op in R.parse(l)}
    missing = sorted(best_ops - tested_ops, key=str)
    assert not missing, missing
    # the op kinds the survey lists for the file
    assert {op for op, *_ in best_ops} == set(":rulcT$^][sD'dpf")
