"""CPU: the library's host logic (parsing with PHP semantics, attempt-list construction, rule parsing) against
the oracle and the golden fixtures -- no device needed."""
import ctypes

import pytest

import dwpa_amd
from dwpa_amd import _lib as L
from tests import synth as S
from dwpa_amd.rulesets import wpa_rules
from oracle import oracle as O
from oracle import rules as R
from tests.conftest import job_args


def test_parse_accepts_exactly_what_php_accepts(mixed):
    for j in mixed:
        line, keys, pmk, nc = job_args(j)
        p = dwpa_amd.parse_m22000(line, nc)
        has_key = any(k is not None for k in keys)
        if j["expect"]:
            assert isinstance(p, dict), j["tag"]
        if isinstance(p, int):
            # a line the library rejects can never produce a PHP hit
            assert not j["expect"], j["tag"]


def test_parse_fields_challenge():
    p = dwpa_amd.parse_m22000(S.CHALLENGE_LINES[1], 8)
    assert p["type"] == 2 and p["keyver"] == 2 and p["essid"] == b"dlink"
    assert p["mac_ap"].hex() == "1c7ee5e2f2d0" and p["mac_sta"].hex() == "0026c72e4900"
    assert p["attempts"] == 1 + 4 * ((8 >> 1) + 1) and p["lists"] == 1
    assert p["hash_m22000"] == O.c_hash_m22000(S.CHALLENGE_LINES[1])
    assert dwpa_amd.parse_m22000(S.CHALLENGE_LINES[0])["type"] == 1


@pytest.mark.parametrize("nc,expect", [(128, 261), (8, 21), (0, 5), (1, 5), (-2, 1), (-1, 1), (4, 13)])
def test_php_attempt_counts(nc, expect):
    # common.php:237,250-300: N+0, then V+k,V-k,N+k,N-k for k = 1..(nc>>1)+1 (do/while)
    assert dwpa_amd.parse_m22000(S.CHALLENGE_LINES[1], nc)["attempts"] == expect


def test_hashcat_attempts_honour_message_pair():
    line = S.CHALLENGE_LINES[1]
    f = line.split(b"*")
    for mp, exp in [(b"00", 1 + 32), (b"10", 1), (b"20", 1 + 16), (b"40", 1 + 16), (b"80", 1 + 32)]:
        l2 = b"*".join(f[:8] + [mp])
        assert dwpa_amd.parse_m22000(l2, 8, L.DWPA_NC_HASHCAT)["attempts"] == exp, mp


def test_short_anonce_needs_several_lists(mixed):
    for j in mixed:
        if j["tag"].startswith("short-anonce-20-"):
            assert dwpa_amd.parse_m22000(j["line"].encode("latin-1"), j["nc"])["lists"] > 1, j["tag"]
    normal = [j for j in mixed if j["tag"].startswith("c5-2")]
    assert all(dwpa_amd.parse_m22000(j["line"].encode("latin-1"), j["nc"])["lists"] == 1 for j in normal)


def test_parse_error_codes():
    assert dwpa_amd.parse_m22000(b"WPA*01*x") == L.DWPA_E_FORMAT
    assert dwpa_amd.parse_m22000(b"WPA*03*00*11*22*33***") == L.DWPA_E_TYPE
    assert dwpa_amd.parse_m22000(b"WPA*01*zz*11*22*33***") == L.DWPA_E_HEX
    f = S.CHALLENGE_LINES[1].split(b"*")
    eap = bytearray(bytes.fromhex(f[7].decode()))
    eap[6] &= 0xFC
    assert dwpa_amd.parse_m22000(b"*".join(f[:7] + [eap.hex().encode()] + f[8:])) == L.DWPA_E_KEYVER


def test_group_by_essid_dedupes():
    lines = S.CHALLENGE_LINES + [S.CHALLENGE_LINES[0], b"garbage"]
    g = dwpa_amd.group_by_essid(lines)
    assert list(g) == [b"dlink"] and len(g[b"dlink"]) == 2


def test_rule_parser_matches_oracle_count():
    lib = L.load()
    rules = wpa_rules() + ["#comment", "", "X9", "s", "$", "T", "Tz", ": :", "sab sbc"]
    text = "\n".join(rules).encode()
    n = ctypes.c_uint32(0)
    assert lib.dwpa_rules_expand(0, text, len(text), None, 0, None, None, ctypes.byref(n)) == 0
    assert n.value == sum(1 for r in rules if R.parse(r))


@pytest.mark.parametrize("rules,coptions,expect", [
    ("", "", (None, 0, None)),
    ("-S -r help_crack.rules", "", ("help_crack.rules", 0, None)),          # help_crack.py:445-447
    ("", "-d 1,3 --force", (None, 0b101, None)),                             # hashcat numbers devices from 1
    ("--rules-file=x.rule", "--backend-devices 2", ("x.rule", 0b10, None)),
    ("", "--nonce-error-corrections=16", (None, 0, 16)),                     # a -co NC value overrides the 8
])
def test_help_crack_option_parsing(rules, coptions, expect):
    from dwpa_amd.help_crack import _parse_options
    assert _parse_options(rules, coptions) == expect


def test_product_package_loads_no_openssl_or_test_code():
    """VERDICT r4 hygiene: the product package (dwpa_amd and its library) pulls in no OpenSSL-backed module and no
    test infrastructure -- the synthetic-line generator lives in tests/, the CPU oracle in oracle/."""
    import subprocess
    import sys
    code = ("import sys, dwpa_amd, dwpa_amd.help_crack, dwpa_amd.device, dwpa_amd.shard, dwpa_amd.rulesets\n"
            "dwpa_amd.load()\n"
            "bad = [m for m in sys.modules if m.split('.')[0] in ('oracle', 'tests', '_hashlib', 'hashlib', 'hmac')]\n"
            "maps = open('/proc/self/maps').read()\n"
            "print(bad, 'libcrypto' in maps, 'libssl' in maps)\n")
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=root, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "[] False False"
