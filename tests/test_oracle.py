"""CPU: the parity oracle pinned against the reference's own KAT and public vectors, and C vs Python oracle."""
import hashlib
import random

import pytest

from oracle import oracle as O
from tests import synth as S
from tests.conftest import dec, job_args


def test_challenge_kat(kat):
    # help_crack.py:690-699: both challenge lines crack with PSK aaaa1234 (run() requires 2 records, :893)
    for c in kat["challenge"]:
        line = c["line"].encode()
        exp = dec(c["expect"])
        assert O.c_check_key_m22000(line, [b"aaaa1234"]) == exp
        assert O.py_check_key_m22000(line, [b"aaaa1234"]) == exp
        assert exp[0] == b"aaaa1234"


def test_challenge_eapol_needs_nonce_correction(kat):
    r = O.c_check_key_m22000(kat["challenge"][1]["line"].encode(), [b"aaaa1234"], False, 8)
    assert r[1:3] == [4, "LE"]
    assert O.c_check_key_m22000(kat["challenge"][1]["line"].encode(), [b"aaaa1234"], False, 2) is False


def test_pbkdf2_vectors(kat):
    for v in kat["pbkdf2"]:
        p, s, dk = bytes.fromhex(v["password"]), bytes.fromhex(v["salt"]), v["dk"]
        assert O.c_pbkdf2(p, s, v["iterations"], len(dk) // 2).hex() == dk
        assert O.c_pbkdf2(p, s, 4096, 32).hex() == v["pmk32"]
        assert hashlib.pbkdf2_hmac("sha1", p, s, 4096, 32).hex() == v["pmk32"]
    assert len(kat["pbkdf2"]) >= 5


def test_cmac_vectors(kat):
    for v in kat["cmac"]:
        k, m = bytes.fromhex(v["key"]), bytes.fromhex(v["msg"])
        assert O.c_omac1_aes_128(m, k).hex() == v["tag"]
        assert O.omac1_aes_128(m, k).hex() == v["tag"]


def test_mixed_golden_both_oracles(mixed):
    for j in mixed:
        line, keys, pmk, nc = job_args(j)
        exp = dec(j["expect"])
        assert O.c_check_key_m22000(line, keys, pmk, nc) == exp, j["tag"]
        assert O.py_check_key_m22000(line, keys, pmk, nc) == exp, j["tag"]


def test_nc_windows_golden(nc_windows):
    """The call sites' nonce windows (common.php:606,919: nc 131 and 258; odd and negative nc): the C oracle on
    every fixture job, the pure-Python oracle on the short ones (its AES makes the 300-key jobs take minutes;
    make_golden.py asserted both on all of them when it wrote the file)."""
    for j in nc_windows:
        line, keys, pmk, nc = job_args(j)
        exp = dec(j["expect"])
        assert O.c_check_key_m22000(line, keys, pmk, nc) == exp, j["tag"]
        if len(keys) <= 4 and (nc < 200 or line[4:6] == b"02" and b"kv3" not in j["tag"].encode()):
            assert O.py_check_key_m22000(line, keys, pmk, nc) == exp, j["tag"]


@pytest.mark.parametrize("seed", [11, 12])
def test_oracles_agree_random(seed):
    rng = random.Random(seed)
    for i in range(6):
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.random_psk(rng)
        kv = rng.choice([1, 2, 3])
        line = S.eapol_line(psk, essid, ap, sta, an, sn, kv, rng.randint(-3, 3), rng.choice(["LE", "BE"]), rng=rng)
        keys = [S.random_psk(rng), psk]
        a = O.c_check_key_m22000(line, keys, False, 8)
        assert a == O.py_check_key_m22000(line, keys, False, 8)
        assert a and a[0] == psk


def test_hash_m22000():
    for line in S.CHALLENGE_LINES:
        f = line.split(b"*")
        assert O.c_hash_m22000(line) == hashlib.md5(b"".join(f[1:8])).digest() == O.hash_m22000(line)
    assert O.c_hash_m22000(b"WPA*01*x") is False


def test_hc_unhex_cases():
    assert O.hc_unhex(b"$HEX[414243]") == b"ABC"
    assert O.hc_unhex(b"$HEX[]") == b"$HEX[]"
    assert O.hc_unhex(b"$HEX[41424]") == b"$HEX[41424]"
    assert O.hc_unhex(b"$HEX[41zz]") == b"$HEX[41zz]"
    assert O.hc_unhex(b"$HEX[4142]x") == b"$HEX[4142]x"
    assert O.hc_unhex(b"plain") == b"plain"


def test_long_keys_both_oracles():
    """Keys longer than the C oracle's 4096-byte result buffer (hash_pbkdf2 takes any length): the C and Python
    restatements agree, and the key comes back whole, plain or from its $HEX[] form."""
    ap, sta = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")
    for n in (4096, 4097, 20000):
        k = bytes(random.Random(n).randrange(256) for _ in range(n))
        pmk = O.c_pbkdf2(k, b"ESSID")
        assert pmk == O.pbkdf2_pmk(k, b"ESSID")
        line = S.pmkid_line(k, b"ESSID", ap, sta, pmk)
        for cand in ([b"x" * 9, k], [b"$HEX[" + k.hex().encode() + b"]"]):
            r = O.c_check_key_m22000(line, cand)
            assert r == O.py_check_key_m22000(line, cand) and r[0] == k and r[3] == pmk
        assert O.c_check_many(line, [b"y" * 8, k])[0] == 1
