"""CPU: the library's host backend (dwpa_amd/csrc/host_check.cpp + host_crypto.cpp) against the oracle.

The host backend answers the check path and dwpa_pbkdf2_pmk on the CPU: small calls always (dwpa_config.host_max_pmks)
and every call when no gfx950 device is usable, if allow_cpu_fallback / DWPA_CPU_FALLBACK=1 asks for it.  It is the
library's own code -- SHA-NI / AES-NI or scalar primitives, the TableBuilder's PHP nonce-correction order -- never the
oracle.  Here (no GPU) every call of this module runs on it; the tuples must equal the C oracle's exactly:
the goldens (challenge KAT, 130 mixed jobs, the call sites' nc windows), 1,500 mutated lines, C5-shaped random
batches, binary ESSIDs and keys, keys up to 64 KiB, ESSIDs of 0-1,000 bytes and EAPOL frames up to 900 bytes.  The
scalar primitives (CPUs without SHA-NI / AES-NI) are checked in a child process with DWPA_HOST_SIMD=0.
"""
import ctypes
import os
import random
import subprocess
import sys
import threading
from concurrent.futures import ThreadPoolExecutor

import pytest

import dwpa_amd
from dwpa_amd import _lib as L
from dwpa_amd import m22000 as M
from oracle import oracle as O
from tests import synth as S
from tests.conftest import ROOT, dec, job_args


def _gpu_present():
    return os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "0") != ""


@pytest.fixture(autouse=True)
def _host_backend(monkeypatch):
    """Every call with a derive on the host backend, and the host backend for the rest when there is no device."""
    monkeypatch.setenv("DWPA_CPU_FALLBACK", "1")
    monkeypatch.setenv("DWPA_HOST_MAX_PMKS", "1000000000")
    yield


def _assert_host():
    if not _gpu_present():
        assert M.check_stats()["backend"] in (L.DWPA_BACKEND_HOST_SMALL, L.DWPA_BACKEND_HOST_FALLBACK)


def _oracle_many(jobs):
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda a: O.c_check_key_m22000(*a), jobs))


def test_challenge_kat(kat):
    for c in kat["challenge"]:
        assert dwpa_amd.check_key_m22000(c["line"], [b"aaaa1234"]) == dec(c["expect"])
        _assert_host()
    r = dwpa_amd.check_key_m22000(kat["challenge"][1]["line"], [b"x" * 8, b"aaaa1234"], False, 8)
    assert r[0] == b"aaaa1234" and r[1:3] == [4, "LE"]


def test_pbkdf2_vectors(kat):
    for v in kat["pbkdf2"]:
        p, s = bytes.fromhex(v["password"]), bytes.fromhex(v["salt"])
        assert dwpa_amd.pbkdf2_pmk([p], s)[0].hex() == v["pmk32"]


def test_mixed_golden(mixed):
    for j in mixed:
        line, keys, pmk, nc = job_args(j)
        assert dwpa_amd.check_key_m22000(line, keys, pmk, nc) == dec(j["expect"]), j["tag"]
    got = dwpa_amd.check_batch([job_args(j) for j in mixed])
    _assert_host()
    for j, g in zip(mixed, got):
        assert g == dec(j["expect"]), j["tag"]


def test_nc_windows_golden(nc_windows):
    for j in nc_windows:
        line, keys, pmk, nc = job_args(j)
        assert dwpa_amd.check_key_m22000(line, keys, pmk, nc) == dec(j["expect"]), j["tag"]
    got = dwpa_amd.check_batch([job_args(j) for j in nc_windows])
    for j, g in zip(nc_windows, got):
        assert g == dec(j["expect"]), j["tag"]


def test_mutated_lines_vs_oracle():
    """Parse semantics by mutation (tests/mutate.py): 1,500 mutated PMKID / keyver 1-3 lines, planted key among
    decoys; one batch, and one call per job for the first 200."""
    from tests.mutate import mutated_jobs
    jobs = mutated_jobs(2, 1500)
    exp = _oracle_many(jobs)
    got = dwpa_amd.check_batch(jobs)
    _assert_host()
    mism = [(i, jobs[i][0], g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, mism[:3]
    for i in range(200):
        assert dwpa_amd.check_key_m22000(*jobs[i]) == exp[i], jobs[i][0]
    assert sum(1 for e in exp if e) > 100


def test_random_and_binary_batches_vs_oracle():
    """C5-shaped jobs (PMKID + keyver 1/2/3, planted corrections, shared ESSIDs, null keys) and binary ESSIDs / keys
    with NUL, '*', ':' and $HEX[] forms."""
    rng = random.Random(2024)
    jobs = []
    nets = [S.random_net(rng) for _ in range(12)]
    for i in range(160):
        essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]
        psk = S.random_psk(rng)
        kind = rng.choice(["pmkid", 1, 2, 3])
        line = (S.pmkid_line(psk, essid, rng.randbytes(6), rng.randbytes(6)) if kind == "pmkid" else
                S.eapol_line(psk, essid, rng.randbytes(6), rng.randbytes(6), rng.randbytes(32), rng.randbytes(32),
                             kind, rng.randint(-9, 9), rng.choice(["LE", "BE"]), rng=rng))
        keys = [S.random_psk(rng) for _ in range(rng.randint(0, 12))]
        if rng.random() < 0.8:
            keys.insert(rng.randint(0, len(keys)), psk)
        if rng.random() < 0.1:
            keys.insert(0, None)
        pmk = S.pmk(psk if rng.random() < 0.5 else S.random_psk(rng), essid) if rng.random() < 0.15 else False
        jobs.append((line, keys, pmk, rng.choice([0, 1, 8, 16, 128, 131, 258])))
    for i in range(120):
        essid = bytes(rng.choice([0, 0x2a, 0x3a, 0xff, 0x80, rng.randrange(256)])
                      for _ in range(rng.choice([1, 2, 13, 31, 32, 33, 47, 64])))
        psk = bytes(rng.choice([0, 0xff, 0x3a, rng.randrange(256)]) for _ in range(rng.choice([0, 1, 8, 31, 63, 64, 80])))
        kind = rng.choice(["pmkid", 1, 2, 3])
        ap, sta = rng.randbytes(6), rng.randbytes(6)
        line = (S.pmkid_line(psk, essid, ap, sta) if kind == "pmkid" else
                S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), kind, rng.randint(-5, 5),
                             rng.choice(["LE", "BE"]), rng=rng))
        keys = [bytes(rng.randrange(256) for _ in range(rng.randint(0, 20))) for _ in range(rng.randint(0, 6))]
        if rng.random() < 0.85:
            keys.insert(rng.randint(0, len(keys)), psk if i % 3 else b"$HEX[" + psk.hex().encode() + b"]")
        jobs.append((line, keys, False, rng.choice([0, 8, 128])))
    exp = _oracle_many(jobs)
    got = dwpa_amd.check_batch(jobs)
    mism = [(i, g, e) for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, mism[:3]
    for i in range(0, len(jobs), 5):
        assert dwpa_amd.check_key_m22000(*jobs[i]) == exp[i]
    assert sum(1 for e in exp if e) > 150


def test_pbkdf2_key_and_essid_lengths():
    """Keys of 0..300 bytes (the 64-byte HMAC block boundary: longer keys are hashed first) and 1 KiB..64 KiB, ESSID
    salts of 0..1,000 bytes (1, 2 and 16+ SHA-1 blocks), against the oracle's OpenSSL PBKDF2."""
    rng = random.Random(7)
    keys = [bytes(rng.randrange(256) for _ in range(n)) for n in list(range(0, 70)) + [100, 127, 128, 200, 300]]
    for essid_len in (0, 1, 7, 32, 47, 51, 52, 60, 120, 1000):
        essid = bytes(rng.randrange(256) for _ in range(essid_len))
        assert b"".join(dwpa_amd.pbkdf2_pmk(keys, essid)) == O.c_pbkdf2_many(keys, essid, threads=8), essid_len
    longk = [bytes(rng.randrange(256) for _ in range(n)) for n in (1000, 4095, 4096, 4097, 65537)] + [b"A" * 65536]
    assert b"".join(dwpa_amd.pbkdf2_pmk(longk, b"ThisIsASSID")) == O.c_pbkdf2_many(longk, b"ThisIsASSID", threads=8)


def test_long_keys_and_essids_check_path():
    """Keys up to 64 KiB (plain and $HEX[]) and ESSIDs of 0..1,000 bytes through the check path, PMKID and EAPOL."""
    rng = random.Random(9)
    ap, sta = bytes.fromhex("020000000001"), bytes.fromhex("020000000002")
    long_key = bytes(rng.randrange(256) for _ in range(65536))
    jobs = []
    for kv, line in ((None, S.pmkid_line(long_key, b"ThisIsASSID", ap, sta)),
                     (2, S.eapol_line(long_key, b"ThisIsASSID", ap, sta, bytes(range(32)), bytes(range(32, 64)), 2,
                                      nc=2, mp=0x80))):
        jobs.append((line, [b"x" * 9, long_key[:4097], long_key], False, 8))
        jobs.append((line, [b"$HEX[" + long_key.hex().encode() + b"]"], False, 8))
    for n in (0, 1, 32, 33, 51, 52, 55, 56, 64, 115, 116, 255, 1000):
        essid = bytes(rng.randrange(256) for _ in range(n))
        psk = S.random_psk(rng)
        jobs.append((S.pmkid_line(psk, essid, ap, sta), [b"wrongpsk1", psk], False, 8))
        jobs.append((S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), 1 + n % 3, -1, "BE",
                                  rng=rng), [psk], False, 8))
    exp = _oracle_many(jobs)
    assert all(e and e[0] == long_key for e in exp[:4])
    assert exp[4] is False and exp[5] is False and all(exp[6:])
    assert [dwpa_amd.check_key_m22000(*j) for j in jobs] == exp
    assert dwpa_amd.check_batch(jobs) == exp


def test_long_eapol_frames_vs_oracle():
    """EAPOL frames of 99..900 bytes (nets.struct is varchar(2000)): up to 15 SHA-1/MD5 blocks, 57 CMAC blocks,
    both CMAC last-block cases, hits at +-nc both endians."""
    rng = random.Random(61)
    jobs = []
    for el in (99, 100, 111, 112, 119, 120, 128, 175, 176, 255, 256, 400, 512, 777, 900):
        for kv in (1, 2, 3):
            essid, ap, sta, an, sn = S.random_net(rng)
            psk = S.random_psk(rng)
            nc = rng.choice([8, 128])
            off = rng.choice([0, 1, -1, 4, -4]) if nc == 8 else rng.choice([0, 30, -65, 65])
            line = S.eapol_line(psk, essid, ap, sta, an, sn, kv, off, rng.choice(["LE", "BE"]), eapol_len=el, rng=rng)
            jobs.append((line, [S.random_psk(rng), psk, S.random_psk(rng)], False, nc))
    exp = _oracle_many(jobs)
    assert all(exp)
    assert dwpa_amd.check_batch(jobs) == exp


def test_concurrent_callers():
    """Reentrant: eight threads calling at once (PHP ZTS / a threaded server) each get their own exact answers."""
    rng = random.Random(33)
    jobs = []
    for i in range(48):
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.random_psk(rng)
        line = (S.pmkid_line(psk, essid, ap, sta) if i % 4 == 0 else
                S.eapol_line(psk, essid, ap, sta, an, sn, 1 + i % 3, i % 7 - 3, "LE", rng=rng))
        jobs.append((line, [S.random_psk(rng), psk] if i % 5 else [S.random_psk(rng)], False, 128))
    exp = _oracle_many(jobs)
    got = [None] * len(jobs)

    def worker(t):
        for i in range(t, len(jobs), 8):
            got[i] = dwpa_amd.check_key_m22000(*jobs[i])

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert got == exp


_SCALAR_CHILD = r"""
import os, sys, json
sys.path.insert(0, sys.argv[1])
import dwpa_amd
from tests.conftest import load_golden, dec, job_args
bad = []
for c in load_golden("kat.json")["challenge"]:
    if dwpa_amd.check_key_m22000(c["line"], [b"aaaa1234"]) != dec(c["expect"]):
        bad.append("kat")
for j in load_golden("mixed.json")["jobs"]:
    if dwpa_amd.check_key_m22000(*job_args(j)) != dec(j["expect"]):
        bad.append(j["tag"])
for v in load_golden("kat.json")["pbkdf2"]:
    if dwpa_amd.pbkdf2_pmk([bytes.fromhex(v["password"])], bytes.fromhex(v["salt"]))[0].hex() != v["pmk32"]:
        bad.append("pbkdf2")
print(json.dumps(bad))
"""


def test_scalar_primitives_subprocess():
    """DWPA_HOST_SIMD=0: the portable SHA-1 / SHA-256 / MD5 / AES-128 (CPUs without SHA-NI / AES-NI) give the same
    results on the KAT, the 130 mixed jobs and the PBKDF2 vectors."""
    import json
    env = dict(os.environ, DWPA_HOST_SIMD="0", DWPA_CPU_FALLBACK="1", DWPA_HOST_MAX_PMKS="1000000000")
    r = subprocess.run([sys.executable, "-c", _SCALAR_CHILD, ROOT], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1]) == []


@pytest.mark.skipif(_gpu_present(), reason="a GPU is visible: the no-device path is not reachable")
def test_routing_without_a_device(monkeypatch):
    """No device here.  allow_cpu_fallback off and host_max_pmks -1: every compute call fails loudly (DWPA_E_NODEV).
    The default threshold: a small call (one key) is answered by the host backend (backend 1); with host_max_pmks 50
    a call of 500 keys (above 8 x 50 before any device call) is DWPA_E_NODEV.  allow_cpu_fallback on: dwpa_init returns 0 and the large
    call is answered too (backend 2).  Caller-PMK calls (no derive) are host calls when their verify work is tiny, and
    need the fallback above that."""
    monkeypatch.delenv("DWPA_CPU_FALLBACK", raising=False)
    monkeypatch.delenv("DWPA_HOST_MAX_PMKS", raising=False)
    lib = L.load()

    def init(fallback, host_max):
        cfg = L.Config(ctypes.sizeof(L.Config), 0, 0, 0, 0, fallback, host_max)
        return lib.dwpa_init(ctypes.byref(cfg))

    rng = random.Random(5)
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.random_psk(rng)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 2, 3, "LE", rng=rng)
    small = (line, [psk], False, 128)
    nlarge = 500
    large = (line, [S.fast_psk(rng) for _ in range(nlarge - 1)] + [psk], False, 128)
    caller = (line, [b""], S.pmk(psk, essid), 2000)  # 4,001 attempts: above the cold host budget for caller-PMK checks
    small_caller = (line, [b""], S.pmk(psk, essid), 8)  # 17 attempts: answered by the host backend
    exp = {k: O.c_check_key_m22000(*j) for k, j in (("small", small), ("large", large), ("caller", caller),
                                                     ("small_caller", small_caller))}
    assert all(exp.values())
    try:
        assert init(-1, -1) == L.DWPA_E_NODEV
        for j in (small, large, caller):
            with pytest.raises(L.DwpaError) as e:
                dwpa_amd.check_key_m22000(*j)
            assert e.value.code == L.DWPA_E_NODEV
        with pytest.raises(L.DwpaError):
            dwpa_amd.pbkdf2_pmk([psk], essid)
        assert lib.dwpa_device_count() == L.DWPA_E_NODEV
        assert init(-1, 0) == L.DWPA_E_NODEV
        assert dwpa_amd.check_key_m22000(*small) == exp["small"]
        assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_SMALL
        assert dwpa_amd.pbkdf2_pmk([psk], essid)[0] == S.pmk(psk, essid)
        assert dwpa_amd.check_key_m22000(*small_caller) == exp["small_caller"]
        assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_SMALL
        assert init(-1, 50) == L.DWPA_E_NODEV
        with pytest.raises(L.DwpaError):
            dwpa_amd.check_key_m22000(*large)
        with pytest.raises(L.DwpaError):
            dwpa_amd.check_key_m22000(*caller)
        assert init(1, 50) == 0
        assert dwpa_amd.check_key_m22000(*large) == exp["large"]
        st = M.check_stats()
        assert st["backend"] == L.DWPA_BACKEND_HOST_FALLBACK and st["pmks"] == nlarge and st["hits"] == 1
        assert dwpa_amd.check_key_m22000(*caller) == exp["caller"]
        assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_FALLBACK
        assert dwpa_amd.check_batch([small, large, caller]) == [exp["small"], exp["large"], exp["caller"]]
    finally:
        init(0, 0)  # back to the environment's / library's defaults
