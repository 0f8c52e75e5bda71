"""GPU box: the library's two check-path backends against each other and the oracle, and its routing between them
(DESIGN.md 1.1).

The same jobs run once with every derive on the host backend (host_max_pmks huge) and once with the host backend off
(host_max_pmks -1: every call on the gfx950 device); both result lists must equal the C oracle's exactly.  Then the
default routing: a one-key call is answered by the host backend, a call far above the threshold by the device, and a
process that allows the host backend and makes only small calls never probes the device (dwpa_init does not start
the HIP runtime).
"""
import json
import os
import random
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

import dwpa_amd
from dwpa_amd import _lib as L
from dwpa_amd import m22000 as M
from oracle import oracle as O
from tests import synth as S
from tests.conftest import ROOT, dec, job_args

pytestmark = [pytest.mark.gpu, pytest.mark.host_routing]


def _oracle_many(jobs):
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda a: O.c_check_key_m22000(*a), jobs))


def _both(jobs):
    """(host results, device results) of one dwpa_check_batch over `jobs`, each checked for the backend it ran on."""
    try:
        M.init(host_max_pmks=1 << 30)
        host = dwpa_amd.check_batch(jobs)
        assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_SMALL
        M.init(host_max_pmks=-1)
        dev = dwpa_amd.check_batch(jobs)
        assert M.check_stats()["backend"] == L.DWPA_BACKEND_DEVICE
    finally:
        M.init()
    return host, dev


def _mixed_jobs(seed, n):
    rng = random.Random(seed)
    nets = [S.random_net(rng) for _ in range(16)]
    jobs = []
    for _ in range(n):
        essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]
        psk = S.random_psk(rng)
        kind = rng.choice(["pmkid", 1, 2, 3])
        line = (S.pmkid_line(psk, essid, ap, sta) if kind == "pmkid" else
                S.eapol_line(psk, essid, ap, sta, an, sn, kind, rng.randint(-70, 70), rng.choice(["LE", "BE"]),
                             rng=rng))
        keys = [S.random_psk(rng) for _ in range(rng.randint(0, 24))]
        if rng.random() < 0.8:
            keys.insert(rng.randint(0, len(keys)), psk)
        if rng.random() < 0.1:
            keys.insert(rng.randint(0, len(keys)), None)
        pmk = S.pmk(psk if rng.random() < 0.5 else S.random_psk(rng), essid) if rng.random() < 0.15 else False
        jobs.append((line, keys, pmk, rng.choice([-3, 0, 1, 8, 17, 128, 131, 258])))
    return jobs


def test_goldens_host_equals_device(mixed, nc_windows, kat):
    jobs = [job_args(j) for j in mixed + nc_windows]
    jobs += [(c["line"], [b"aaaa1234"], False, 128) for c in kat["challenge"]]
    exp = [dec(j["expect"]) for j in mixed + nc_windows] + [dec(c["expect"]) for c in kat["challenge"]]
    host, dev = _both(jobs)
    assert host == exp
    assert dev == exp


def test_mutated_and_random_host_equals_device():
    from tests.mutate import mutated_jobs
    jobs = mutated_jobs(5, 600) + _mixed_jobs(11, 400)
    exp = _oracle_many(jobs)
    host, dev = _both(jobs)
    assert [i for i, (h, e) in enumerate(zip(host, exp)) if h != e] == []
    assert [i for i, (d, e) in enumerate(zip(dev, exp)) if d != e] == []
    assert sum(1 for e in exp if e) > 200


def test_pbkdf2_host_equals_device():
    rng = random.Random(3)
    essid = rng.randbytes(rng.randint(1, 32))
    keys = [rng.randbytes(rng.randint(8, 63)) for _ in range(300)] + [b"", b"k" * 64, rng.randbytes(1000)]
    try:
        M.init(host_max_pmks=1 << 30)
        host = dwpa_amd.pbkdf2_pmk(keys, essid)
        M.init(host_max_pmks=-1)
        dev = dwpa_amd.pbkdf2_pmk(keys, essid)
    finally:
        M.init()
    assert host == dev
    assert b"".join(host) == O.c_pbkdf2_many(keys, essid, threads=8)


def test_default_routing():
    """One key: the host backend.  Thousands of keys: the device, cold or warm (8 x the default budget is far below).
    Caller-PMK checks: a PMKID line's one HMAC on the host, a 521-attempt EAPOL window on the (warm) device."""
    rng = random.Random(8)
    essid, ap, sta, an, sn = S.random_net(rng)
    psk = S.fast_psk(rng)
    line = S.eapol_line(psk, essid, ap, sta, an, sn, 2, 5, "BE", rng=rng)
    M.init()
    assert dwpa_amd.check_key_m22000(line, [psk]) == [psk, 5, "BE", S.pmk(psk, essid)]
    assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_SMALL
    keys = [S.fast_psk(rng) for _ in range(40000)] + [psk]
    assert dwpa_amd.check_key_m22000(line, keys) == [psk, 5, "BE", S.pmk(psk, essid)]
    assert M.check_stats()["backend"] == L.DWPA_BACKEND_DEVICE
    # caller-PMK checks (common.php:592,606,919): a PMKID line's one HMAC on the host, a 521-attempt EAPOL window
    # (the device is warm now) on the GPU
    pline = S.pmkid_line(psk, essid, ap, sta)
    pmk = S.pmk(psk, essid)
    r = dwpa_amd.check_key_m22000(pline, [b""], pmk, 258)
    assert r == O.c_check_key_m22000(pline, [b""], pmk, 258) and r
    assert M.check_stats()["backend"] == L.DWPA_BACKEND_HOST_SMALL
    r = dwpa_amd.check_key_m22000(line, [b""], pmk, 258)
    assert r == O.c_check_key_m22000(line, [b""], pmk, 258) and r
    assert M.check_stats()["backend"] == L.DWPA_BACKEND_DEVICE


_CHILD = r"""
import json, random, sys
sys.path.insert(0, sys.argv[1])
import dwpa_amd
from dwpa_amd import _lib as L, m22000 as M
from tests import synth as S
assert M.init(allow_cpu_fallback=1) == 0
rng = random.Random(9)
essid, ap, sta, an, sn = S.random_net(rng)
psk = S.fast_psk(rng)
line = S.pmkid_line(psk, essid, ap, sta)
out = {"small": []}
for _ in range(5):
    out["small"].append([dwpa_amd.check_key_m22000(line, [S.fast_psk(rng), psk]) == [psk, None, None, S.pmk(psk, essid)],
                         M.check_stats()["backend"]])
out["devices_after_small"] = M.resource_stats()["devices"]
keys = [S.fast_psk(rng) for _ in range(30000)] + [psk]
out["large_ok"] = dwpa_amd.check_key_m22000(line, keys) == [psk, None, None, S.pmk(psk, essid)]
out["large_backend"] = M.check_stats()["backend"]
out["devices_after_large"] = M.resource_stats()["devices"]
print(json.dumps(out))
"""


def test_small_calls_never_start_the_device():
    """A fresh process that allows the host backend (as the PHP wrapper's ffi() does) and makes small calls has not
    probed the device; its first large call does, and runs there."""
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, DWPA_HOST_MAX_PMKS="", DWPA_CPU_FALLBACK=""))
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["small"] == [[True, L.DWPA_BACKEND_HOST_SMALL]] * 5
    assert out["devices_after_small"] == 0
    assert out["large_ok"] and out["large_backend"] == L.DWPA_BACKEND_DEVICE
    assert out["devices_after_large"] >= 1
