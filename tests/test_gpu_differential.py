"""Differential test at scale: random m22000 check jobs of every shape through the HIP path, each result tuple
compared with the oracle (web/common.php:157-307 restated).  North_star asks for zero mismatches against the PHP
check path on mixed m22000 sets.  The other parity tests each cover one dimension. This one mixes all of them in
the same batches:

* PMKID and keyver 1/2/3 lines, with planted corrections of either endianness;
* ESSIDs of 1..64 arbitrary bytes, and keys of 0..80 bytes (NUL, 0xff, ':' and '*' included), plain, as `$HEX[..]`
  or null;
* caller PMKs: right, wrong or all-zero (submission's zero-PMK probe, common.php:592);
* the call sites' nc values, -9..258;
* mutated lines from tests/mutate.py.

Jobs run as check_batch calls of 1..400 jobs, plus single calls for a sample.  The size is
DWPA_DIFF_JOBS (default 1,500, ~20 s on one MI355X); round 5 ran it once at 60,000 jobs
(profiles/r05/differential/), round 6 at 30,000 on the device and 30,000 on the host backend
(DWPA_TEST_HOST_BACKEND=1, tests/conftest.py; profiles/r06/differential/)."""
import os
import random
from concurrent.futures import ThreadPoolExecutor

import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from tests.mutate import mutate  # noqa: E402
from oracle import oracle as O  # noqa: E402

NCS = [-9, -1, 0, 1, 2, 7, 8, 16, 127, 128, 131, 258]


def _bytes(rng, lo, hi):
    return bytes(rng.choice([0, 0x2a, 0x3a, 0xff, 0x80, rng.randrange(256)]) for _ in range(rng.randint(lo, hi)))


def _job(rng, nets):
    if rng.random() < 0.3:
        essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]  # shared ESSIDs: PMKs derived once per pair
    else:
        essid, ap, sta, an, sn = _bytes(rng, 1, 64), rng.randbytes(6), rng.randbytes(6), rng.randbytes(32), \
            rng.randbytes(32)
    psk = _bytes(rng, 0, 80) if rng.random() < 0.3 else S.fast_psk(rng)
    kind = rng.choice(["pmkid", 1, 2, 3])
    if kind == "pmkid":
        line = S.pmkid_line(psk, essid, ap, sta)
    else:
        line = S.eapol_line(psk, essid, ap, sta, an, sn, kind, rng.randint(-70, 70), rng.choice(["LE", "BE"]),
                            mp=rng.choice([0x00, 0x02, 0x80, 0x10, 0x20, 0x40]), eapol_len=rng.choice([99, 121, 200]),
                            rng=rng)
    if rng.random() < 0.08:
        line = mutate(rng, line)
    keys = [S.fast_psk(rng, 0, 20) if rng.random() < 0.9 else None for _ in range(rng.randint(0, 12))]
    if rng.random() < 0.75:
        form = psk if rng.random() < 0.8 else b"$HEX[" + psk.hex().encode() + b"]"
        keys.insert(rng.randint(0, len(keys)), form)
    r = rng.random()
    pmk = False if r < 0.8 else (S.pmk(psk, essid) if r < 0.9 else (bytes(32) if r < 0.95 else rng.randbytes(32)))
    return (line, keys, pmk, rng.choice(NCS))


def test_differential_mixed_jobs():
    n = int(os.environ.get("DWPA_DIFF_JOBS", "1500"))
    rng = random.Random(int(os.environ.get("DWPA_DIFF_SEED", "55")))
    nets = [S.random_net(rng) for _ in range(24)]
    jobs = [_job(rng, nets) for _ in range(n)]
    with ThreadPoolExecutor(16) as ex:
        exp = list(ex.map(lambda a: O.c_check_key_m22000(*a), jobs, chunksize=64))
    got, i = [], 0
    while i < n:
        k = rng.choice([1, 7, 60, 400])
        got += dwpa_amd.check_batch(jobs[i:i + k])
        i += k
    mism = [(j, g, e) for j, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not mism, (len(mism), mism[:3])
    for j in range(0, n, 97):
        assert dwpa_amd.check_key_m22000(*jobs[j]) == exp[j], j
    hits = sum(1 for e in exp if e)
    backend = {0: "device", 1: "host backend", 2: "host fallback"}[dwpa_amd.check_stats()["backend"]]
    print(f"differential: {n} jobs, {hits} hits, "
          f"{sum(1 for e in exp if e and e[1] not in (None, 0))} with a nonce correction, 0 mismatches "
          f"(last call on the {backend})")
    assert hits > n // 4
