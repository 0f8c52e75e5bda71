"""GPU parity at the BASELINE.json sizes of the FFI-shaped configs.

C1 = 10,000 PSKs against one PMKID line through dwpa_check_m22000 (the PHP FFI call, common.php:157).
C5 = 1,010 mixed jobs x 202 keys through dwpa_check_batch, PHP nonce window nc=128 (261 attempts).

The oracle is checked on the *prefix* of each job's key list up to the key the GPU reported (all keys for a
miss).  check_key_m22000 returns the first key in input order that verifies (common.php:169-306), so the prefix
decides the result by itself: the GPU tuple is correct iff the oracle returns the same tuple on that prefix.
This keeps the whole C5 batch checked bit-exact in the full [key, nc, endian, PMK] tuple at about half the
oracle cost of a full re-check.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from oracle import oracle as O  # noqa: E402

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))
SUBSET = 8  # C5: prefix-oracle every 8th job (plus every zero-PMK job, at the tail) unless DWPA_FULL_ORACLE=1


def _prefix_oracle(job, got):
    line, keys, pmk, nc = job
    if got is False:
        return O.c_check_key_m22000(line, keys, pmk, nc) is False
    # the GPU names the key by value; find its first occurrence (the oracle returns the first hit, too)
    k = next(i for i, key in enumerate(keys) if key is not None and O.hc_unhex(key) == got[0])
    return O.c_check_key_m22000(line, keys[:k + 1], pmk, nc) == got


def test_c1_pmkid_10k_keys():
    line, keys, psk = S.c1_workload()
    got = dwpa_amd.check_key_m22000(line, keys)
    assert got and got[0] == psk and got[1] is None and got[2] is None
    idx, exp = O.c_check_many(line, keys, 128, THREADS)
    assert idx == len(keys) - 1
    assert got == exp


def c5_expected(job, plant):
    """What check_key_m22000 must return for a C5 job: False when no key was planted, else the planted key's tuple
    with (nc, endian, PMK) re-derived by the oracle from that key alone (a caller PMK applies to the first key
    only, common.php:178,188).  The other keys are random 8..63-byte PSKs, so none of them can match first."""
    line, keys, pmk, nc = job
    if plant is None:
        return False
    r = O.c_check_key_m22000(line, [keys[plant]], pmk if plant == 0 else False, nc)
    assert r, ("planted key does not verify", line[:40])
    return r


def test_c5_mixed_batch_full_size():
    """All 1,010 jobs run on the GPU at full size and every job's result is checked exactly: the planted key's
    [key, nc, endian, PMK] tuple (synth.c5_plan records where each PSK was planted) or False for the ~10 % of jobs
    without one.  A deterministic 1-in-SUBSET slice also gets the full prefix check (first-key-in-order rule over
    the real key list).  DWPA_FULL_ORACLE=1 prefix-checks all 1,010 jobs (~100k OpenSSL PBKDF2s: minutes on the
    box's host share, so it is opt-in)."""
    jobs, plants = S.c5_plan()
    assert len(jobs) == 1010 and sum(len(j[1]) for j in jobs) == 1000 * 202 + 10
    got = dwpa_amd.check_batch(jobs)
    # every EAPOL hit carries an NC and endian inside the planted window
    assert all(g[1] is not None and abs(g[1]) <= 8 for g, j in zip(got, jobs) if g and j[0][4:6] == b"02")

    full = os.environ.get("DWPA_FULL_ORACLE") == "1"
    sel = [i for i in range(len(jobs)) if full or i % SUBSET == 0 or i >= 1000]
    with ThreadPoolExecutor(THREADS) as ex:
        exp = list(ex.map(lambda i: c5_expected(jobs[i], plants[i]), range(len(jobs))))
        ok = list(ex.map(lambda i: _prefix_oracle(jobs[i], got[i]), sel))
    bad = [i for i in range(len(jobs)) if got[i] != exp[i]]
    assert not bad, [(i, jobs[i][0][:40], got[i], exp[i]) for i in bad[:3]]
    assert sum(1 for e in exp if e) == sum(1 for p in plants if p is not None) >= 0.85 * len(jobs)
    bad = [sel[n] for n, o in enumerate(ok) if not o]
    assert not bad, [(i, jobs[i][0][:40], got[i]) for i in bad[:3]]
    if full:
        print(f"DWPA_FULL_ORACLE: {len(sel)} jobs prefix-checked, {len(jobs)} exact, 0 mismatches")


def test_batch_head_tail_split():
    """A derive of >= 4 waves per SIMD of unique (ESSID, key) pairs is split: the head (whole waves per SIMD) and
    the tail (the remainder, on the second stream, overlapping the head's verify).  Hits are planted in head slots,
    in tail slots that derive a tail PMK, and in tail slots that re-use a head PMK (same ESSID, later job), and
    re-derived by the oracle from the winning key alone; the random keys around them never match."""
    import random
    rng = random.Random(91)
    n_per = 36000  # 4 ESSIDs x 36,000 unique keys = 144,000 > 4 x 32,768 (MI355X: 256 CUs x 4 SIMDs x 64 / 2)
    nets = [S.random_net(rng, essid_len=9 + e) for e in range(4)]
    keyset = [[b"k%d-%06d-" % (e, i) + S.fast_psk(rng, 8, 20) for i in range(n_per)] for e in range(4)]
    jobs, want = [], []
    for e, (essid, ap, sta, an, sn) in enumerate(nets):
        keys = list(keyset[e])
        hit = [100, 20000, 1000, 30000][e]  # ESSID 3: the key sits past the head boundary (tail PMK)
        line = (S.pmkid_line(keys[hit], essid, ap, sta) if e % 2 else
                S.eapol_line(keys[hit], essid, ap, sta, an, sn, 2, -2 if e else 5, "LE", rng=rng))
        jobs.append((line, keys, False, 8))
        want.append(hit)
    essid, ap, sta, an, sn = nets[3]
    late = keyset[3]
    # later jobs of ESSID 3 (all their slots are tail slots): a key derived by the head, one derived by the tail
    for src in (5, 35000):
        keys = [b"miss-%05d-" % i + S.fast_psk(rng, 8, 12) for i in range(300)]
        keys[150] = late[src]
        jobs.append((S.eapol_line(late[src], essid, ap, sta, an, sn, 2, 3, "BE", rng=rng), keys, False, 8))
        want.append(150)
    got = dwpa_amd.check_batch(jobs)
    for job, g, w in zip(jobs, got, want):
        line, keys, _, nc = job
        assert g and g[0] == keys[w], (line[:30], g)
        assert O.c_check_key_m22000(line, [keys[w]], False, nc) == g


def test_batch_host_tail():
    """A derive of 6 whole waves per SIMD plus a small remainder: the remainder (the tail) is derived on the host
    backend while the head runs (the box's EPYC derives it in well under the head's time), so no
    device tail wave runs.  Hits planted in head PMKs, in host-derived PMKs, and in later jobs re-using both."""
    import random
    rng = random.Random(92)
    n_per = 50000  # 4 ESSIDs x 50,000 = 200,000 = 6 x 32,768 + 3,392 (MI355X: 256 CUs x 4 SIMDs x 64 / 2)
    nets = [S.random_net(rng, essid_len=9 + e) for e in range(4)]
    keyset = [[b"h%d-%06d-" % (e, i) + S.fast_psk(rng, 8, 20) for i in range(n_per)] for e in range(4)]
    jobs, want = [], []
    for e, (essid, ap, sta, an, sn) in enumerate(nets):
        keys = keyset[e]
        hit = [10, 25000, 40000, 49990][e]  # ESSID 3's key is one of the last derived: a host-tail PMK
        line = (S.pmkid_line(keys[hit], essid, ap, sta) if e % 2 else
                S.eapol_line(keys[hit], essid, ap, sta, an, sn, 3 if e else 2, -4, "BE", rng=rng))
        jobs.append((line, keys, False, 8))
        want.append(hit)
    essid, ap, sta, an, sn = nets[3]
    for src in (7, 49995):  # later jobs re-using a head PMK and a host-tail PMK
        keys = [b"again-%05d-" % i + S.fast_psk(rng, 8, 12) for i in range(100)]
        keys[60] = keyset[3][src]
        jobs.append((S.eapol_line(keyset[3][src], essid, ap, sta, an, sn, 1, 2, "LE", rng=rng), keys, False, 8))
        want.append(60)
    got = dwpa_amd.check_batch(jobs)
    st = dwpa_amd.check_stats()
    for job, g, w in zip(jobs, got, want):
        line, keys, _, nc = job
        assert g and g[0] == keys[w], (line[:30], g)
        assert O.c_check_key_m22000(line, [keys[w]], False, nc) == g
    assert st["pmks"] == 4 * n_per + 200 - 2 and st["tail_pmks"] == 4 * n_per + 200 - 2 - 6 * 32768
    if os.environ.get("DWPA_HOST_TAIL") == "0":
        assert st["tail_waves"] > 0, st  # the switch keeps the remainder on the GPU
    else:
        assert st["tail_waves"] == 0, st  # the remainder came from the host backend


def test_batch_host_tail_switch_off():
    """The same batch with DWPA_HOST_TAIL=0 (read once per process, so in a child): the remainder runs as GPU tail
    waves and every result is the same."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(root, "tests", "test_gpu_configs.py") + "::test_batch_host_tail"],
                       cwd=root, env=dict(os.environ, DWPA_HOST_TAIL="0"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "1 passed" in r.stdout


def test_batch_fanout_dedup_and_mixed_salt_lengths():
    """put_work shape (common.php:879-902): one submitted key checked against every net of an ESSID, plus PMK
    re-use jobs (:919) -- the engine derives each (ESSID, key) once.  ESSIDs of 1..60 bytes put 1- and 2-block
    salts into the same multi-salt launch."""
    import random
    rng = random.Random(77)
    jobs = []
    for essid_len in (1, 7, 32, 51, 52, 60):
        essid = bytes(rng.randrange(0x20, 0x7f) for _ in range(essid_len))
        psk = S.fast_psk(rng)
        shared = [S.fast_psk(rng) for _ in range(5)] + [psk]
        pmk = S.pmk(psk, essid)
        for k in range(24):
            ap, sta = rng.randbytes(6), rng.randbytes(6)
            right = k % 3 != 2
            the = pmk if right else S.pmk(b"other-" + psk, essid)
            if k % 2:
                line = S.pmkid_line(psk, essid, ap, sta, the_pmk=the)
            else:
                line = S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), 1 + k % 3,
                                    rng.randint(-4, 4), rng.choice(["LE", "BE"]), the_pmk=the, rng=rng)
            jobs.append((line, [psk], False, 128))
            jobs.append((line, shared, False, 16))
            jobs.append((line, [b""], pmk, 9))  # PMK re-use: caller PMK, no derivation
    got = dwpa_amd.check_batch(jobs)
    with ThreadPoolExecutor(THREADS) as ex:
        exp = list(ex.map(lambda j: O.c_check_key_m22000(*j), jobs))
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, [(i, got[i], exp[i]) for i in bad[:3]]
    assert sum(1 for e in exp if e) >= len(jobs) // 2


def test_batch_dedup_hex_forms_nulls_and_key_index():
    """The check path's slot table (engine.cpp SlotTable): keys are deduplicated per ESSID on their decoded bytes, so
    "$HEX[..]" (either hex case) and the plain form of one key share a PMK, while malformed $HEX[ forms stay literal
    (hc_unhex, common.php:3-25); null keys are skipped but still count in the returned key index
    (common.php:172,240), and a caller PMK applies to the first non-null key only (:178).  Every job against the
    oracle."""
    import random
    rng = random.Random(91)
    essid = b"dedup-net"
    psk = b"Pa55:w\xc3\xb6rd!"
    hexl, hexu = b"$HEX[" + psk.hex().encode() + b"]", b"$HEX[" + psk.hex().upper().encode() + b"]"
    near = [b"$HEX[" + psk.hex().encode()[:-1] + b"]", b"$HEX[" + psk.hex().encode() + b"", b"$HEX[zz]", b"$HEX[]",
            psk + b" ", b""]
    pmk = S.pmk(psk, essid)
    jobs = []
    for k in range(40):
        ap, sta = rng.randbytes(6), rng.randbytes(6)
        if k % 2:
            line = S.pmkid_line(psk, essid, ap, sta)
        else:
            line = S.eapol_line(psk, essid, ap, sta, rng.randbytes(32), rng.randbytes(32), 1 + k % 3,
                                rng.randint(-3, 3), rng.choice(["LE", "BE"]), rng=rng)
        keys = [None] * (k % 4) + rng.sample(near, 3) + [None]
        form = (psk, hexl, hexu)[k % 3]
        keys.insert(rng.randrange(len(keys) + 1), form)
        if k % 5 == 0:
            keys.append(psk)  # a second copy later in the same job
        caller = pmk if k % 7 == 0 else (b"\x11" * 32 if k % 7 == 1 else False)
        jobs.append((line, keys, caller, 8))
    jobs.append((S.pmkid_line(psk, essid, b"\x01" * 6, b"\x02" * 6), [None, None], False, 8))  # only nulls
    got = dwpa_amd.check_batch(jobs)
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    bad = [i for i, (g, e) in enumerate(zip(got, exp)) if g != e]
    assert not bad, [(i, got[i], exp[i]) for i in bad[:3]]
    assert sum(1 for e in exp if e) >= 30


def test_batch_chunked_across_essid_groups():
    """dwpa_init(batch=...) caps the slots per derive, so one call runs in several chunks whose boundaries cut
    through ESSID groups (the per-group dedup and key-byte counts are then clipped to the chunk); the results
    equal the oracle's job by job."""
    import ctypes
    import random
    from dwpa_amd import _lib as L
    rng = random.Random(93)
    nets = [S.random_net(rng) for _ in range(5)]
    jobs = []
    for i in range(60):
        essid, ap, sta, an, sn = nets[i % 5]
        psk = S.fast_psk(rng)
        line = (S.pmkid_line(psk, essid, rng.randbytes(6), sta) if i % 3 == 0 else
                S.eapol_line(psk, essid, rng.randbytes(6), sta, rng.randbytes(32), rng.randbytes(32), 1 + i % 3,
                             rng.randint(-4, 4), rng.choice(["LE", "BE"]), rng=rng))
        keys = [S.fast_psk(rng, 8, 12) for _ in range(rng.randint(20, 90))]
        keys[rng.randrange(len(keys))] = psk
        keys += keys[:5]  # duplicates inside the job, and (same ESSID) across jobs
        jobs.append((line, keys, False, rng.choice([8, 128])))
    lib = L.load()
    cfg = L.Config(ctypes.sizeof(L.Config), 0, 1000, 0)
    assert lib.dwpa_init(ctypes.byref(cfg)) == 0
    try:
        got = dwpa_amd.check_batch(jobs)
    finally:
        cfg = L.Config(ctypes.sizeof(L.Config), 0, 0, 0)
        lib.dwpa_init(ctypes.byref(cfg))
    with ThreadPoolExecutor(THREADS) as ex:
        exp = list(ex.map(lambda j: O.c_check_key_m22000(*j), jobs))
    assert got == exp
    assert all(exp)


def test_pbkdf2_pmk_duplicate_keys():
    keys = [b"password", b"password", b"12345678", b"password", b"x" * 63, b"12345678"]
    essid = b"linksys"
    got = dwpa_amd.pbkdf2_pmk(keys, essid)
    assert got == [O.c_pbkdf2(k, essid) for k in keys]


@pytest.mark.parametrize("nkeys", [70000, 66800])
def test_pbkdf2_pmk_head_tail_split(nkeys):
    """dwpa_pbkdf2_pmk over > 2 waves per SIMD of keys (the head/tail split of the derive, joined before the PMKs are
    copied out), with duplicates and the empty key: every PMK in its input position, a sample of 300 spread over head
    and tail against the oracle and every duplicate equal to its first copy.  70,000 keys leave a ~4,400-PMK tail for
    the GPU; 66,800 a ~1,200-PMK one, which the host backend derives beside the head."""
    import random
    rng = random.Random(97)
    keys = [b"p%06d-" % i + S.fast_psk(rng, 4, 30) for i in range(nkeys)]
    for i in range(0, nkeys, 997):
        keys[i] = keys[i // 2]  # duplicates of earlier keys (head and tail positions)
    keys[12345] = b""
    essid = b"split-essid"
    got = dwpa_amd.pbkdf2_pmk(keys, essid)
    assert len(got) == len(keys)
    idx = sorted(set(rng.sample(range(len(keys)), 300)) | {0, 12345, nkeys - 1, 65535, 65536})
    with ThreadPoolExecutor(THREADS) as ex:
        exp = list(ex.map(lambda i: O.c_pbkdf2(keys[i], essid), idx))
    assert [got[i] for i in idx] == exp
    first = {}
    for i, k in enumerate(keys):
        first.setdefault(k, i)
        assert got[i] == got[first[k]]


def test_batch_concurrent_callers():
    """Concurrent dwpa_check_batch calls (PHP ZTS threads, a threaded server) run on separate call contexts of one
    device (DWPA_CALLS_PER_DEVICE, default 2) and overlap on the GPU.  Four threads call three times each, on job
    sets large enough for the head/tail split (>= 2 waves per SIMD of unique keys); every call must equal the
    single-caller result, whose hits are re-derived by the oracle from the winning key alone."""
    import random
    import threading
    rng = random.Random(95)
    sets = []
    for t in range(4):
        jobs = []
        for e in range(3):
            essid, ap, sta, an, sn = S.random_net(rng, essid_len=5 + t + e)
            keys = [b"c%d%d-%06d-" % (t, e, i) + S.fast_psk(rng, 8, 12) for i in range(24000)]
            hit = rng.randrange(len(keys))
            line = (S.pmkid_line(keys[hit], essid, ap, sta) if e == 0 else
                    S.eapol_line(keys[hit], essid, ap, sta, an, sn, e, rng.randint(-6, 6),
                                 rng.choice(["LE", "BE"]), rng=rng))
            jobs.append((line, keys, False, 16))
        sets.append(jobs)
    serial = [dwpa_amd.check_batch(j) for j in sets]
    for jobs, got in zip(sets, serial):
        for (line, keys, pmk, nc), g in zip(jobs, got):
            assert g, line[:30]
            assert O.c_check_key_m22000(line, [g[0]], False, nc) == g
    results = [[] for _ in sets]

    def caller(t):
        for _ in range(3):
            results[t].append(dwpa_amd.check_batch(sets[t]))

    threads = [threading.Thread(target=caller, args=(t,)) for t in range(len(sets))]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    for t in range(len(sets)):
        assert len(results[t]) == 3 and all(r == serial[t] for r in results[t]), t
