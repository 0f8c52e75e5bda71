"""A server process's lifetime in miniature: many check calls of every shape, from several threads at once, on the
call contexts of one device (engine.cpp: DWPA_CALLS_PER_DEVICE contexts per GPU, their buffers grown and reused
from call to call).  PHP-FPM workers and a threaded server call check_key_m22000 (common.php:157) and the batched
put_work loop (:900-925) millions of times with sizes that vary from call to call; a buffer kept from a larger call,
a stale first-hit word (k_verify_att's early exit), a hit counter or a tail flag left over from the previous call
would show up here as a wrong tuple.  Every result is checked against the oracle (the key-prefix rule of
test_gpu_configs.py for the large jobs)."""
import random
import threading
from concurrent.futures import ThreadPoolExecutor

import pytest

pytestmark = pytest.mark.gpu

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from oracle import oracle as O  # noqa: E402


def _job(rng, nets, nkeys, nc, plant_at=None, caller=False):
    essid, ap, sta, an, sn = nets[rng.randrange(len(nets))]
    ap, sta = rng.randbytes(6), rng.randbytes(6)
    psk = S.fast_psk(rng)
    kind = rng.choice(["pmkid", 1, 2, 3])
    line = (S.pmkid_line(psk, essid, ap, sta) if kind == "pmkid" else
            S.eapol_line(psk, essid, ap, sta, an, sn, kind, rng.randint(-6, 6), rng.choice(["LE", "BE"]), rng=rng))
    keys = [S.fast_psk(rng, 8, 24) for _ in range(nkeys)]
    if plant_at is not None and nkeys:
        keys[min(plant_at, nkeys - 1)] = psk
    elif nkeys and rng.random() < 0.7:
        keys[rng.randrange(nkeys)] = psk
    pmk = S.pmk(psk, essid) if caller and rng.random() < 0.5 else (b"\x07" * 32 if caller else False)
    return (line, keys, pmk, nc)


def _calls(seed):
    """One caller's sequence: single checks, small and mid batches, and a large derive (head/tail split)."""
    rng = random.Random(seed)
    nets = [S.random_net(rng) for _ in range(6)]
    seq = []
    for r in range(16):
        shape = "big" if r in (3, 11) else "bigt" if r == 7 else rng.choice(["one", "one", "batch", "batch", "mid"])
        if shape == "one":
            seq.append(("one", [_job(rng, nets, rng.randint(0, 20), rng.choice([0, 8, 128]),
                                     caller=rng.random() < 0.3)]))
        elif shape == "batch":
            seq.append(("batch", [_job(rng, nets, rng.randint(0, 16), rng.choice([0, 8, 16, 128]),
                                       caller=rng.random() < 0.2) for _ in range(rng.randint(1, 24))]))
        elif shape == "mid":
            seq.append(("batch", [_job(rng, nets, rng.randint(50, 100), 128) for _ in range(rng.randint(4, 8))]))
        elif shape == "big":  # > 2 waves per SIMD of unique keys: the head/tail split, a tail the GPU derives
            seq.append(("batch", [_job(rng, nets, 36000, 8, plant_at=rng.randrange(600)) for _ in range(2)]))
        else:  # a head of 2 waves per SIMD and a small remainder: the tail derived on the host beside the head
            seq.append(("batch", [_job(rng, nets, 33000, 8, plant_at=rng.randrange(600)) for _ in range(2)]))
    return seq


def _run(seq):
    out = []
    for kind, jobs in seq:
        if kind == "one":
            out.append([dwpa_amd.check_key_m22000(*jobs[0])])
        else:
            out.append(dwpa_amd.check_batch(jobs))
    return out


def _expected(job, got):
    line, keys, pmk, nc = job
    if len(keys) > 1000:  # the first key in input order decides: check the prefix up to the reported key
        if got is False:
            return O.c_check_key_m22000(line, keys, pmk, nc)
        k = next(i for i, key in enumerate(keys) if key == got[0])
        return O.c_check_key_m22000(line, keys[:k + 1], pmk, nc)
    return O.c_check_key_m22000(line, keys, pmk, nc)


def test_many_calls_of_every_shape_from_three_threads():
    _soak()


@pytest.mark.host_routing
def test_many_calls_with_the_library_routing_from_three_threads():
    """The same lifetime with the library's own routing: small calls on the host backend, the rest
    on the device with host-derived tails, three threads sharing the host pool and the call contexts."""
    from dwpa_amd import m22000 as M
    M.init()
    _soak()


def _soak():
    seqs = [_calls(1000 + t) for t in range(3)]
    results = [None] * 3

    def caller(t):
        results[t] = _run(seqs[t])

    threads = [threading.Thread(target=caller, args=(t,)) for t in range(3)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    # the same sequences once more from one thread: contexts reused with other sizes in between
    again = _run(seqs[0])
    assert again == results[0]
    flat = [(job, got) for t in range(3) for (kind, jobs), res in zip(seqs[t], results[t]) for job, got in
            zip(jobs, res)]
    with ThreadPoolExecutor(16) as ex:
        exp = list(ex.map(lambda jg: _expected(*jg), flat))
    bad = [(i, flat[i][0][0][:30], flat[i][1], e) for i, e in enumerate(exp) if flat[i][1] != e]
    assert not bad, bad[:3]
    assert sum(1 for _, g in flat if g) > len(flat) // 3
