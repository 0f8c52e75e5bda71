"""TEST / BENCH INFRASTRUCTURE ONLY -- the CPU baseline's process pool.  Never imported by the product path.

PHP-FPM serves each request in its own worker process, and one request runs check_key_m22000
(web/common.php:157-307) on one core.  The baseline therefore times the OpenSSL C restatement (oracle/) in worker
*processes*, one single-threaded check per task, instead of threads of one process: in round 2 the threaded
figure scaled 12-14x over 16 threads on PMKID legs but only 6-7x on EAPOL legs (OpenSSL 3's per-call HMAC/EVP
fetches contend inside one process).  Workers are started with the "spawn" method (fresh interpreters: nothing of
a GPU-initialised parent is inherited) and warmed before timing, as pre-forked PHP-FPM workers are.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import time
from concurrent.futures import ProcessPoolExecutor


def _init():
    from oracle import oracle as O
    O.lib()


def _noop(_):
    return os.getpid()


def _check_chunk(args):
    """check_key_m22000(line, [key], False, nc) per key of the chunk; index of the first match or -1."""
    line, keys, nc = args
    from oracle import oracle as O
    return O.c_check_many(line, keys, nc, 1)[0]


def _job_pmks(job):
    """check_key_m22000 on one job; returns the PMKs it derived (it stops at the first matching key)."""
    from oracle import oracle as O
    line, keys, pmk, nc = job
    r = O.c_check_key_m22000(line, keys, pmk, nc)
    if r is False:
        return sum(1 for k in keys if k is not None)
    k = next(i for i, x in enumerate(keys) if x is not None and O.hc_unhex(x) == r[0])
    return sum(1 for x in keys[:k + 1] if x is not None)


def physical_cores(cpus) -> int:
    """Distinct (physical id, core id) pairs among `cpus` (/proc/cpuinfo); len(cpus) if unknown."""
    try:
        seen, cur = set(), {}
        with open("/proc/cpuinfo") as f:
            for line in list(f) + [""]:
                if not line.strip():
                    if "processor" in cur and int(cur["processor"]) in cpus:
                        seen.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
        return len(seen) or len(cpus)
    except OSError:
        return len(cpus)


class PhpPool:
    """`workers` single-threaded oracle processes (PHP-FPM children)."""

    def __init__(self, workers: int):
        self.workers = max(1, int(workers))
        self.ex = ProcessPoolExecutor(self.workers, mp_context=mp.get_context("spawn"), initializer=_init)
        list(self.ex.map(_noop, range(4 * self.workers)))  # start and warm every worker before timing

    def check_keys(self, line: bytes, keys, nc: int):
        """One check per key over all workers; returns (index of the first match in `keys` or -1, seconds)."""
        n = len(keys)
        parts = max(1, min(n, 4 * self.workers))
        bounds = [n * j // parts for j in range(parts + 1)]
        t0 = time.perf_counter()
        idx = list(self.ex.map(_check_chunk, [(line, keys[bounds[j]:bounds[j + 1]], nc) for j in range(parts)]))
        dt = time.perf_counter() - t0
        first = next((bounds[j] + i for j, i in enumerate(idx) if i >= 0), -1)
        return first, dt

    def job_pmks(self, jobs, budget_s: float):
        """check_key_m22000 per job, one job per free worker as PHP-FPM hands requests out, until `budget_s`
        elapses (then the jobs in flight finish); returns (jobs done, PMKs derived, seconds).  Two jobs per worker
        stay queued so no worker idles between jobs of different lengths."""
        from concurrent.futures import FIRST_COMPLETED, wait
        done = nk = nxt = 0
        pending = set()
        t0 = time.perf_counter()
        while True:
            while nxt < len(jobs) and len(pending) < 2 * self.workers and time.perf_counter() - t0 < budget_s:
                pending.add(self.ex.submit(_job_pmks, jobs[nxt]))
                nxt += 1
            if not pending:
                break
            fin, pending = wait(pending, return_when=FIRST_COMPLETED)
            for f in fin:
                nk += f.result()
                done += 1
        return done, nk, time.perf_counter() - t0

    def close(self):
        self.ex.shutdown(wait=True)
