"""Host backend figures on this machine's CPU (dwpa_amd/csrc/host_check.cpp): which primitives CPUID selected,
PBKDF2 throughput at 1 thread and at the pool's threads, and the latency of the server's small check calls (one key
vs a PMKID / EAPOL keyver 2 / keyver 3 line at nc=128, caller-PMK checks), each beside the same call through the C
oracle (OpenSSL, one PHP request's core).  Every result is checked against the oracle.  Prints one JSON line.

    python tools/host_backend_bench.py [--reps N]

PBKDF2 runs in chunks of 2 keys on SHA-NI chains, or 8 / 16 keys on AVX-512, whichever the library's measured
per-chunk costs say finishes the call first (host_check.cpp derive_chunk); the one-thread rows (a child with
DWPA_HOST_THREADS=1) give the per-core rates: 2 keys = SHA-NI, 32 and 256 keys = AVX-512 where present.
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DWPA_HOST_MAX_PMKS", "1000000000")  # every call with a derive on the host backend


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--pbkdf2-only", action="store_true")
    args = ap.parse_args()
    import dwpa_amd
    from dwpa_amd import m22000 as M
    from oracle import oracle as O
    from tests import synth as S

    rng = random.Random(11)
    essid, apm, sta, an, sn = S.random_net(rng, essid_len=10)

    def med(fn, n):
        fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts) * 1e3

    out = {"cpu_model": next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
                             None),
           "flags": sorted({f for l in open("/proc/cpuinfo") if l.startswith("flags") for f in l.split()}
                           & {"sha_ni", "aes", "avx2", "avx512f"}),
           "host_threads_cap": int(os.environ.get("DWPA_HOST_THREADS", "16"))}
    rows = []
    threads = max(1, min(out["host_threads_cap"], len(os.sched_getaffinity(0)), os.cpu_count() or 1))
    sizes = (2, 32, 256) if args.pbkdf2_only else (1, 2, 16, 64, 256, 512, 1024, 4096)
    for n in sizes:
        keys = [S.fast_psk(rng) for _ in range(n)]
        ms = med(lambda: dwpa_amd.pbkdf2_pmk(keys, essid), max(3, args.reps // (1 + n // 16)))
        ok = b"".join(dwpa_amd.pbkdf2_pmk(keys, essid)) == O.c_pbkdf2_many(keys, essid, threads=8)
        rows.append({"call": f"dwpa_pbkdf2_pmk, {n} key(s)", "threads": threads, "ms": round(ms, 3),
                     "pmk_per_s": round(n / ms * 1e3), "same_result": ok})
    if args.pbkdf2_only:
        out["rows"] = rows
        print(json.dumps(out))
        sys.exit(0 if all(r["same_result"] for r in rows) else 3)
    import subprocess
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--pbkdf2-only", "--reps", str(args.reps)],
                       env=dict(os.environ, DWPA_HOST_THREADS="1"), capture_output=True, text=True, timeout=300)
    if r.returncode not in (0, 3):
        raise SystemExit(f"one-thread child failed: {r.stderr[-2000:]}")
    rows += json.loads(r.stdout)["rows"]
    psk = S.fast_psk(rng)
    pmk = S.pmk(psk, essid)
    lines = {"pmkid": S.pmkid_line(psk, essid, apm, sta),
             "eapol-kv2": S.eapol_line(psk, essid, apm, sta, an, sn, 2, -5, "BE", rng=rng),
             "eapol-kv3": S.eapol_line(psk, essid, apm, sta, an, sn, 3, 7, "LE", rng=rng)}
    for kind, line in lines.items():
        for label, job in (("1 key, hit", (line, [psk], False, 128)),
                           ("1 key, miss", (line, [S.fast_psk(rng)], False, 128)),
                           ("caller PMK, miss, nc=258", (line, [b""], bytes(32), 258))):
            ms = med(lambda: dwpa_amd.check_key_m22000(*job), args.reps)
            got = dwpa_amd.check_key_m22000(*job)
            backend = M.check_stats()["backend"]
            cpu = med(lambda: O.c_check_key_m22000(*job), max(3, args.reps // 4))
            rows.append({"call": f"check_key_m22000, {kind}, {label}", "ms": round(ms, 3),
                         "oracle_openssl_1core_ms": round(cpu, 3), "backend": backend,
                         "same_result": got == O.c_check_key_m22000(*job)})
    # a GPU-less server's bulk call: a C5-shaped batch (PMKID + keyver 1/2/3, nc=128, 202 keys per job), all on the
    # host backend (DWPA_HOST_MAX_PMKS above: every call with a derive is a host call), every result vs the oracle
    jobs, _ = S.c5_plan(seed=9, per_kind=25, essids=20, zero_pmk=1)
    nkeys = sum(len(j[1]) for j in jobs)
    ms = med(lambda: dwpa_amd.check_batch(jobs), 3)
    got = dwpa_amd.check_batch(jobs)
    backend = M.check_stats()["backend"]
    exp = [O.c_check_key_m22000(*j) for j in jobs]
    rows.append({"call": f"check_batch, C5-shaped {len(jobs)} jobs x 202 keys, nc=128 (a GPU-less server's bulk call)",
                 "keys": nkeys, "ms": round(ms, 1), "pmk_per_s": round(nkeys / ms * 1e3), "backend": backend,
                 "same_result": got == exp})
    out["rows"] = rows
    out["all_same"] = all(r["same_result"] for r in rows)
    print(json.dumps(out))
    sys.exit(0 if out["all_same"] else 3)


if __name__ == "__main__":
    main()
