"""Why is a one-key server call slower than a 202-key call?  (profiles/r03/legs_k/c1lat.json:
10.36 ms for 1 key against 8.70 ms for 202.)

Three views of the same FFI call (dwpa_check_m22000, one EAPOL keyver-2 line and one PMKID line, nc=128):
  * sequential: 9 calls of one key count back to back, then the next count (the c1lat order of round 3);
  * interleaved: rounds of one call per key count, so every count sees the same GPU state;
  * after idle: one call after the GPU has been idle for `gap` seconds (the gap between two server requests).
Run it under `rocprofv3 --kernel-trace` to split each call into its kernels; the JSON line carries the host wall
time per call with CLOCK_MONOTONIC stamps so the trace can be cut per call.
    python tools/small_call_probe.py > out.json
"""
from __future__ import annotations

import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402

KS = (1, 2, 16, 202)


def main():
    rng = random.Random(7)
    essid, ap, sta, an, sn = S.random_net(rng, essid_len=10)
    calls = []

    def call(kind, k, tag):
        keys = [S.fast_psk(rng) for _ in range(k - 1)]
        psk = S.fast_psk(rng)
        keys.append(psk)
        line = (S.pmkid_line(psk, essid, ap, sta) if kind == "pmkid" else
                S.eapol_line(psk, essid, ap, sta, an, sn, 2, -5, "BE", rng=rng))
        t0 = time.monotonic_ns()
        r = dwpa_amd.check_key_m22000(line, keys)
        t1 = time.monotonic_ns()
        assert r and r[0] == psk
        calls.append({"tag": tag, "kind": kind, "keys": k, "t0_ns": t0, "t1_ns": t1, "ms": (t1 - t0) / 1e6})

    for kind in ("eapol", "pmkid"):
        call(kind, 1, "warm")
    for kind in ("eapol", "pmkid"):  # round 3's order: one count at a time
        for k in KS:
            for _ in range(9):
                call(kind, k, "sequential")
    for _ in range(9):
        for kind in ("eapol", "pmkid"):
            for k in KS:
                call(kind, k, "interleaved")
    for gap in (0.0, 0.02, 0.1, 0.3, 1.0):
        for _ in range(5):
            for k in (1, 202):
                time.sleep(gap)
                call("eapol", k, f"gap{gap}")
    summary = {}
    for c in calls:
        summary.setdefault(f"{c['tag']}/{c['kind']}/{c['keys']}", []).append(c["ms"])
    out = {"summary_median_ms": {k: round(statistics.median(v), 3) for k, v in summary.items()},
           "calls": calls}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
