"""Child process of test_gpu_parity.py::test_first_key_exit_across_chunks: the first-key early exit is
read once per process (DWPA_FIRST_KEY_EXIT), so each setting runs in its own process.  Prints one JSON line: the
library's results and the CPU oracle's for jobs whose PSK appears several times, with the call cut into 128-slot
chunks (dwpa_init batch) so a job spans chunks and attempt-parallel segments."""
import ctypes
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dwpa_amd  # noqa: E402
from dwpa_amd import _lib as L  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests import synth as S  # noqa: E402


# (copies of the PSK at these key indices, null keys at these indices)
PLAN = (([20, 100, 130, 250], [3, 50]), ([250, 140], [0, 139]), ([5, 6, 299], []), ([299], [10, 20, 30]), ([], [7]))


def jobs():
    rng = random.Random(77)
    out = []
    for copies, nulls in PLAN:
        essid, ap, sta, an, sn = S.random_net(rng)
        psk = S.fast_psk(rng)
        kv = 2 + len(out) % 2  # keyver 2 and 3, both attempt-parallel at nc=128
        line = S.eapol_line(psk, essid, ap, sta, an, sn, kv, rng.choice([-7, 3, 0, 40]), rng.choice(["LE", "BE"]),
                            rng=rng)
        keys = [S.fast_psk(rng) for _ in range(300)]
        for i in copies:
            keys[i] = psk
        for i in nulls:
            keys[i] = None
        out.append((line, keys, False, 128))
    return out


def main():
    cfg = L.Config(ctypes.sizeof(L.Config), 0, 128, 0)
    L.check(L.load().dwpa_init(ctypes.byref(cfg)), "init")
    js = jobs()
    b = dwpa_amd.BatchJobs(js)
    b.run()
    got = b.results()
    key_index = [int(b.out[i].key_index) if b.rcs[i] == L.DWPA_HIT else None for i in range(len(js))]
    single = [dwpa_amd.check_key_m22000(*j) for j in js]
    exp = [O.c_check_key_m22000(*j) for j in js]

    def enc(r):
        return r if r is False else [r[0].hex(), r[1], r[2], r[3].hex()]
    print(json.dumps({"exit": os.environ.get("DWPA_FIRST_KEY_EXIT", "1"), "got": [enc(r) for r in got],
                      "single": [enc(r) for r in single], "exp": [enc(r) for r in exp],
                      "key_index": key_index,
                      "first_copy": [min(c) if c else None for c, _ in PLAN]}))


if __name__ == "__main__":
    main()
