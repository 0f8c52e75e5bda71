"""partial_round.py -- k_pbkdf2 duration against batch size around one resident wave round (524,288 lanes =
262,144 PMKs at 8 waves/SIMD on 256 CUs).  Shows how a partial round (C1, C5) is dispatched.  Workgroup size comes
from DWPA_PBKDF2_WG.  Prints one JSON line per batch size."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import dwpa_amd  # noqa: E402
from tests import synth as S  # noqa: E402
from dwpa_amd.device import Dictionary, Event, Stream  # noqa: E402


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [262144, 229376, 202752, 196608, 163840, 131072, 65536, 524288]
    n = max(sizes)
    rng = np.random.default_rng(5)
    lens = np.full(n, 10, dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    data = rng.integers(0x61, 0x7B, int(off[-1]) + 64, dtype=np.uint8)
    d = Dictionary(off, data, device=0)
    import random
    r = random.Random(3)
    essid, ap, sta, _, _ = S.random_net(r, essid_len=10)
    line = S.pmkid_line(b"notthekey1", essid, ap, sta)
    st = Stream(0)
    for cnt in sizes:
        sc = dwpa_amd.Scan([line], device=0, nc=0, batch=cnt)
        sc.load_dict(d.off.ptr, d.data.ptr, 0, cnt, 8, 63, st.handle)
        sc.pbkdf2(0, st.handle)  # warm
        ms = []
        for _ in range(3):
            a, b = Event(0), Event(0)
            a.record(st)
            sc.pbkdf2(0, st.handle)
            b.record(st)
            st.synchronize()
            ms.append(a.elapsed_ms(b))
        sc.close()
        best = min(ms)
        print(json.dumps({"wg": int(os.environ.get("DWPA_PBKDF2_WG", "256")), "pmks": cnt, "ms": round(best, 3),
                          "pmk_per_s": round(cnt / best * 1e3), "round_frac": round(cnt / 262144, 3)}), flush=True)


if __name__ == "__main__":
    main()
