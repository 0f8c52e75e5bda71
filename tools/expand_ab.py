"""A/B of dwpa_rules_expand_file between two builds of the library (GPU box): the same synthetic source as
`bench.py --workload expand` (5M words of 6..16 printable bytes x the 148-rule WPA set), each library called through
raw ctypes (no dwpa_amd signature table, so an older build loads too), in alternating order (A B, B A, ...) with a
sync between calls, `reps` times each.  Output goes
to OUT_DIR (default: a temporary directory).  Prints one JSON line per call and a summary."""
import ctypes
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dwpa_amd.rulesets import wpa_rules  # noqa: E402


def main():
    libs = sys.argv[1:3]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n = 5_000_000
    rng = np.random.default_rng(9)
    lens = rng.integers(6, 17, n).astype(np.int64)
    ends = np.cumsum(lens + 1)
    text = rng.integers(0x21, 0x7F, int(ends[-1]), dtype=np.uint8)
    text[text == ord("$")] = ord("%")
    text[ends - 1] = 0x0A
    tmp = tempfile.mkdtemp(prefix="dwpa_expand_ab_", dir=os.environ.get("OUT_DIR"))
    spath, rpath, opath = (os.path.join(tmp, x) for x in ("source.txt", "bestWPA.rule", "cracked.txt.gz"))
    with open(spath, "wb") as f:
        f.write(text.tobytes())
    with open(rpath, "w") as f:
        f.write("\n".join(wpa_rules()) + "\n")
    handles = []
    for p in libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        fn = lib.dwpa_rules_expand_file
        fn.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                       ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        handles.append(fn)
    src = (ctypes.c_char_p * 1)(spath.encode())
    res = {p: [] for p in libs}
    for rep in range(reps + 1):  # rep 0 warms each library; the order alternates (A B, B A, ...)
        order = list(zip(libs, handles))
        if rep % 2:
            order.reverse()
        for p, fn in order:
            w, c = ctypes.c_uint64(0), ctypes.c_uint64(0)
            t0 = time.perf_counter()
            rc = fn(0, rpath.encode(), src, 1, opath.encode(), 0, ctypes.byref(w), ctypes.byref(c))
            el = time.perf_counter() - t0
            size = os.path.getsize(opath)
            print(json.dumps({"lib": p, "rep": rep, "rc": rc, "s": round(el, 3), "words": w.value,
                              "cands": c.value, "bytes": size, "cands_per_s": round(c.value / el, 1)}), flush=True)
            if rep:
                res[p].append(el)
            os.remove(opath)
            os.sync()  # the next call starts without the last one's 10 GB of dirty pages still being written back
            time.sleep(2)
    for x in (spath, rpath):
        os.remove(x)
    os.rmdir(tmp)
    print(json.dumps({"summary": {p: sorted(v) for p, v in res.items()}}))


if __name__ == "__main__":
    main()
