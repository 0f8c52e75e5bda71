"""Kernel timeline of one call period from a rocprofv3 SQLite trace (rocprofv3 >= 7 writes *_results.db by default):
kernels between the n-th and (n+1)-th launch of `head`, relative to the n-th head's start, plus the GPU-busy share
of every full period.   python tools/trace_db.py RESULTS.db [n] [head-prefix]"""
import sqlite3
import sys


def main(path, n=5, head="k_pbkdf2_gfx950_ms"):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end, queue_id from kernels order by start").fetchall()
    heads = [i for i, r in enumerate(rows) if r[0].startswith(head) and "tail" not in r[0]]
    i0, i1 = heads[n], heads[n + 1]
    base = rows[i0][1]
    for name, s, e, q in rows[max(0, i0 - 6):i1]:
        print("%-44s %9.3f %9.3f %8.3f  q%s" % (name[:44], (s - base) / 1e6, (e - base) / 1e6, (e - s) / 1e6, q))
    busy = []
    for a, b in zip(heads[2:-1], heads[3:]):
        lo, hi = rows[a][1] - 200_000, rows[b][1] - 200_000
        iv = sorted((max(s, lo), min(e, hi)) for _, s, e, _ in rows if e > lo and s < hi)
        tot, cs, ce = 0, None, None
        for s, e in iv:
            if cs is None or s > ce:
                if cs is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        tot += ce - cs
        busy.append((tot / (hi - lo), (hi - lo) / 1e6))
    print("busy share per call: " + " ".join("%.3f/%.1fms" % b for b in busy))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5,
         sys.argv[3] if len(sys.argv) > 3 else "k_pbkdf2_gfx950_ms")
