"""Print one call period of a rocprofv3 kernel trace (csv): kernels between the n-th and (n+1)-th launch of `head`,
relative to the n-th head's start.  python tools/trace_window.py TRACE.csv [n] [head-prefix]"""
import csv
import sys


def main(path, n=5, head="k_pbkdf2_gfx950_ms"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    heads = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(head)]
    i0, i1 = heads[n], heads[n + 1]
    base = int(rows[i0]["Start_Timestamp"])
    for r in rows[max(0, i0 - 4):i1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Stream_Id") or r.get("Queue_Id")
        print("%-40s %9.3f %9.3f %8.3f  %s" % (r["Kernel_Name"][:40], (s - base) / 1e6, (e - base) / 1e6,
                                                (e - s) / 1e6, q))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5,
         sys.argv[3] if len(sys.argv) > 3 else "k_pbkdf2_gfx950_ms")
