"""GPU-busy fraction of each check-path call from a rocprofv3 kernel trace (bench.py --workload c5 under
`rocprofv3 --kernel-trace`): the union of all kernel intervals inside one call period (head PBKDF2 launch to the
next one, shifted to include the call's prep kernel) divided by that period.  Warmup calls are skipped.

    python tools/busy_fraction.py profiles/r02/c5_tail_beside_head/c5prof/run_kernel_trace.csv
"""
import csv
import json
import sys


def busy(path, head="k_pbkdf2_gfx950_ms", skip=2, lead_ns=200_000):
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    heads = sorted(int(r["Start_Timestamp"]) for r in rows if r["Kernel_Name"].startswith(head))
    out = []
    for a, b in zip(heads[skip:-1], heads[skip + 1:]):
        lo, hi = a - lead_ns, b - lead_ns
        tot, cs, ce = 0, None, None
        for s, e in iv:
            s, e = max(s, lo), min(e, hi)
            if e <= s:
                continue
            if ce is None or s > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if ce is not None:
            tot += ce - cs
        out.append({"period_ms": round((hi - lo) / 1e6, 3), "busy_frac": round(tot / (hi - lo), 4)})
    return out


if __name__ == "__main__":
    print(json.dumps(busy(sys.argv[1])))
