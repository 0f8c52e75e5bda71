"""Summarise tools/profile_traffic.sh output: per-kernel mean duration (kernel trace) and HBM bytes per dispatch
from FETCH_SIZE / WRITE_SIZE (KB units in rocprofv3's derived counters; FETCH_SIZE doubled on gfx950 for wide
coalesced reads, MI355X_MICROARCH.md "HBM [CDNA4]")."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def main(out):
    res = {}
    dur = defaultdict(list)
    for r in rows(os.path.join(out, "stats", "**", "*kernel_trace.csv")):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        per = defaultdict(list)
        for r in rows(os.path.join(out, name, "**", "*counter_collection.csv")):
            if r["Counter_Name"] == counter:
                per[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)
        for k, v in per.items():
            d = res.setdefault(k, {})
            d[counter + "_bytes_per_dispatch_raw"] = sum(v) / len(v)
            d["dispatches_" + name] = len(v)
    for k, v in dur.items():
        d = res.setdefault(k, {})
        d["dispatches_trace"] = len(v)
        d["mean_ms"] = sum(v) / len(v)
    for k, d in res.items():
        f = d.get("FETCH_SIZE_bytes_per_dispatch_raw")
        w = d.get("WRITE_SIZE_bytes_per_dispatch_raw")
        if f is not None and w is not None:
            d["hbm_bytes_per_dispatch"] = 2 * f + w
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
