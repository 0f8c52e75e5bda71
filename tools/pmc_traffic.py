"""Summarise tools/profile_traffic.sh output per kernel: dispatch durations from the kernel trace, and HBM bytes
per dispatch from the FETCH_SIZE / WRITE_SIZE passes.  rocprofv3 reports both counters in KiB.  On gfx950
FETCH_SIZE reads half the bytes of a wide coalesced stream, so the corrected figure doubles it
(MI355X_MICROARCH.md "HBM [CDNA4]").  Medians are over dispatches: the bench's untimed last batch (the one
holding the planted PSK) is partial and shorter, so the median is the full-batch launch the bench line reports."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def rows(pattern):
    for path in glob.glob(pattern, recursive=True):
        with open(path) as f:
            yield from csv.DictReader(f)


def short(name):
    return name.split("(")[0]


def main(out):
    res = defaultdict(dict)
    dur = defaultdict(list)
    for r in rows(os.path.join(out, "stats", "**", "*kernel_trace.csv")):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    for name, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        per = defaultdict(list)
        for r in rows(os.path.join(out, name, "**", "*counter_collection.csv")):
            if r["Counter_Name"] == counter:
                per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
        for k, v in per.items():
            res[k][counter + "_raw_bytes_median"] = statistics.median(v)
            res[k][counter + "_raw_bytes_all"] = v
    for k, v in dur.items():
        res[k]["dispatches"] = len(v)
        res[k]["mean_ms"] = sum(v) / len(v)
        res[k]["median_ms"] = statistics.median(v)
        res[k]["all_ms"] = [round(x, 4) for x in v]
    for k, d in res.items():
        f = d.get("FETCH_SIZE_raw_bytes_median")
        w = d.get("WRITE_SIZE_raw_bytes_median")
        if f is not None and w is not None:
            d["hbm_bytes_per_dispatch_raw"] = f + w
            d["hbm_bytes_per_dispatch_corrected"] = 2 * f + w
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
