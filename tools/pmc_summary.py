"""Per-kernel mean of rocprofv3 --pmc counters (one row per kernel name: counters averaged over its dispatches,
plus the mean dispatch duration from the PMC run's timestamps, i.e. the kernel alone).
python tools/pmc_summary.py PASS1.csv [PASS2.csv ...]"""
import collections
import csv
import sys


def main(paths):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    for k in sorted(vals, key=lambda k: -sum(dur[k].values())):
        d = list(dur[k].values())
        cs = " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(vals[k].items()))
        print("%-44s n=%d ms=%.3f %s" % (k, len(d), sum(d) / len(d), cs))


if __name__ == "__main__":
    main(sys.argv[1:])
