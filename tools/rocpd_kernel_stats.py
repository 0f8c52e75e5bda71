"""Kernel statistics (the rocprofv3 --stats kernel_stats.csv columns) from a rocprofv3 SQLite database (rocpd, the
default output format of ROCm 7's rocprofv3):  python tools/rocpd_kernel_stats.py results.db > kernel_stats.csv"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 4), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
