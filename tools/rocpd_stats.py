"""Kernel statistics (rocprofv3 --stats' kernel_stats.csv columns) from a rocprofv3 SQLite output
(run_results.db, the default --output-format of this rocprofv3): one row per kernel name with
calls, total / average / min / max duration in ns and the percentage of kernel time.

usage: python tools/rocpd_stats.py <run_results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1:3]
    cur = sqlite3.connect(db).cursor()
    rows = cur.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                       "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, calls, tot, avg, mn, mx in rows:
            w.writerow([name, calls, tot, round(avg, 3), round(100.0 * tot / total, 4), mn, mx])
    for name, calls, tot, avg, *_ in rows[:8]:
        print(f"{calls:6d} {avg / 1e3:12.3f} us  {name[:110]}")


if __name__ == "__main__":
    main()
