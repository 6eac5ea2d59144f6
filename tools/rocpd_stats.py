"""Kernel statistics (the rocprofv3 --stats kernel_stats.csv columns) from a rocprofv3 SQLite
results database (rocpd format, the default output of `rocprofv3 --kernel-trace --stats -d DIR`).

    python tools/rocpd_stats.py gpurun_out/prof_train/run_results.db > profiles/rXX/kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                     "max(end - start) from kernels group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, n, tot, avg, mn, mx in rows:
        w.writerow([name, n, tot, round(avg, 1), round(100.0 * tot / total, 2), mn, mx])


if __name__ == "__main__":
    main(sys.argv[1])
