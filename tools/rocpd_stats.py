"""Kernel statistics (the rocprofv3 --stats kernel_stats.csv columns) from a rocprofv3 SQLite
results database (rocpd format, the default output of `rocprofv3 --kernel-trace --stats -d DIR`).

    python tools/rocpd_stats.py gpurun_out/prof_train/run_results.db > profiles/rXX/kernel_stats.csv
    python tools/rocpd_stats.py --step <db> [first kernel of a step]   # the last step, launch by launch
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




def last_step(path, first_kernel="dense_kernel"):
    """the kernel sequence of the last step in a trace (from the last launch of `first_kernel`):
    duration (us), workgroups, name -- where a step's time goes, launch by launch"""
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    i0 = max(i for i, r in enumerate(rows) if first_kernel in r[0])
    out = []
    for k, (n, s, e, g, w) in enumerate(rows[i0:]):
        gap = (s - rows[i0 + k - 1][2]) / 1e3 if k else 0.0   # from the previous kernel's end
        out.append(((e - s) / 1e3, g // max(1, w), n, gap))
    return out


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--step":
        seq = last_step(sys.argv[2], *(sys.argv[3:4]))
        for us, wg, name, gap in seq:
            print(f"{us:8.2f} us (gap {gap:5.2f}) {wg:7d} WG  {name[:90]}")
        span = sum(s[0] + s[3] for s in seq)
        print(f"{sum(s[0] for s in seq):8.2f} us in kernels, {span:8.2f} us first start -> last end, "
              f"{len(seq)} launches")
    else:
        main(sys.argv[1])
