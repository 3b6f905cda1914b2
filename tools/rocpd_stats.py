"""rocprofv3 --kernel-trace --stats summary from its rocpd SQLite output.

    python tools/rocpd_stats.py <run_results.db> <out.csv>

ROCm 7's rocprofv3 writes the trace as a rocpd database by default; this
writes the same columns as its kernel_stats.csv (Name, Calls, TotalDurationNs,
AverageNs, Percentage, MinNs, MaxNs, StdDev), sorted by total time.
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration),"
        " avg(duration*duration) from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                    "StdDev"])
        for name, n, s, a, mn, mx, a2 in rows:
            sd = max(a2 - a * a, 0.0) ** 0.5
            w.writerow([name, n, s, f"{a:.1f}", f"{100.0 * s / tot:.3f}", mn, mx, f"{sd:.1f}"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
