"""Kernel stats (rocprofv3 --stats' columns) from a rocprofv3 rocpd database, for runs whose output format
was the default .db: python tools/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], r[3], r[4], r[5], 100.0 * r[2] / tot])


if __name__ == "__main__":
    main()
