"""Read rocprofv3's rocpd SQLite output (run_results.db) without the rocpd CLI.
  rocpd_report.py stats DB OUT.csv         per-kernel stats (calls, total/avg/min/max ns, %)
  rocpd_report.py counter DB NAME KERNEL   print per-dispatch values of counter NAME for kernels matching KERNEL"""
import csv
import glob
import os
import sqlite3
import sys


def find_db(path):
    if os.path.isfile(path):
        return path
    dbs = sorted(glob.glob(os.path.join(path, "**", "*.db"), recursive=True))
    if not dbs:
        raise FileNotFoundError(f"no rocpd .db under {path}")
    return dbs[0]


def kernel_stats(db):
    c = sqlite3.connect(find_db(db))
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": r[3], "MinNs": r[4], "MaxNs": r[5],
             "Percentage": 100.0 * r[2] / tot} for r in rows]


def counter_values(db, name, kernel):
    c = sqlite3.connect(find_db(db))
    return [r[0] for r in c.execute("select value from counters_collection where counter_name = ? and "
                                    "kernel_name like ? order by dispatch_id", (name, f"%{kernel}%"))]


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        st = kernel_stats(sys.argv[2])
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(st[0].keys()))
            w.writeheader()
            w.writerows(st)
        for r in st[:12]:
            print(f"{r['Percentage']:6.2f}% {r['Calls']:7d} {r['AverageNs'] / 1e3:10.2f} us  {r['Name'][:100]}")
    else:
        print(counter_values(sys.argv[2], sys.argv[3], sys.argv[4]))
