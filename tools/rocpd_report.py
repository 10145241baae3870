"""Read rocprofv3's rocpd SQLite output (run_results.db) without the rocpd CLI.
  rocpd_report.py stats DB OUT.csv         per-kernel stats (calls, total/avg/min/max ns, %)
  rocpd_report.py counter DB NAME KERNEL   print per-dispatch values of counter NAME for kernels matching KERNEL
  rocpd_report.py timeline DB OUT.csv      every kernel in start order: name, start/end (ns from the first), stream/queue
                                           columns as the db names them
  rocpd_report.py gaps DB OUT.json         per acting step (kernels between two ctx_advance_kernel launches): span,
                                           busy time (sum of kernel durations), idle gaps between consecutive kernels"""
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


def step_gaps(db):
    c = sqlite3.connect(find_db(db))
    cur = c.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    ks = "start" if "start" in cols else [x for x in cols if "start" in x][0]
    ke = "end" if "end" in cols else [x for x in cols if x.endswith("end")][0]
    rows = c.execute(f"select name, {ks}, {ke} from kernels order by {ks}").fetchall()
    steps, cur_step = [], []
    for name, t0, t1 in rows:
        cur_step.append((name, t0, t1))
        if "ctx_advance_kernel" in name:
            steps.append(cur_step)
            cur_step = []
    out = []
    for st in steps:
        span = st[-1][2] - st[0][1]
        busy = sum(t1 - t0 for _, t0, t1 in st)
        gaps = [max(0, st[i][1] - st[i - 1][2]) for i in range(1, len(st))]
        tg = [max(0, st[i][1] - st[i - 1][2]) for i in range(1, len(st)) if "tower8" in st[i][0]]
        out.append({"kernels": len(st), "span_us": span / 1e3, "busy_us": busy / 1e3, "idle_us": sum(gaps) / 1e3,
                    "gap_median_us": sorted(gaps)[len(gaps) // 2] / 1e3 if gaps else None,
                    "gap_before_tower_median_us": sorted(tg)[len(tg) // 2] / 1e3 if tg else None})
    return out


def timeline(db, out):
    c = sqlite3.connect(find_db(db))
    cur = c.execute("select * from kernels limit 1")
    cols = [d[0] for d in cur.description]
    ks = "start" if "start" in cols else [x for x in cols if "start" in x][0]
    ke = "end" if "end" in cols else [x for x in cols if x.endswith("end")][0]
    extra = [x for x in cols if any(t in x.lower() for t in ("stream", "queue"))]
    rows = c.execute(f"select name, {ks}, {ke}{''.join(', ' + x for x in extra)} from kernels order by {ks}").fetchall()
    t0 = rows[0][1] if rows else 0
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "start_ns", "end_ns"] + extra)
        for r in rows:
            w.writerow([r[0], r[1] - t0, r[2] - t0] + list(r[3:]))
    print(f"{len(rows)} kernels, columns {cols}")


if __name__ == "__main__":
    if sys.argv[1] == "timeline":
        timeline(sys.argv[2], sys.argv[3])
        sys.exit(0)
    if sys.argv[1] == "gaps":
        import json
        res = step_gaps(sys.argv[2])
        json.dump(res, open(sys.argv[3], "w"), indent=1)
        for r in res:
            print(json.dumps(r))
        sys.exit(0)
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
