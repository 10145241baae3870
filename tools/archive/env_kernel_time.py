"""Kernel-duration record of the env step kernel for bench.py's env workload (configs 1/3): reads the rocprofv3
--kernel-trace --stats CSVs of `bench.py --workload env` runs and writes profiles/env_kernel_time.json, one entry per
geometry, so the bench line reports the HBM fraction from the kernel's own duration beside the event-timed one.
  python tools/env_kernel_time.py profiles/r05/r5env/env84_kernel_stats.csv:84:84:4 profiles/r05/r5env/env16_kernel_stats.csv:16:20:32"""
import csv
import json
import os
import re
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    out = []
    for spec in sys.argv[1:]:
        path, H, W, hist = spec.split(":")
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if "env_step_compact_kernel" in r["Name"]]
        assert len(rows) == 1, rows
        r = rows[0]
        kname = re.search(r"env_step_compact_kernel<\d+>", r["Name"]).group(0)
        out.append({"envs": 4096, "H": int(H), "W": int(W), "hist": int(hist), "kernel": kname,
                    "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                    "source": os.path.relpath(path, ROOT)})
    with open(os.path.join(ROOT, "profiles", "env_kernel_time.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
