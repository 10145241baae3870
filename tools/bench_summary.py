"""One-line summary of a bench.py JSON record (used by tools/gpu_run.sh after each bench step).
usage: bench_summary.py FILE.json"""
import json
import sys

if __name__ == "__main__":
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    out = [sys.argv[1], f"{d['value']:.1f} {d['unit']}", f"{d['ms_per_step']:.2f} ms/step", f"frac {r.get('frac')}"]
    if d.get("visit_count_match_full") is not None:
        out.append(f"match_full {d['visit_count_match_full']}")
    pp = d.get("parity_path")
    if pp:
        out.append(f"parity[{pp.get('form', 'x6')}] {pp['value']:.1f} on {pp.get('envs')} envs (frac {pp['frac']:.3f}")
        for k in ("vs_x6_path", "vs_f32_mfma_path"):
            vm = pp.get(k)
            if vm:
                out.append(f"{k[3:]} {vm['value']:.1f} match {vm['visit_count_match']}")
    if d.get("ranks_seen") is not None:
        out.append(f"ranks_seen {d['ranks_seen']} ({d.get('backend')})")
    if d.get("cpu_baseline"):
        out.append(f"cpu {d['cpu_baseline']['value']:.2f}")
    print(" | ".join(out))
