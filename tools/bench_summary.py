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
        out.append(f"parity {pp['value']:.1f} (frac {pp['frac']:.3f}, f32mfma {pp['vs_f32_mfma_path']['value']:.1f}, "
                   f"x6==f32mfma {pp['vs_f32_mfma_path']['visit_count_match']})")
    if d.get("cpu_baseline"):
        out.append(f"cpu {d['cpu_baseline']['value']:.2f}")
    print(" | ".join(out))
