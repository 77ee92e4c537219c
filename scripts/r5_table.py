"""Round-5 closing-pass table: one row per shape from gpurun_out/r5_final
(bench JSON line, kernel stats CSV)."""
import csv
import glob
import json
import os
import sys

O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r5_final"


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("lkf::", "")
    return n


for f in sorted(glob.glob(os.path.join(O, "bench_*.json"))):
    name = os.path.basename(f)[6:-5]
    try:
        d = json.loads(open(f).read())
    except Exception:
        continue
    r = d.get("roofline", {})
    cb = d.get("cpu_baseline") or {}
    g = d.get("parity_gate") or {}
    top = ""
    ks = os.path.join(O, "kernel_stats_%s.csv" % name)
    if os.path.exists(ks):
        rows = sorted(csv.DictReader(open(ks)), key=lambda x: -float(x["TotalDurationNs"]))
        rows = [x for x in rows if not x["Name"].startswith("__amd")][:3]
        top = ", ".join("%s %.0f us" % (short(x["Name"]), float(x["AverageNs"]) / 1e3) for x in rows)
    tr = r.get("traffic")
    b = r.get("algorithmic_bytes_per_step")
    print("| %s | %.3g | %.4f | %.3f | %s | %s | %s (%s) | %s |" % (
        name, d["value"], d["ms_per_step"], r.get("frac", 0),
        ("%.2f GB / %.2f GB (%.2fx)" % (tr / 1e9, b / 1e9, tr / b)) if tr and b else "-",
        "%s (%s DT differ)" % (d.get("parity"), g.get("downtracks_differing")) if g else d.get("parity"),
        ("%.3g M/s" % (cb.get("value", 0) / 1e6)) if cb else "-", cb.get("cores"), top))
