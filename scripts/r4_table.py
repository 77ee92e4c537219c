"""Markdown table of the round-4 closing pass (profiles/r4_final_bench_<shape>.json
plus the dominant kernel's time from profiles/r4_final_kernel_stats_<shape>.csv).
usage: python3 scripts/r4_table.py <shape> [<shape> ...]"""
import csv
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def kernels(shape, top=3):
    p = os.path.join(ROOT, "profiles", "r4_final_kernel_stats_%s.csv" % shape)
    if not os.path.exists(p):
        return ""
    rows = [r for r in csv.DictReader(open(p)) if "lkf::" in r["Name"]]
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    out = []
    for r in rows[:top]:
        n = r["Name"].replace("void ", "").replace("lkf::", "").replace("(anonymous namespace)::", "").split("(")[0]
        out.append("%s %.0f µs" % (n, float(r["AverageNs"]) / 1e3))
    return ", ".join(out)


print("| shape | workload / step | fwd pkts/s | ms/step | frac | PMC traffic / step | CPU baseline (threads, eff) | top kernels (rocprof avg) |")
print("|---|---|---:|---:|---:|---:|---:|---|")
for shape in sys.argv[1:]:
    d = json.load(open(os.path.join(ROOT, "profiles", "r4_final_bench_%s.json" % shape)))
    r = d["roofline"]
    c = d.get("cpu_baseline") or {}
    tr = r.get("traffic")
    cpu = "%.3g (%s, %s)" % (c["value"], c.get("cores"), c.get("thread_scaling_eff")) if c else "—"
    print("| %s | %s; %s | %.3g | %.4f | %.3f | %s | %s | %s |" % (
        shape, d["config"]["workload"][:60], d["config"]["step"][:40], d["value"], d["ms_per_step"], r["frac"],
        "%.3g GB" % (tr / 1e9) if tr else "—", cpu, kernels(shape)))
