"""Summarise rocprofv3 --pmc CSV passes per kernel (mean per dispatch) and
optionally delete the raw CSVs (the raw files include every setup copy kernel
and can exceed gpurun's 64 MiB copy-back limit).

usage: python3 scripts/pmc_summary.py <pmc_dir> [--delete-raw]
Writes <pmc_dir>/summary.json.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "lkf::" not in name:
                    continue
                short = name.split("(")[0]
                acc[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "lkf::" in name:
                    dur[name.split("(")[0]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["_dispatch_samples"] = max(len(v) for v in cs.values())
    for k, v in dur.items():
        out.setdefault(k, {})["_mean_duration_ns_profiled"] = sum(v) / len(v)
    # HBM traffic per launch (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
    # WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies half the bytes of wide
    # coalesced reads, so it is doubled.
    for k in list(out.keys()):
        c = out[k]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            out[k.split("::")[-1] + "_hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
    # whole-step traffic: every engine kernel's bytes over all its dispatches,
    # per batch (one k_decide_dt dispatch per batch)
    nsteps = out.get("lkf::k_decide_dt", {}).get("_dispatch_samples", 0)
    if nsteps:
        tot = 0.0
        for k, c in out.items():
            if k.startswith("lkf::") and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                tot += (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 * c["_dispatch_samples"]
        out["hbm_bytes_per_step"] = int(tot / nsteps)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_sources_sha
    out["kernel_sources_sha"] = kernel_sources_sha()
    out["bench_args_rooms"] = int(os.environ.get("PMC_ROOMS", "100"))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))
    if "--delete-raw" in sys.argv:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            os.remove(f)


if __name__ == "__main__":
    main()
