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


def short_name(name):
    """'void lkf::k_emit<96>(lkf::EmitArgs)' -> 'lkf::k_emit<96>' (template kernels carry a return type)"""
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n[5:] if n.startswith("void ") else n


RD = ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")
WR = ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum")


def exact_bytes(c):
    """Read and write bytes from the L2's memory-side request counters by
    request size (the passes EXACT=1 of scripts/gpu_final.sh collects):
    32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B, and 64 x WRREQ_64B +
    32 x (WRREQ - WRREQ_64B).  FETCH_SIZE's rocprofv3 expression counts a
    128-B request (not in TCC_BUBBLE on gfx950) as 64 B, which is why the
    guide doubles it; the by-size sum needs no correction.  -> (read, write)
    or None."""
    if not all(k in c for k in RD + WR):
        return None
    rd = 32 * c[RD[0]] + 64 * c[RD[1]] + 128 * c[RD[2]]
    wr = 64 * c[WR[1]] + 32 * (c[WR[0]] - c[WR[1]])
    return rd, wr


def totals(out):
    """per-launch HBM bytes per kernel and the whole step's (per k_decide_dt<false> dispatch = per batch)"""
    for k in list(out.keys()):
        c = out[k]
        if isinstance(c, dict) and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            out[short_name(k).split("::")[-1] + "_hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        if isinstance(c, dict) and exact_bytes(c):
            rd, wr = exact_bytes(c)
            out[short_name(k).split("::")[-1] + "_hbm_exact_rd_wr_per_launch"] = [int(rd), int(wr)]
            if "TCC_EA0_RDREQ_sum" in c:  # the by-size counts should add up to all read requests
                c["_rdreq_by_size_over_all"] = (c[RD[0]] + c[RD[1]] + c[RD[2]]) / max(1.0, c["TCC_EA0_RDREQ_sum"])
    dec = [c for k, c in out.items() if isinstance(c, dict) and short_name(k).startswith("lkf::k_decide_dt")]
    nsteps = max((c.get("_dispatch_samples", 0) for c in dec), default=0)
    if nsteps:
        tot = 0.0
        for k, c in out.items():
            if isinstance(c, dict) and short_name(k).startswith("lkf::") and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                tot += (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 * c["_dispatch_samples"]
        out["hbm_bytes_per_step"] = int(tot / nsteps)
        ex = [(exact_bytes(c), c["_dispatch_samples"]) for k, c in out.items()
              if isinstance(c, dict) and short_name(k).startswith("lkf::")]
        if ex and all(e for e, _ in ex):
            out["hbm_exact_read_per_step"] = int(sum(e[0] * n for e, n in ex) / nsteps)
            out["hbm_exact_write_per_step"] = int(sum(e[1] * n for e, n in ex) / nsteps)
            out["hbm_exact_bytes_per_step"] = out["hbm_exact_read_per_step"] + out["hbm_exact_write_per_step"]
    return out


def bench_shape(argstr):
    """The workload a bench.py command line measures (the keys bench.py matches
    before quoting this summary's traffic): config, rooms, batch length, and
    whether the step ingests raw datagrams or protects with SRTP."""
    import argparse
    import shlex
    from bench import CONFIGS
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--rooms", type=int, default=0)
    ap.add_argument("--batch-s", type=float, default=1.0)
    ap.add_argument("--extpackets", action="store_true")
    ap.add_argument("--host-io", action="store_true")
    ap.add_argument("--srtp", action="store_true")
    a, _ = ap.parse_known_args(shlex.split(argstr))
    ingress = (not a.extpackets or a.config == 3) and not (a.host_io and a.config != 3)
    return {"bench_args": argstr, "bench_args_config": a.config, "bench_args_rooms": a.rooms or CONFIGS[a.config]["rooms"],
            "bench_args_batch_s": a.batch_s, "bench_args_ingress": ingress, "bench_args_srtp": a.srtp}


def main():
    d = sys.argv[1]
    if "--from-summary" in sys.argv:  # re-derive the totals of an existing summary.json (raw CSVs deleted)
        out = {short_name(k) if isinstance(v, dict) else k: v for k, v in json.load(open(os.path.join(d, "summary.json"))).items()}
        json.dump(totals(out), open(os.path.join(d, "summary.json"), "w"), indent=1, sort_keys=True)
        return
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "lkf::" not in name:
                    continue
                acc[short_name(name)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "lkf::" in name:
                    dur[short_name(name)].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["_dispatch_samples"] = max(len(v) for v in cs.values())
    for k, v in dur.items():
        out.setdefault(k, {})["_mean_duration_ns_profiled"] = sum(v) / len(v)
    # HBM traffic per launch (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
    # WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies half the bytes of wide
    # coalesced reads, so it is doubled.
    totals(out)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_sources_sha
    out["kernel_sources_sha"] = kernel_sources_sha()
    out.update(bench_shape(os.environ.get("BENCH_ARGS", "")))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))
    if "--delete-raw" in sys.argv:
        for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            os.remove(f)


if __name__ == "__main__":
    main()
