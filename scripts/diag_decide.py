"""Diagnostic: k_decide_dt per-wave counters from a -DLKF_DIAG=1 build.

    make -C livekit-server_amd/csrc diag && python3 scripts/diag_decide.py [rooms] [batches] [config] [batch_s]
"""
import ctypes as C
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["waves", "chunks", "runs", "serial", "serial_drain", "cyc_classify", "cyc_runbody", "cyc_prologue",
         "fw_translate", "fw_common", "seq_push", "cyc_load", "cyc_runs", "cyc_serial", "cyc_total", "packets",
         "why_kf_switch", "why_svc", "why_cls_other", "why_ssrc", "why_padding", "why_reorder_dup", "why_gap_late",
         "why_picid_wrap", "why_tsw", "why_tdrop_offset", "why_other_ok", "why_seq", "pro_round1", "pro_hot", "pro_maps",
         "serial_total"]


def main():
    rooms = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    bs = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
    tr = wl.Trace(cfg, duration_s=nb * bs, batch_s=bs, rooms=rooms)
    lib = os.path.join(ROOT, "livekit-server_amd", "lib", os.environ.get("DIAG_LIB", "liblkfwd_diag.so"))
    eng = pkg.Engine.for_trace(tr, lib_path=lib)
    fn = eng.lib.lkf_debug_counters
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]
    wl.load_topology(eng.api, eng.h, tr)
    out = (C.c_uint64 * 32)()
    for b in range(nb):
        wl.queue_events(eng.api, eng.h, tr, b)
        pk, n, ar, alen = tr.batch(b)
        eng.submit(pk, n, ar, alen)
        if b == 1:
            fn(eng.h, out, 1)  # reset after the first (warm-up) batch
        eng.run()
        eng.sync()
    rc = fn(eng.h, out, 0)
    print("rc", rc)
    v = list(out)
    for i, nm in enumerate(NAMES):
        if nm:
            print("%-14s %14d  per-wave %10.1f" % (nm, v[i], v[i] / max(1, v[0])))
    st = eng.stats()
    print("last batch:", st)
    eng.close()


if __name__ == "__main__":
    main()
