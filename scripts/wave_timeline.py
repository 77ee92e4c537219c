"""Diagnostic: k_decide_dt per-wave lifetimes from a -DLKF_WTIME=1 build.

    make -C livekit-server_amd/csrc wtime && python3 scripts/wave_timeline.py [rooms] [batches] [batch_s]

Runs configs[1] batches (1 s each by default) through liblkfwd_wtime.so, then reads the
last decide launch's per-wave stamps (s_memrealtime, 100 MHz): the occupancy
curve (waves alive over time), wave lifetime vs packets / serial steps.
"""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rooms = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    pkg = importlib.import_module("livekit-server_amd")
    wl = importlib.import_module("livekit-server_amd.workload")
    bs = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    cfg = int(os.environ.get("WT_CONFIG", "2"))
    tr = wl.Trace(cfg, duration_s=nb * bs, batch_s=bs, rooms=rooms)
    lib = os.path.join(ROOT, "livekit-server_amd", "lib", os.environ.get("WTIME_LIB", "liblkfwd_wtime.so"))
    eng = pkg.Engine.for_trace(tr, lib_path=lib)
    fn = eng.lib.lkf_debug_wtime
    fn.restype = C.c_int
    fn.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint32]
    wl.load_topology(eng.api, eng.h, tr)
    for b in range(nb):
        wl.queue_events(eng.api, eng.h, tr, b)
        pk, n, ar, alen = tr.batch(b)
        eng.submit(pk, n, ar, alen, tr.batch_dd(b)[0] if tr.has_dd() else None)
        eng.run()
        eng.sync()
    nw = 1 << 17
    buf = (C.c_uint32 * (16 * nw))()
    assert fn(eng.h, buf, nw) == 0
    a = np.frombuffer(buf, dtype=np.uint32).reshape(-1, 16).astype(np.int64)
    a = a[(a[:, 0] != 0) | (a[:, 1] != 0)]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) * 10  # ns
    en = (a[:, 1] - t0) * 10
    life = en - st
    pk = a[:, 2]
    ser = a[:, 3] & 0xFFFF
    ch = a[:, 3] >> 16
    print("waves %d  kernel span %.1f us" % (len(a), en.max() / 1e3))
    print("lifetime us: mean %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f" % (
        life.mean() / 1e3, *(np.percentile(life, q) / 1e3 for q in (50, 90, 99)), life.max() / 1e3))
    print("start us: p50 %.1f p90 %.1f max %.1f ; end us: p10 %.1f p50 %.1f p90 %.1f" % (
        *(np.percentile(st, q) / 1e3 for q in (50, 90)), st.max() / 1e3,
        *(np.percentile(en, q) / 1e3 for q in (10, 50, 90))))
    # occupancy curve
    T = int(en.max() // 1000) + 1
    occ = np.zeros(T + 1)
    for s_, e_ in zip(st // 1000, en // 1000):
        occ[s_:e_ + 1] += 1
    print("waves alive per 10 us:", " ".join("%d" % occ[i] for i in range(0, T, 10)))
    print("mean alive %.0f" % (life.sum() / en.max()))
    for lo, hi in ((0, 100), (100, 200), (200, 400), (400, 100000)):
        m = (pk >= lo) & (pk < hi)
        if m.any():
            print("packets [%d,%d): %5d waves  life %.1f us  serial %.2f  chunks %.2f" % (
                lo, hi, m.sum(), life[m].mean() / 1e3, ser[m].mean(), ch[m].mean()))
    for k in range(0, 6):
        m = ser == k
        if m.any():
            print("serial=%d: %5d waves  life %.1f us" % (k, m.sum(), life[m].mean() / 1e3))
    m = ser >= 6
    if m.any():
        print("serial>=6: %5d waves  life %.1f us" % (m.sum(), life[m].mean() / 1e3))
    pro, stp, drn, tot = a[:, 4], a[:, 5], a[:, 6], a[:, 7]
    print("cycles per wave: total %.0f prologue %.0f serial-steps %.0f drains %.0f (%.0f%% / %.0f%% / %.0f%%)" % (
        tot.mean(), pro.mean(), stp.mean(), drn.mean(), 100 * pro.sum() / tot.sum(), 100 * stp.sum() / tot.sum(),
        100 * drn.sum() / tot.sum()))
    ms = ser > 0
    print("per serial step: %.0f cycles + drain %.0f (svc DownTracks: 'drain' = cycles in svc_run)" % (
        stp[ms].sum() / ser[ms].sum(), drn[ms].sum() / ser[ms].sum()))
    if os.environ.get("WT_PART1"):  # the k_decide_dt<true> waves only (slots past the plain part)
        pass
    top = np.argsort(-life)[:10]
    for i in top:
        lay = a[i, 13]
        print("  long wave: life %.1f us pk %d serial %d (reorder %d kf %d ssrc/pad %d other %d) runs %d chunks %d "
              "pro %d step %d tot %d  S %d->%d T %d->%d" % (
                  life[i] / 1e3, pk[i], ser[i], a[i, 9], a[i, 10], a[i, 11], a[i, 12], a[i, 8], ch[i], pro[i],
                  stp[i], tot[i], np.int8(lay & 255), np.int8((lay >> 8) & 255), np.int8((lay >> 16) & 255),
                  np.int8((lay >> 24) & 255)))
    re = a[:, 14]
    ends = [(re & 255).sum(), ((re >> 8) & 255).sum(), ((re >> 16) & 255).sum(), ((re >> 24) & 255).sum(),
            a[:, 15].sum()]
    print("run ends: chunk end %d, control op %d, temporal switch %d, later gap %d, full step %d" % tuple(ends))
    print("runs per wave %.2f; serial reasons: reorder %d kf %d ssrc/pad %d other %d" % (
        a[:, 8].mean(), a[:, 9].sum(), a[:, 10].sum(), a[:, 11].sum(), a[:, 12].sum()))
    nonrun = tot - stp - drn - pro
    print("non-serial cycles per run: %.0f" % (nonrun.sum() / max(1, a[:, 8].sum())))
    eng.close()


if __name__ == "__main__":
    main()
