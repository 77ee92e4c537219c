"""(diagnosis) Per-wave phase stamps of k_ing_nack on the headline trace:
needs a build with -DLKF_NACK_DBG=2 (make ab ABNAME=ndbg ABINGFLAGS=-DLKF_NACK_DBG=2)
loaded with LKF_LIB=liblkfwd_ndbg.so.  One ingest + run at a time; prints, per
batch, the kernel span and the median / p90 of each phase of a wave."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
pkg = importlib.import_module("livekit-server_amd")
workload = importlib.import_module("livekit-server_amd.workload")

tr = workload.Trace(int(os.environ.get("NS_CFG", "2")), duration_s=float(os.environ.get("NS_DUR", "6")), batch_s=1.0)
workload.events_at_batch_start(tr)
lp = os.path.join(os.path.dirname(pkg.__file__), "lib", os.environ.get("LKF_LIB", "liblkfwd_ndbg.so"))
eng = pkg.Engine.for_trace(tr, device=0, lib_path=lp)
lib = eng.lib
f = lib.lkf_debug_nack_stamps
f.restype, f.argtypes = C.c_int, [C.POINTER(C.c_ulonglong), C.c_uint]
buf = (C.c_ulonglong * (7 * 65536))()
workload.load_topology(eng.api, eng.h, tr)
workload.load_streams(eng.api, eng.h, tr)
for b in range(tr.nbatches):
    workload.queue_events(eng.api, eng.h, tr, b)
    rp, n, ar, alen = tr.batch_raw(b)
    eng.ingest(rp, n, ar, alen)
    eng.run()
    eng.sync()
    k = f(buf, 65536)
    assert k > 0, k
    a = np.ctypeslib.as_array(buf)[: 7 * k].reshape(k, 7).astype(np.int64)
    nIdx = a[:, 0] >> 32
    t0, tA, tB, tC = a[:, 1], a[:, 2], a[:, 3], a[:, 4]
    tD = a[:, 5]
    M = a[:, 6] & 0xFFFFFFFF
    E = a[:, 6] >> 32
    T0 = t0.min()
    d = (tD - t0) / 100
    st = (t0 - T0) / 100
    print("batch %d: waves %d span %.1f us; wave %.1f med %.1f p90 %.1f max; last start %.1f us" %
          (b, k, (tD.max() - T0) / 100, np.median(d), np.percentile(d, 90), d.max(), st.max()))
    ph = np.stack([tA - t0, tB - tA, tC - tB, tD - tC]) / 100
    print("   median: loads %.1f  hash/remove %.1f  life+sort %.1f  pairs/queue %.1f" % tuple(np.median(ph, axis=1)))
    print("   p90   : loads %.1f  hash/remove %.1f  life+sort %.1f  pairs/queue %.1f" % tuple(np.percentile(ph, 90, axis=1)))
    print("   nIdx med %d max %d; M med %d max %d; E med %d max %d" %
          (np.median(nIdx), nIdx.max(), np.median(M), M.max(), np.median(E), E.max()))
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([tD, -np.ones_like(tD)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    print("   most waves alive at once: %d" % np.cumsum(ev[:, 1]).max())
    for q in (5, 10, 20, 40, 80):
        print("   started by %3d us: %d  finished by: %d" % (q, (st < q).sum(), ((tD - T0) / 100 < q).sum()))
eng.close()
tr.close()
