"""Debug: config-4 parity, first wire-byte difference in detail."""
import ctypes as C, importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.oracle_lib import load as load_oracle
pkg = importlib.import_module("livekit-server_amd")
wl = importlib.import_module("livekit-server_amd.workload")
abi = importlib.import_module("livekit-server_amd.abi")
for rep in range(int(os.environ.get("REPS", "2"))):
    tr = wl.Trace(4, duration_s=2.0, batch_s=1.0, rooms=1, participants=600)
    o = load_oracle(); eng = pkg.Engine.for_trace(tr); oh = o.create(500)
    wl.load_topology(eng.api, eng.h, tr); wl.load_topology(o.api, oh, tr)
    for b in range(tr.nbatches):
        wl.queue_events(eng.api, eng.h, tr, b); wl.queue_events(o.api, oh, tr, b)
        pk, n, ar, alen = tr.batch(b)
        eng.submit(pk, n, ar, alen); eng.run(); eng.sync(); o.run(oh, pk, n, ar, alen)
        grec, gar = eng.drain(); orec, oar = pkg.drain_arrays(o.api, oh)
        bad = np.nonzero(gar != oar)[0]
        print("rep", rep, "batch", b, "records", len(grec), "bad bytes", len(bad))
        if len(bad):
            recs = np.unique(np.searchsorted(grec["out_off"], bad, side="right") - 1)
            print(" bad records:", len(recs), recs[:20])
            r = recs[0]
            off, ln = int(grec["out_off"][r]), int(grec["out_len"][r])
            print(" rec", grec[r])
            print(" gpu", gar[off:off + 48].tobytes().hex())
            print(" orc", oar[off:off + 48].tobytes().hex())
            pi = int(grec["pkt"][r])
            arr = np.ctypeslib.as_array(C.cast(pk, C.POINTER(C.c_uint8)), shape=(n * 64,))
            d = arr[pi * 64:(pi + 1) * 64]
            aoff = int(d[24:28].view(np.uint32)[0]); poff = int(d[36:38].view(np.uint16)[0]); plen = int(d[38:40].view(np.uint16)[0])
            raw = np.ctypeslib.as_array(C.cast(ar, C.POINTER(C.c_uint8)), shape=(alen,))
            print(" raw", raw[aoff:aoff + 48].tobytes().hex(), "arena_off", aoff, "poff", poff, "plen", plen, "vhs", d[47])
    eng.close(); o.destroy(oh)
