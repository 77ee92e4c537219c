"""RED for Opus on the GPU (lkf_red_encode / lkf_red_decode), engine vs oracle.

Opus tracks of lossy, reordered synthetic traces are RED-encoded batch after
batch (the two-packet history carries across batches), the RED stream is
decoded with packets dropped and reordered (recovery from the redundant
blocks, the 8-packet receive history across batches), and the RED batch is
forwarded to the tracks' DownTracks: descriptors, raw bytes and the forwarded
wire packets must be identical."""
import ctypes as C

import numpy as np
import pytest

from tests import red_lib
from tests.oracle_lib import load as load_oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [dict(config=2, rooms=3, seed=4), dict(config=3, rooms=2, seed=6)])
def test_red_encode_decode_match_oracle(pkg, workload, cfg):
    o = load_oracle()
    kw = dict(cfg)
    tr = workload.Trace(kw.pop("config"), duration_s=3.0, batch_s=1.0, **kw)
    m = red_lib.opus_map(tr)
    eng = pkg.Engine.for_trace(tr, headroom=3.5)  # RED payloads carry up to three Opus frames
    oh = o.create(500)
    rng = np.random.default_rng(1)
    try:
        workload.load_topology(eng.api, eng.h, tr)
        workload.load_topology(o.api, oh, tr)
        for b in range(tr.nbatches):
            pkts, n, arena, alen = red_lib.batch_arrays(tr, b)
            g = red_lib.red(eng.api, eng.h, "red_encode", pkts, n, arena, alen, m)
            r = red_lib.red(o.api, oh, "red_encode", pkts, n, arena, alen, m)
            assert g[1] == r[1] > 0 and np.array_equal(g[0], r[0]) and np.array_equal(g[2], r[2]), b
            rp, k, rar = r
            # the RED batch forwarded to the tracks' DownTracks (RedReceiver's WriteRTP fan-out)
            ar = (C.c_uint8 * (len(rar) + 64)).from_buffer_copy(rar.tobytes() + bytes(64))
            pk = (pkg.abi.lkf_pkt * k).from_buffer_copy(rp.tobytes())
            eng.submit(pk, k, ar, len(rar))
            eng.run()
            eng.sync()
            o.run(oh, pk, k, ar, len(rar))
            grec, gw = eng.drain()
            orec, ow = pkg.drain_arrays(o.api, oh)
            assert len(grec) == len(orec) > 0
            for f in pkg.abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gw, ow), b
            # decode with losses (and a few swaps inside each track's run)
            keep = rng.random(k) > 0.3
            idx = np.nonzero(keep)[0]
            f = red_lib.fields(rp, k)
            for j in range(0, len(idx) - 1, 7):
                if f["track"][idx[j]] == f["track"][idx[j + 1]]:
                    idx[j], idx[j + 1] = idx[j + 1], idx[j]
            lp = rp.reshape(k, 64)[idx].reshape(-1).copy()
            g = red_lib.red(eng.api, eng.h, "red_decode", lp, len(idx), rar, len(rar), m)
            r = red_lib.red(o.api, oh, "red_decode", lp, len(idx), rar, len(rar), m)
            assert g[1] == r[1] > len(idx) and np.array_equal(g[0], r[0]) and np.array_equal(g[2], r[2]), b
    finally:
        eng.close()
        o.destroy(oh)
        tr.close()
