"""Sender-report-driven reference-layer offsets as packet-indexed control ops
(VERDICT r4 item 6), engine vs oracle.

Simulcast publishers send an RTCP sender report per layer about once a
second; StreamTrackerManager.SetRTCPSenderReportData recomputes the
layerOffsets that processSourceSwitch reads through
GetReferenceLayerRTPTimestamp on every layer switch (streamtrackermanager.go
:561-627, :660-679; forwarder.go:1512-1520).  Here every 3-layer video track
gets sender reports in every batch, each applied at a packet index inside the
batch (lkf_sender_report, no pipeline drain), with RTP timestamps jittered so
that the offsets change between switches; some tracks also get a whole table
(lkf_set_layer_offsets) between batches.  Every record, wire byte, counter and
exported Forwarder state must equal the oracle's, and the run must differ from
one without the reports (the offsets were used)."""
import ctypes as C

import numpy as np
import pytest

from tests.oracle_lib import load as load_oracle
from tests.test_parity_gpu import _state_tuple

pytestmark = pytest.mark.gpu


def _reports(tr, b, n, rng):
    """(track, layer, ntp, rtp, at_pkt) for batch b (n packets)."""
    out = []
    for t in range(tr.ntracks):
        p = tr.tracks[t]
        if p.kind != 1 or not p.has_ref_ts:
            continue
        base = ((3_900_000_000 + b) << 32) + int(rng.integers(0, 1 << 31))
        x = int(rng.integers(0, 1 << 32))
        for layer in range(3):
            if rng.random() < 0.3:
                continue
            frac = int(rng.integers(0, 1 << 30))
            ntp = base + frac
            rtp = (x - int(p.layer_offsets[0][layer]) + frac * 90000 // (1 << 32) +
                   int(rng.integers(-400, 400))) & 0xFFFFFFFF
            out.append((t, layer, ntp, rtp, int(rng.integers(0, max(1, n)))))
    return out


def _run(api, h, tr, with_reports, seed, drain):
    rng = np.random.default_rng(seed)
    outs = []
    for b in range(tr.nbatches):
        pk, n, ar, alen = tr.batch(b)
        reps = _reports(tr, b, n, rng)
        if with_reports:
            for t, layer, ntp, rtp, at in reps:
                assert api["sender_report"](h, t, layer, ntp, rtp, at) == 0
            if b == 2:  # a whole table between batches (from the next batch's first packet)
                for t in range(0, tr.ntracks, 5):
                    if tr.tracks[t].kind == 1:
                        tab = (C.c_uint32 * 9)(*[(int(tr.tracks[t].layer_offsets[r][l]) + 7 * (r - l)) & 0xFFFFFFFF
                                                 for r in range(3) for l in range(3)])
                        assert api["set_layer_offsets"](h, t, tab) == 0
        outs.append(drain(b, pk, n, ar, alen))
    return outs


def test_sender_reports_mid_trace(pkg, workload, abi):
    tr = workload.Trace(2, duration_s=5.0, batch_s=1.0, rooms=4, seed=77)
    o = load_oracle()
    eng = pkg.Engine.for_trace(tr)
    oh, oh0 = o.create(500), o.create(500)
    try:
        for api, h in ((eng.api, eng.h), (o.api, oh), (o.api, oh0)):
            workload.load_topology(api, h, tr)

        def eng_batch(b, pk, n, ar, alen):
            workload.queue_events(eng.api, eng.h, tr, b)
            eng.submit(pk, n, ar, alen)
            eng.run()
            eng.sync()
            return eng.drain()

        def orc_batch(h):
            def f(b, pk, n, ar, alen):
                workload.queue_events(o.api, h, tr, b)
                o.run(h, pk, n, ar, alen)
                return pkg.drain_arrays(o.api, h)
            return f

        g = _run(eng.api, eng.h, tr, True, 9, eng_batch)
        r = _run(o.api, oh, tr, True, 9, orc_batch(oh))
        r0 = _run(o.api, oh0, tr, False, 9, orc_batch(oh0))
        differs = 0
        for b in range(tr.nbatches):
            (grec, gar), (orec, oar), (zrec, zar) = g[b], r[b], r0[b]
            assert len(grec) == len(orec), b
            for f in abi.OUT_DTYPE.names:
                assert np.array_equal(grec[f], orec[f]), (b, f)
            assert np.array_equal(gar, oar), b
            differs += int(len(zrec) != len(orec) or not np.array_equal(zrec["ext_ts"], orec["ext_ts"]))
        assert differs > 0, "the reports changed nothing: no switch read the new offsets"
        for d in range(tr.ndts):
            assert _state_tuple(eng.api, eng.h, d, abi) == _state_tuple(o.api, oh, d, abi), d
    finally:
        o.destroy(oh)
        o.destroy(oh0)
        eng.close()
