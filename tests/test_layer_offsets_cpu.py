"""Sender-report-driven reference-layer offsets, CPU side.

StreamTrackerManager.SetRTCPSenderReportData (streamtrackermanager.go:603-627)
recomputes layerOffsets[ref][other] for the reporting layer against every
other layer, both ways, with updateLayerOffsetLocked (:561-601).  The oracle's
restatement (oracle/oracle_engine.cpp orc_sender_report) is checked here
against an independent Python restatement with Go's integer semantics
(truncating int64 division, uint32 wrap, time.Duration.Seconds,
mediatransportutil NtpTime.Time).  No reference test covers the function:
parity unpinned beyond the two restatements; the NTP conversion follows
mediatransportutil's published source (the module is not vendored)."""
import ctypes as C

import numpy as np

from tests.oracle_lib import load as load_oracle

M32 = 0xFFFFFFFF


def go_quo(a, b):  # Go's truncating integer division
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def ntp_duration(t):
    sec = (t >> 32) * 10**9
    frac = (t & M32) * 10**9
    nsec = frac >> 32
    if (frac & M32) >= 0x80000000:
        nsec += 1
    return sec + nsec


def seconds(d):
    sec = go_quo(d, 10**9)
    return float(sec) + float(d - sec * 10**9) / 1e9


class PyManager:
    def __init__(self, clock, offs):
        self.clock = clock
        self.sr = [None, None, None]
        self.offs = [list(r) for r in offs]

    def _update(self, ref, other):
        a, b = self.sr[ref], self.sr[other]
        if a is None or a[0] == 0 or b is None or b[0] == 0:
            return
        d = ntp_duration(a[0]) - ntp_duration(b[0])
        if abs(seconds(d)) > 60.0:
            return
        rtp_diff = go_quo(d * self.clock, 10**9)
        norm = (b[1] + (rtp_diff & M32)) & M32
        off = (a[1] - norm) & M32
        self.offs[ref][other] = off or 1

    def report(self, layer, ntp, rtp):
        if layer < 0 or layer > 2:
            return
        self.sr[layer] = (ntp, rtp)
        for i in range(3):
            if i != layer:
                self._update(layer, i)
                self._update(i, layer)


def test_sender_report_offsets_match_python_restatement():
    o = load_oracle()
    abi = o.abi
    o.lib.orc_debug_layer_offsets.restype = C.c_int
    o.lib.orc_debug_layer_offsets.argtypes = [C.c_void_p, C.c_int32, C.c_int, C.c_void_p]
    rng = np.random.default_rng(5)
    h = o.create(500)
    try:
        for trial in range(6):
            tp = abi.lkf_track_params()
            tp.kind = abi.LKF_KIND_VIDEO
            tp.codec = 2  # LKF_CODEC_VP8
            tp.clock_rate = 90000
            tp.has_ref_ts = 1
            init = rng.integers(0, 2**32, (3, 3), dtype=np.uint64)
            for r in range(3):
                for l in range(3):
                    tp.layer_offsets[r][l] = int(init[r][l]) if r != l else 0
            t = o.api["add_track"](h, C.byref(tp))
            py = PyManager(90000, [[tp.layer_offsets[r][l] for l in range(3)] for r in range(3)])
            base = (3_900_000_000 << 32) + int(rng.integers(0, 2**32))
            rtp0 = int(rng.integers(0, 2**32))
            for k in range(200):
                layer = int(rng.integers(-1, 4))  # -1 and 3: ignored
                jump = int(rng.choice([0, 1, 1, 1, 70, -70])) * (1 << 32)  # seconds; 70 s apart: not used
                ntp = (base + k * (1 << 30) + int(rng.integers(0, 1 << 31)) + jump) & ((1 << 64) - 1)
                rtp = (rtp0 + k * 22500 + int(rng.integers(-3000, 3000)) - (int(init[0][layer]) if 0 <= layer < 3 else 0)) & M32
                if k % 37 == 5:
                    ntp = 0  # a report without NTP time: no offset from or against it
                py.report(layer, ntp, rtp)
                assert o.api["sender_report"](h, t, layer, ntp, rtp, k) == 0
                out = (C.c_uint32 * 9)()
                assert o.lib.orc_debug_layer_offsets(h, t, 1, out) == 0
                assert [out[i] for i in range(9)] == [py.offs[r][l] for r in range(3) for l in range(3)], (trial, k)
            # the applied table changes only with the next batch (at its packet indices)
            applied = (C.c_uint32 * 9)()
            assert o.lib.orc_debug_layer_offsets(h, t, 0, applied) == 0
            assert [applied[i] for i in range(9)] == [tp.layer_offsets[r][l] for r in range(3) for l in range(3)]
            o.run(h, None, 0, None, 0)
            assert o.lib.orc_debug_layer_offsets(h, t, 0, applied) == 0
            assert [applied[i] for i in range(9)] == [py.offs[r][l] for r in range(3) for l in range(3)]
    finally:
        o.destroy(h)
