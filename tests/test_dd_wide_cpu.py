"""The wide dependency-descriptor workload (synth svc_dd=2) reaches the
reference reader's maxima that the engine's old fixed limits refused
(dependencydescriptorreader.go:217-303 takes up to NumDecodeTargets chains and
unbounded frame-diff lists): an attached structure with 9 chains and T2
templates of 17 frame diffs, frames with custom lists of 9-10 and 18 frame
diffs and 9 custom chain diffs.  The descriptors are read back here by a
small bit reader (the AV1 dependency descriptor syntax), so the GPU parity
tests on this workload (test_parity_gpu / test_ingress_gpu *_dd_wide) are
known to exercise the pooled and spilled frame-diff paths.  The oracle runs
the workload end to end."""
import ctypes as C

from tests.oracle_lib import load as load_oracle

LKF_PKT_DD = 0x10  # include/lkfwd.h


class Bits:
    def __init__(self, b):
        self.b, self.i = b, 0

    def get(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.i >> 3] >> (7 - (self.i & 7))) & 1)
            self.i += 1
        return v

    def ns(self, n):
        if n <= 1:
            return 0
        w = n.bit_length()
        m = (1 << w) - n
        v = self.get(w - 1)
        return v if v < m else ((v << 1) + self.get(1)) - m


def read_dd(buf, st):
    """-> (structure or None, frame fields).  st: the structure in force."""
    r = Bits(buf)
    r.get(1), r.get(1)
    tid = r.get(6)
    r.get(16)
    out = dict(custom_fd=None, custom_chains=None, tmpl=(tid - st["offset"]) % 64 if st else None)
    if len(buf) <= 3:
        return None, out
    att, act, cdti, cfd, cch = (r.get(1) for _ in range(5))
    if att:
        st = dict(offset=r.get(6), ndt=r.get(5) + 1)
        n = 1
        while r.get(2) != 3:
            n += 1
        st["ntmpl"] = n
        for _ in range(n * st["ndt"]):
            r.get(2)
        fds = []
        for _ in range(n):
            k = 0
            while r.get(1):
                r.get(4)
                k += 1
            fds.append(k)
        st["tmpl_fd"] = fds
        st["chains"] = r.ns(st["ndt"] + 1)
        if st["chains"]:
            for _ in range(st["ndt"]):
                r.ns(st["chains"])
            for _ in range(n * st["chains"]):
                r.get(4)
        if r.get(1):
            for _ in range(3):
                r.get(32)
    if act:
        r.get(st["ndt"])
    if cdti:
        r.get(2 * st["ndt"])
    if cfd:
        k = 0
        while True:
            s = r.get(2)
            if s == 0:
                break
            r.get(4 * s)
            k += 1
        out["custom_fd"] = k
    if cch:
        out["custom_chains"] = st["chains"]
    out["tmpl"] = (tid - st["offset"]) % 64 if st else None
    return (st if att else None), out


def test_dd_wide_trace_reaches_reference_maxima(pkg, workload):
    abi = pkg.abi
    tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=3, svc_dd=2, seed=61)
    try:
        structs, cfd, cch, tmpl_long = [], [], [], 0
        cur, cur_by_track = None, {}
        for b in range(tr.nbatches):
            pk, n, ar, alen = tr.batch(b)
            dd, nd = tr.batch_dd(b)
            arena = C.string_at(ar, alen)
            for i in range(nd):
                if not (pk[i].flags & LKF_PKT_DD) or dd[i].dd_len == 0:
                    continue
                off = pk[i].arena_off + dd[i].dd_off
                buf = arena[off:off + dd[i].dd_len]
                assert dd[i].dd_len <= 255
                st, f = read_dd(buf, cur_by_track.get(pk[i].track, cur))
                if st:
                    structs.append(st)
                    cur_by_track[pk[i].track] = st
                    cur = st
                s = st or cur_by_track.get(pk[i].track, cur)
                if f["custom_fd"] is not None:
                    cfd.append(f["custom_fd"])
                elif s and f["tmpl"] is not None and s["tmpl_fd"][f["tmpl"]] > 8:
                    tmpl_long += 1
                if f["custom_chains"] is not None:
                    cch.append(f["custom_chains"])
        assert structs and all(s["chains"] == 9 and s["ndt"] == 9 for s in structs)
        assert max(max(s["tmpl_fd"]) for s in structs) == 17  # > kDDFdInline: the structure's pool
        assert tmpl_long > 0  # frames that use a long template list
        assert max(cfd) == 18 and any(9 <= k <= 10 for k in cfd)  # custom lists -> the spill array
        assert cch and set(cch) == {9}
    finally:
        tr.close()


def test_dd_wide_oracle_runs(pkg, workload):
    """The oracle forwards the wide workload; its selection differs from the
    3-chain one (long frame-diff lists reference more frames)."""
    abi = pkg.abi
    fw = {}
    for mode in (1, 2):
        tr = workload.Trace(5, duration_s=3.0, batch_s=0.5, rooms=3, svc_dd=mode, seed=61)
        o = load_oracle()
        h = o.create(500)
        try:
            workload.load_topology(o.api, h, tr)
            fw[mode] = 0
            for b in range(tr.nbatches):
                workload.queue_events(o.api, h, tr, b)
                pk, n, ar, alen = tr.batch(b)
                dd, _ = tr.batch_dd(b)
                o.run(h, pk, n, ar, alen, dd)
                st = abi.lkf_stats()
                assert o.lib.orc_get_stats(h, C.byref(st)) == 0
                fw[mode] += st.forwarded
        finally:
            o.destroy(h)
            tr.close()
    assert fw[2] > 0 and fw[2] != fw[1]
