"""A CPU stand-in for `Engine` in bench.py's launcher rehearsal (`--dry-run`).

Test infrastructure only: it drives the CPU oracle (oracle/, loaded through
tests/oracle_lib.py) behind the few Engine methods bench.py's step loop calls,
so that the multi-process launcher, the room plan, the per-tick summary
all-gathers and the max-over-ranks reduction can run on a machine without a
GPU (gloo backend).  The numbers such a run prints are not a measurement and
the JSON line says so ("dry_run": true).  Nothing in the product path imports
this module.
"""
import ctypes as C

from tests.oracle_lib import load as load_oracle


class DryRunEngine:
    """Engine's bench-facing surface over one oracle engine (host pointers)."""

    def __init__(self, seq_size=500):
        self.o = load_oracle()
        self.api = self.o.api
        self.h = self.o.create(seq_size)
        self._cum = None
        self._pending = None
        self.reset_cum()

    @classmethod
    def for_trace(cls, trace, **kw):
        return cls()

    def reset_cum(self):
        self._cum = {"tuples": 0, "forwarded": 0, "out_bytes": 0, "arena_bytes": 0,
                     "drops": [0] * self.o.abi.LKF_DROP_NREASONS}

    def ingest_device(self, raws, n, raw, raw_len):
        rc = self.api["ingest"](self.h, C.cast(raws, C.c_void_p), n, C.cast(raw, C.c_void_p), raw_len)
        assert rc == 0, rc
        # the ingested ExtPacket batch (oracle-owned) over the same raw arena
        p, m = C.c_void_p(), C.c_uint32()
        f = self.o.lib.orc_ingested_ptr
        f.restype, f.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]
        assert f(self.h, C.byref(p), C.byref(m)) == 0
        self._pending = (p, m.value, raw, raw_len)

    def submit_device(self, pkts, n, arena, arena_len):
        self._pending = (pkts, n, arena, arena_len)

    def run(self, stream=None):
        pk, n, ar, alen = self._pending
        rc = self.o.lib.orc_run(self.h, C.cast(pk, C.c_void_p), n, C.cast(ar, C.c_void_p), alen)
        assert rc == 0, rc
        self._pending = None
        st = self.o.abi.lkf_stats()
        assert self.api["get_stats"](self.h, C.byref(st)) == 0
        d = st.as_dict()
        for k in ("tuples", "forwarded", "out_bytes", "arena_bytes"):
            self._cum[k] += d[k]
        self._cum["drops"] = [a + b for a, b in zip(self._cum["drops"], d["drops"])]

    def sync(self):
        pass

    def cumulative(self, reset=False):
        out = dict(self._cum, drops=list(self._cum["drops"]))
        if reset:
            self.reset_cum()
        return out

    def timing_window(self, n):
        return 0.0, 0.0, 0.0

    def close(self):
        if self.h:
            self.o.destroy(self.h)
            self.h = None
