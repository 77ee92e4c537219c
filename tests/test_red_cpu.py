"""RED for Opus on the CPU oracle (the checker of the GPU kernels; the
restatement itself is pinned by redreceiver_test.go in oracle/kat_red.inc):
encode -> decode over a synthetic trace's Opus tracks returns every primary
payload unchanged, and with packets dropped between the two the redundant
blocks recover them (RFC 2198, redreceiver.go / redprimaryreceiver.go)."""
import numpy as np

from tests import red_lib
from tests.oracle_lib import load as load_oracle


def test_red_round_trip_and_recovery(workload):
    o = load_oracle()
    tr = workload.Trace(2, duration_s=2.0, batch_s=1.0, rooms=2, seed=3, loss=0.0, reorder=0.0)
    m = red_lib.opus_map(tr)
    enc_h, dec_h, dec2_h = o.create(500), o.create(500), o.create(500)
    try:
        for h in (enc_h, dec_h, dec2_h):
            workload.load_topology(o.api, h, tr)
        recovered = 0
        for b in range(tr.nbatches):
            pkts, n, arena, alen = red_lib.batch_arrays(tr, b)
            rp, k, rar = red_lib.red(o.api, enc_h, "red_encode", pkts, n, arena, alen, m)
            src = red_lib.fields(pkts, n)
            audio = np.isin(src["track"], np.nonzero(m >= 0)[0])
            assert k == int(audio.sum()) > 0
            # no loss: the primaries come back, byte for byte
            dp, dk, dar = red_lib.red(o.api, dec_h, "red_decode", rp, k, rar, len(rar), m)
            f = red_lib.fields(dp, dk)
            assert dk == k
            assert np.array_equal(f["ext_sn"], src["ext_sn"][audio])
            for j, i in enumerate(np.nonzero(audio)[0]):
                a = arena[src["arena_off"][i] + src["payload_off"][i]:][:src["payload_len"][i]]
                g = dar[f["arena_off"][j] + f["payload_off"][j]:][:f["payload_len"][j]]
                assert np.array_equal(a, g)
            # every third RED packet lost: recovered from the next packets' blocks
            keep = np.arange(k) % 3 != 1
            kp, kk = red_lib.drop(rp, k, keep)
            lp, lk, _ = red_lib.red(o.api, dec2_h, "red_decode", kp, kk, rar, len(rar), m)
            recovered += lk - kk
        assert recovered > 100
    finally:
        for h in (enc_h, dec_h, dec2_h):
            o.destroy(h)
        tr.close()
