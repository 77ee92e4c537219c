"""SRTP test helpers (test infrastructure).

- bind_transports: one transport per (room, subscriber) of a synthetic trace
  with seeded master keys; every seventh DownTrack stays unbound (its packets
  go out unprotected), identically on the engine and the oracle.
- An independent RFC 3711 AES_CM_128_HMAC_SHA1_80 protect built from OpenSSL's
  AES-128 (libcrypto, ECB single blocks) and Python's hmac/hashlib: the
  checker for the oracle's restatement (oracle/srtp_oracle.h).
"""
import ctypes as C
import hashlib
import hmac

import numpy as np


def bind_transports(pkg, api, h, trace, seed, unbound_every=7):
    rng = np.random.default_rng(seed)
    keys, tmap = {}, {}
    for d in range(trace.ndts):
        p = trace.downtracks[d]
        if d % unbound_every == 0:
            continue
        k = (int(trace.tracks[p.track].room), int(p.subscriber))
        if k not in keys:
            mk = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
            ms = rng.integers(0, 256, 14, dtype=np.uint8).tobytes()
            t = api["add_transport"](h, C.byref(pkg.transport_params(mk, ms)))
            assert t >= 0, t
            keys[k] = (t, mk, ms)
        assert api["set_downtrack_transport"](h, d, keys[k][0]) == 0
        tmap[d] = keys[k]
    return tmap


class OpenSSLAes:
    """AES-128 block encryption from the system libcrypto (EVP, ECB)."""

    def __init__(self):
        c = C.CDLL("libcrypto.so.3")
        c.EVP_CIPHER_CTX_new.restype = C.c_void_p
        c.EVP_aes_128_ecb.restype = C.c_void_p
        c.EVP_EncryptInit_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_char_p]
        c.EVP_CIPHER_CTX_set_padding.argtypes = [C.c_void_p, C.c_int]
        c.EVP_EncryptUpdate.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int), C.c_char_p, C.c_int]
        c.EVP_CIPHER_CTX_free.argtypes = [C.c_void_p]
        self.c = c

    def ecb(self, key, data):
        ctx = self.c.EVP_CIPHER_CTX_new()
        try:
            assert self.c.EVP_EncryptInit_ex(ctx, self.c.EVP_aes_128_ecb(), None, bytes(key), None) == 1
            self.c.EVP_CIPHER_CTX_set_padding(ctx, 0)
            out = C.create_string_buffer(len(data) + 16)
            n = C.c_int(0)
            assert self.c.EVP_EncryptUpdate(ctx, out, C.byref(n), bytes(data), len(data)) == 1
            return out.raw[:n.value]
        finally:
            self.c.EVP_CIPHER_CTX_free(ctx)


def kdf(aes, label, mk, ms, n):
    """RFC 3711 §4.3.1 / §4.3.3 AES-CM PRF with key_derivation_rate 0."""
    out = b""
    i = 0
    while len(out) < n:
        x = bytearray(ms + b"\0\0")
        x[7] ^= label
        x[14], x[15] = i >> 8, i & 255
        out += aes.ecb(mk, bytes(x))
        i += 1
    return out[:n]


def session(aes, mk, ms):
    return kdf(aes, 0, mk, ms, 16), kdf(aes, 2, mk, ms, 14), kdf(aes, 1, mk, ms, 20)


def header_len(pkt):
    n = 12 + 4 * (pkt[0] & 15)
    if pkt[0] & 0x10:
        n += 4 + 4 * ((pkt[n + 2] << 8) | pkt[n + 3])
    return n


def abs_send_time(unix_ns):
    ntp = ((unix_ns // 10**9 + 0x83AA7E80) << 32) | (((unix_ns % 10**9) << 32) // 10**9)
    return (ntp >> 14) & 0xFFFFFF


def stamp_abs(pkt, ext, v):
    """The abs-send-time element (id `ext`, 3 bytes) of a one- or two-byte
    extension block set to v."""
    pkt = bytearray(pkt)
    if not ext or not (pkt[0] & 0x10):
        return bytes(pkt)
    x = 12 + 4 * (pkt[0] & 15)
    prof = (pkt[x] << 8) | pkt[x + 1]
    end = header_len(pkt)
    p = x + 4
    while p < end:
        if pkt[p] == 0:
            p += 1
            continue
        if prof == 0xBEDE:
            i, ln, dat = pkt[p] >> 4, (pkt[p] & 15) + 1, p + 1
            if i == 15:
                break
        else:
            i, ln, dat = pkt[p], pkt[p + 1], p + 2
        if i == ext and ln == 3:
            pkt[dat:dat + 3] = bytes([(v >> 16) & 255, (v >> 8) & 255, v & 255])
            break
        p = dat + ln
    return bytes(pkt)


def protect(aes, sess, pkt, roc):
    key, salt, auth = sess
    h = header_len(pkt)
    seq = (pkt[2] << 8) | pkt[3]
    iv = int.from_bytes(salt + b"\0\0", "big") ^ (int.from_bytes(pkt[8:12], "big") << 64) \
        ^ (((roc << 16) | seq) << 16)
    nblk = (len(pkt) - h + 15) // 16
    ks = aes.ecb(key, b"".join(((iv + j) % (1 << 128)).to_bytes(16, "big") for j in range(nblk)))
    ct = bytes(a ^ b for a, b in zip(pkt[h:], ks))
    m = pkt[:h] + ct
    tag = hmac.new(auth, m + roc.to_bytes(4, "big"), hashlib.sha1).digest()[:10]
    return m + tag


class Checker:
    """Replays a DownTrack-ordered record stream: ROC = (ext SN >> 16) minus
    that of the DownTrack's first protected packet."""

    def __init__(self, trace, tmap, aes=None):
        self.aes = aes or OpenSSLAes()
        self.trace = trace
        self.tmap = tmap
        self.sess = {}
        self.base = {}
        self.n_roc = 0  # protected packets with a nonzero rollover counter

    def expect(self, rec, plain, send_ns):
        d = int(rec["dt"])
        pkt = stamp_abs(plain, int(self.trace.downtracks[d].ext_abs_send_time), abs_send_time(send_ns))
        if d not in self.tmap:
            return pkt
        t, mk, ms = self.tmap[d]
        if t not in self.sess:
            self.sess[t] = session(self.aes, mk, ms)
        b = self.base.setdefault(d, int(rec["ext_sn"]) >> 16)
        roc = ((int(rec["ext_sn"]) >> 16) - b) & 0xFFFFFFFF
        self.n_roc += roc != 0
        return protect(self.aes, self.sess[t], pkt, roc)
