"""SRTP test helpers (test infrastructure).

- bind_transports: one transport per (room, subscriber) of a synthetic trace
  with seeded master keys; every seventh DownTrack stays unbound (its packets
  go out unprotected), identically on the engine and the oracle.
- An independent RFC 3711 AES_CM_128_HMAC_SHA1_80 protect built from OpenSSL's
  AES-128 (libcrypto, ECB single blocks) and Python's hmac/hashlib, and an
  RFC 7714 AEAD_AES_128_GCM protect on OpenSSL's EVP AES-128-GCM: the checkers
  for the oracle's restatement (oracle/srtp_oracle.h).
"""
import ctypes as C
import hashlib
import hmac

import numpy as np

AES_CM, GCM = 1, 2  # LKF_SRTP_AES128_CM_HMAC_SHA1_80, LKF_SRTP_AEAD_AES_128_GCM


def bind_transports(pkg, api, h, trace, seed, unbound_every=7, gcm_every=0):
    """gcm_every: every gcm_every-th transport (in creation order) is
    AEAD_AES_128_GCM (12-byte master salt), the rest AES_CM_128_HMAC_SHA1_80;
    the map holds (transport, master key, master salt, profile)."""
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
            prof = GCM if gcm_every and len(keys) % gcm_every == gcm_every - 1 else AES_CM
            if prof == GCM:
                ms = ms[:12]
            t = api["add_transport"](h, C.byref(pkg.transport_params(mk, ms, prof)))
            assert t >= 0, t
            keys[k] = (t, mk, ms, prof)
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

    def gcm_seal(self, key, iv, aad, pt):
        """AES-128-GCM (96-bit IV): ciphertext || 16-byte tag."""
        c = self.c
        if not hasattr(self, "_gcm"):
            c.EVP_aes_128_gcm.restype = C.c_void_p
            c.EVP_CIPHER_CTX_ctrl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
            c.EVP_EncryptFinal_ex.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_int)]
            self._gcm = True
        ctx = c.EVP_CIPHER_CTX_new()
        try:
            assert c.EVP_EncryptInit_ex(ctx, c.EVP_aes_128_gcm(), None, None, None) == 1
            assert c.EVP_CIPHER_CTX_ctrl(ctx, 0x9, 12, None) == 1  # EVP_CTRL_GCM_SET_IVLEN
            assert c.EVP_EncryptInit_ex(ctx, None, None, bytes(key), bytes(iv)) == 1
            n = C.c_int(0)
            if aad:
                assert c.EVP_EncryptUpdate(ctx, None, C.byref(n), bytes(aad), len(aad)) == 1
            out = C.create_string_buffer(len(pt) + 32)
            got = 0
            if pt:
                assert c.EVP_EncryptUpdate(ctx, out, C.byref(n), bytes(pt), len(pt)) == 1
                got = n.value
            tail = C.create_string_buffer(32)
            assert c.EVP_EncryptFinal_ex(ctx, tail, C.byref(n)) == 1
            ct = out.raw[:got] + tail.raw[:n.value]
            tag = C.create_string_buffer(16)
            assert c.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag) == 1  # EVP_CTRL_GCM_GET_TAG
            return ct + tag.raw
        finally:
            c.EVP_CIPHER_CTX_free(ctx)


def kdf(aes, label, mk, ms, n):
    """RFC 3711 §4.3.1 / §4.3.3 AES-CM PRF with key_derivation_rate 0."""
    out = b""
    i = 0
    while len(out) < n:
        x = bytearray(ms + bytes(16 - len(ms)))
        x[7] ^= label
        x[14], x[15] = i >> 8, i & 255
        out += aes.ecb(mk, bytes(x))
        i += 1
    return out[:n]


def session(aes, mk, ms, prof=AES_CM):
    if prof == GCM:  # RFC 7714 §12: 12-byte session salt, no auth key
        return kdf(aes, 0, mk, ms, 16), kdf(aes, 2, mk, ms, 12), None
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


def protect_gcm(aes, sess, pkt, roc):
    """RFC 7714 §8.1: IV = (00 00 || SSRC || ROC || SEQ) XOR salt, AAD = the
    header, ciphertext || tag after it."""
    key, salt, _ = sess
    h = header_len(pkt)
    seq = (pkt[2] << 8) | pkt[3]
    iv = bytes(2) + bytes(pkt[8:12]) + roc.to_bytes(4, "big") + seq.to_bytes(2, "big")
    iv = bytes(a ^ b for a, b in zip(iv, salt))
    return bytes(pkt[:h]) + aes.gcm_seal(key, iv, pkt[:h], pkt[h:])


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
        t, mk, ms, prof = self.tmap[d]
        if t not in self.sess:
            self.sess[t] = session(self.aes, mk, ms, prof)
        b = self.base.setdefault(d, int(rec["ext_sn"]) >> 16)
        roc = ((int(rec["ext_sn"]) >> 16) - b) & 0xFFFFFFFF
        self.n_roc += roc != 0
        return (protect_gcm if prof == GCM else protect)(self.aes, self.sess[t], pkt, roc)
