// =============================================================================
//  srtp_oracle.h — TEST INFRASTRUCTURE ONLY (checker for the SRTP protect stage).
//
//  Scalar restatement of the SRTP protect path behind pacer/base.go:59
//  (p.WriteStream.WriteRTP after writeRTPHeaderExtensions, base.go:71-100).
//  The algorithm lives in third-party code that is not in /root/reference:
//  github.com/pion/srtp/v2 v2.0.18 (go.mod:87, pulled in by pion/webrtc/v3
//  v3.2.24, go.mod:37).  Restated from its published algorithm:
//    - RFC 3711 §4.1.1 AES Counter Mode keystream and §4.3.1 key derivation
//      (pion: key_derivation.go aesCmKeyDerivation, srtp.go generateCounter),
//    - RFC 3711 §4.2 HMAC-SHA1 authentication, 80-bit tag over the
//      authenticated portion || ROC (pion: srtp_cipher_aes_cm_hmac_sha1.go
//      encryptRTP / generateSrtpAuthTag),
//    - the sender-side rollover counter of pion's srtpSSRCState
//      (context.go nextRolloverCount / updateRolloverCount),
//    - pion/rtp NewAbsSendTimeExtension (abssendtimeextension.go) for the
//      abs-send-time value the pacer writes.
//  Block cipher, hash and MAC are textbook FIPS-197 (byte-oriented, no
//  tables), FIPS 180-4 and RFC 2104.  Pinned by the FIPS-197 C.1 and RFC 3711
//  B.2 / B.3 known answers and RFC 2202 HMAC-SHA1 vectors (oracle/kat.cpp),
//  and in tests/test_srtp_cpu.py against OpenSSL's AES-128 and HMAC-SHA1.
// =============================================================================
#pragma once
#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

namespace orc_srtp {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;

// ---- AES-128 (FIPS-197 §5.1-5.2, byte oriented) -----------------------------
inline u8 xtime(u8 a) { return u8((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
inline u8 gmul(u8 a, u8 b) {
  u8 p = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) p ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return p;
}
// S-box: multiplicative inverse in GF(2^8) followed by the affine map (§5.1.1)
inline const std::array<u8, 256> &sbox() {
  static const std::array<u8, 256> s = [] {
    std::array<u8, 256> t{};
    for (int x = 0; x < 256; x++) {
      u8 inv = 0;
      for (int y = 1; y < 256 && x; y++)
        if (gmul(u8(x), u8(y)) == 1) {
          inv = u8(y);
          break;
        }
      u8 b = inv, r = 0x63;
      for (int i = 0; i < 5; i++) {
        r ^= b;
        b = u8((b << 1) | (b >> 7));
      }
      t[size_t(x)] = r;
    }
    return t;
  }();
  return s;
}

struct Aes128 {
  u8 rk[176];
  explicit Aes128(const u8 key[16]) {  // KeyExpansion §5.2
    const auto &S = sbox();
    std::memcpy(rk, key, 16);
    u8 rcon = 1;
    for (int i = 4; i < 44; i++) {
      u8 t[4];
      std::memcpy(t, rk + 4 * (i - 1), 4);
      if (i % 4 == 0) {
        const u8 t0 = t[0];
        t[0] = u8(S[t[1]] ^ rcon);
        t[1] = S[t[2]];
        t[2] = S[t[3]];
        t[3] = S[t0];
        rcon = xtime(rcon);
      }
      for (int j = 0; j < 4; j++) rk[4 * i + j] = u8(rk[4 * (i - 4) + j] ^ t[j]);
    }
  }
  void encrypt(const u8 in[16], u8 out[16]) const {  // Cipher §5.1
    const auto &S = sbox();
    u8 s[16];
    for (int i = 0; i < 16; i++) s[i] = u8(in[i] ^ rk[i]);
    for (int r = 1; r <= 10; r++) {
      u8 t[16];
      for (int i = 0; i < 16; i++) t[i] = S[s[i]];  // SubBytes
      for (int c = 0; c < 4; c++)                   // ShiftRows: row k rotates left by k
        for (int k = 0; k < 4; k++) s[4 * c + k] = t[4 * ((c + k) % 4) + k];
      if (r != 10)
        for (int c = 0; c < 4; c++) {  // MixColumns
          const u8 a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
          s[4 * c] = u8(gmul(a0, 2) ^ gmul(a1, 3) ^ a2 ^ a3);
          s[4 * c + 1] = u8(a0 ^ gmul(a1, 2) ^ gmul(a2, 3) ^ a3);
          s[4 * c + 2] = u8(a0 ^ a1 ^ gmul(a2, 2) ^ gmul(a3, 3));
          s[4 * c + 3] = u8(gmul(a0, 3) ^ a1 ^ a2 ^ gmul(a3, 2));
        }
      for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];  // AddRoundKey
    }
    std::memcpy(out, s, 16);
  }
};

// ---- SHA-1 (FIPS 180-4 §6.1) and HMAC (RFC 2104) ----------------------------
struct Sha1 {
  u32 h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  std::vector<u8> buf;
  u64 total = 0;
  static u32 rol(u32 x, int n) { return (x << n) | (x >> (32 - n)); }
  void block(const u8 *p) {
    u32 w[80];
    for (int t = 0; t < 16; t++) w[t] = u32(p[4 * t]) << 24 | u32(p[4 * t + 1]) << 16 | u32(p[4 * t + 2]) << 8 | p[4 * t + 3];
    for (int t = 16; t < 80; t++) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
      u32 f, k;
      if (t < 20) {
        f = (b & c) | (~b & d);
        k = 0x5A827999u;
      } else if (t < 40) {
        f = b ^ c ^ d;
        k = 0x6ED9EBA1u;
      } else if (t < 60) {
        f = (b & c) | (b & d) | (c & d);
        k = 0x8F1BBCDCu;
      } else {
        f = b ^ c ^ d;
        k = 0xCA62C1D6u;
      }
      const u32 tmp = rol(a, 5) + f + e + k + w[t];
      e = d;
      d = c;
      c = rol(b, 30);
      b = a;
      a = tmp;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
    h[4] += e;
  }
  void update(const u8 *p, size_t n) {
    total += n;
    buf.insert(buf.end(), p, p + n);
    size_t off = 0;
    for (; off + 64 <= buf.size(); off += 64) block(buf.data() + off);
    buf.erase(buf.begin(), buf.begin() + long(off));
  }
  std::array<u8, 20> final() {
    const u64 bits = total * 8;
    const u8 one = 0x80, zero = 0;
    update(&one, 1);
    while (buf.size() != 56) update(&zero, 1);
    u8 len[8];
    for (int i = 0; i < 8; i++) len[i] = u8(bits >> (56 - 8 * i));
    update(len, 8);
    std::array<u8, 20> d{};
    for (int i = 0; i < 5; i++)
      for (int j = 0; j < 4; j++) d[size_t(4 * i + j)] = u8(h[i] >> (24 - 8 * j));
    return d;
  }
};

inline std::array<u8, 20> hmac_sha1(const u8 *key, size_t klen, const u8 *msg, size_t n) {
  u8 k0[64] = {0};
  if (klen > 64) {
    Sha1 s;
    s.update(key, klen);
    auto d = s.final();
    std::memcpy(k0, d.data(), 20);
  } else {
    std::memcpy(k0, key, klen);
  }
  u8 ip[64], op[64];
  for (int i = 0; i < 64; i++) {
    ip[i] = u8(k0[i] ^ 0x36);
    op[i] = u8(k0[i] ^ 0x5c);
  }
  Sha1 in;
  in.update(ip, 64);
  in.update(msg, n);
  const auto id = in.final();
  Sha1 out;
  out.update(op, 64);
  out.update(id.data(), 20);
  return out.final();
}

// ---- pion/srtp v2.0.18 ------------------------------------------------------
// key_derivation.go aesCmKeyDerivation (indexOverKdr == 0): PRF input = master
// salt with the label XORed into byte 7, the last two bytes a block counter.
inline std::vector<u8> kdf(u8 label, const u8 mk[16], const u8 *ms, size_t outLen, size_t saltLen = 14) {
  Aes128 a(mk);
  std::vector<u8> out;
  u8 in[16] = {0};
  std::memcpy(in, ms, saltLen);
  in[7] ^= label;
  for (u16 i = 0; out.size() < outLen; i++) {
    in[14] = u8(i >> 8);
    in[15] = u8(i);
    u8 b[16];
    a.encrypt(in, b);
    out.insert(out.end(), b, b + 16);
  }
  out.resize(outLen);
  return out;
}

struct Session {  // newSrtpCipherAesCmHmacSha1 (labelSRTPEncryption 0, AuthenticationTag 1, Salt 2)
  u8 key[16];
  u8 salt[14];
  u8 auth[20];
  Session(const u8 mk[16], const u8 ms[14]) {
    auto k = kdf(0x00, mk, ms, 16), a = kdf(0x01, mk, ms, 20), s = kdf(0x02, mk, ms, 14);
    std::memcpy(key, k.data(), 16);
    std::memcpy(auth, a.data(), 20);
    std::memcpy(salt, s.data(), 14);
  }
};

// context.go srtpSSRCState: the sender's guess of the rollover counter
// (seqNumMedian 1 << 15, seqNumMax 1 << 16; the replay detector is receive-only)
struct SSRCState {
  u64 index = 0;
  bool rolloverHasProcessed = false;
  // nextRolloverCount: (roc, difference)
  void next(u16 sequenceNumber, u32 &roc, int32_t &difference) const {
    const int32_t seq = int32_t(sequenceNumber);
    const u32 localRoc = u32(index >> 16);
    const int32_t localSeq = int32_t(index & 0xFFFF);
    u32 guessRoc = localRoc;
    difference = 0;
    if (rolloverHasProcessed) {
      if (index > (1u << 15)) {
        if (localSeq < (1 << 15)) {
          if (seq - localSeq > (1 << 15)) {
            guessRoc = localRoc - 1;
            difference = seq - localSeq - (1 << 16);
          } else {
            difference = seq - localSeq;
          }
        } else {
          if (localSeq - (1 << 15) > seq) {
            guessRoc = localRoc + 1;
            difference = seq - localSeq + (1 << 16);
          } else {
            difference = seq - localSeq;
          }
        }
      } else {
        difference = seq - localSeq;  // localRoc is 0
      }
    }
    roc = guessRoc;
  }
  // updateRolloverCount
  void update(u16 sequenceNumber, int32_t difference) {
    if (!rolloverHasProcessed) {
      index |= sequenceNumber;
      rolloverHasProcessed = true;
      return;
    }
    if (difference > 0) index += u64(difference);
  }
};

// Context.EncryptRTP -> encryptRTP (srtp.go) -> srtpCipherAesCmHmacSha1.encryptRTP:
// header copied, payload XORed with the AES-CM keystream of
// generateCounter(SEQ, ROC, SSRC, salt) (incrementing the 128-bit counter per
// block), tag = HMAC-SHA1(k_a, header || ciphertext || ROC)[0:10] appended.
// `pkt` is the marshalled RTP packet (header incl. extensions, then payload).
inline std::vector<u8> protect(const Session &s, SSRCState &st, const std::vector<u8> &pkt) {
  const size_t cc = pkt[0] & 0x0f;
  size_t h = 12 + 4 * cc;
  if (pkt[0] & 0x10) h += 4 + 4 * ((size_t(pkt[h + 2]) << 8) | pkt[h + 3]);
  const u16 seq = u16((pkt[2] << 8) | pkt[3]);
  u32 roc;
  int32_t diff;
  st.next(seq, roc, diff);
  st.update(seq, diff);
  u8 ctr[16] = {0};
  std::memcpy(ctr, s.salt, 14);
  for (int i = 0; i < 4; i++) {
    ctr[4 + i] ^= pkt[8 + size_t(i)];   // SSRC
    ctr[8 + i] ^= u8(roc >> (24 - 8 * i));
  }
  ctr[12] ^= u8(seq >> 8);
  ctr[13] ^= u8(seq);
  Aes128 a(s.key);
  std::vector<u8> out(pkt.begin(), pkt.end());
  for (size_t off = h; off < pkt.size(); off += 16) {
    u8 ks[16];
    a.encrypt(ctr, ks);
    for (size_t j = 0; j < 16 && off + j < pkt.size(); j++) out[off + j] ^= ks[j];
    for (int i = 15; i >= 0; i--)  // incrementCTR
      if (++ctr[i] != 0) break;
  }
  std::vector<u8> m(out.begin(), out.end());
  for (int i = 0; i < 4; i++) m.push_back(u8(roc >> (24 - 8 * i)));
  const auto tag = hmac_sha1(s.auth, 20, m.data(), m.size());
  out.insert(out.end(), tag.begin(), tag.begin() + 10);
  return out;
}

// ---- AEAD_AES_128_GCM (RFC 7714; pion srtp_cipher_aead_aes_gcm.go) --------
// GCM per NIST SP 800-38D: GHASH over GF(2^128) with the bit-reflected
// convention (bit 0 = the most significant bit of byte 0), R = 11100001 || 0^120
inline void gf_mul(const u8 X[16], const u8 Y[16], u8 out[16]) {
  u8 Z[16] = {0}, V[16];
  std::memcpy(V, Y, 16);
  for (int i = 0; i < 128; i++) {
    if (X[i / 8] & (0x80 >> (i % 8)))
      for (int k = 0; k < 16; k++) Z[k] ^= V[k];
    const bool lsb = V[15] & 1;
    for (int k = 15; k > 0; k--) V[k] = u8((V[k] >> 1) | (V[k - 1] << 7));
    V[0] >>= 1;
    if (lsb) V[0] ^= 0xE1;
  }
  std::memcpy(out, Z, 16);
}
inline void ghash_update(const u8 H[16], u8 Y[16], const u8 *data, size_t n) {  // zero-padded 16-B blocks
  for (size_t off = 0; off < n; off += 16) {
    u8 b[16] = {0};
    std::memcpy(b, data + off, std::min<size_t>(16, n - off));
    for (int k = 0; k < 16; k++) Y[k] ^= b[k];
    gf_mul(Y, H, Y);
  }
}
// GCM-AE(K, IV (96 bits), P, A) -> C || T (128-bit tag)
inline std::vector<u8> gcm_seal(const u8 key[16], const u8 iv[12], const u8 *p, size_t np, const u8 *a, size_t na) {
  Aes128 c(key);
  u8 H[16] = {0}, J0[16];
  c.encrypt(H, H);
  std::memcpy(J0, iv, 12);
  J0[12] = J0[13] = J0[14] = 0;
  J0[15] = 1;
  std::vector<u8> out(np + 16);
  u8 ctr[16];
  std::memcpy(ctr, J0, 16);
  for (size_t off = 0; off < np; off += 16) {
    for (int i = 15; i >= 12; i--)  // inc32
      if (++ctr[i] != 0) break;
    u8 ks[16];
    c.encrypt(ctr, ks);
    for (size_t j = 0; j < 16 && off + j < np; j++) out[off + j] = p[off + j] ^ ks[j];
  }
  u8 Y[16] = {0};
  ghash_update(H, Y, a, na);
  ghash_update(H, Y, out.data(), np);
  u8 L[16];
  const u64 la = u64(na) * 8, lc = u64(np) * 8;
  for (int i = 0; i < 8; i++) {
    L[i] = u8(la >> (56 - 8 * i));
    L[8 + i] = u8(lc >> (56 - 8 * i));
  }
  ghash_update(H, Y, L, 16);
  u8 E[16];
  c.encrypt(J0, E);
  for (int k = 0; k < 16; k++) out[np + k] = E[k] ^ Y[k];
  return out;
}
// newSrtpCipherAeadAesGcm: session key and 12-byte session salt from the
// AES-CM PRF over the 12-byte master salt (labels 0 and 2)
struct SessionGcm {
  u8 key[16];
  u8 salt[12];
  SessionGcm(const u8 mk[16], const u8 ms[12]) {
    auto k = kdf(0x00, mk, ms, 16, 12), sl = kdf(0x02, mk, ms, 12, 12);
    std::memcpy(key, k.data(), 16);
    std::memcpy(salt, sl.data(), 12);
  }
};
// srtpCipherAeadAesGcm.encryptRTP: IV = (0^16 || SSRC || ROC || SEQ) XOR salt
// (RFC 7714 §8.1), AAD = the RTP header (extensions included), output =
// header || GCM ciphertext || 16-byte tag; the rollover guess as for AES-CM
inline std::vector<u8> protect_gcm(const SessionGcm &s, SSRCState &st, const std::vector<u8> &pkt) {
  const size_t cc = pkt[0] & 0x0f;
  size_t h = 12 + 4 * cc;
  if (pkt[0] & 0x10) h += 4 + 4 * ((size_t(pkt[h + 2]) << 8) | pkt[h + 3]);
  const u16 seq = u16((pkt[2] << 8) | pkt[3]);
  u32 roc;
  int32_t diff;
  st.next(seq, roc, diff);
  st.update(seq, diff);
  u8 iv[12] = {0};
  for (int i = 0; i < 4; i++) {
    iv[2 + i] = pkt[8 + size_t(i)];
    iv[6 + i] = u8(roc >> (24 - 8 * i));
  }
  iv[10] = u8(seq >> 8);
  iv[11] = u8(seq);
  for (int i = 0; i < 12; i++) iv[i] ^= s.salt[i];
  std::vector<u8> out(pkt.begin(), pkt.begin() + long(h));
  const auto ct = gcm_seal(s.key, iv, pkt.data() + h, pkt.size() - h, pkt.data(), h);
  out.insert(out.end(), ct.begin(), ct.end());
  return out;
}

// pion/rtp NewAbsSendTimeExtension(t).Marshal(): NTP time >> 14, low 24 bits
inline u32 abs_send_time(int64_t unixNs) {
  const u64 u = u64(unixNs);
  u64 sec = u / 1000000000ull + 0x83AA7E80ull;
  u64 frac = ((u % 1000000000ull) << 32) / 1000000000ull;
  const u64 ntp = (sec << 32) | frac;
  return u32((ntp >> 14) & 0xFFFFFF);
}

// Writes the abs-send-time element (id `ext`) of a marshalled header in place
// (pacer/base.go:86-97 sets it on the header before WriteRTP).
inline void set_abs_send_time(std::vector<u8> &pkt, u8 ext, u32 v) {
  if (!ext || !(pkt[0] & 0x10)) return;
  const size_t x = 12 + 4 * size_t(pkt[0] & 0x0f);
  const u16 prof = u16((pkt[x] << 8) | pkt[x + 1]);
  const size_t end = x + 4 + 4 * ((size_t(pkt[x + 2]) << 8) | pkt[x + 3]);
  size_t p = x + 4;
  while (p < end) {
    if (prof == 0xBEDE) {
      const u8 b = pkt[p];
      if (b == 0) {
        p++;
        continue;
      }
      const u8 id = u8(b >> 4);
      const size_t l = size_t(b & 0x0f) + 1;
      if (id == 15) return;
      if (id == ext && l == 3) {
        pkt[p + 1] = u8(v >> 16);
        pkt[p + 2] = u8(v >> 8);
        pkt[p + 3] = u8(v);
        return;
      }
      p += 1 + l;
    } else {  // two-byte profile 0x100x
      const u8 id = pkt[p];
      if (id == 0) {
        p++;
        continue;
      }
      const size_t l = pkt[p + 1];
      if (id == ext && l == 3) {
        pkt[p + 2] = u8(v >> 16);
        pkt[p + 3] = u8(v >> 8);
        pkt[p + 4] = u8(v);
        return;
      }
      p += 2 + l;
    }
  }
}
}  // namespace orc_srtp
