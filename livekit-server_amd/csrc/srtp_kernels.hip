// =============================================================================
// srtp_kernels.hip — SRTP protect of forwarded packets on gfx950
// (the step after the pacer, pacer/base.go:59-100).
//
// pion/srtp/v2 v2.0.18 (go.mod:87) protects each packet with the subscriber
// transport's context, profile SRTP_AES128_CM_HMAC_SHA1_80 (RFC 3711):
//   keystream  AES-128 in counter mode, IV = salt ^ SSRC<<64 ^ (ROC<<16|SEQ)<<16
//   tag        HMAC-SHA1(k_a, header || ciphertext || ROC), first 10 bytes
//   ROC        the sender's rollover guess per SSRC (srtpSSRCState)
//
//   k_aes_tables   S-box and T-table (computed, FIPS-197 §5.1.1), once
//   k_srtp_keys    one lane per transport: AES-CM key derivation (RFC 3711
//                  §4.3.1: session key, salt, auth key), session key
//                  schedule, HMAC ipad/opad midstates (two SHA-1 blocks saved
//                  per packet)
//   k_srtp_roc     one lane per DownTrack: a bound DownTrack's first protected
//                  packet fixes its rollover base (pion starts the SSRC's
//                  index at that packet's SEQ with ROC 0, so ROC = (munged
//                  ext SN >> 16) - (first ext SN >> 16) while the munged
//                  sequence moves by less than 2^15 between packets)
//   k_srtp_protect one lane per output record: header copy with the
//                  abs-send-time element stamped, payload XOR keystream
//                  (T-table AES, tables in LDS), then HMAC-SHA1 over the
//                  written packet + ROC and the 10-byte tag.  The work is
//                  VALU/LDS-bound (≈10 AES rounds per 16 B and 80 SHA-1 rounds
//                  per 64 B), not HBM-bound.
// =============================================================================
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace lkf {
namespace {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;

__device__ __forceinline__ u32 ror32(u32 x, u32 n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ u32 rol32(u32 x, u32 n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ u32 bswap(u32 x) { return __builtin_bswap32(x); }

__device__ __forceinline__ u8 xtime(u8 a) { return u8((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

// ---- AES-128, big-endian column words (T-table form of FIPS-197 §5.1) ------
// te[x] = (2·S[x], S[x], S[x], 3·S[x]); the other three tables are its byte
// rotations.  sb = the S-box.
struct AesTab {
  const u32 *te;
  const u8 *sb;
  __device__ __forceinline__ u32 T0(u32 x) const { return te[x]; }
  __device__ __forceinline__ u32 T1(u32 x) const { return ror32(te[x], 8); }
  __device__ __forceinline__ u32 T2(u32 x) const { return ror32(te[x], 16); }
  __device__ __forceinline__ u32 T3(u32 x) const { return ror32(te[x], 24); }
  __device__ __forceinline__ u32 S(u32 x) const { return sb[x]; }
};

__device__ __forceinline__ void aes_expand(const AesTab &t, const u32 key[4], u32 rk[44]) {
  for (int i = 0; i < 4; i++) rk[i] = key[i];
  u32 rcon = 0x01000000u;
#pragma unroll
  for (int i = 4; i < 44; i++) {
    u32 w = rk[i - 1];
    if (i % 4 == 0) {
      w = (t.S((w >> 16) & 255) << 24) | (t.S((w >> 8) & 255) << 16) | (t.S(w & 255) << 8) | t.S(w >> 24);
      w ^= rcon;
      rcon = u32(xtime(u8(rcon >> 24))) << 24;
    }
    rk[i] = rk[i - 4] ^ w;
  }
}

// round keys read where they are used (the transport's session in global
// memory, L1-resident: every lane of a wave mostly shares one) instead of 44
// registers per lane — the protect kernel's occupancy
struct RkG {
  const u32 *p;
  __device__ __forceinline__ u32 operator[](int i) const { return p[i]; }
};

template <class Tab, class RK>
__device__ __forceinline__ void aes_encrypt(const Tab &t, const RK &rk, u32 &s0, u32 &s1, u32 &s2, u32 &s3) {
  s0 ^= rk[0];
  s1 ^= rk[1];
  s2 ^= rk[2];
  s3 ^= rk[3];
#pragma unroll
  for (int r = 1; r < 10; r++) {
    const u32 t0 = t.T0(s0 >> 24) ^ t.T1((s1 >> 16) & 255) ^ t.T2((s2 >> 8) & 255) ^ t.T3(s3 & 255) ^ rk[4 * r];
    const u32 t1 = t.T0(s1 >> 24) ^ t.T1((s2 >> 16) & 255) ^ t.T2((s3 >> 8) & 255) ^ t.T3(s0 & 255) ^ rk[4 * r + 1];
    const u32 t2 = t.T0(s2 >> 24) ^ t.T1((s3 >> 16) & 255) ^ t.T2((s0 >> 8) & 255) ^ t.T3(s1 & 255) ^ rk[4 * r + 2];
    const u32 t3 = t.T0(s3 >> 24) ^ t.T1((s0 >> 16) & 255) ^ t.T2((s1 >> 8) & 255) ^ t.T3(s2 & 255) ^ rk[4 * r + 3];
    s0 = t0;
    s1 = t1;
    s2 = t2;
    s3 = t3;
  }
  const u32 o0 = (t.S(s0 >> 24) << 24) | (t.S((s1 >> 16) & 255) << 16) | (t.S((s2 >> 8) & 255) << 8) | t.S(s3 & 255);
  const u32 o1 = (t.S(s1 >> 24) << 24) | (t.S((s2 >> 16) & 255) << 16) | (t.S((s3 >> 8) & 255) << 8) | t.S(s0 & 255);
  const u32 o2 = (t.S(s2 >> 24) << 24) | (t.S((s3 >> 16) & 255) << 16) | (t.S((s0 >> 8) & 255) << 8) | t.S(s1 & 255);
  const u32 o3 = (t.S(s3 >> 24) << 24) | (t.S((s0 >> 16) & 255) << 16) | (t.S((s1 >> 8) & 255) << 8) | t.S(s2 & 255);
  s0 = o0 ^ rk[40];
  s1 = o1 ^ rk[41];
  s2 = o2 ^ rk[42];
  s3 = o3 ^ rk[43];
}

// ---- SHA-1 compression (FIPS 180-4 §6.1.2), message words big-endian --------
__device__ __forceinline__ void sha1_block(u32 h[5], u32 w[16]) {
  u32 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
  for (int t = 0; t < 80; t++) {
    if (t >= 16) w[t & 15] = rol32(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
    u32 f, k;
    if (t < 20) {
      f = d ^ (b & (c ^ d));
      k = 0x5A827999u;
    } else if (t < 40) {
      f = b ^ c ^ d;
      k = 0x6ED9EBA1u;
    } else if (t < 60) {
      f = (b & c) | (d & (b | c));
      k = 0x8F1BBCDCu;
    } else {
      f = b ^ c ^ d;
      k = 0xCA62C1D6u;
    }
    const u32 tmp = rol32(a, 5) + f + e + k + w[t & 15];
    e = d;
    d = c;
    c = rol32(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a;
  h[1] += b;
  h[2] += c;
  h[3] += d;
  h[4] += e;
}

// ---- tables ------------------------------------------------------------------
__device__ u8 gmul(u8 a, u8 b) {
  u8 p = 0;
  for (int i = 0; i < 8; i++) {
    if (b & 1) p ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return p;
}

__global__ void k_aes_tables(u32 *tab) {  // tab: te[256], then the S-box packed 4 per word
  const u32 x = threadIdx.x;
  u8 inv = 0;
  for (u32 y = 1; y < 256 && x; y++)
    if (gmul(u8(x), u8(y)) == 1) {
      inv = u8(y);
      break;
    }
  u8 b = inv, s = 0x63;
  for (int i = 0; i < 5; i++) {
    s ^= b;
    b = u8((b << 1) | (b >> 7));
  }
  const u8 m2 = xtime(s), m3 = u8(m2 ^ s);
  tab[x] = (u32(m2) << 24) | (u32(s) << 16) | (u32(s) << 8) | m3;
  reinterpret_cast<u8 *>(tab + 256)[x] = s;
}

// ---- per-transport session keys ---------------------------------------------
__device__ __forceinline__ u32 be32(const u8 *p) {
  return (u32(p[0]) << 24) | (u32(p[1]) << 16) | (u32(p[2]) << 8) | p[3];
}

__global__ void k_srtp_keys(const lkf_transport_params *__restrict__ in, u32 first, u32 n, const u32 *__restrict__ tab,
                            SrtpKeys *__restrict__ keys) {
  const u32 i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const lkf_transport_params &p = in[i];
  const AesTab t{tab, reinterpret_cast<const u8 *>(tab + 256)};
  u32 mk[4], mrk[44];
  for (int k = 0; k < 4; k++) mk[k] = be32(p.master_key + 4 * k);
  aes_expand(t, mk, mrk);
  // PRF input: master salt (14 B) with the label XORed into byte 7, then a
  // 16-bit block counter (pion key_derivation.go aesCmKeyDerivation)
  const bool gcm = p.profile == LKF_SRTP_AEAD_AES_128_GCM;  // 12-byte master salt
  u8 ms[16] = {0};
  for (int k = 0; k < (gcm ? 12 : 14); k++) ms[k] = p.master_salt[k];
  u32 prf[4];
  auto derive = [&](u32 label, u32 ctr, u32 out[4]) {
    for (int k = 0; k < 4; k++) prf[k] = be32(ms + 4 * k);
    prf[1] ^= label;  // byte 7
    prf[3] |= ctr;    // bytes 14-15
    out[0] = prf[0];
    out[1] = prf[1];
    out[2] = prf[2];
    out[3] = prf[3];
    aes_encrypt(t, mrk, out[0], out[1], out[2], out[3]);
  };
  u32 sk[4], a0[4], a1[4], sl[4];
  derive(0, 0, sk);
  derive(1, 0, a0);
  derive(1, 1, a1);
  derive(2, 0, sl);
  SrtpKeys &K = keys[first + i];
  u32 rk[44];
  aes_expand(t, sk, rk);
  for (int k = 0; k < 44; k++) K.rk[k] = rk[k];
  K.salt[0] = sl[0];
  K.salt[1] = sl[1];
  K.salt[2] = sl[2];
  K.salt[3] = sl[3] & 0xFFFF0000u;  // 14-byte salt
  K.profile = p.profile;
  if (gcm) {  // newSrtpCipherAeadAesGcm: 12-byte session salt, GHASH key H = E(K, 0^128)
    K.salt[3] = 0;
    u32 h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    aes_encrypt(t, rk, h0, h1, h2, h3);
    K.ih[0] = h0;
    K.ih[1] = h1;
    K.ih[2] = h2;
    K.ih[3] = h3;
    K.ih[4] = 0;
    return;
  }
  // HMAC-SHA1 with the 20-byte auth key: midstates after the ipad / opad blocks
  const u32 ak[5] = {a0[0], a0[1], a0[2], a0[3], a1[0]};
  u32 w[16], hi[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  u32 ho[5] = {hi[0], hi[1], hi[2], hi[3], hi[4]};
  for (int k = 0; k < 16; k++) w[k] = (k < 5 ? ak[k] : 0u) ^ 0x36363636u;
  sha1_block(hi, w);
  for (int k = 0; k < 16; k++) w[k] = (k < 5 ? ak[k] : 0u) ^ 0x5c5c5c5cu;
  sha1_block(ho, w);
  for (int k = 0; k < 5; k++) {
    K.ih[k] = hi[k];
    K.oh[k] = ho[k];
  }
}

// ---- rollover bases -----------------------------------------------------------
__global__ void k_srtp_roc(SrtpDT *__restrict__ sd, const u32 *__restrict__ perm, const u64 *__restrict__ recBase,
                           const u32 *__restrict__ fwdCnt, const lkf_out *__restrict__ out, u32 ndts) {
  const u32 p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ndts) return;
  const u32 d = perm[p];
  SrtpDT s = sd[d];
  if (s.tp1 == 0 || s.init || fwdCnt[d] == 0) return;
  s.rocBase = out[recBase[p]].ext_sn >> 16;
  s.init = 1;
  sd[d] = s;
}

// ---- protect ------------------------------------------------------------------
// One lane per record, one pass over the packet in 64-byte message blocks
// (aligned to the packet start, so the source loads and the protected stores
// are whole 16-B chunks): per block, four new AES-CM keystream blocks (the
// keystream window is offset from the message block by the header length, so
// a 5-block window carries one block to the next message block; the same four
// AES calls for every lane, whatever its header length), the ciphertext words,
// and one SHA-1 compression of the inner HMAC over them (the tail words append
// ROC, 0x80 and the length).  The T-table lives in LDS replicated 32 times,
// word-interleaved (entry x of copy c at 32x + c, c = lane % 32): every lane
// reads its own bank, so the random lookups of AES never conflict.
constexpr u32 SRTP_T = 256;

struct AesLds {
  const u32 *t;  // 32 interleaved copies of te
  u32 c;         // this lane's copy
  __device__ __forceinline__ u32 T0(u32 x) const { return t[(x << 5) | c]; }
  __device__ __forceinline__ u32 T1(u32 x) const { return ror32(T0(x), 8); }
  __device__ __forceinline__ u32 T2(u32 x) const { return ror32(T0(x), 16); }
  __device__ __forceinline__ u32 T3(u32 x) const { return ror32(T0(x), 24); }
  __device__ __forceinline__ u32 S(u32 x) const { return (T0(x) >> 16) & 255; }
};

// ---- AEAD_AES_128_GCM -----------------------------------------------------
// GHASH (NIST SP 800-38D §6.4; bit 0 = the most significant bit of byte 0, the
// block as big-endian words) with Shoup's 4-bit tables: M[n] = n * H for the 16
// nibbles (M[8] = H, M[4] = H*x, M[2] = H*x^2, M[1] = H*x^3, the rest XORs),
// Y * H one nibble at a time from the last byte, each step shifting Z right by
// 4 and folding the 4 bits shifted out back in through R = last4[rem] << 112.
// A wave's GCM lanes are grouped by transport: one 256-B table per wave in LDS
// (16 entries, one bank row: lanes reading different entries never conflict),
// rebuilt per distinct transport among the wave's records (records of a
// DownTrack are contiguous, so a wave sees one or two).
struct GcmDefer {  // a GCM record's GHASH inputs, carried from the CTR pass
  uint4 *dst;
  u32 len, hw, key;
  u32 ej[4];  // E(K, J0)
};

__device__ __forceinline__ void gf_mul_tab(u32 y[4], const uint4 *M, const u32 *L4) {
  u32 z0, z1, z2, z3;
  {
    const uint4 m = M[y[3] & 15];
    z0 = m.x, z1 = m.y, z2 = m.z, z3 = m.w;
  }
  auto step = [&](u32 nib) {
    const u32 rem = z3 & 15;
    z3 = (z3 >> 4) | (z2 << 28);
    z2 = (z2 >> 4) | (z1 << 28);
    z1 = (z1 >> 4) | (z0 << 28);
    z0 = (z0 >> 4) ^ (L4[rem] << 16);
    const uint4 m = M[nib];
    z0 ^= m.x, z1 ^= m.y, z2 ^= m.z, z3 ^= m.w;
  };
  step((y[3] >> 4) & 15);
#pragma unroll
  for (int i = 14; i >= 0; i--) {
    const u32 xb = (y[i >> 2] >> (24 - 8 * (i & 3))) & 255;
    step(xb & 15);
    step(xb >> 4);
  }
  y[0] = z0, y[1] = z1, y[2] = z2, y[3] = z3;
}

// GHASH(H, A = header, C) for the wave's deferred GCM records, then each tag
// E(K, J0) ^ S after its ciphertext.  Every lane of the wave calls it (the
// loop over transports is wave-uniform).
__device__ void gcm_ghash_wave(const SrtpKeys *keys, const GcmDefer &g, bool on, uint4 *M, const u32 *L4) {
  const u32 lane = threadIdx.x & 63;
  u64 pend = __ballot(on);
  while (pend) {
    const u32 key = __shfl(g.key, __ffsll((long long)pend) - 1);
    if (lane < 16) {  // this transport's table: lane n builds M[n]
      const SrtpKeys &K = keys[key];
      u32 b[4] = {K.ih[0], K.ih[1], K.ih[2], K.ih[3]};  // H = M[8]
      u32 m[4] = {0, 0, 0, 0};
#pragma unroll
      for (int bit = 3; bit >= 0; bit--) {
        if ((lane >> bit) & 1) m[0] ^= b[0], m[1] ^= b[1], m[2] ^= b[2], m[3] ^= b[3];
        const u32 r = 0xE1000000u & (0u - (b[3] & 1u));  // * x
        b[3] = (b[3] >> 1) | (b[2] << 31);
        b[2] = (b[2] >> 1) | (b[1] << 31);
        b[1] = (b[1] >> 1) | (b[0] << 31);
        b[0] = (b[0] >> 1) ^ r;
      }
      M[lane] = make_uint4(m[0], m[1], m[2], m[3]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool mine = on && g.key == key;
    if (mine) {
      const u32 *ow = reinterpret_cast<const u32 *>(g.dst);
      const u32 hw = g.hw, lc = g.len - 4 * g.hw;  // ciphertext bytes
      u32 y[4] = {0, 0, 0, 0};
      for (u32 blk = 0; 4 * blk < hw; blk++) {
#pragma unroll
        for (int j = 0; j < 4; j++) y[j] ^= (4 * blk + j < hw) ? bswap(ow[4 * blk + j]) : 0u;
        gf_mul_tab(y, M, L4);
      }
      for (u32 blk = 0; 16 * blk < lc; blk++) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int left = int(lc) - int(16 * blk + 4 * j);  // bytes of this word inside the ciphertext
          const u32 v = left > 0 ? bswap(ow[hw + 4 * blk + j]) : 0u;
          y[j] ^= left >= 4 ? v : left > 0 ? (v & (0xFFFFFFFFu << (8 * (4 - left)))) : 0u;
        }
        gf_mul_tab(y, M, L4);
      }
      y[1] ^= 32u * hw;  // len(A) || len(C) in bits
      y[3] ^= 8u * lc;
      gf_mul_tab(y, M, L4);
      u8 *tag = reinterpret_cast<u8 *>(g.dst) + g.len;
#pragma unroll
      for (int k = 0; k < 16; k++) tag[k] = u8((g.ej[k / 4] ^ y[k / 4]) >> (24 - 8 * (k & 3)));
    }
    pend &= ~__ballot(mine);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // table reads done before the next rebuild
    __builtin_amdgcn_wave_barrier();
  }
}

// AEAD_AES_128_GCM (RFC 7714 §8, pion srtpCipherAeadAesGcm.encryptRTP) of one
// record, CTR half: IV = (0^16 || SSRC || ROC || SEQ) XOR salt, counter blocks
// IV || 2, 3, ..; writes the header (abs-send-time stamped) and the ciphertext
// in whole 16-B chunks (one new keystream block per chunk: the window is offset
// from the chunk by the header length, a whole number of words), and E(K, J0)
// for the tag.  GHASH over the header and the ciphertext read back from the
// output follows in gcm_ghash_wave.
template <class Tab>
__device__ void protect_gcm(const Tab &tb, const SrtpKeys *K, const uint4 *src, uint4 *dst, u32 len, u32 hw,
                            u32 absPos, u32 absVal, u32 ssrc, u32 seq, u32 roc, GcmDefer &g) {
  const RkG rk{K->rk};
  const u32 iv0 = (ssrc >> 16) ^ K->salt[0], iv1 = ((ssrc << 16) | (roc >> 16)) ^ K->salt[1],
            iv2 = ((roc << 16) | seq) ^ K->salt[2];
  const u32 ch0 = (hw + 3) >> 2, sft = 4 * ch0 - hw;
  u32 win[8];
  auto ks = [&](int q, u32 *o) {
    u32 a0 = iv0, a1 = iv1, a2 = iv2, a3 = u32(2 + q);
    aes_encrypt(tb, rk, a0, a1, a2, a3);
    o[0] = a0, o[1] = a1, o[2] = a2, o[3] = a3;
  };
  ks(-int(ch0), win);
  ks(1 - int(ch0), win + 4);
  const u32 nch = (len + 15) / 16;
  for (u32 c = 0; c < nch; c++) {
    if (c) {
#pragma unroll
      for (int k = 0; k < 4; k++) win[k] = win[4 + k];
      ks(int(c) + 1 - int(ch0), win + 4);
    }
    uint4 ch = src[c];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      u32 &v = j == 0 ? ch.x : j == 1 ? ch.y : j == 2 ? ch.z : ch.w;
      const u32 w = 4 * c + u32(j);
      if (w < hw) {  // header word: abs-send-time stamped
        for (u32 k = 0; k < 3; k++) {
          const u32 pos = absPos + k;
          if (pos / 4 == w) {
            const u32 sh = 8 * (pos & 3);
            v = (v & ~(255u << sh)) | (((absVal >> (16 - 8 * k)) & 255) << sh);
          }
        }
      } else {
        const u32 kw = sft + u32(j);
        v ^= bswap(kw == 0 ? win[0] : kw == 1 ? win[1] : kw == 2 ? win[2] : kw == 3 ? win[3] : kw == 4 ? win[4]
                                                                                                 : kw == 5 ? win[5] : win[6]);
      }
    }
    dst[c] = ch;
  }
  u32 e0 = iv0, e1 = iv1, e2 = iv2, e3 = 1u;  // E(K, J0)
  aes_encrypt(tb, rk, e0, e1, e2, e3);
  g.dst = dst;
  g.len = len;
  g.hw = hw;
  g.ej[0] = e0, g.ej[1] = e1, g.ej[2] = e2, g.ej[3] = e3;
}

// One record; a GCM record's GHASH half is deferred to the wave pass (g, true).
__device__ bool protect_record(const SrtpProtectArgs &A, const AesLds &tb, u64 i, GcmDefer &g) {
  const lkf_out r = A.out[i];
  const u32 len = r.out_len;
  const uint4 *src = reinterpret_cast<const uint4 *>(A.arena + r.out_off);
  uint4 *dst = reinterpret_cast<uint4 *>(A.prot + r.out_off + 16 * i);
  const u8 *sb = A.arena + r.out_off;
  const DevDT dt = A.dts[r.dt];
  const uint4 c0v = src[0];
  const u32 w0 = c0v.x;
  const u32 cc = w0 & 15, hasX = w0 & 0x10;
  u32 h = 12 + 4 * cc;
  // abs-send-time element (pacer/base.go:86-97): 3 bytes at byte `absPos`
  u32 absPos = 0xffff0000u;
  if (hasX) {
    const u32 xw = reinterpret_cast<const u32 *>(sb)[h / 4];
    const u32 prof = ((xw & 255) << 8) | ((xw >> 8) & 255);
    const u32 end = h + 4 + 4 * ((((xw >> 16) & 255) << 8) | (xw >> 24));
    if (dt.extAbs) {
      u32 q = h + 4;
      while (q < end) {
        const u32 b = sb[q];
        if (b == 0) {  // padding
          q++;
          continue;
        }
        u32 id, l, data;
        if (prof == 0xBEDE) {
          id = b >> 4;
          l = (b & 15) + 1;
          data = q + 1;
          if (id == 15) break;
        } else {  // two-byte profile
          id = b;
          l = sb[q + 1];
          data = q + 2;
        }
        if (id == dt.extAbs && l == 3) {
          absPos = data;
          break;
        }
        q = data + l;
      }
    }
    h = end;
  }
  const u32 hw = h / 4;
  const SrtpDT s = A.sd[r.dt];
  const bool prot = s.tp1 != 0;
  u32 roc = 0, ctr0 = 0, ctr1 = 0, ctr2 = 0, ctr3 = 0;
  u32 hs[5] = {0, 0, 0, 0, 0};
  const SrtpKeys *K = prot ? A.keys + (s.tp1 - 1) : A.keys;
  if (prot && K->profile == LKF_SRTP_AEAD_AES_128_GCM) {
    protect_gcm(tb, K, src, dst, len, hw, absPos, A.absVal, bswap(c0v.z), bswap(w0) & 0xFFFF,
                u32((r.ext_sn >> 16) - s.rocBase), g);
    g.key = s.tp1 - 1;
    return true;
  }
  const RkG rk{K->rk};
  if (prot) {
    roc = u32((r.ext_sn >> 16) - s.rocBase);
    const u32 ssrc = bswap(c0v.z);
    const u32 seq = bswap(w0) & 0xFFFF;
    ctr0 = K->salt[0];
    ctr1 = K->salt[1] ^ ssrc;
    ctr2 = K->salt[2] ^ roc;
    ctr3 = K->salt[3] ^ (seq << 16);
    for (int k = 0; k < 5; k++) hs[k] = K->ih[k];
  }
  const u32 sft = (0u - hw) & 3;  // keystream window offset of message word 0
  int blk0 = -int((hw + 3) >> 2);   // AES block index of window slot 0
  u32 win[20];
#pragma unroll
  for (int k = 0; k < 4; k++) win[k] = 0;
  const u32 L = len + 4;
  const u64 bits = u64(64 + L) * 8;
  const u32 nb = prot ? (L + 9 + 63) / 64 : (len + 63) / 64;
  const u64 tail = (u64(roc) << 32) | 0x80000000ull;
  for (u32 b = 0; b < nb; b++) {
    uint4 ch[4];
#pragma unroll
    for (int c = 0; c < 4; c++) ch[c] = (64 * b + 16 * c < len) ? src[4 * b + c] : make_uint4(0, 0, 0, 0);
    if (prot) {
#pragma unroll
      for (int k = 1; k <= 4; k++) {
        u32 a0 = ctr0, a1 = ctr1, a2 = ctr2, a3 = ctr3 + u32(blk0 + k);
        aes_encrypt(tb, rk, a0, a1, a2, a3);
        win[4 * k] = a0;
        win[4 * k + 1] = a1;
        win[4 * k + 2] = a2;
        win[4 * k + 3] = a3;
      }
    }
#pragma unroll
    for (int j = 0; j < 16; j++) {  // ciphertext (little-endian words, in place)
      u32 &v = (j & 3) == 0 ? ch[j >> 2].x : (j & 3) == 1 ? ch[j >> 2].y : (j & 3) == 2 ? ch[j >> 2].z : ch[j >> 2].w;
      const u32 w = 16 * b + u32(j);
      if (w < hw) {  // header word: abs-send-time stamped
        for (u32 k = 0; k < 3; k++) {
          const u32 pos = absPos + k;
          if (pos / 4 == w) {
            const u32 sh = 8 * (pos & 3);
            v = (v & ~(255u << sh)) | (((A.absVal >> (16 - 8 * k)) & 255) << sh);
          }
        }
      } else if (prot) {
        const u32 ks = sft == 0 ? win[j] : sft == 1 ? win[j + 1] : sft == 2 ? win[j + 2] : win[j + 3];
        v ^= bswap(ks);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; c++)
      if (64 * b + 16 * c < len) dst[4 * b + c] = ch[c];
    if (prot) {
      // inner HMAC message words (in place): packet || ROC || 0x80 || 0... || length
#pragma unroll
      for (int j = 0; j < 16; j++) {
        u32 &v = (j & 3) == 0 ? ch[j >> 2].x : (j & 3) == 1 ? ch[j >> 2].y : (j & 3) == 2 ? ch[j >> 2].z : ch[j >> 2].w;
        const int dlt = int(len) - int(4 * (16 * b + u32(j)));
        if (dlt >= 4) {
          v = bswap(v);
        } else if (dlt > 0) {
          v = (bswap(v) & (0xFFFFFFFFu << (8 * (4 - dlt)))) | u32(tail >> (32 + 8 * dlt));
        } else {
          const int q = -dlt;
          v = q < 8 ? u32((tail << (8 * q)) >> 32) : 0u;
        }
      }
      if (b == nb - 1) {
        ch[3].z = u32(bits >> 32);
        ch[3].w = u32(bits);
      }
      u32 W[16] = {ch[0].x, ch[0].y, ch[0].z, ch[0].w, ch[1].x, ch[1].y, ch[1].z, ch[1].w,
                   ch[2].x, ch[2].y, ch[2].z, ch[2].w, ch[3].x, ch[3].y, ch[3].z, ch[3].w};
      sha1_block(hs, W);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) win[k] = win[16 + k];
    blk0 += 4;
  }
  if (!prot) return false;  // no transport: the packet goes out as is (abs-send-time stamped)
  // outer hash, then the 80-bit tag after the payload
  u32 ho[5] = {K->oh[0], K->oh[1], K->oh[2], K->oh[3], K->oh[4]};
  {
    u32 w[16] = {hs[0], hs[1], hs[2], hs[3], hs[4], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, (64 + 20) * 8};
    sha1_block(ho, w);
  }
  u8 *tag = reinterpret_cast<u8 *>(dst) + len;
#pragma unroll
  for (int k = 0; k < 10; k++) tag[k] = u8(ho[k / 4] >> (24 - 8 * (k & 3)));
  return false;
}

__global__ void __launch_bounds__(SRTP_T) k_srtp_protect(SrtpProtectArgs A) {
  __shared__ u32 sTe[256 * 32];
  __shared__ uint4 sGt[SRTP_T / 64][16];  // per-wave GHASH table
  __shared__ u32 sL4[16];
  const u32 tid = threadIdx.x;
  for (u32 k = tid; k < 256 * 32; k += SRTP_T) sTe[k] = A.tab[k >> 5];
  if (tid < 16)  // last4[r] = r (carry-less) * 0xE1 << 5
    sL4[tid] = ((tid & 1) ? 0x1C20u : 0u) ^ ((tid & 2) ? 0x3840u : 0u) ^ ((tid & 4) ? 0x7080u : 0u) ^
               ((tid & 8) ? 0xE100u : 0u);
  __syncthreads();
  const u64 n = A.totals[0];
  const u64 i = u64(blockIdx.x) * SRTP_T + tid;
  const AesLds tb{sTe, tid & 31};
  GcmDefer g{};
  const bool gcm = (i < n && i < A.cap) ? protect_record(A, tb, i, g) : false;
  gcm_ghash_wave(A.keys, g, gcm, sGt[tid >> 6], sL4);
}

}  // namespace

hipError_t launch_aes_tables(hipStream_t s, uint32_t *tab) {
  hipLaunchKernelGGL(k_aes_tables, dim3(1), dim3(256), 0, s, tab);
  return hipGetLastError();
}

hipError_t launch_srtp_keys(hipStream_t s, const lkf_transport_params *in, uint32_t first, uint32_t n,
                            const uint32_t *tab, SrtpKeys *keys) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_srtp_keys, dim3((n + 63) / 64), dim3(64), 0, s, in, first, n, tab, keys);
  return hipGetLastError();
}

hipError_t launch_srtp_protect(hipStream_t s, const SrtpProtectArgs &a, uint32_t ndts, const uint32_t *perm,
                               const uint64_t *recBase, const uint32_t *fwdCnt) {
  if (ndts) hipLaunchKernelGGL(k_srtp_roc, dim3((ndts + 255) / 256), dim3(256), 0, s, a.sd, perm, recBase, fwdCnt, a.out, ndts);
  const u64 g = (a.cap + SRTP_T - 1) / SRTP_T;
  if (g) hipLaunchKernelGGL(k_srtp_protect, dim3(u32(g)), dim3(SRTP_T), 0, s, a);
  return hipGetLastError();
}

}  // namespace lkf
