// red_kernels.hip — RED (RFC 2198) for Opus on the GPU:
//   k_red_encode  RedReceiver.ForwardRTP's encodeRedForPrimary
//                 (redreceiver.go:58-79, :124-207): primary -> RED with up to
//                 two redundant blocks from the track's history
//   k_red_decode  RedPrimaryReceiver.ForwardRTP / getSendPktsFromRed /
//                 extractPktsFromRed (redprimaryreceiver.go:60-88, :145-269):
//                 RED -> primary, plus the lost packets its blocks recover
// Both are serial per track (a two-packet history / an 8-packet receive
// bitmap), parallel over tracks: one thread per mapped track of the batch.
// Each input packet owns a reserved output slot (records and 16-B aligned
// wire bytes); the host packs them.
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace lkf {
namespace {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
constexpr int kRedCount = 2;   // maxRedCount redreceiver.go:31
constexpr u32 kMtu = 1500;     // mtuSize :32
constexpr u8 kOpusPT = 111;    // opusPT :37

__device__ void copy_bytes(u8 *d, const u8 *s, u32 n) {
  for (u32 i = 0; i < n; i++) d[i] = s[i];
}

__global__ void k_red_encode(RedLaunch a) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.ngroups) return;
  const u32 b = a.gBegin[g], e = a.gEnd[g];
  const u32 src = a.in[b].track;
  RedEncState &st = a.enc[src];
  for (u32 i = b; i < e; i++) {
    const lkf_pkt p = a.in[i];
    const u8 *raw = a.inArena + p.arena_off;
    const u8 *pay = raw + p.payload_off;
    const u16 sn = u16(p.ext_sn);
    const u32 ts = u32(p.ext_ts);
    // redundant blocks: the non-nil suffix of the history that is close enough
    int lastNil = -1;
    for (int k = kRedCount - 1; k >= 0; k--)
      if (!st.has[k]) {
        lastNil = k;
        break;
      }
    int sel[kRedCount], ns = 0;
    for (int k = lastNil + 1; k < kRedCount; k++) {
      if (sn == st.sn[k] || u16(sn - st.sn[k]) > u16(kRedCount) || u32(ts - st.ts[k]) >= (1u << 14)) continue;
      sel[ns++] = k;
    }
    u32 size = u32(p.payload_len) + 1;
    for (int k = 0; k < ns; k++) size += u32(st.len[sel[k]]) + 4;
    if (size > kMtu) ns = 0;
    // write the RED packet before the history rotates (its blocks are history entries)
    u8 *w = a.outArena + a.byteOff[i];
    copy_bytes(w, raw, p.payload_off);  // the source header (the ExtPacket's RTP header is reused)
    u8 *q = w + p.payload_off;
    u32 n = 0;
    for (int k = 0; k < ns; k++) {
      const int s = sel[k];
      u32 h = u32(0x80 | kOpusPT);
      h = (h << 14) | ((ts - st.ts[s]) & 0x3FFF);
      h = (h << 10) | (u32(st.len[s]) & 0x3FF);
      q[n++] = u8(h >> 24);
      q[n++] = u8(h >> 16);
      q[n++] = u8(h >> 8);
      q[n++] = u8(h);
    }
    q[n++] = kOpusPT;
    bool ok = true;
    for (int k = 0; k < ns; k++) {
      copy_bytes(q + n, st.pay[sel[k]], st.len[sel[k]]);
      n += st.len[sel[k]];
    }
    if (n + p.payload_len > kMtu) ok = false;  // copy() short of space: the packet is not forwarded
    else {
      copy_bytes(q + n, pay, p.payload_len);
      n += p.payload_len;
    }
    // insert the primary into the history (redreceiver.go:144-158)
    for (int k = kRedCount - 1; k >= 0; k--) {
      if (!st.has[k] || u16(sn - st.sn[k]) < (1u << 15)) {
        for (int j = 0; j < k; j++) {
          st.has[j] = st.has[j + 1];
          st.sn[j] = st.sn[j + 1];
          st.ts[j] = st.ts[j + 1];
          st.len[j] = st.len[j + 1];
          copy_bytes(st.pay[j], st.pay[j + 1], st.len[j + 1]);
        }
        st.has[k] = 1;
        st.sn[k] = sn;
        st.ts[k] = ts;
        const u32 keep = p.payload_len < kMtu ? p.payload_len : kMtu;
        st.len[k] = u16(keep);
        copy_bytes(st.pay[k], pay, keep);
        break;
      }
    }
    a.cnt[i] = ok ? 1 : 0;
    if (ok) {
      lkf_pkt o = p;
      o.track = a.map[src];
      o.arena_off = u32(a.byteOff[i]);
      o.payload_len = u16(n);
      a.out[a.recOff[i]] = o;
    }
  }
}

__global__ void k_red_decode(RedLaunch a) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= a.ngroups) return;
  const u32 b = a.gBegin[g], e = a.gEnd[g];
  const u32 src = a.in[b].track;
  RedDecState &st = a.dec[src];
  for (u32 i = b; i < e; i++) {
    const lkf_pkt p = a.in[i];
    const u8 *raw = a.inArena + p.arena_off;
    const u8 *pay = raw + p.payload_off;
    const u16 sn = u16(p.ext_sn);
    // getSendPktsFromRed :145-198
    bool need = false;
    if (!st.first) {
      st.lastSeq = sn;
      st.hist = 0;
      st.first = 1;
    } else {
      const u16 diff = u16(sn - st.lastSeq);
      if (diff == 0) {
      } else if (diff > 0x8000) {
        if (u16(65535 - diff) < 8) {
          st.hist |= u8(1u << (65535 - diff));
          need = true;
        }
      } else if (diff > 8) {
        st.lastSeq = sn;
        st.hist = 0;
        need = true;
      } else {
        st.lastSeq = sn;
        st.hist = u8((u32(st.hist) << diff) | (1u << (diff - 1)));
        need = true;
      }
    }
    u32 rb = 0;
    if (need) {
      u16 bit = u16(st.lastSeq - sn);
      for (int k = 0; k < kRedCount; k++) {
        if (bit > 7) break;
        if ((st.hist & u8(1u << bit)) == 0) rb |= 1u << k;
        bit++;
      }
    }
    // extractPktsFromRed :200-269 (block headers, then the blocks in order)
    u32 nb = 0, blockLen = 0, pos = 0, len[17], tso[17];
    u8 pt[17];
    bool ok = true;
    const u32 L = p.payload_len;
    for (;;) {
      if (L - pos < 1) {
        ok = false;
        break;
      }
      if ((pay[pos] & 0x80) == 0) {
        pt[nb] = pay[pos] & 0x7F;
        len[nb] = 0;
        tso[nb] = 0;
        nb++;
        pos++;
        break;
      }
      if (L - pos < 4 || nb >= 16) {  // (more than 16 redundant blocks: beyond this engine)
        ok = false;
        break;
      }
      u32 h = (u32(pay[pos]) << 24) | (u32(pay[pos + 1]) << 16) | (u32(pay[pos + 2]) << 8) | u32(pay[pos + 3]);
      len[nb] = h & 0x03FF;
      h >>= 10;
      tso[nb] = h & 0x3FFF;
      h >>= 14;
      pt[nb] = u8(h & 0x7F);
      blockLen += len[nb];
      nb++;
      pos += 4;
    }
    if (ok && L - pos < blockLen) ok = false;
    u32 k = 0;
    if (ok) {
      const u32 slot = (u32(p.payload_off) + L + 15) & ~15u;
      for (u32 j = 0; j < nb; j++) {
        const bool primary = j == nb - 1;
        const u32 recoverIndex = nb - j - 1;
        if (!primary && (recoverIndex < 1 || (rb & (1u << (recoverIndex - 1))) == 0)) {
          pos += len[j];
          continue;
        }
        const u32 bl = primary ? L - pos : len[j];
        u8 *w = a.outArena + a.byteOff[i] + u64(k) * slot;
        copy_bytes(w, raw, p.payload_off);
        copy_bytes(w + p.payload_off, pay + pos, bl);
        lkf_pkt o = p;
        o.track = a.map[src];
        o.arena_off = u32(a.byteOff[i] + u64(k) * slot);
        o.payload_len = u16(bl);
        if (!primary) {  // the recovered packet (the primary keeps the RED header as the reference does)
          o.ext_sn = p.ext_sn - recoverIndex;
          o.ext_ts = p.ext_ts - tso[j];
          o.hdr1 = u8((p.hdr1 & 0x80) | pt[j]);
        }
        a.out[a.recOff[i] + k] = o;
        k++;
        pos += bl;
        if (primary) break;
      }
    }
    a.cnt[i] = k;
  }
}
}  // namespace

hipError_t launch_red(hipStream_t s, bool decode, const RedLaunch &a) {
  if (!a.ngroups) return hipSuccess;
  if (decode)
    hipLaunchKernelGGL(k_red_decode, dim3((a.ngroups + 63) / 64), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_red_encode, dim3((a.ngroups + 63) / 64), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace lkf
