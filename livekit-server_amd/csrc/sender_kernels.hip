// sender_kernels.hip — DownTrack.rtpStats on the GPU for the packets the host
// lists: buffer.RTPStatsSender.Update (rtpstats_sender.go:229-432) for the
// padding, blank frames and RTX DownTrack.sendingPacket accounts
// (downtrack.go:1930-1959), SURVEY.md §8(f) 2.
//
//   k_sender_updates  one thread per DownTrack, its packets in call order.
//
// The forwarded packets of a batch are accounted inside their DownTrack's
// decide wave (k_decide_dt, ss_fold in forward_kernels.hip), which has every
// input at hand; both use the scalar Update of sender_device.h.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "sender_device.h"

namespace lkf {
namespace {
using u8 = uint8_t;
using u16 = uint16_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;
using namespace ss;

__global__ void k_sender_updates(SenderListLaunch A) {
  const u32 g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= A.ngroups) return;
  const u32 b = A.gBegin[g], e = A.gBegin[g + 1];
  if (b >= e) return;
  const u32 d = A.list[b].dt;
  SenderStats S = A.ss[d];
  u32 *ring = A.ring + size_t(d) * kSnInfoSize;
  u32 *gap = A.gap + size_t(d) * kGapWords;
  for (u32 i = b; i < e; i++) {
    const SenderUpd &u = A.list[i];
    ss_update(S, ring, gap, u.t, u.esn, u.ets, u.marker != 0, u.hdr, u.pay, u.pad);
  }
  A.ss[d] = S;
}
}  // namespace

hipError_t launch_sender_updates(hipStream_t s, const SenderListLaunch &a) {
  if (!a.ngroups) return hipSuccess;
  hipLaunchKernelGGL(k_sender_updates, dim3((a.ngroups + 63) / 64), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace lkf
