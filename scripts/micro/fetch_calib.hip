// fetch_calib.hip — known-byte calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE
// for k_emit's access pattern (MI355X_MICROARCH.md, HBM section: "Other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern"), and the bandwidth a byte-shifted fan-out copy reaches.
//
// Kernels (each moves a known number of bytes, 1 GiB-class, beyond the 256 MiB
// Infinity Cache):
//   k_copy_aligned   out[i] = in[i], 16 B per lane, nt stores
//   k_copy_shifted   out chunk = bytes [3 + 16c, 19 + 16c) of in: two 16-B loads
//                    + v_alignbyte per 16-B store (k_emit's payload chunks)
//   k_fanout_shifted every input packet (1 KiB) copied byte-shifted into F
//                    consecutive output packets (k_emit's track-major reuse:
//                    F DownTracks read one payload, copies of one DownTrack
//                    adjacent)
//   k_fanout_pktmajor the same copies in packet-major output order (the F
//                    copies of a packet adjacent)
// Prints per kernel: algorithmic read/write bytes and the time (HIP events);
// run under `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` for the counters.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t r_ = (x);                                                               \
    if (r_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(r_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using u32 = uint32_t;
using u64 = uint64_t;

__device__ __forceinline__ void st_nt(uint4 *p, uint4 v) {
  __builtin_nontemporal_store(v.x, reinterpret_cast<u32 *>(p));
  __builtin_nontemporal_store(v.y, reinterpret_cast<u32 *>(p) + 1);
  __builtin_nontemporal_store(v.z, reinterpret_cast<u32 *>(p) + 2);
  __builtin_nontemporal_store(v.w, reinterpret_cast<u32 *>(p) + 3);
}
__device__ __forceinline__ uint4 shift3(uint4 a, uint4 b) {  // bytes [3, 19) of a:b
  uint4 v;
  v.x = __builtin_amdgcn_alignbyte(a.y, a.x, 3);
  v.y = __builtin_amdgcn_alignbyte(a.z, a.y, 3);
  v.z = __builtin_amdgcn_alignbyte(a.w, a.z, 3);
  v.w = __builtin_amdgcn_alignbyte(b.x, a.w, 3);
  return v;
}

__global__ void k_copy_aligned(const uint4 *__restrict__ in, uint4 *__restrict__ out, u64 n16) {
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += u64(gridDim.x) * blockDim.x)
    st_nt(out + i, in[i]);
}

__global__ void k_copy_shifted(const uint4 *__restrict__ in, uint4 *__restrict__ out, u64 n16) {
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += u64(gridDim.x) * blockDim.x)
    st_nt(out + i, shift3(in[i], in[i + 1]));
}

// pkt16 = 16-B chunks per packet, F copies per packet, npkt packets.
// track-major: output copy k of packet p at (k * npkt + p) within a block of
// `trackPkts` packets (all copies of one "DownTrack" adjacent).
__global__ void k_fanout_shifted(const uint4 *__restrict__ in, uint4 *__restrict__ out, u32 pkt16, u32 F, u64 npkt,
                                 u32 trackPkts) {
  const u64 total = npkt * F * pkt16;
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += u64(gridDim.x) * blockDim.x) {
    const u64 c = i % pkt16, rec = i / pkt16;  // output record (track-major)
    const u64 track = rec / (u64(trackPkts) * F), inTrack = rec % (u64(trackPkts) * F);
    const u64 k = inTrack / trackPkts, p = track * trackPkts + inTrack % trackPkts;
    (void)k;
    const uint4 *src = in + p * (pkt16 + 1) + c;
    st_nt(out + i, shift3(src[0], src[1]));
  }
}

__global__ void k_fanout_pktmajor(const uint4 *__restrict__ in, uint4 *__restrict__ out, u32 pkt16, u32 F, u64 npkt) {
  const u64 total = npkt * F * pkt16;
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += u64(gridDim.x) * blockDim.x) {
    const u64 c = i % pkt16, rec = i / pkt16;
    const u64 p = rec / F;
    const uint4 *src = in + p * (pkt16 + 1) + c;
    st_nt(out + i, shift3(src[0], src[1]));
  }
}

__global__ void k_write_nt(uint4 *__restrict__ out, u64 n16) {
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += u64(gridDim.x) * blockDim.x)
    st_nt(out + i, make_uint4(u32(i), 1, 2, 3));
}
__global__ void k_write_plain(uint4 *__restrict__ out, u64 n16) {
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += u64(gridDim.x) * blockDim.x)
    out[i] = make_uint4(u32(i), 1, 2, 3);
}
__global__ void k_read(const uint4 *__restrict__ in, u64 n16, u32 *sink) {
  u32 acc = 0;
  for (u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += u64(gridDim.x) * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// XCD-aware fan-out: block b runs on XCD b % 8; each XCD copies a contiguous
// eighth of the (track-major) output, its waves walking it in order, so a
// payload's F copies are read by one XCD close together in time
__global__ void k_fanout_xcd(const uint4 *__restrict__ in, uint4 *__restrict__ out, u32 pkt16, u32 F, u64 npkt,
                             u32 trackPkts, int nt) {
  const u64 total = npkt * F * pkt16;
  const u32 xcd = blockIdx.x % 8, slot = blockIdx.x / 8, perX = gridDim.x / 8;
  const u64 per = (total + 7) / 8, beg = u64(xcd) * per, end = min(total, beg + per);
  for (u64 i = beg + u64(slot) * blockDim.x + threadIdx.x; i < end; i += u64(perX) * blockDim.x) {
    const u64 c = i % pkt16, rec = i / pkt16;
    const u64 track = rec / (u64(trackPkts) * F), inTrack = rec % (u64(trackPkts) * F);
    const u64 p = track * trackPkts + inTrack % trackPkts;
    const uint4 *src = in + p * (pkt16 + 1) + c;
    const uint4 v = shift3(src[0], src[1]);
    if (nt)
      st_nt(out + i, v);
    else
      out[i] = v;
  }
}

int main(int argc, char **argv) {
  const u64 inBytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024ull) << 20;  // MiB
  const u32 F = 9, pkt16 = 64;                                                       // 1 KiB packets
  const u64 npkt = inBytes / ((pkt16 + 1) * 16) / 200 * 200;  // whole 200-packet tracks
  const u64 outBytes = npkt * F * pkt16 * 16;
  uint4 *in, *out;
  CK(hipMalloc(&in, inBytes + 64));
  CK(hipMalloc(&out, outBytes > inBytes ? outBytes : inBytes));
  CK(hipMemset(in, 1, inBytes + 64));
  CK(hipMemset(out, 0, outBytes > inBytes ? outBytes : inBytes));
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 grid(cus * 16), block(256);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char *name, u64 rd, u64 wr, auto launch) {
    launch();  // warm
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int reps = 5;
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-18s read %12llu B  write %12llu B  %8.3f ms  %7.1f GB/s (read+write)\n", name, (unsigned long long)rd,
           (unsigned long long)wr, ms, double(rd + wr) / (ms * 1e-3) / 1e9);
  };
  const u64 n16 = inBytes / 16;
  run("copy_aligned", inBytes, inBytes, [&] { hipLaunchKernelGGL(k_copy_aligned, grid, block, 0, 0, in, out, n16); });
  run("copy_shifted", inBytes, inBytes,
      [&] { hipLaunchKernelGGL(k_copy_shifted, grid, block, 0, 0, in, out, n16 - 1); });
  run("fanout_trackmajor", npkt * pkt16 * 16, outBytes,
      [&] { hipLaunchKernelGGL(k_fanout_shifted, grid, block, 0, 0, in, out, pkt16, F, npkt, 200u); });
  run("fanout_pktmajor", npkt * pkt16 * 16, outBytes,
      [&] { hipLaunchKernelGGL(k_fanout_pktmajor, grid, block, 0, 0, in, out, pkt16, F, npkt); });
  const u64 w16 = outBytes / 16;
  run("write_nt", 0, outBytes, [&] { hipLaunchKernelGGL(k_write_nt, grid, block, 0, 0, out, w16); });
  run("write_plain", 0, outBytes, [&] { hipLaunchKernelGGL(k_write_plain, grid, block, 0, 0, out, w16); });
  u32 *sink;
  CK(hipMalloc(&sink, 4));
  run("read", inBytes, 0, [&] { hipLaunchKernelGGL(k_read, grid, block, 0, 0, in, n16, sink); });
  run("fanout_xcd_nt", npkt * pkt16 * 16, outBytes,
      [&] { hipLaunchKernelGGL(k_fanout_xcd, grid, block, 0, 0, in, out, pkt16, F, npkt, 200u, 1); });
  run("fanout_xcd_plain", npkt * pkt16 * 16, outBytes,
      [&] { hipLaunchKernelGGL(k_fanout_xcd, grid, block, 0, 0, in, out, pkt16, F, npkt, 200u, 0); });
  CK(hipFree(sink));
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
