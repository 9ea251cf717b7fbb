// tools/timeline.hip -- per-wave timelines of the RX verify kernels (VERDICT
// r3 "do this" 2: attribute the single-queue gap).  A DIAGNOSTIC build, in a
// translation unit of its own: the product kernels carry no stamps.
//
// The kernels are the product's verify bodies (cksum_device.h building blocks,
// the same code as verify_body / k_ipv4_verify_multi in cksum_kernels.hip)
// with three stamps per wave from the 100 MHz constant clock (s_memrealtime):
// when the wave starts, when its first datagram is folded (its first loads
// have returned), and when it ends; plus the wave's XCC id, hardware id word
// (CU / SIMD / SE) and the number of datagrams it folded.  Lane 0 writes them
// with a vector store into a buffer no other code reads.
//
//   tl_run(mode, ...)  mode 0: one k_ipv4_verify<G,U>-shaped launch per batch
//                      mode 1: one k_ipv4_verify_multi<8,2>-shaped launch over
//                              `per_launch` batches (one grid)
//   launches go round-robin over `nstreams` HIP streams, like the bench.
//
// Read the SHARES (ramp / steady / tail), not the run time: the stamps' waits
// make the build a little slower than the product.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../libunsod_amd/csrc/cksum_device.h"

namespace {

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ uint32_t hw_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(v));
  return v;
}
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xfu;
}
// one record per wave: t0, t1, t2 (u64 ticks), then xcc | pkts << 8, hw_id
constexpr uint32_t kRec = 8;  // u32 words per wave
__device__ __forceinline__ void put_rec(uint32_t *tl, uint32_t bytes, uint32_t w, uint64_t t0, uint64_t t1,
                                        uint64_t t2, uint32_t pkts) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(tl, 0, (int)bytes, 0x00020000);
  if ((threadIdx.x & 63u) == 0) {
    const uint32_t o = 4u * kRec * w;
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t0, r, o, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(t0 >> 32), r, o + 4u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t1, r, o + 8u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(t1 >> 32), r, o + 12u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)t2, r, o + 16u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(t2 >> 32), r, o + 20u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(xcc_id() | (pkts << 8), r, o + 24u, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(hw_id(), r, o + 28u, 0, 0);
  }
}

// verify_body (cksum_kernels.hip) with stamps
template <int G, int U>
__global__ __launch_bounds__(kBlock) void tl_verify(Desc d, uint16_t *ip_out, uint16_t *l4_out, uint8_t *st_out,
                                                    uint32_t *tl, uint32_t tl_bytes, uint32_t w0) {
  const uint64_t t0 = stamp();
  uint64_t t1 = 0;
  uint32_t pkts = 0;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(d);
  const int lane = threadIdx.x & (G - 1);
  for_each_packet<G, U>(d, r, lane, [&](uint32_t i, uint32_t off, uint32_t flen, u32x4 (&v)[U]) {
    IpHdr ih;
    bool hdr_ok, l4_ok;
    uint32_t sum_h, sum_l;
    ipv4_sums<G, U, false>(r, off, flen, lane, v, ih, hdr_ok, l4_ok, sum_h, sum_l);
    if (lane == 0)
      verify_emit(verify_result(i, ((uintptr_t)d.base + off) & 1u, ih, hdr_ok, l4_ok, sum_h, sum_l, d, r, off), ip_out,
                  l4_out, st_out, nullptr, d);
    if (!pkts) t1 = stamp();
    ++pkts;
  });
  if (!pkts) t1 = stamp();
  const uint64_t t2 = stamp();
  put_rec(tl, tl_bytes, w0 + blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), t0, t1, t2, pkts * (64u / G));
}

// k_ipv4_verify_multi (cksum_kernels.hip) with stamps (held to 5 waves per SIMD,
// not the product's 6: the stamps cost a register and 6 would spill one)
template <int G, int U>
__global__ __launch_bounds__(kBlock, 5) void tl_multi(MultiArgs a, uint32_t *tl, uint32_t tl_bytes, uint32_t w0) {
  const uint64_t t0 = stamp();
  uint64_t t1 = 0;
  uint32_t units = 0;
  constexpr uint32_t gpw = 64u / G;
  const int lane = threadIdx.x & (G - 1);
  const uint32_t gid = (threadIdx.x & 63u) / G;
  const uint32_t nwaves = gridDim.x * (kBlock / 64);
  uint32_t j = 0, u0 = a.e[0].unit0;
  uint32_t next = a.nb > 1 ? a.e[1].unit0 : 0xffffffffu;
  Desc d = a.e[0].d;
  uint16_t *ipo = a.e[0].ip, *l4o = a.e[0].l4;
  uint8_t *sto = a.e[0].st;
  for (uint32_t u = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); u < a.units; u += nwaves) {
    if (u >= next) {
      do {
        ++j;
      } while (j + 1 < a.nb && a.e[j + 1].unit0 <= u);
      d = a.e[j].d;
      u0 = a.e[j].unit0;
      next = j + 1 < a.nb ? a.e[j + 1].unit0 : 0xffffffffu;
      ipo = a.e[j].ip;
      l4o = a.e[j].l4;
      sto = a.e[j].st;
    }
    const __amdgpu_buffer_rsrc_t r = rsrc_of(d);
    const uint32_t i = (u - u0) * gpw + gid;
    if (i < d.n) {
      const uint32_t off = pkt_off(d, i), flen = pkt_len(d, i);
      u32x4 v[U];
      issue_first<G, U>(r, off, flen, lane, v);
      IpHdr ih;
      bool hdr_ok, l4_ok;
      uint32_t sum_h, sum_l;
      ipv4_sums<G, U, false>(r, off, flen, lane, v, ih, hdr_ok, l4_ok, sum_h, sum_l);
      if (lane == 0)
        verify_emit(verify_result(i, ((uintptr_t)d.base + off) & 1u, ih, hdr_ok, l4_ok, sum_h, sum_l, d, r, off), ipo,
                    l4o, sto, nullptr, d);
    }
    if (!units) t1 = stamp();
    ++units;
  }
  if (!units) t1 = stamp();
  const uint64_t t2 = stamp();
  put_rec(tl, tl_bytes, w0 + blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), t0, t1, t2, units * gpw);
}

// verify_dyn_body (dealt units, round 5) with stamps: the first stamp after
// the wave's first unit, the unit count in the record
template <int G, int U>
__global__ __launch_bounds__(kBlock) void tl_dyn(Desc d, uint16_t *ip_out, uint16_t *l4_out, uint8_t *st_out,
                                                 uint32_t *deal, uint32_t *tl, uint32_t tl_bytes, uint32_t w0) {
  const uint64_t t0 = stamp();
  uint64_t t1 = 0;
  uint32_t units = 0;
  verify_dyn_body<G, U>(d, ip_out, l4_out, st_out, nullptr, deal, [&]() {
    if (!units) t1 = stamp();
    ++units;
  });
  if (!units) t1 = stamp();
  const uint64_t t2 = stamp();
  put_rec(tl, tl_bytes, w0 + blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6), t0, t1, t2, units * (64u / G));
}

Desc desc_of(const mi_pkt_batch &b) {
  Desc d{};
  d.base = (const uint8_t *)b.base;
  d.bytes = (uint32_t)((b.bytes + 15u) & ~15ull);
  d.n = b.n;
  d.stride = b.stride;
  d.first_off = b.first_off;
  d.fixed_len = b.fixed_len;
  d.len_hi = ~0u;
  return d;
}

}  // namespace

extern "C" {

// Waves one launch of `mode` has (for sizing the record buffer).
uint32_t tl_waves(int mode, uint32_t n, int grid) {
  (void)n;
  return (uint32_t)grid * (kBlock / 64);
  (void)mode;
}

// `launches` launches; launch k covers batches starting at (k * per) % nb
// (per = 1 in mode 0) on stream k % nstreams; records of launch k start at
// wave k * waves.  Fixed-stride batches only.  Returns the GPU span in us
// (events), < 0 on error.
float tl_run(int mode, const mi_pkt_batch *b, int nb, uint16_t *const *ip, uint16_t *const *l4,
             uint8_t *const *st, int per, int launches, int nstreams, int grid, int shape_g, int shape_u,
             uint32_t *tl, uint32_t tl_bytes) {
  if (nstreams < 1 || nstreams > 4 || nb < 1 || per < 1 || per > kMaxMulti) return -2.f;
  hipStream_t s[4];
  hipEvent_t e0, e1[4];
  for (int q = 0; q < nstreams; ++q) {
    if (hipStreamCreateWithFlags(&s[q], hipStreamNonBlocking) != hipSuccess) return -3.f;
    if (hipEventCreate(&e1[q]) != hipSuccess) return -3.f;
  }
  if (hipEventCreate(&e0) != hipSuccess) return -3.f;
  const uint32_t waves = (uint32_t)grid * (kBlock / 64);
  uint32_t *deal = nullptr;  // mode 2: one counter set per stream, zeroed (each launch leaves it zeroed)
  if (mode == 2) {
    if (hipMalloc(&deal, (size_t)kDealSetBytes * nstreams) != hipSuccess) return -3.f;
    (void)hipMemset(deal, 0, (size_t)kDealSetBytes * nstreams);
    (void)hipDeviceSynchronize();
  }
  (void)hipEventRecord(e0, s[0]);
  for (int q = 1; q < nstreams; ++q) hipStreamWaitEvent(s[q], e0, 0);
  for (int k = 0; k < launches; ++k) {
    hipStream_t q = s[k % nstreams];
    const uint32_t w0 = (uint32_t)k * waves;
    if (mode == 2) {
      const int j = k % nb;
      hipLaunchKernelGGL((tl_dyn<16, 6>), dim3(grid), dim3(kBlock), 0, q, desc_of(b[j]), ip[j], l4[j], st[j],
                         deal + (k % nstreams) * (kDealSetBytes / 4u), tl, tl_bytes, w0);
    } else if (mode == 0) {
      const int j = k % nb;
      const Desc d = desc_of(b[j]);
      if (shape_g == 16 && shape_u == 6)
        hipLaunchKernelGGL((tl_verify<16, 6>), dim3(grid), dim3(kBlock), 0, q, d, ip[j], l4[j], st[j], tl, tl_bytes, w0);
      else if (shape_g == 8 && shape_u == 4)
        hipLaunchKernelGGL((tl_verify<8, 4>), dim3(grid), dim3(kBlock), 0, q, d, ip[j], l4[j], st[j], tl, tl_bytes, w0);
      else if (shape_g == 8 && shape_u == 2)
        hipLaunchKernelGGL((tl_verify<8, 2>), dim3(grid), dim3(kBlock), 0, q, d, ip[j], l4[j], st[j], tl, tl_bytes, w0);
      else
        return -5.f;
    } else {
      MultiArgs a{};
      uint32_t units = 0;
      constexpr uint32_t gpw = 64u / 8u;
      for (int m = 0; m < per; ++m) {
        const int j = (k * per + m) % nb;
        a.e[m].d = desc_of(b[j]);
        a.e[m].ip = ip[j];
        a.e[m].l4 = l4[j];
        a.e[m].st = st[j];
        a.e[m].unit0 = units;
        units += (b[j].n + gpw - 1) / gpw;
      }
      a.nb = (uint32_t)per;
      a.units = units;
      hipLaunchKernelGGL((tl_multi<8, 2>), dim3(grid), dim3(kBlock), 0, q, a, tl, tl_bytes, w0);
    }
  }
  for (int q = 0; q < nstreams; ++q) hipEventRecord(e1[q], s[q]);
  float span = 0.f;
  for (int q = 0; q < nstreams; ++q) {
    hipEventSynchronize(e1[q]);
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1[q]);
    if (t > span) span = t;
  }
  if (hipGetLastError() != hipSuccess) span = -4.f / 1000.f;
  for (int q = 0; q < nstreams; ++q) {
    hipEventDestroy(e1[q]);
    hipStreamDestroy(s[q]);
  }
  hipEventDestroy(e0);
  if (deal) (void)hipFree(deal);
  return span * 1000.f;
}

// Occupancy of the instrumented kernels (blocks per CU), for the grid choice.
int tl_occupancy(int mode) {
  int per_cu = 0;
  if (mode == 2)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)tl_dyn<16, 6>, kBlock, 0);
  else if (mode == 0)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)tl_verify<16, 6>, kBlock, 0);
  else
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)tl_multi<8, 2>, kBlock, 0);
  return per_cu;
}

}  // extern "C"
