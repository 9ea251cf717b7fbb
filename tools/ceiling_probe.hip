// tools/ceiling_probe.hip -- the read ceiling for the bench's exact pattern
// (VERDICT r1 item 2): what does a kernel that only READS the bytes the verify
// kernel reads get, submitted the way bench.py submits verify (back-to-back
// launches of one BASELINE-sized batch each, alternating over 2 streams, R
// rotating batches)?  Built as tools/libceiling.so and driven from
// tools/ceiling.py, which runs the real verify kernel on the same batches in
// the same process so the two numbers sit side by side.
//
//   mode 0  slot envelopes: chunk c of the flat envelope index space (nch
//           16-byte chunks per datagram, slot * stride + env_off), grid-stride,
//           U nontemporal buffer loads in flight per lane -- the verify
//           kernel's bytes without its arithmetic;
//   mode 1  one contiguous run of the same byte count per batch (no slot
//           gaps): the best case for the same traffic.
//
// ceil_copy (the TX copy's ceiling): chunk c of the flat
// slot space is read at src slot * sstride + soff + 16 k (soff may be
// misaligned: one unaligned 16-byte load, as k_tx_flat issues) and written at
// dst slot * dstride + doff + 16 k -- the same bytes as the fused TX copy
// without its gather arithmetic.
#include <hip/hip_runtime.h>

#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void rd_env(const uint8_t *p, uint32_t bytes, uint32_t nslots, uint32_t stride,
                                             uint32_t env_off, uint32_t nch, uint32_t *sink) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, (int)bytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t total = nslots * nch;
  uint32_t acc = 0;
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < total; c += nthr * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      const uint32_t slot = cc / nch, k = cc - slot * nch;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, cc < total ? slot * stride + env_off + 16u * k : 0xFFFFF000u,
                                                   0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads; practically never stores
}

// The same read plus in-place writes, to price TX finalize's stores alone:
// WMODE 1: the lane holding chunk 0 of a slot stores 4 bytes into it (the
// ip_sum / L4 sum patch of in_delayed_cksum + ip_sum); WMODE 2: the lanes
// holding chunks 0..3 store them back whole (one full 64 B block per slot);
// WMODE 3: 4 bytes per slot into a separate dense array (what verify writes).
// SAUX: the stores' cache policy (gfx950 CPol bits: 1 = sc0, 2 = nt, 16 = sc1).
template <int U, int WMODE, int SAUX = 0>
__global__ __launch_bounds__(256) void rdw_env(uint8_t *p, uint32_t bytes, uint32_t nslots, uint32_t stride,
                                              uint32_t env_off, uint32_t nch, uint32_t *side) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t total = nslots * nch;
  uint32_t acc = 0;  // every load is consumed (a load used only under a branch may be sunk into it)
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < total; c += nthr * U) {
    u32x4 v[U];
    uint32_t slot[U], k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      slot[u] = cc / nch;
      k[u] = cc - slot[u] * nch;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, cc < total ? slot[u] * stride + env_off + 16u * k[u] : 0xFFFFF000u,
                                                   0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      if (cc >= total) continue;
      const uint32_t a = slot[u] * stride + env_off + 16u * k[u];
      const uint32_t x = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
      acc += x;
      if (WMODE == 1 && k[u] == 0) __builtin_amdgcn_raw_buffer_store_b32(x | 1u, r, a + 8u, 0, SAUX);
      if (WMODE == 2 && k[u] < 4) __builtin_amdgcn_raw_buffer_store_b128(v[u], r, a, 0, SAUX);
      if (WMODE == 3 && k[u] == 0)
        __builtin_amdgcn_raw_buffer_store_b32(x, __builtin_amdgcn_make_buffer_rsrc(side, 0, (int)(nslots * 4u), 0x00020000),
                                              4u * slot[u], 0, SAUX);
    }
  }
  if (acc == 0x9E3779B9u) side[0] = acc;
}

// A write-only pass of the same in-place patches (no reads): 4 bytes at
// slot * stride + env_off + 8 per slot -- the second half of a finalize split
// into a read-only sum pass (sums to a side array) and a patch pass.
__global__ __launch_bounds__(256) void wr_patch(uint8_t *p, uint32_t bytes, uint32_t nslots, uint32_t stride,
                                               uint32_t env_off) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(p, 0, (int)bytes, 0x00020000);
  for (uint32_t s = blockIdx.x * 256u + threadIdx.x; s < nslots; s += gridDim.x * 256u)
    __builtin_amdgcn_raw_buffer_store_b32(s | 1u, r, s * stride + env_off + 8u, 0, 0);
}

template <int U>
__global__ __launch_bounds__(256) void rd_flat(const uint8_t *p, uint32_t bytes, uint32_t *sink) {
  auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), 0, (int)bytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t total = bytes / 16u;
  uint32_t acc = 0;
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < total; c += nthr * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, cc < total ? 16u * cc : 0xFFFFF000u, 0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int U, int SAUX>
__global__ __launch_bounds__(256) void cp_env(const uint8_t *src, uint32_t sbytes, uint8_t *dst, uint32_t dbytes,
                                             uint32_t nslots, uint32_t sstride, uint32_t soff, uint32_t dstride,
                                             uint32_t doff, uint32_t nch) {
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(src), 0, (int)sbytes, 0x00020000);
  auto rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)dbytes, 0x00020000);
  const uint32_t nthr = gridDim.x * 256u;
  const uint32_t total = nslots * nch;
  for (uint32_t c = blockIdx.x * 256u + threadIdx.x; c < total; c += nthr * U) {
    u32x4 v[U];
    uint32_t slot[U], k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      slot[u] = cc / nch;
      k[u] = cc - slot[u] * nch;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, cc < total ? slot[u] * sstride + soff + 16u * k[u] : 0xFFFFF000u,
                                                   0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t cc = c + (uint32_t)u * nthr;
      __builtin_amdgcn_raw_buffer_store_b128(v[u], rd, cc < total ? slot[u] * dstride + doff + 16u * k[u] : 0xFFFFF000u,
                                             0, SAUX);
    }
  }
}

extern "C" {

// steps copy launches over (srcs[k % nb], dsts[k % nb]) alternating over
// nstreams streams; returns the GPU span in us.
float ceil_copy(void *const *srcs, void *const *dsts, int nb, uint32_t sbytes, uint32_t dbytes, uint32_t nslots,
                uint32_t sstride, uint32_t soff, uint32_t dstride, uint32_t doff, uint32_t nch, int unroll, int grid,
                int steps, int nstreams, int saux) {
  if (nstreams < 1 || nstreams > 8 || nb < 1) return -2.f;
  hipStream_t s[8];
  hipEvent_t e0, e1[8];
  for (int q = 0; q < nstreams; ++q) {
    if (hipStreamCreateWithFlags(&s[q], hipStreamNonBlocking) != hipSuccess) return -3.f;
    if (hipEventCreate(&e1[q]) != hipSuccess) return -3.f;
  }
  if (hipEventCreate(&e0) != hipSuccess) return -3.f;
  hipEventRecord(e0, s[0]);
  for (int q = 1; q < nstreams; ++q) hipStreamWaitEvent(s[q], e0, 0);
  for (int k = 0; k < steps; ++k) {
    const uint8_t *a = (const uint8_t *)srcs[k % nb];
    uint8_t *b = (uint8_t *)dsts[k % nb];
    hipStream_t st = s[k % nstreams];
#define L(U, A) hipLaunchKernelGGL((cp_env<U, A>), dim3(grid), dim3(256), 0, st, a, sbytes, b, dbytes, nslots, sstride, soff, dstride, doff, nch);
#define LA(U) if (saux == 0) { L(U, 0) } else if (saux == 1) { L(U, 1) } else if (saux == 2) { L(U, 2) } else { L(U, 3) }
    if (unroll == 2) { LA(2) } else if (unroll == 4) { LA(4) } else { LA(8) }
#undef LA
#undef L
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
  return span * 1000.f;
}

// steps launches, launch k over bases[k % nb] on stream k % nstreams (created
// here, non-blocking); returns the GPU span of all launches in us (events),
// or a negative value on error.
float ceil_run(void *const *bases, int nb, uint32_t bytes, uint32_t nslots, uint32_t stride, uint32_t env_off,
               uint32_t nch, int mode, int unroll, int grid, int steps, int nstreams) {
  static uint32_t *sink = nullptr, *side = nullptr;
  if (!sink && hipMalloc(&sink, 256) != hipSuccess) return -1.f;
  if (!side && hipMalloc(&side, 64u << 20) != hipSuccess) return -1.f;  // >= 4 B per slot of any batch
  if (nslots > (16u << 20)) return -2.f;
  if (nstreams < 1 || nstreams > 8 || nb < 1) return -2.f;
  hipStream_t s[8];
  hipEvent_t e0, e1[8];
  for (int q = 0; q < nstreams; ++q) {
    if (hipStreamCreateWithFlags(&s[q], hipStreamNonBlocking) != hipSuccess) return -3.f;
    if (hipEventCreate(&e1[q]) != hipSuccess) return -3.f;
  }
  if (hipEventCreate(&e0) != hipSuccess) return -3.f;
  hipEventRecord(e0, s[0]);
  for (int q = 1; q < nstreams; ++q) hipStreamWaitEvent(s[q], e0, 0);
  const uint32_t flat = nslots * nch * 16u;
  for (int k = 0; k < steps; ++k) {
    uint8_t *p = (uint8_t *)bases[k % nb];
    hipStream_t st = s[k % nstreams];
#define L(U)                                                                                         \
  if (mode == 0)                                                                                     \
    hipLaunchKernelGGL((rd_env<U>), dim3(grid), dim3(256), 0, st, (const uint8_t *)p, bytes, nslots, stride, env_off, nch, sink); \
  else if (mode == 1)                                                                                \
    hipLaunchKernelGGL((rd_flat<U>), dim3(grid), dim3(256), 0, st, (const uint8_t *)p, flat, sink);                  \
  else if (mode == 2)                                                                                \
    hipLaunchKernelGGL((rdw_env<U, 1>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  else if (mode == 3)                                                                                \
    hipLaunchKernelGGL((rdw_env<U, 2>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  else if (mode == 4)                                                                                \
    hipLaunchKernelGGL((rdw_env<U, 3>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  else if (mode == 5)                                                                                \
    hipLaunchKernelGGL((rdw_env<U, 1, 2>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  else if (mode == 6)                                                                                \
    hipLaunchKernelGGL((rdw_env<U, 2, 2>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  else if (mode >= 8 && mode <= 12) {                                                                \
    const int aux = mode == 8 ? 2 : mode == 9 ? 1 : mode == 10 ? 16 : mode == 11 ? 17 : 3;          \
    if (aux == 2) hipLaunchKernelGGL((rdw_env<U, 3, 2>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
    else if (aux == 1) hipLaunchKernelGGL((rdw_env<U, 3, 1>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
    else if (aux == 16) hipLaunchKernelGGL((rdw_env<U, 3, 16>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
    else if (aux == 17) hipLaunchKernelGGL((rdw_env<U, 3, 17>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
    else hipLaunchKernelGGL((rdw_env<U, 3, 3>), dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off, nch, side); \
  } else                                                                                             \
    hipLaunchKernelGGL(wr_patch, dim3(grid), dim3(256), 0, st, (uint8_t *)p, bytes, nslots, stride, env_off);
    if (unroll == 2) { L(2) } else if (unroll == 4) { L(4) } else if (unroll == 8) { L(8) } else { L(16) }
#undef L
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
  return span * 1000.f;
}

}  // extern "C"
