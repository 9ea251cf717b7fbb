// libunsod_amd/csrc/cksum_device.h -- the device-side building blocks of the
// library's kernels (cksum_kernels.hip; kept apart so that an experimental
// kernel can live in a translation unit of its own and compile in seconds):
// the fold arithmetic,
// the batch descriptor and its buffer resource, the IPv4 header parse, the
// per-datagram RX verify results and their stores.  Internal; not part of
// the C ABI.
#ifndef MI_CKSUM_DEVICE_H
#define MI_CKSUM_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_cksum.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

namespace {


constexpr int kBlock = 256;           // 4 waves
constexpr int kU = 4;                 // chunks per lane per pass (scalar path)
constexpr uint32_t kOOB = 0xFFFFF000u;  // offset the bounds check always rejects
constexpr uint64_t kMaxBytes = MI_BATCH_MAX_BYTES;  // == kOOB - 4096: offsets past it stay 32-bit
static_assert(kMaxBytes == 0xFFFFF000ull - 4096, "kOOB must lie beyond every valid byte");

// ---------------------------------------------------------------- device math
__device__ __forceinline__ uint32_t fold16(uint32_t x) {
  x = (x & 0xffffu) + (x >> 16);
  x = (x & 0xffffu) + (x >> 16);
  return x;
}
__device__ __forceinline__ uint32_t fold16_64(uint64_t s) {
  s = (s & 0xffffffffull) + (s >> 32);
  s = (s & 0xffffffffull) + (s >> 32);
  return fold16((uint32_t)s);
}
__device__ __forceinline__ uint32_t swap16(uint32_t x) {
  return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}
// A dword's two 16-bit lanes, added: the absolute-address lanes of in_cksumdata.
// v_dot2_u32_u16 with (1, 1): lo16 + hi16 + acc in one VALU op.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t halves_acc(uint32_t w, uint32_t acc) {
  const u16x2 one = {1, 1};
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), one, acc, false);
}
__device__ __forceinline__ uint32_t halves(uint32_t w) { return halves_acc(w, 0u); }
__device__ __forceinline__ uint32_t sum4(const u32x4 &v) {
  return halves_acc(v.w, halves_acc(v.z, halves_acc(v.y, halves(v.x))));
}
// Bytes [a, b) of dword w, 0 <= a, b <= 4 (64-bit shifts: a shift by 32 is legal).
__device__ __forceinline__ uint32_t keep(uint32_t w, int a, int b) {
  return w & (uint32_t)((~0ull << (8 * a)) & ~(~0ull << (8 * b)));
}
// Slow path for chunks that straddle a boundary: the bytes of chunk v (which
// starts `rel` bytes after the packet start) that lie in [r0, r1) of the packet.
__device__ __forceinline__ uint32_t range_sum(const u32x4 &v, int rel, int r0, int r1) {
  const int lo = r0 - rel, hi = r1 - rel;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    s += halves(keep(w[k], min(max(lo - 4 * k, 0), 4), min(max(hi - 4 * k, 0), 4)));
  return s;
}

// x of lane i + n within its 16-lane row (0 past the row end): DPP row_shl.
template <int N>
__device__ __forceinline__ uint32_t row_shl(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + N, 0xf, 0xf, false);
}

// Sum of the G lanes of this lane's group, valid in the group's LEADER lane
// (lane % G == 0) only.  DPP row shifts inside a 16-lane row (plain VALU ops,
// no LDS round trip), one cross-row step for G = 32 / 64.
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t x) {
  if constexpr (G >= 2) x += row_shl<1>(x);
  if constexpr (G >= 4) x += row_shl<2>(x);
  if constexpr (G >= 8) x += row_shl<4>(x);
  if constexpr (G >= 16) x += row_shl<8>(x);
  if constexpr (G == 32) x += __shfl_down(x, 16, 64);
  if constexpr (G == 64)
    x = __builtin_amdgcn_readlane(x, 0) + __builtin_amdgcn_readlane(x, 16) +
        __builtin_amdgcn_readlane(x, 32) + __builtin_amdgcn_readlane(x, 48);
  return x;
}

// x as held by lane k of this lane's group (k group-uniform).
template <int G>
__device__ __forceinline__ uint32_t group_lane(uint32_t x, uint32_t k) {
  if constexpr (G == 64) {
    return __builtin_amdgcn_readlane(x, __builtin_amdgcn_readfirstlane(k));
  } else {
    return __shfl(x, (int)((threadIdx.x & 63u & ~(unsigned)(G - 1)) + k), 64);
  }
}

// A DPP move computed by EVERY lane at this point.  A DPP result consumed only
// under a condition may otherwise be sunk into a branch, where the lanes it
// reads from are switched off and read back as 0.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_all(uint32_t x) {
  uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
  asm volatile("" : "+v"(y));
  return y;
}

// Inclusive prefix sum inside each G-lane group (DPP, no LDS).
template <int G>
__device__ __forceinline__ uint32_t group_scan(uint32_t x) {
  const uint32_t lg = threadIdx.x & (G - 1);
  if constexpr (G >= 2) { const uint32_t y = dpp_all<0x111>(x); x += lg >= 1 ? y : 0u; }  // row_shr:1
  if constexpr (G >= 4) { const uint32_t y = dpp_all<0x112>(x); x += lg >= 2 ? y : 0u; }  // row_shr:2
  if constexpr (G >= 8) { const uint32_t y = dpp_all<0x114>(x); x += lg >= 4 ? y : 0u; }  // row_shr:4
  if constexpr (G >= 16) { const uint32_t y = dpp_all<0x118>(x); x += (lg & 15u) >= 8 ? y : 0u; }  // row_shr:8
  if constexpr (G >= 32) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  if constexpr (G == 64) x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Inclusive prefix sum over the wave: row shifts inside 16-lane rows, then
// the row_bcast:15 / row_bcast:31 carries across rows.
__device__ __forceinline__ uint32_t wave_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

struct Desc {
  const uint8_t *base;
  uint32_t bytes;  // bounds-check size (rounded up to 16)
  uint32_t n;
  const uint64_t *offs;
  uint64_t stride, first_off;
  const uint32_t *lens;
  uint32_t fixed_len;
  uint32_t len_lo, len_hi;  // length class filter: only lo <= lens[i] < hi (lens != NULL)
  uint32_t flags;           // MI_BATCH_*
  uint32_t *cflags, *cdata; // RX offload outputs (m_pkthdr.csum_flags / csum_data), or NULL
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const Desc &d) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(d.base), 0, (int)d.bytes,
                                           0x00020000);
}

// ------------------------------------------------------------ bounded arrays
//
// Every array a kernel of this library reads or writes -- the packets (rsrc_of
// above), the descriptors (offsets, lengths, chain and TX tables, seeds), the
// outputs, the bad counter, the drop-in mailbox and result words, the
// multi-batch argument table -- is reached through a buffer resource that
// carries the array's extent.  The hardware range-checks every access against
// it: past the extent a load reads zeros and a store or atomic is dropped.  So
// no index -- one read from a descriptor, a stale one, a wrong one -- can
// address memory outside the arrays the caller handed over, and no kernel has
// a global_ / flat_ / scratch_ memory instruction or a scalar load through a
// user pointer (tools/isa_audit.py; tests/test_isa_audit.py reads the built
// code object on every build).  Extents: n elements for the per-datagram
// arrays (the host keeps n * 8 below 4 GiB, make_desc), what the host measured
// for the others (the chain / TX segment tables: the allocation holding them,
// alloc_extent).  A NULL array has extent 0.
//
// MI_DEBUG_BOUNDS=1 (`make debug`, lib/debug/libmicksum.so): every access
// through an Arr that falls outside its extent -- other than the kOOB
// sentinel the kernels use for "no access" -- is reported with a device printf
// naming the function and line, the offset, the extent and the lane.
#ifndef MI_DEBUG_BOUNDS
#define MI_DEBUG_BOUNDS 0
#endif
struct Arr {
  __amdgpu_buffer_rsrc_t r;
  uint32_t bytes;
};
__device__ __forceinline__ Arr arr_of(const void *p, uint64_t bytes) {
  const uint32_t b = !p ? 0u : bytes < kOOB ? (uint32_t)bytes : kOOB;
  return {__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)b, 0x00020000), b};
}
#if MI_DEBUG_BOUNDS
#define MI_AT , const char *fn_ = __builtin_FUNCTION(), int line_ = __builtin_LINE()
#define MI_AT_FWD , fn_, line_
__device__ __noinline__ void arr_oob(const char *fn, int line, uint32_t off, uint32_t size, uint32_t bytes) {
  printf("libmicksum: out-of-range access in %s:%d: offset %u + %u of an array of %u bytes (block %u thread %u)\n",
         fn, line, off, size, bytes, blockIdx.x, threadIdx.x);
}
#define ARR_CHECK(a, off, size) \
  do { if ((off) < kOOB && (uint64_t)(off) + (size) > (a).bytes) arr_oob(fn_, line_, (off), (size), (a).bytes); } while (0)
#else
#define MI_AT
#define MI_AT_FWD
#define ARR_CHECK(a, off, size) do { } while (0)
#endif
// Cache policies (gfx950 CPol bits): 0 default; kSys = sc0 | sc1, the
// system-scope coherent access a relaxed __hip_atomic at system scope compiles
// to (the host-shared mailbox and result words); bit 31 volatile (a poll the
// compiler must not hoist).
constexpr int kSys = 1 | 16, kVolatile = (int)(1u << 31);
// Byte offset of element i of SZ-byte elements, or kOOB when it does not fit
// 32 bits: a corrupt index (a descriptor's segment number of 2^29 and up)
// must read the out-of-range zero, not wrap to another, valid, entry.
template <uint32_t SZ>
__device__ __forceinline__ uint32_t elem_off(uint32_t i) {
  return i < kOOB / SZ ? SZ * i : kOOB;
}
template <int AUX = 0>
__device__ __forceinline__ uint32_t ld_u32(const Arr &a, uint32_t i MI_AT) {
  const uint32_t o = elem_off<4>(i);
  ARR_CHECK(a, o, 4u);
  return __builtin_amdgcn_raw_buffer_load_b32(a.r, o, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ uint64_t ld_u64(const Arr &a, uint32_t i MI_AT) {
  const uint32_t o = elem_off<8>(i);
  ARR_CHECK(a, o, 8u);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(a.r, o, 0, AUX);
  return (uint64_t)v.x | ((uint64_t)v.y << 32);
}
__device__ __forceinline__ uint32_t ld_u8(const Arr &a, uint32_t i MI_AT) {
  ARR_CHECK(a, i, 1u);
  return __builtin_amdgcn_raw_buffer_load_b8(a.r, i, 0, 0);
}
template <int AUX = 0>
__device__ __forceinline__ void st_u32(const Arr &a, uint32_t i, uint32_t v MI_AT) {
  const uint32_t o = elem_off<4>(i);
  ARR_CHECK(a, o, 4u);
  __builtin_amdgcn_raw_buffer_store_b32(v, a.r, o, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st_u64(const Arr &a, uint32_t i, uint64_t v MI_AT) {
  const uint32_t o = elem_off<8>(i);
  ARR_CHECK(a, o, 8u);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)v, (uint32_t)(v >> 32)}, a.r, o, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st_u16(const Arr &a, uint32_t i, uint32_t v MI_AT) {
  const uint32_t o = elem_off<2>(i);
  ARR_CHECK(a, o, 2u);
  __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, a.r, o, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void st_u8(const Arr &a, uint32_t i, uint32_t v MI_AT) {
  ARR_CHECK(a, i, 1u);
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, a.r, i, 0, AUX);
}
__device__ __forceinline__ void add_u32(const Arr &a, uint32_t i, uint32_t v MI_AT) {
  const uint32_t o = elem_off<4>(i);
  ARR_CHECK(a, o, 4u);
  (void)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32((int)v, a.r, (int)o, 0, 0);
}

// A wave-uniform struct of dwords at byte `off` of an array (the multi-batch
// argument table, a burst's arguments): vector loads, each dword made uniform
// (so the fields can build buffer resources without a waterfall loop).
template <typename T>
__device__ __forceinline__ T ld_uniform(const Arr &a, uint32_t off) {
  static_assert(sizeof(T) % 4 == 0, "dwords");
  uint32_t w[sizeof(T) / 4];
#pragma unroll
  for (uint32_t k = 0; k < sizeof(T) / 4; ++k)
    w[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)__builtin_amdgcn_raw_buffer_load_b32(a.r, off + 4u * k, 0, 0));
  T t;
  __builtin_memcpy(&t, w, sizeof t);
  return t;
}

// The batch's descriptor arrays: n offsets (u64, or u32 with MI_BATCH_OFFS32)
// and n lengths.  The flag is a kernel argument, so the branch is uniform.
__device__ __forceinline__ Arr offs_arr(const Desc &d) {
  return arr_of(d.offs, (uint64_t)d.n * ((d.flags & MI_BATCH_OFFS32) ? 4u : 8u));
}
__device__ __forceinline__ Arr lens_arr(const Desc &d) { return arr_of(d.lens, (uint64_t)d.n * 4u); }
// (AUX: the descriptor loads' cache policy -- kSys for descriptors the host
// rewrites under a resident kernel, svc_burst)
template <int AUX = 0>
__device__ __forceinline__ uint64_t desc_off(const Desc &d, uint32_t i) {
  if (!d.offs) return d.first_off + (uint64_t)i * d.stride;
  const Arr a = offs_arr(d);
  return (d.flags & MI_BATCH_OFFS32) ? (uint64_t)ld_u32<AUX>(a, i) : ld_u64<AUX>(a, i);
}
template <int AUX = 0>
__device__ __forceinline__ uint32_t pkt_off(const Desc &d, uint32_t i) {
  const uint64_t o = desc_off<AUX>(d, i);
  return o < kOOB ? (uint32_t)o : kOOB;
}
template <int AUX = 0>
__device__ __forceinline__ uint32_t pkt_len(const Desc &d, uint32_t i) {
  const uint32_t l = d.lens ? ld_u32<AUX>(lens_arr(d), i) : d.fixed_len;
  return l < 0x7fff0000u ? l : 0x7fff0000u;
}
// Packet bytes are read once: nontemporal loads (aux = 2, `nt`) measured +10 %
// over the default policy on a 2 GiB stream (tools/hbm_probe.hip, profiles/).
__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
}

// Issue the U loads of pass p for a packet whose envelope starts at byte c0
// and has nch chunks; chunks past the envelope get the out-of-range offset.
template <int G, int U, int AUX = 2>
__device__ __forceinline__ void issue_pass(__amdgpu_buffer_rsrc_t r, uint32_t c0, uint32_t nch,
                                           uint32_t p, int lane, u32x4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t ci = p * (G * U) + u * G + lane;
    v[u] = __builtin_amdgcn_raw_buffer_load_b128(r, ci < nch ? c0 + 16u * ci : kOOB, 0, AUX);
  }
}

// Header fields of an IPv4 datagram that starts h bytes into the envelope,
// read from the chunks lanes 0..2 of the group hold (pass 0, u = 0): six
// group-lane reads of the dwords that cover bytes h .. h+23.
struct IpHdr {
  uint32_t hl, iplen, proto, src, dst;
  uint32_t w[5];  // the 20 header bytes as little-endian dwords, stream-aligned
};
template <int G, int U>
__device__ __forceinline__ IpHdr parse_ipv4(const u32x4 (&v)[U], uint32_t h) {
  const uint32_t q = h >> 2, rb = h & 3u;
  uint32_t T[6];
  if constexpr (G == 1) {
    // lane-per-packet: chunks 0..2 are this lane's v[0..2]
    static_assert(U >= 3, "a lone lane needs the 35-byte header window in one pass");
    const uint32_t D[12] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y,
                            v[1].z, v[1].w, v[2].x, v[2].y, v[2].z, v[2].w};
#pragma unroll
    for (int j = 0; j < 6; ++j)
      T[j] = q == 0 ? D[j] : q == 1 ? D[j + 1] : q == 2 ? D[j + 2] : D[j + 3];
  } else {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const uint32_t idx = q + j, c = idx & 3u;
      const u32x4 &v0 = v[0];
      const uint32_t mine = c == 0 ? v0.x : c == 1 ? v0.y : c == 2 ? v0.z : v0.w;
      T[j] = group_lane<G>(mine, idx >> 2);
    }
  }
  IpHdr ih;
  // little-endian u32 at byte h + 4k = alignbyte({T[k+1], T[k]}, rb)
#pragma unroll
  for (int k = 0; k < 5; ++k) ih.w[k] = __builtin_amdgcn_alignbyte(T[k + 1], T[k], rb);
  ih.hl = (ih.w[0] & 0x0fu) << 2;
  ih.iplen = ((ih.w[0] >> 8) & 0xff00u) | (ih.w[0] >> 24);
  ih.proto = (ih.w[2] >> 8) & 0xffu;
  ih.src = ih.w[3];
  ih.dst = ih.w[4];
  return ih;
}

// Absolute-lane sum of stream-aligned dwords: even stream bytes go to the low
// lane unless the datagram starts at an odd address.
__device__ __forceinline__ uint32_t abs_halves(uint32_t w, bool odd) {
  const uint32_t e = halves(w & 0x00ff00ffu), o = halves((w >> 8) & 0x00ff00ffu);
  return odd ? (e << 8) + o : e + (o << 8);
}

// ------------------------------------------------------------------ kernels
//
// Chunk classes inside a pass: a chunk wholly inside the summed range is
// "pure" and costs one unmasked sum4; only chunks that straddle the envelope
// head, a header/L4 cut or the end take the masked slow path, under a branch
// that the wave skips (s_cbranch_execz) when none of its lanes has one --
// about two of every ~25 chunk slots for a 1500 B datagram.

// Generic spans: in_cksum_skip / in_cksum_pseudo_header / in_cksum_hdr.
struct SpanSeeds {
  const uint32_t *seeds, *src, *dst;
  const uint8_t *proto;
  const uint32_t *plens;
};
// Span i's output from its folded bytes S (stream lanes): the seeds (n-element
// arrays) added, folded, complemented, stored into out (n u16).
__device__ __forceinline__ void span_emit(const Desc &d, const SpanSeeds &s, uint32_t i, uint32_t len, uint64_t sum,
                                          uint16_t *out) {
  const uint64_t n4 = (uint64_t)d.n * 4u;
  if (s.seeds) sum += ld_u32(arr_of(s.seeds, n4), i);
  if (s.src) {
    const uint32_t pl = s.plens ? ld_u32(arr_of(s.plens, n4), i) : len;
    sum += (uint64_t)ld_u32(arr_of(s.src, n4), i) + ld_u32(arr_of(s.dst, n4), i) +
           (ld_u8(arr_of(s.proto, d.n), i) << 8) + swap16(pl & 0xffffu);
  }
  st_u16(arr_of(out, (uint64_t)d.n * 2u), i, ~fold16_64(sum) & 0xffffu);
}

template <int G, int U>
__global__ __launch_bounds__(kBlock) void k_span(Desc d, uint32_t abs_lanes, SpanSeeds s,
                                                 uint16_t *out) {
  const __amdgpu_buffer_rsrc_t r = rsrc_of(d);
  const int lane = threadIdx.x & (G - 1);
  const uint32_t stride = gridDim.x * (kBlock / G);
  for (uint32_t i = blockIdx.x * (kBlock / G) + threadIdx.x / G; i < d.n; i += stride) {
    const uint32_t off = pkt_off(d, i), len = pkt_len(d, i);
    const uint32_t c0 = off & ~15u, h = off & 15u;
    const uint32_t nch = len ? (h + len + 15u) >> 4 : 0u;
    const uint32_t npass = (nch + G * U - 1) / (G * U);
    uint32_t acc = 0;
    for (uint32_t p = 0; p < npass; ++p) {
      u32x4 v[U];
      issue_pass<G, U>(r, c0, nch, p, lane, v);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rel = (int)(16u * (p * (G * U) + u * G + lane)) - (int)h;
        const bool pure = rel >= 0 && rel + 16 <= (int)len;
        acc += pure ? sum4(v[u]) : 0u;
        if (!pure && rel < (int)len) acc += range_sum(v[u], rel, 0, (int)len);
      }
      acc = fold16(acc);
    }
    acc = group_sum<G>(acc);
    if (lane == 0) {
      uint64_t sum = fold16(acc);
      if (!abs_lanes && (((uintptr_t)d.base + off) & 1u)) sum = swap16((uint32_t)sum);
      span_emit(d, s, i, len, sum, out);
    }
  }
}

// One pass's chunks of an IPv4 datagram whose first byte sits h bytes into
// the group's first chunk: acc_t += bytes [0, lend), and for datagrams with IP
// options acc_h += header bytes [0, hend) (TX: acc_f += the ip_sum field).
template <int G, int U, bool TX>
__device__ __forceinline__ void fold_pass(const u32x4 (&v)[U], uint32_t p, int lane, uint32_t h,
                                          int lend, int hend, bool opts, uint32_t &acc_t,
                                          uint32_t &acc_h, uint32_t &acc_f) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int rel = (int)(16u * (p * (G * U) + u * G + lane)) - (int)h;
    const bool pure = rel >= 0 && rel + 16 <= lend;
    acc_t += pure ? sum4(v[u]) : 0u;
    if (!pure && rel < lend) acc_t += range_sum(v[u], rel, 0, lend);
    if (opts && rel < hend) {
      acc_h += range_sum(v[u], rel, 0, hend);
      if (TX) acc_f += range_sum(v[u], rel, 10, 12);
    }
  }
}

// Sums of one IPv4 datagram: header [0, hl) and L4 [hl, ip_len) (absolute
// lanes, unfolded group totals), plus the parsed header.  TX excludes the
// ip_sum field (bytes 10..11) from the header sum.
//
// The chunks fold ONE range, [0, ip_len): a datagram is at most 65535 bytes, so
// its unfolded 16-bit-lane total is < 2^31 and the L4 sum is that total minus
// the header sum, exactly (disjoint byte sets, no modular wrap, zero-ness kept).
// A 20-byte header -- the common case -- is summed from the five dwords the
// header parse already holds; only datagrams with IP options (hl > 20) fold
// their header from the chunks.
// COH: every load of the datagram's bytes system-coherent (kSys) instead of
// nontemporal -- bytes the host rewrites under a resident kernel (svc_burst),
// read with no acquire fence.
template <int G, int U, bool TX, bool COH = false>
__device__ __forceinline__ void ipv4_sums(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t flen,
                                          int lane, u32x4 (&v)[U], IpHdr &ih, bool &hdr_ok,
                                          bool &l4_ok, uint32_t &sum_h, uint32_t &sum_l,
                                          bool demux = false) {
  const uint32_t c0 = off & ~15u, h = off & 15u;
  const uint32_t nch = (h + flen + 15u) >> 4;
  const uint32_t npass = (nch + G * U - 1) / (G * U);
  ih = parse_ipv4<G, U>(v, h);
  const bool odd = h & 1u;  // base is 16-byte aligned
  hdr_ok = flen >= 20u && ih.hl >= 20u && ih.hl <= flen;
  const bool len_ok = hdr_ok && ih.iplen >= ih.hl && ih.iplen <= flen;
  // TX: the protocols whose senders sum their message (TCP / UDP; with
  // MI_BATCH_DEMUX also ICMP, IGMP, CARP)
  l4_ok = TX ? len_ok && (ih.proto == 6u || ih.proto == 17u ||
                          (demux && (ih.proto == 1u || ih.proto == 2u || ih.proto == 112u)))
             : len_ok;
  const int hend = hdr_ok && (!TX || len_ok) ? (int)ih.hl : 0;
  const int lend = l4_ok ? (int)ih.iplen : hend;
  const bool opts = hend > 20;  // group-uniform
  uint32_t acc_t = 0, acc_h = 0, acc_f = 0;
  for (uint32_t p = 0;;) {
    fold_pass<G, U, TX>(v, p, lane, h, lend, hend, opts, acc_t, acc_h, acc_f);
    if (++p >= npass) break;
    issue_pass<G, U, COH ? kSys : 2>(r, c0, nch, p, lane, v);
  }
  const uint32_t total = group_sum<G>(acc_t);
  uint32_t hdr, field;
  if (opts) {
    hdr = group_sum<G>(acc_h);
    field = TX ? group_sum<G>(acc_f) : 0u;
  } else if (hend) {
    hdr = abs_halves(ih.w[0], odd) + abs_halves(ih.w[1], odd) + abs_halves(ih.w[2], odd) +
          abs_halves(ih.w[3], odd) + abs_halves(ih.w[4], odd);
    field = TX ? abs_halves(ih.w[2] & 0xffff0000u, odd) : 0u;
  } else {
    hdr = field = 0u;
  }
  sum_h = hdr - field;  // TX: ip_sum is zeroed before in_cksum (ip_output.c:670-672)
  sum_l = total - hdr;
}

// Grid-stride walk over the packets of a batch, one packet per lane group at a
// time, with the FIRST pass of the group's next packet issued before the
// current packet is folded: a group keeps two packets' loads in flight, which
// is what small datagrams (one pass each) need to cover HBM latency.
template <int G, int U, int AUX = 2>
__device__ __forceinline__ void issue_first(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t flen,
                                            int lane, u32x4 (&v)[U]) {
  issue_pass<G, U, AUX>(r, off & ~15u, flen ? ((off & 15u) + flen + 15u) >> 4 : 0u, 0, lane, v);
}

// AUX0: cache policy of each packet's FIRST pass (2 = nontemporal, as every
// other read; TX finalize may keep the header lines it writes back into)
template <int G, int U, typename Body, int AUX0 = 2>
__device__ __forceinline__ void for_each_packet(const Desc &d, __amdgpu_buffer_rsrc_t r, int lane,
                                                Body body) {
  if (d.lens && (d.len_lo != 0u || d.len_hi != ~0u)) {
    // Length-class launch: each wave scans windows of 64 packets with one
    // coalesced load of lens[], ballots the members of this launch's class,
    // compacts their indices through 64 words of LDS, and hands them to its
    // groups round-robin.  Rare classes cost one load per 64 packets.
    __shared__ uint32_t sel[kBlock];
    const uint32_t lane64 = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t gpw = 64u / G, gid = lane64 / G;  // groups per wave, group id in wave
    const uint32_t nwaves = gridDim.x * (kBlock / 64);
    for (uint32_t base = (blockIdx.x * (kBlock / 64) + wv) * 64u; base < d.n; base += nwaves * 64u) {
      const uint32_t k = base + lane64;
      const uint32_t l = k < d.n ? ld_u32(lens_arr(d), k) : 0u;
      const bool in = k < d.n && l >= d.len_lo && l < d.len_hi;
      const uint64_t m = __ballot(in);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (in) sel[wv * 64u + below] = k;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const uint32_t cnt = __popcll(m);
      for (uint32_t q = gid; q < cnt; q += gpw) {
        const uint32_t i = sel[wv * 64u + q];
        const uint32_t off = pkt_off(d, i), flen = pkt_len(d, i);
        u32x4 v[U];
        issue_first<G, U, AUX0>(r, off, flen, lane, v);
        body(i, off, flen, v);
      }
      __builtin_amdgcn_wave_barrier();  // sel[] is rewritten by the next window
    }
    return;
  }
  const uint32_t stride = gridDim.x * (kBlock / G);
  uint32_t i = blockIdx.x * (kBlock / G) + threadIdx.x / G;
  if (i >= d.n) return;
  if constexpr (U > 4) {
    // wide shapes already keep U loads per lane in flight; double-buffering
    // them costs occupancy and measured slower (16x6: 91 -> 111 VGPRs, 2-stream
    // 15.7 -> 16.5 us per 1500 B batch, profiles/db6_r02.jsonl; 8x12: 121 -> 172)
    for (; i < d.n; i += stride) {
      const uint32_t off = pkt_off(d, i), flen = pkt_len(d, i);
      u32x4 v[U];
      issue_first<G, U, AUX0>(r, off, flen, lane, v);
      body(i, off, flen, v);
    }
    return;
  }
  uint32_t off = pkt_off(d, i), flen = pkt_len(d, i);
  u32x4 v[U];
  issue_first<G, U, AUX0>(r, off, flen, lane, v);
  for (;;) {
    const uint32_t in = i + stride;
    const bool more = in < d.n;
    uint32_t offn = 0, flenn = 0;
    if (more) {
      offn = pkt_off(d, in);
      flenn = pkt_len(d, in);
    }
    u32x4 vn[U];
    issue_first<G, U, AUX0>(r, offn, flenn, lane, vn);
    body(i, off, flen, v);
    if (!more) break;
    i = in;
    off = offn;
    flen = flenn;
    for (int u = 0; u < U; ++u) v[u] = vn[u];
  }
}

// RX verify outputs of one datagram from its absolute-lane header / L4 sums
// (ip_input.c:459-471, tcp_input.c:697-720).
// RX offload: the m_pkthdr.csum_flags / csum_data a
// checksumming NIC hands the stack (if_loop.c:255-276 is the in-tree model),
// chosen so every consumer reaches the decision it would reach computing the
// sums itself:
//  * ip_input.c:459-460 takes sum = !(flags & CSUM_IP_VALID): IP_CHECKED for
//    every well-formed header, IP_VALID iff ip_sum folds to 0;
//  * tcp_input.c:698-709 / udp_usrreq.c:431-438 take th_sum = csum_data ^ 0xffff
//    under DATA_VALID|PSEUDO_HDR: csum_data = fold(pseudo + S(l4)) = l4 ^ 0xffff
//    reproduces in_cksum_pseudo_header's value bit for bit.  Set for TCP, and
//    for UDP when uh_ulen == ip_len - hl (otherwise udp_input sums uh_ulen
//    bytes, udp_usrreq.c:406-414); never for fragments (ip_reass sums csum_data of the
//    pieces, no pseudo header) or other protocols.
// Malformed headers get no flags: the stack's own length checks drop them.
template <bool COH = false>
__device__ __forceinline__ void rx_offload_flags(__amdgpu_buffer_rsrc_t r, uint32_t off, const IpHdr &ih,
                                                 bool hdr_ok, bool l4_ok, uint32_t ip, uint32_t l4, uint32_t &fl,
                                                 uint32_t &cd) {
  fl = 0;
  cd = 0;
  if (hdr_ok) {
    fl = MI_CSUM_IP_CHECKED | (ip ? 0u : MI_CSUM_IP_VALID);
    const uint32_t ip_off = ((ih.w[1] >> 8) & 0xff00u) | (ih.w[1] >> 24);
    const uint32_t plen = ih.iplen - ih.hl;
    bool l4v = l4_ok && (ip_off & 0x3fffu) == 0u;  // IP_MF | IP_OFFMASK
    if (l4v && ih.proto == 17u) {
      const uint32_t u = off + ih.hl + 4u;  // uh_ulen, big-endian
      const uint32_t ulen = plen >= 8u ? ((uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, u, 0, COH ? kSys : 0) << 8) |
                                             __builtin_amdgcn_raw_buffer_load_b8(r, u + 1u, 0, COH ? kSys : 0)
                                       : ~0u;
      l4v = ulen == plen;
    } else {
      l4v = l4v && ih.proto == 6u;
    }
    if (l4v) {
      fl |= MI_CSUM_DATA_VALID | MI_CSUM_PSEUDO_HDR;
      cd = l4 ^ 0xffffu;
    }
  }
}

// ---- small-header callers (MI_BATCH_DEMUX).  Rare
// per-datagram work done by one lane after the datagram's single pass: the
// bytes it re-reads were just streamed, so they come from L2.

// Absolute-lane sum of bytes [a, b) of the datagram at off.
template <bool COH = false>
__device__ __forceinline__ uint32_t dgram_range(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t a,
                                                uint32_t b) {
  uint32_t s = 0;
  for (uint32_t c = (off + a) & ~15u; c < off + b; c += 16u)
    s += range_sum(__builtin_amdgcn_raw_buffer_load_b128(r, c, 0, COH ? kSys : 0), (int)(c - off), (int)a, (int)b);
  return s;
}
template <bool COH = false>
__device__ __forceinline__ uint32_t ld_byte(__amdgpu_buffer_rsrc_t r, uint32_t o) {
  return __builtin_amdgcn_raw_buffer_load_b8(r, o, 0, COH ? kSys : 0);
}
template <bool COH = false>
__device__ __forceinline__ uint32_t ld_be16(__amdgpu_buffer_rsrc_t r, uint32_t o) {
  return (ld_byte<COH>(r, o) << 8) | ld_byte<COH>(r, o + 1u);
}
// Absolute-lane sum of the span [hl, hl + span) given S = sum of [hl, ip_len):
// whichever of the span or the rest is shorter is re-read (S is exact, < 2^31).
template <bool COH = false>
__device__ __forceinline__ uint32_t l4_span_sum(__amdgpu_buffer_rsrc_t r, uint32_t off, const IpHdr &ih,
                                                uint32_t span, uint32_t S) {
  const uint32_t plen = ih.iplen - ih.hl;
  if (span >= plen) return S;
  if (span <= plen - span) return dgram_range<COH>(r, off, ih.hl, ih.hl + span);
  return S - dgram_range<COH>(r, off, ih.hl + span, ih.iplen);
}

// RX: the L4 value the protocol input routine tests (mi_cksum.h, MI_BATCH_DEMUX).
template <bool COH = false>
__device__ __forceinline__ void demux_l4(__amdgpu_buffer_rsrc_t r, uint32_t off, const IpHdr &ih,
                                         bool odd, uint32_t sum_l, uint32_t &l4, uint32_t &st) {
  const uint32_t plen = ih.iplen - ih.hl;
  const uint32_t ip_off = ((ih.w[1] >> 8) & 0xff00u) | (ih.w[1] >> 24);
  uint32_t need = 0, span = plen;
  bool none = (ip_off & 0x3fffu) != 0u, pseudo = false;  // IP_MF | IP_OFFMASK: ip_reass first
  if (!none) {
    switch (ih.proto) {
      case 6u: need = 20u; pseudo = true; break;    // tcp_input.c:688-693
      case 17u: need = 8u; pseudo = true; break;    // udp_usrreq.c:375-381
      case 1u: need = 36u; break;                   // ip_icmp.c:374-378
      case 2u: need = 8u; break;                    // igmp.c:1448-1452
      case 112u: need = 36u; span = 36u; break;     // ip_carp.c:600-607, :641-643
      default: none = true;
    }
  }
  l4 = 0;
  if (none) {
    st |= MI_ST_L4_NONE;
    return;
  }
  if (plen < need) {
    st |= MI_ST_MALFORMED;
    return;
  }
  if (ih.proto == 17u) {
    const uint32_t ulen = ld_be16<COH>(r, off + ih.hl + 4u);  // udp_usrreq.c:406-414
    if (ulen != plen) {
      if (ulen > plen || ulen < 8u) {
        st |= MI_ST_MALFORMED;
        return;
      }
      span = ulen;  // m_adj to uh_ulen
    }
    if (ld_be16<COH>(r, off + ih.hl + 6u) == 0u) {  // uh_sum == 0: udps_nosum
      st |= MI_ST_L4_NONE;
      return;
    }
  }
  uint32_t sl = fold16(l4_span_sum<COH>(r, off, ih, span, sum_l));
  if (odd) sl = swap16(sl);
  if (pseudo) {
    const uint64_t seed = (uint64_t)ih.src + ih.dst + (ih.proto << 8) + swap16(span);
    l4 = ~fold16_64(seed + sl) & 0xffffu;
  } else {
    l4 = ~sl & 0xffffu;
  }
}

// One datagram's RX outputs, computed (verify_result) apart from their
// stores (verify_emit).  On gfx950 vmcnt counts stores with loads, so a store
// issued before the NEXT datagram's loads makes the wait for those loads wait
// for the store's acknowledgement too; the kernels therefore emit a
// datagram's outputs after the next datagram's loads are in flight.
// MI_DEFER=1 emits each datagram's outputs only after the next datagram's
// loads are issued.  Measured on MI355X (profiles/defer_ab_r02.jsonl, same box,
// interleaved): verify 1500 B 15.2 vs 14.6 us, Pareto 206 vs 203 us, finalize
// unchanged -- holding the outputs costs more than the store wait saves, so it
// is off.
#ifndef MI_DEFER
#define MI_DEFER 0
#endif
constexpr bool kDefer = MI_DEFER;
// MI_OUT_AUX: the cache policy of the ip / l4 / status buffer stores (gfx950
// CPol bits: 1 = sc0, 2 = nt, 16 = sc1; -1 or 0: default).  Measured
// (profiles/r03/serial_floor_r03.jsonl), 1500 B verify per launch on one stream
// / two queues: default 18.5 / 14.24, sc0 18.3-18.7, sc1 19.3-19.6 / 15.0,
// sc0+sc1 19.2-19.6 / 15.1, nt 20.2-20.7 / 18.5-18.7 (partial-line nt writes),
// plain global stores 18.3-18.9 -- the default policy stays.
#ifndef MI_OUT_AUX
#define MI_OUT_AUX -1
#endif
struct VOut {
  uint32_t i = ~0u;  // ~0u: nothing pending
  uint32_t ip = 0, l4 = 0, st = 0, fl = 0, cd = 0;
};
template <bool COH = false>
__device__ __forceinline__ VOut verify_result(uint32_t i, bool odd, const IpHdr &ih, bool hdr_ok, bool l4_ok,
                                              uint32_t sum_h, uint32_t sum_l, const Desc &d,
                                              __amdgpu_buffer_rsrc_t r, uint32_t off) {
  VOut o;
  o.i = i;
  uint32_t ip = 0, l4 = 0, st = 0;
  if (!hdr_ok) {
    st = MI_ST_MALFORMED;
  } else {
    uint32_t sh = fold16(sum_h);
    if (ih.hl != 20u && odd) sh = swap16(sh);  // in_cksum (stream) vs in_cksum_hdr (abs)
    ip = ~sh & 0xffffu;
    if (!l4_ok) {
      st = MI_ST_MALFORMED;
    } else if (d.flags & MI_BATCH_DEMUX) {
      demux_l4<COH>(r, off, ih, odd, sum_l, l4, st);
    } else {
      uint32_t sl = fold16(sum_l);
      if (odd) sl = swap16(sl);
      const uint32_t plen = ih.iplen - ih.hl;
      const uint64_t seed = (uint64_t)ih.src + ih.dst + (ih.proto << 8) + swap16(plen);
      l4 = ~fold16_64(seed + sl) & 0xffffu;
    }
    st |= (ip ? MI_ST_IP_BAD : 0u) | (l4 ? MI_ST_L4_BAD : 0u);
  }
  o.ip = ip;
  o.l4 = l4;
  o.st = st;
  if (d.cflags) rx_offload_flags<COH>(r, off, ih, hdr_ok, l4_ok, ip, l4, o.fl, o.cd);
  return o;
}

// The stores: each output through a resource over its n elements (bad: one
// counter), so a datagram index can only ever land inside its own array.
// (Plain global stores and buffer stores of the default policy measured the
// same, profiles/r03/serial_floor_r03.jsonl.)
// (COH: system-coherent stores -- write-through, so a wait for their acks
// orders them before a result word with no release fence, svc_burst)
template <bool COH = false>
__device__ __forceinline__ void verify_emit(const VOut &o, uint16_t *ip_out, uint16_t *l4_out, uint8_t *st_out,
                                            uint32_t *bad, const Desc &d) {
  if (o.i == ~0u) return;
  constexpr int kOA = COH ? kSys : MI_OUT_AUX >= 0 ? MI_OUT_AUX : 0;
  const uint64_t n = d.n;
  if (ip_out) st_u16<kOA>(arr_of(ip_out, 2u * n), o.i, o.ip);
  if (l4_out) st_u16<kOA>(arr_of(l4_out, 2u * n), o.i, o.l4);
  if (st_out) st_u8<kOA>(arr_of(st_out, n), o.i, o.st);
  if (bad && (o.st & ~MI_ST_L4_NONE)) add_u32(arr_of(bad, 4u), 0u, 1u);
  if (d.cflags) {
    st_u32<COH ? kSys : 0>(arr_of(d.cflags, 4u * n), o.i, o.fl);
    if (d.cdata) st_u32<COH ? kSys : 0>(arr_of(d.cdata, 4u * n), o.i, o.cd);
  }
}

// RX verify with DEALT units (round 5, VERDICT r4 "do this" 5): one launch in
// flight -- the reference's single RX kthread on one queue -- ends with a
// second, partial generation of waves (a 2048-workgroup grid is 8192 waves for
// 5120 slots: a 10.5 us tail).  Here the grid is ONE resident
// generation.  A unit is one wave's 64 / G datagrams; wave w takes unit w,
// then deals itself further units from one of kDealCtrs counters (counter c
// serves the workgroups b with b % kDealCtrs == c, and deals slice c of the
// units past the first generation's), so every wave stays busy until the
// units run out and the launch ends within about one unit of its steady rate.
// Why this shape (tools/xcd_probe.hip, profiles/r05/xcd_probe_r05.jsonl):
// same-address atomics serialize at ~66 per us whatever their scope, so one
// counter per launch (or per XCD) would be the bottleneck and a first grab by
// every wave at once would queue for ~10 us; with the first unit static and 64
// counters each sees ~250 grabs per 1500 B launch, spread over it.  The next
// ticket is fetched while the current unit is folded.  A set of counters must
// not be shared by launches in flight together: the prepared submissions own
// one set per stream / queue, and a launch leaves its counters at 0 -- each
// counter is taken exactly units_c + waves_c times (every wave ends with one
// failing grab), and the wave that draws the last ticket resets it.
constexpr uint32_t kDealCtrs = 64;                 // counters per set, 64 bytes apart
constexpr uint32_t kDealSetBytes = kDealCtrs * 64u;
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};
// (hook: called after each unit -- tools/timeline.hip stamps the waves)
template <int G, int U, typename Hook = NoHook>
__device__ __forceinline__ void verify_dyn_body(const Desc &d, uint16_t *ip_out, uint16_t *l4_out, uint8_t *st_out,
                                                uint32_t *bad, uint32_t *deal, Hook hook = Hook()) {
  constexpr uint32_t gpw = 64u / G, wpb = kBlock / 64;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(d);
  const int lane = threadIdx.x & (G - 1);
  const uint32_t lane64 = threadIdx.x & 63u, gid = lane64 / G;
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * wpb;
  const uint32_t T = (d.n + gpw - 1) / gpw;  // units
  const uint32_t c = blockIdx.x % kDealCtrs;
  // counter c deals units nw + c, nw + c + kDealCtrs, ...: the counters
  // advance together, so the waves keep sweeping ONE window of the batch in
  // order (units dealt from kDealCtrs separate slices -- that many regions
  // read at once -- measured 1-2 us slower per launch)
  const uint32_t s0 = nw + c, sc = s0 < T ? (T - s0 + kDealCtrs - 1) / kDealCtrs : 0u;
  const uint32_t nb_c = gridDim.x / kDealCtrs + (c < gridDim.x % kDealCtrs ? 1u : 0u);
  const uint32_t last = sc + nb_c * wpb - 1u;  // the counter's last ticket this launch
  const Arr ctr = arr_of(deal, kDealSetBytes);
  auto grab = [&]() -> uint32_t {
    uint32_t t = 0;
    if (lane64 == 0) t = (uint32_t)__builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, ctr.r, (int)(64u * c), 0, 0);
    return t;
  };
  uint32_t u = blockIdx.x * wpb + wv;  // the static first unit
  uint32_t t = grab();                 // the next ticket, in flight
  for (;;) {
    const uint32_t i = u * gpw + gid;
    if (u < T && i < d.n) {
      const uint32_t off = pkt_off(d, i), flen = pkt_len(d, i);
      u32x4 v[U];
      issue_first<G, U>(r, off, flen, lane, v);
      IpHdr ih;
      bool hdr_ok, l4_ok;
      uint32_t sum_h, sum_l;
      ipv4_sums<G, U, false>(r, off, flen, lane, v, ih, hdr_ok, l4_ok, sum_h, sum_l);
      if (lane == 0)
        verify_emit(verify_result(i, ((uintptr_t)d.base + off) & 1u, ih, hdr_ok, l4_ok, sum_h, sum_l, d, r, off),
                    ip_out, l4_out, st_out, bad, d);
    }
    hook();
    const uint32_t tk = (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
    if (tk >= sc) {
      if (tk == last && lane64 == 0) st_u32(ctr, 16u * c, 0u);  // every other grab of this launch is done
      break;
    }
    u = s0 + tk * kDealCtrs;
    t = grab();
  }
}
// The kernel-argument table of a multi-batch launch (k_ipv4_verify_multi):
// up to kMaxMulti batches with their outputs.
constexpr int kMaxMulti = 16;
struct MultiEnt {
  Desc d;
  uint16_t *ip, *l4;
  uint8_t *st;
  uint32_t unit0;  // first unit of this batch
  uint32_t pad;
};
struct MultiArgs {
  uint32_t nb, units;
  uint32_t *bad;
  MultiEnt e[kMaxMulti];
};

}  // namespace

#endif  // MI_CKSUM_DEVICE_H
