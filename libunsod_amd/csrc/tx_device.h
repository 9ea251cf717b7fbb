// libunsod_amd/csrc/tx_device.h -- the fused TX copy + checksum kernels
// (m_copydata + in_delayed_cksum + ip_sum in one pass),
// included by cksum_kernels.hip inside its anonymous namespace; kept in a
// header of its own so a tool translation unit can compile one TX kernel in
// seconds (tools/ab builds, register studies).  Internal; not part of the C
// ABI.  Needs cksum_device.h first.
#ifndef MI_TX_DEVICE_H
#define MI_TX_DEVICE_H

// ------------------------------------------- TX: fused copy + checksum offload
//
// SURVEY.md 8(f) rank 2.  With if_hwassist = CSUM_IP | CSUM_TCP | CSUM_UDP the
// stack leaves the sums to the device (ip_output.c:649-672) and the driver
// copies every outgoing frame out of its mbuf chain into an rte_mbuf
// (m_copydata(m, 0, len, rm_data), uinet_if_dpdk.c:594-597).  Here both are
// one pass: a lane group per frame gathers the chain into 16-byte chunks
// aligned to the DESTINATION slot (so stores are whole dwordx4 except at the
// frame's two ends), folds the IP header and the L4 range from those same
// registers, patches ip_sum and the L4 sum field (in_delayed_cksum,
// ip_output.c:958-983: UDP 0 -> 0xffff, stored only if it lies inside the IP
// mbuf's m_len) into the chunk registers, and stores.  Read L, write L.
//
// Gather: lane j of the group builds destination chunk ci = p*G*U + u*G + j.
// The segment table (m_data, m_len of each mbuf of the chain) sits one
// segment per lane; a group scan turns lengths into frame positions.  For each
// chunk the lane keeps the segment holding its first byte ("prim") and, when
// the chunk straddles a segment boundary, the next non-empty one ("sec"); a
// chunk touching three or more segments (tiny mbufs) takes a slow loop.  A
// piece of a segment is read as the two aligned source chunks around it and
// funnel-shifted (v_alignbyte) into destination alignment; bytes outside the
// piece are masked off.
struct TxDesc {
  const uint8_t *src;
  uint32_t src_bytes;
  uint32_t n;
  const uint64_t *seg_off;
  const int32_t *seg_len;
  const uint32_t *pkt_seg;
  const uint32_t *pkt_len;
  const uint32_t *cflags, *cdata;
  uint8_t *dst;
  uint32_t dst_bytes;
  uint32_t room, l3;
  uint64_t dst_stride, dst_first;
  uint8_t *status;
  uint32_t nseg;  // segments the seg_off / seg_len tables hold (host: their allocation)
};
// The TX batch's tables as bounded arrays (cksum_device.h, Arr).
struct TxArrs {
  Arr pkt_len, pkt_seg, seg_len, seg_off, cflags, cdata, status;
};
__device__ __forceinline__ TxArrs tx_arrs(const TxDesc &t) {
  const uint64_t n = t.n;
  return {arr_of(t.pkt_len, 4u * n),          arr_of(t.pkt_seg, 4u * (n + 1u)), arr_of(t.seg_len, 4ull * t.nseg),
          arr_of(t.seg_off, 8ull * t.nseg),   arr_of(t.cflags, 4u * n),        arr_of(t.cdata, 4u * n),
          arr_of(t.status, n)};
}

// The 16 bytes at source address a (any alignment): the aligned chunk at
// a & ~15 and (unless aligned) the next one, funnel-shifted.
struct Raw2 {
  u32x4 x, y;
};
__device__ __forceinline__ Raw2 ld_pair(__amdgpu_buffer_rsrc_t r, uint32_t a) {
  const uint32_t A = a & ~15u;
  return {ld16(r, A), ld16(r, (a & 15u) ? A + 16u : kOOB)};
}
__device__ __forceinline__ u32x4 shift2(const u32x4 &x, const u32x4 &y, uint32_t a) {
  // named registers and selects only: an array here gets a select-of-index
  // turned into a dynamic (scratch) access by the optimiser
  const uint32_t s = a & 15u, b = s & 3u;
  const bool h8 = s & 8u, h4 = s & 4u;
  const uint32_t t0 = h8 ? x.z : x.x, t1 = h8 ? x.w : x.y, t2 = h8 ? y.x : x.z;
  const uint32_t t3 = h8 ? y.y : x.w, t4 = h8 ? y.z : y.x, t5 = h8 ? y.w : y.y;
  const uint32_t z0 = h4 ? t1 : t0, z1 = h4 ? t2 : t1, z2 = h4 ? t3 : t2;
  const uint32_t z3 = h4 ? t4 : t3, z4 = h4 ? t5 : t4;
  return {__builtin_amdgcn_alignbyte(z1, z0, b), __builtin_amdgcn_alignbyte(z2, z1, b),
          __builtin_amdgcn_alignbyte(z3, z2, b), __builtin_amdgcn_alignbyte(z4, z3, b)};
}
__device__ __forceinline__ u32x4 shift_pair(const Raw2 &p, uint32_t a) { return shift2(p.x, p.y, a); }
// Bytes [a, b) of a dword as a mask, 0 <= a, b <= 4 (32-bit shifts only).
__device__ __forceinline__ uint32_t byte_mask(int a, int b) {
  const uint32_t lo = a >= 4 ? 0u : 0xffffffffu << (8 * a);
  const uint32_t hi = b >= 4 ? 0xffffffffu : ~(0xffffffffu << (8 * b));
  return lo & hi;
}
// acc |= bytes [lo, hi) of chunk v (any lo, hi; clamped to the chunk)
__device__ __forceinline__ void merge_bytes(u32x4 &acc, const u32x4 &v, int lo, int hi) {
  if (lo <= 0 && hi >= 16) {
    acc.x |= v.x; acc.y |= v.y; acc.z |= v.z; acc.w |= v.w;
    return;
  }
  acc.x |= v.x & byte_mask(min(max(lo, 0), 4), min(max(hi, 0), 4));
  acc.y |= v.y & byte_mask(min(max(lo - 4, 0), 4), min(max(hi - 4, 0), 4));
  acc.z |= v.z & byte_mask(min(max(lo - 8, 0), 4), min(max(hi - 8, 0), 4));
  acc.w |= v.w & byte_mask(min(max(lo - 12, 0), 4), min(max(hi - 12, 0), 4));
}
// Byte b (0..15) of chunk v := x, if 0 <= b < 16.
__device__ __forceinline__ void put_byte(u32x4 &v, int b, uint32_t x) {
  if (b < 0 || b >= 16) return;
  const uint32_t sh = 8u * (b & 3), m = ~(0xffu << sh), y = (x & 0xffu) << sh;
  const int j = b >> 2;
  v.x = j == 0 ? (v.x & m) | y : v.x;
  v.y = j == 1 ? (v.y & m) | y : v.y;
  v.z = j == 2 ? (v.z & m) | y : v.z;
  v.w = j == 3 ? (v.w & m) | y : v.w;
}
// Store bytes [lo, hi) of chunk v at destination address a (16-aligned).
// Copied frames are written once and not read back by this kernel:
// nontemporal stores (aux = 2, `nt`) lift a plain slot copy of the TX
// geometry from 0.51 to 0.62 of HBM (tools/ceiling_copy.py,
// profiles/ceiling_copy_r02.jsonl).
#ifndef MI_TX_STORE_AUX
#define MI_TX_STORE_AUX 2
#endif
// Bytes [b0, b1) of dword w (clamped to [0, 4)) at destination address at.
__device__ __forceinline__ void store_dword_part(__amdgpu_buffer_rsrc_t r, uint32_t w, uint32_t at, int b0, int b1) {
  constexpr int kAux = MI_TX_STORE_AUX;
  if (b0 <= 0 && b1 >= 4) {
    __builtin_amdgcn_raw_buffer_store_b32(w, r, at, 0, kAux);
    return;
  }
  if (b0 <= 0 && b1 > 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)w, r, at, 0, kAux);
  if (b0 <= 1 && b1 > 1) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> 8), r, at + 1u, 0, kAux);
  if (b0 <= 2 && b1 > 2) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> 16), r, at + 2u, 0, kAux);
  if (b0 <= 3 && b1 > 3) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(w >> 24), r, at + 3u, 0, kAux);
}
__device__ __forceinline__ void store_chunk(__amdgpu_buffer_rsrc_t r, uint32_t a, const u32x4 &v, int lo,
                                            int hi) {
  constexpr int kAux = MI_TX_STORE_AUX;
  if (lo <= 0 && hi >= 16) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, a, 0, kAux);
    return;
  }
  // per dword: one whole-dword store, or its covered bytes one by one, each
  // under its own condition -- straight-line code (a byte loop with run-time
  // bounds here kept every chunk of a pass live across it: ~45 VGPRs more in
  // the TX kernels)
  store_dword_part(r, v.x, a, lo, hi);
  store_dword_part(r, v.y, a + 4u, lo - 4, hi - 4);
  store_dword_part(r, v.z, a + 8u, lo - 8, hi - 8);
  store_dword_part(r, v.w, a + 12u, lo - 12, hi - 12);
}

// TX sums from the group's absolute-lane accumulators (in_delayed_cksum's
// in_cksum_skip(m, ip_len, hl) and in_cksum(m, hl) with ip_sum = 0), both
// returned in every lane of the group.
template <int G>
__device__ __forceinline__ void tx_sums(uint32_t acc_t, uint32_t acc_h, uint32_t acc_f, int hend,
                                        const IpHdr &ih, bool odd, bool udp, uint32_t &c_ip,
                                        uint32_t &c_l4) {
  const uint32_t total = group_sum<G>(acc_t);
  uint32_t hdr, field;
  if (hend > 20) {
    hdr = group_sum<G>(acc_h);
    field = group_sum<G>(acc_f);
  } else if (hend) {
    hdr = abs_halves(ih.w[0], odd) + abs_halves(ih.w[1], odd) + abs_halves(ih.w[2], odd) +
          abs_halves(ih.w[3], odd) + abs_halves(ih.w[4], odd);
    field = abs_halves(ih.w[2] & 0xffff0000u, odd);
  } else {
    hdr = field = 0u;
  }
  uint32_t sh = fold16(hdr - field), sl = fold16(total - hdr);
  if (odd) {
    sh = swap16(sh);
    sl = swap16(sl);
  }
  c_ip = ~sh & 0xffffu;
  c_l4 = ~sl & 0xffffu;
  if (udp && c_l4 == 0u) c_l4 = 0xffffu;
  c_ip = group_lane<G>(c_ip, 0);
  c_l4 = group_lane<G>(c_l4, 0);
}

// Fold one chunk of an IPv4 datagram whose first byte is rel bytes after the
// datagram start (fold_pass for a single chunk; bytes outside the piece the
// chunk carries are zero, so whole-chunk arithmetic stays exact).
__device__ __forceinline__ void fold_chunk(const u32x4 &v, int rel, int lend, int hend, bool opts,
                                           uint32_t &acc_t, uint32_t &acc_h, uint32_t &acc_f) {
  const bool pure = rel >= 0 && rel + 16 <= lend;
  acc_t += pure ? sum4(v) : 0u;
  if (!pure && rel < lend) acc_t += range_sum(v, rel, 0, lend);
  if (opts && rel < hend) {
    acc_h += range_sum(v, rel, 0, hend);
    acc_f += range_sum(v, rel, 10, 12);
  }
}

// x as held by the next lane of this lane's G-lane group (G = 8 or 16), or,
// for the group's last lane, by the group's first lane of xn: DPP row shifts.
template <int G>
__device__ __forceinline__ uint32_t next_lane(uint32_t x, uint32_t xn, bool last) {
  static_assert(G == 8 || G == 16, "row-local groups only");
  const uint32_t in = dpp_all<0x101>(x);             // row_shl:1
  const uint32_t ed = dpp_all<0x110 + (G - 1)>(xn);  // row_shr:G-1
  return last ? ed : in;
}
template <int G>
__device__ __forceinline__ u32x4 next_lane4(const u32x4 &x, const u32x4 &xn, bool last) {
  return {next_lane<G>(x.x, xn.x, last), next_lane<G>(x.y, xn.y, last), next_lane<G>(x.z, xn.z, last),
          next_lane<G>(x.w, xn.w, last)};
}

// A piece of one segment: destination chunks [cfirst, clast) carrying frame
// bytes [pa, pe), the byte at frame position q read from source address q + del.
struct Piece {
  uint32_t cfirst, clast, del;
  int pa, pe;
};

// Pass p of a piece: each lane loads ONE aligned source chunk per destination
// chunk ci = cfirst + p*G*U + u*G + lane (source chunks are consecutive across
// the group's lanes, like the destination chunks); x[U] is the chunk after
// the pass, loaded by the group's last lane only.  A misaligned piece also
// needs the source chunk of clast.
template <int G, int U>
__device__ __forceinline__ void load_pass(__amdgpu_buffer_rsrc_t rs, const Piece &pc, uint32_t p, int lane,
                                          uint32_t h, u32x4 (&x)[U + 1]) {
  const uint32_t cb = pc.cfirst + p * (G * U);
  const uint32_t lim = pc.clast + (((pc.del - h) & 15u) ? 1u : 0u);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t ci = cb + u * G + lane;
    x[u] = ld16(rs, ci < lim ? (16u * ci - h + pc.del) & ~15u : kOOB);
  }
  const uint32_t ci = cb + U * G;
  x[U] = ld16(rs, lane == G - 1 && ci < lim ? (16u * ci - h + pc.del) & ~15u : kOOB);
}
// Destination chunk u of pass p, shifted into destination alignment (the
// second source chunk is the next lane's, fetched with a DPP row shift) and
// masked to the piece.
template <int G, int U>
__device__ __forceinline__ u32x4 make_chunk(const u32x4 (&x)[U + 1], int u, const Piece &pc, uint32_t p,
                                            int lane, uint32_t h) {
  const uint32_t ci = pc.cfirst + p * (G * U) + u * G + lane;
  const int cs = (int)(16u * ci) - (int)h;
  const bool last = lane == G - 1;
  // (computed by every lane before the select: a ternary arm is evaluated only
  // by the lanes that take it, and the DPP would read switched-off lanes)
  const u32x4 nl = next_lane4<G>(x[u], x[u + 1 < U ? u + 1 : u], last);
  const u32x4 nx = u + 1 < U ? nl : (last ? x[U] : nl);
  u32x4 v{0, 0, 0, 0};
  if (ci < pc.clast) merge_bytes(v, shift2(x[u], nx, (uint32_t)cs + pc.del), pc.pa - cs, pc.pe - cs);
  return v;
}

// Fast path of k_tx_copy: chunk-major gather with unaligned loads.  Every
// nonempty mbuf of the frame (at most kTxSeg of them: the header mbuf and the
// payload's cluster pieces) is kept as (frame position, source - position) in
// registers; destination chunk ci (frame bytes [q0, q0 + 16), q0 = 16 ci - h)
// takes each overlapping segment's bytes with ONE 16-byte load at the
// segment's source address of q0 (gfx950 buffer loads accept any byte
// address, tools/unaligned_probe.hip) -- no funnel shifts, no neighbour-lane
// exchange -- and all of a pass's loads are issued before any is used.  A
// load that would start before the source buffer or run past its end takes a
// per-byte path instead (the first / last bytes of the buffer only).
constexpr int kTxSeg = 4;
// The source loads of the TX gather.  A group's 16-byte loads start at any
// byte, so each wave-instruction's window of a frame straddles one more
// 128-byte line than it covers, and the next pass's window starts in that same
// line: with nontemporal loads (which do not keep the line in L2) every such
// line came from HBM twice -- 1.45x the algorithmic read bytes, from the
// request-size counters (32 B x RDREQ_32B + 64 B x RDREQ_64B + 128 B x
// RDREQ_128B; profiles/r03/pmc_reqsize_r03.jsonl).  With the default policy
// (MI_TX_LOAD_AUX 0) the straddled line is an L2 hit: 1.15x, and socket frames
// 51.5 -> 47.1 us per 65536 x 1514 B batch (0.48 -> 0.53 of 8 TB/s),
// single-segment frames 48.1 -> 44.4 us (0.51 -> 0.56); profiles/r03/tx_r03.jsonl.
#ifndef MI_TX_LOAD_AUX
#define MI_TX_LOAD_AUX 0
#endif
__device__ __forceinline__ u32x4 ld16_src(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, MI_TX_LOAD_AUX);
}
// (A software-pipelined variant -- pass p+1's loads issued before pass p is
// built -- measured slower: the second register set spilled at the 128-VGPR
// bound, socket frames 57.9 vs 51.3 us; profiles/tx_pipe_r02.jsonl.)

// A frame's first kTxSeg nonempty segments: segment e covers frame bytes
// [S_e, S_e+1) (S_0 = 0, the last one to L), frame byte q of segment e sits
// at source offset q + D_e.  A 16-byte load at source offset A (u32; a
// negative offset wraps past lim) is inside the source buffer iff A <= lim.
struct TxSegs {
  int S1, S2, S3, L;
  uint32_t D0, D1, D2, D3, lim;
};
// Destination chunk ci (frame bytes [q0, q0 + 16), q0 = 16 ci - h): bytes
// [max(q0, 0), q0 + B) come from segment j (the one holding the first byte,
// loaded at A1), [q0 + B, min(q0 + 16, L)) from segment j + 1 (at A2) when
// `two`.  clip: the chunk is cut by the frame's ends.  slow: it touches three
// segments or a load would leave the source buffer.
struct TxCut {
  int q0, B;
  uint32_t A1, A2;
  bool two, clip, slow;
};
__device__ __forceinline__ TxCut tx_cut(const TxSegs &g, uint32_t ci, uint32_t h) {
  const int S1 = g.S1, S2 = g.S2, S3 = g.S3, L = g.L;
  const uint32_t D0 = g.D0, D1 = g.D1, D2 = g.D2, D3 = g.D3;
  TxCut c;
  c.q0 = (int)(16u * ci) - (int)h;
  const int q = max(c.q0, 0), hi = min(c.q0 + 16, L);
  const bool j1 = q >= S1, j2 = q >= S2, j3 = q >= S3;
  const uint32_t d0 = j3 ? D3 : j2 ? D2 : j1 ? D1 : D0;
  const uint32_t d1 = j2 ? D3 : j1 ? D2 : D1;
  const int s1 = j3 ? L : j2 ? S3 : j1 ? S2 : S1;
  const int s2 = j2 ? L : j1 ? S3 : S2;
  c.A1 = (uint32_t)c.q0 + d0;
  c.A2 = (uint32_t)c.q0 + d1;
  c.B = s1 - c.q0;
  c.two = s1 < hi;
  c.clip = c.q0 < 0 || c.q0 + 16 > L;
  c.slow = q < hi && (c.A1 > g.lim || (c.two && (s2 < hi || c.A2 > g.lim)));
  return c;
}
// The chunk from its (at most two) loads: one mask per dword in the common
// case, byte masks at the frame's ends, byte loads in the rare slow case.
__device__ __forceinline__ u32x4 tx_build(const TxSegs &g, const TxCut &c, const u32x4 &xa, const u32x4 &xb,
                                          __amdgpu_buffer_rsrc_t rs) {
  u32x4 v{0, 0, 0, 0};
  if (!c.clip && !c.slow) {
    // bytes [0, B) from xa, [B, 16) from xb
    const uint32_t b = (uint32_t)min(max(c.B, 0), 16);
    const uint64_t lo = b >= 8u ? ~0ull : (1ull << (8u * b)) - 1u;
    const uint64_t hm = b <= 8u ? 0ull : b >= 16u ? ~0ull : (1ull << (8u * (b - 8u))) - 1u;
    v.x = (xa.x & (uint32_t)lo) | (xb.x & ~(uint32_t)lo);
    v.y = (xa.y & (uint32_t)(lo >> 32)) | (xb.y & ~(uint32_t)(lo >> 32));
    v.z = (xa.z & (uint32_t)hm) | (xb.z & ~(uint32_t)hm);
    v.w = (xa.w & (uint32_t)(hm >> 32)) | (xb.w & ~(uint32_t)(hm >> 32));
  } else if (!c.slow) {
    const int lo = max(c.q0, 0) - c.q0, hi = min(c.q0 + 16, g.L) - c.q0;
    merge_bytes(v, xa, lo, min(c.B, hi));
    if (c.two) merge_bytes(v, xb, c.B, hi);
  } else {
    for (int q = max(c.q0, 0); q < min(c.q0 + 16, g.L); ++q) {
      const uint32_t d = q >= g.S3 ? g.D3 : q >= g.S2 ? g.D2 : q >= g.S1 ? g.D1 : g.D0;
      put_byte(v, q - c.q0, __builtin_amdgcn_raw_buffer_load_b8(rs, (uint32_t)(q + (int)d), 0, 0));
    }
  }
  return v;
}

// What ip_output decides for a frame from its IP header and m_pkthdr
// (ip_output.c:649-672 with in_delayed_cksum, ip_output.c:958-983): which sums
// to do, where the L4 one goes (at = hl + csum_data), and whether the datagram
// is well-formed enough to be summed at all.
struct TxPlan {
  bool ok, do_ip, do_l4, udp;
  uint32_t at;
  int hend, lend;  // header / datagram length when ok, else 0
};
__device__ __forceinline__ TxPlan tx_plan(const TxDesc &t, uint32_t i, uint32_t len, const IpHdr &ih) {
  TxPlan pl;
  const uint32_t flen = len >= t.l3 ? len - t.l3 : 0u;
  pl.ok = flen >= 20u && ih.hl >= 20u && ih.hl <= flen && ih.iplen >= ih.hl && ih.iplen <= flen;
  const TxArrs ta = tx_arrs(t);
  const uint32_t fl =
      t.cflags ? ld_u32(ta.cflags, i) : MI_CSUM_IP | (ih.proto == 6u ? MI_CSUM_TCP : ih.proto == 17u ? MI_CSUM_UDP : 0u);
  pl.do_ip = pl.ok && (fl & MI_CSUM_IP);
  pl.do_l4 = pl.ok && (fl & (MI_CSUM_TCP | MI_CSUM_UDP));
  pl.udp = fl & MI_CSUM_UDP;
  pl.at = ih.hl + (t.cdata ? ld_u32(ta.cdata, i) : (fl & MI_CSUM_TCP) ? MI_CSUM_DATA_TCP : MI_CSUM_DATA_UDP);
  pl.hend = pl.ok ? (int)ih.hl : 0;
  pl.lend = pl.ok ? (int)ih.iplen : 0;
  return pl;
}
__device__ __forceinline__ uint8_t tx_status(const TxPlan &pl, bool l4_store) {
  return (uint8_t)((pl.ok ? 0u : MI_TX_NOSUM) | (pl.do_l4 && !l4_store ? MI_TX_L4_SKIPPED : 0u));
}

// (forceinline: as a real call its TxDesc argument is passed through the
// stack -- a private segment, which no kernel of this library may have)
// Generic gather of frame i by a G-lane group (long chains, an IP header split
// over mbufs, sum fields far from the header): chunk-major over the whole
// frame, every piece of every chunk gathered by walking the chain; chunks
// stored as they are built, the sum fields patched once they have landed.
// len, the chain [k0, k1) and ip_mlen come from the caller's chain walk.
template <int G, int U>
__device__ __forceinline__ void tx_frame_generic(const TxDesc &t, __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t rd, uint32_t i,
                                 int lane, uint32_t len, uint32_t k0, uint32_t k1, uint32_t ip_mlen) {
  const TxArrs ta = tx_arrs(t);
  const uint32_t l3 = t.l3;
  const uint32_t D = (uint32_t)(t.dst_first + (uint64_t)i * t.dst_stride);  // host-checked < 4 GiB
  const uint32_t h = D & 15u, c0 = D & ~15u;
  const bool odd = (h + l3) & 1u;
  IpHdr ih{};
  TxPlan pl{};
  uint32_t acc_t = 0, acc_h = 0, acc_f = 0;
  const uint32_t nch = (h + len + 15u) >> 4;
  const uint32_t npass = (nch + G * U - 1) / (G * U);
  for (uint32_t p = 0; p < npass; ++p) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int cs = (int)(16u * (p * (G * U) + u * G + lane)) - (int)h;
      v[u] = u32x4{0, 0, 0, 0};
      int pos = 0;
      for (uint32_t k = k0; k < k1; ++k) {
        const int l = max((int32_t)ld_u32(ta.seg_len, k), 0);
        const int lo = max(pos - cs, 0), hi = min(min(pos + l, (int)len) - cs, 16);
        if (hi > lo) {
          const uint32_t a = (uint32_t)cs + ((uint32_t)ld_u64(ta.seg_off, k) - (uint32_t)pos);
          merge_bytes(v[u], shift_pair(ld_pair(rs, a), a), lo, hi);
        }
        pos += l;
      }
    }
    if (p == 0) {
      const u32x4 hv[1] = {v[0]};
      ih = parse_ipv4<G, 1>(hv, h + l3);
      pl = tx_plan(t, i, len, ih);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t ci = p * (G * U) + u * G + lane;
      const int cs = (int)(16u * ci) - (int)h;
      fold_chunk(v[u], cs - (int)l3, pl.lend, pl.hend, pl.hend > 20, acc_t, acc_h, acc_f);
      if (ci < nch) store_chunk(rd, c0 + 16u * ci, v[u], -cs, (int)len - cs);
    }
  }
  if (npass == 0) pl = TxPlan{};
  const bool l4_store = pl.do_l4 && (uint64_t)pl.at + 2u <= ip_mlen;
  uint32_t c_ip, c_l4;
  tx_sums<G>(acc_t, acc_h, acc_f, pl.hend, ih, odd, pl.udp, c_ip, c_l4);
  if (pl.do_ip || l4_store) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's chunk stores have landed
    if (lane == 0) {
      const uint32_t pip = l3 + 10u, pl4 = l3 + pl.at;
      if (pl.do_ip) {
        if (pip < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)c_ip, rd, D + pip, 0, 0);
        if (pip + 1u < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c_ip >> 8), rd, D + pip + 1u, 0, 0);
      }
      if (l4_store) {
        if (pl4 < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)c_l4, rd, D + pl4, 0, 0);
        if (pl4 + 1u < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c_l4 >> 8), rd, D + pl4 + 1u, 0, 0);
      }
    }
  }
  if (lane == 0) st_u8(ta.status, i, tx_status(pl, l4_store));
}

// Pass p's two loads per destination chunk (tx_cut) into xa / xb, its cuts
// into cut.
template <int G, int U>
__device__ __forceinline__ void tx_issue(const TxSegs &sg, uint32_t p, int lane, uint32_t h, __amdgpu_buffer_rsrc_t rs,
                                         u32x4 (&xa)[U], u32x4 (&xb)[U], TxCut (&cut)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const TxCut c = tx_cut(sg, p * (G * U) + u * G + lane, h);
    xa[u] = ld16_src(rs, c.q0 < sg.L && !c.slow ? c.A1 : kOOB);
    xb[u] = ld16_src(rs, c.two && !c.slow ? c.A2 : kOOB);
    cut[u] = c;
  }
}
// (on by default since round 6: +6 % on socket chains, +3 % on single
// segments in the interleaved A/B, profiles/r06/tx_ab_r06.jsonl; round 5 had
// it off on a misread of the fault record)
#ifndef MI_TX_EARLY_LOADS
#define MI_TX_EARLY_LOADS 1
#endif

// U <= 2 shapes are held to 4 waves per SIMD (128 VGPRs; the descriptor
// prefetch costs ~10 and a few spill to scratch): profiles/tx_copy_r02.jsonl,
// socket frames 59-64 us per launch against 64-66 without the prefetch and
// 69 with it at 3 waves per SIMD.
template <int G, int U, bool EL = MI_TX_EARLY_LOADS>
__global__ __launch_bounds__(kBlock, (U <= 2 ? 4 : 1)) void k_tx_copy(TxDesc t) {
  static_assert(G >= 8, "the header window needs lanes 0..6 of the group");
  __shared__ uint32_t s_seg[kBlock / G][kTxSeg][2];
  Desc ds{}, dd{};
  ds.base = t.src;
  ds.bytes = t.src_bytes;
  dd.base = t.dst;
  dd.bytes = t.dst_bytes;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(ds), rd = rsrc_of(dd);
  const TxArrs ta = tx_arrs(t);
  const int lane = threadIdx.x & (G - 1);
  const uint32_t grp = (threadIdx.x & 255u) / G;
  const uint32_t stride = gridDim.x * (kBlock / G);
  // Descriptor prefetch: a frame's descriptors are a chain of two dependent
  // loads (pkt_seg -> seg_len / seg_off) ahead of its first data load, so the
  // NEXT frame's chain is walked while this frame's data is in flight -- the
  // first level at the top of the iteration, the second level right after this
  // frame's first data pass is issued (its wait then covers only the older
  // descriptor loads; vmcnt is in order).  Lane j holds segment k0 + j.
  uint32_t i = blockIdx.x * (kBlock / G) + threadIdx.x / G;
  uint32_t len_c = 0, k0_c = 0, k1_c = 0;
  int32_t sl_c = 0;
  uint32_t so_c = 0;
  if (i < t.n) {
    len_c = ld_u32(ta.pkt_len, i);
    k0_c = ld_u32(ta.pkt_seg, i);
    k1_c = ld_u32(ta.pkt_seg, i + 1);
    if (k0_c + lane < k1_c) {
      sl_c = (int32_t)ld_u32(ta.seg_len, k0_c + lane);
      so_c = (uint32_t)ld_u64(ta.seg_off, k0_c + lane);
    }
  }
  for (; i < t.n; i += stride) {
    const uint32_t len = len_c;
    const uint32_t k0 = k0_c, k1 = k1_c;
    const int32_t sl0 = sl_c;
    const uint32_t so0 = so_c;
    const uint32_t in = i + stride;
    uint32_t len_n = 0, k0_n = 0, k1_n = 0;
    if (in < t.n) {
      len_n = ld_u32(ta.pkt_len, in);
      k0_n = ld_u32(ta.pkt_seg, in);
      k1_n = ld_u32(ta.pkt_seg, in + 1);
    }
    bool pre2 = false;
    auto prefetch2 = [&]() {
      if (pre2) return;
      pre2 = true;
      sl_c = 0;
      so_c = 0;
      if (in < t.n && k0_n + lane < k1_n) {
        sl_c = (int32_t)ld_u32(ta.seg_len, k0_n + lane);
        so_c = (uint32_t)ld_u64(ta.seg_off, k0_n + lane);
      }
      len_c = len_n;
      k0_c = k0_n;
      k1_c = k1_n;
    };
    const uint32_t l3 = t.l3;
    const uint32_t D = (uint32_t)(t.dst_first + (uint64_t)i * t.dst_stride);  // host-checked < 4 GiB
    const uint32_t h = D & 15u, c0 = D & ~15u;
    uint32_t st = len > t.room ? MI_TX_NOBUFS : 0u;
    // walk 1: bytes in the chain, the IP mbuf (segment holding frame byte l3)
    // and its m_len from the IP header on, and the first kTxSeg nonempty
    // segments (frame start, source offset - frame start) into LDS
    uint32_t total = 0, ip_mlen = 0, m = 0;
    for (uint32_t w = k0; w < k1 && !st; w += G) {
      const uint32_t k = w + lane;
      const uint32_t l = k < k1 ? (uint32_t)max(w == k0 ? sl0 : (int32_t)ld_u32(ta.seg_len, k), 0) : 0u;
      const uint32_t inc = group_scan<G>(l);
      const uint32_t a = total + inc - l, e = total + inc;
      const uint32_t nz = l ? 1u : 0u;
      const uint32_t zi = group_scan<G>(nz);
      const uint32_t idx = m + zi - nz;
      if (nz && idx < (uint32_t)kTxSeg) {
        s_seg[grp][idx][0] = a;
        s_seg[grp][idx][1] = (w == k0 ? so0 : (uint32_t)ld_u64(ta.seg_off, k)) - a;
      }
      const bool isip = l && a <= l3 && l3 < e;
      ip_mlen += group_sum<G>(isip ? e - l3 : 0u);  // leader only
      total += group_lane<G>(inc, G - 1);
      m += group_lane<G>(zi, G - 1);
    }
    if (!st && total < len) st = MI_TX_SHORT;
    if (st) {
      if (lane == 0) st_u8(ta.status, i, st);
      prefetch2();
      continue;
    }
    ip_mlen = group_lane<G>(ip_mlen, 0);
    const bool odd = (h + l3) & 1u;  // parity of the IP header's destination address
    IpHdr ih{};
    bool ok = false, do_ip = false, do_l4 = false, udp = false, done = false;
    uint32_t at = 0;
    int hend = 0, lend = 0;
    uint32_t acc_t = 0, acc_h = 0, acc_f = 0;
    auto decide1 = [&](const u32x4 &h0, uint32_t hoff) {
      const u32x4 hv[1] = {h0};
      ih = parse_ipv4<G, 1>(hv, hoff);
      const TxPlan pl = tx_plan(t, i, len, ih);
      ok = pl.ok;
      do_ip = pl.do_ip;
      do_l4 = pl.do_l4;
      udp = pl.udp;
      at = pl.at;
      hend = pl.hend;
      lend = pl.lend;
    };
    auto fold_all = [&](const u32x4 (&v)[U], uint32_t cfirst, uint32_t p) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rel = (int)(16u * (cfirst + p * (G * U) + u * G + lane)) - (int)(h + l3);
        fold_chunk(v[u], rel, lend, hend, hend > 20, acc_t, acc_h, acc_f);
      }
    };
    auto store_all = [&](const u32x4 (&v)[U], uint32_t cfirst, uint32_t clast, uint32_t p, int pa, int pe,
                         int u0 = 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (u < u0) continue;
        const uint32_t ci = cfirst + p * (G * U) + u * G + lane;
        const int cs = (int)(16u * ci) - (int)h;
        if (ci < clast) store_chunk(rd, c0 + 16u * ci, v[u], pa - cs, pe - cs);
      }
    };
    if (m <= (uint32_t)kTxSeg) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // segment e covers frame bytes [S[e], S[e+1]) (the last one: to len),
      // frame byte q sits at source offset q + Dl[e]
      static_assert(kTxSeg == 4, "segment registers S1..S3 / D0..D3");
      auto seg_start = [&](uint32_t e) { return e < m ? min((int)s_seg[grp][e][0], (int)len) : (int)len; };
      auto seg_delta = [&](uint32_t e) { return e < m ? s_seg[grp][e][1] : 0u; };
      const uint32_t nch = (h + len + 15u) >> 4;
      const uint32_t npass = (nch + G * U - 1) / (G * U);
      // Chunk ci of the frame is gathered from at most two loads (tx_cut,
      // tx_build above).
      const int S1 = seg_start(1), S2 = seg_start(2), S3 = seg_start(3);
      const uint32_t D0 = seg_delta(0), D1 = seg_delta(1), D2 = seg_delta(2), D3 = seg_delta(3);
      const uint32_t lim = t.src_bytes - 16u;  // A (u32, negatives wrap) is loadable iff A <= lim
      const TxSegs sg{S1, S2, S3, (int)len, D0, D1, D2, D3, lim};
      u32x4 held{0, 0, 0, 0};
      u32x4 xa[U], xb[U];
      TxCut cut[U];
      if (npass) tx_issue<G, U>(sg, 0u, lane, h, rs, xa, xb, cut);
      for (uint32_t p = 0; p < npass; ++p) {
        u32x4 v[U];
        if (p == 0) prefetch2();
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = tx_build(sg, cut[u], xa[u], xb[u], rs);
        // the next pass's loads go out BEFORE this pass's stores: vmcnt counts
        // stores too and retires in order, so loads issued after the stores
        // could not be waited for without also waiting for the stores' acks
        if (EL && p + 1 < npass) tx_issue<G, U>(sg, p + 1, lane, h, rs, xa, xb, cut);
        if (p == 0) {
          decide1(v[0], h + l3);
          const uint32_t pip = l3 + 10u, pl4 = l3 + at;
          const bool l4s = do_l4 && (uint64_t)at + 2u <= ip_mlen;
          const uint32_t need = max(do_ip ? pip + 2u : 0u, l4s ? pl4 + 2u : 0u);
          if ((uint64_t)need + h > 16ull * G) break;  // a sum field beyond the held chunks: generic path
          done = true;
          held = v[0];
        }
        fold_all(v, 0, p);
        store_all(v, 0, nch, p, 0, (int)len, p == 0 ? 1 : 0);
        if (!EL && p + 1 < npass) tx_issue<G, U>(sg, p + 1, lane, h, rs, xa, xb, cut);
      }
      if (npass == 0) {
        ok = do_ip = do_l4 = false;
        done = true;
      }
      if (done) {
        const bool l4_store = do_l4 && (uint64_t)at + 2u <= ip_mlen;
        uint32_t c_ip, c_l4;
        tx_sums<G>(acc_t, acc_h, acc_f, hend, ih, odd, udp, c_ip, c_l4);
        const uint32_t pip = l3 + 10u, pl4 = l3 + at;
        const int b0 = (int)h - (int)(16u * lane);  // frame position -> byte of held
        if (do_ip) {
          if (pip < len) put_byte(held, (int)pip + b0, c_ip);
          if (pip + 1u < len) put_byte(held, (int)pip + 1 + b0, c_ip >> 8);
        }
        if (l4_store) {
          if (pl4 < len) put_byte(held, (int)pl4 + b0, c_l4);
          if (pl4 + 1u < len) put_byte(held, (int)pl4 + 1 + b0, c_l4 >> 8);
        }
        const uint32_t ci = lane;
        const int cs = (int)(16u * ci) - (int)h;
        if (ci < nch) store_chunk(rd, c0 + 16u * ci, held, -cs, (int)len - cs);
        if (lane == 0) st_u8(ta.status, i, (ok ? 0u : MI_TX_NOSUM) | (do_l4 && !l4_store ? MI_TX_L4_SKIPPED : 0u));
      }
      __builtin_amdgcn_wave_barrier();  // s_seg is rewritten by the group's next frame
    }
    prefetch2();
    if (!done) tx_frame_generic<G, U>(t, rs, rd, i, lane, len, k0, k1, ip_mlen);
  }
}

// Slot s of a frame's piece-flat walk (k_tx_wave, below): destination chunk ci,
// the piece's bytes [lo, hi) of that chunk, the source offset A of the
// chunk's first byte position.  Every piece value is a separate scalar
// argument: a select among the fields of a captured aggregate (a lambda's
// closure) becomes a load through a selected address, i.e. a stack table
// read at run time (scratch).
struct TxSlot {
  uint32_t ci, A;
  int lo, hi;
  bool in, slow;
};
__device__ __forceinline__ TxSlot tx_slot(uint32_t s, uint32_t P1, uint32_t P2, uint32_t P3, uint32_t T, uint32_t cf0,
                                          uint32_t cf1, uint32_t cf2, uint32_t cf3, int S1, int S2, int S3, int L,
                                          uint32_t D0, uint32_t D1, uint32_t D2, uint32_t D3, uint32_t h,
                                          uint32_t lim) {
  const bool j1 = s >= P1, j2 = s >= P2, j3 = s >= P3;
  const uint32_t Ps = j3 ? P3 : j2 ? P2 : j1 ? P1 : 0u;
  const uint32_t cfs = j3 ? cf3 : j2 ? cf2 : j1 ? cf1 : cf0;
  const int Sa = j3 ? S3 : j2 ? S2 : j1 ? S1 : 0;
  const int Sb = j3 ? L : j2 ? S3 : j1 ? S2 : S1;
  const uint32_t Dl = j3 ? D3 : j2 ? D2 : j1 ? D1 : D0;
  TxSlot o;
  o.ci = cfs + (s - Ps);
  const int q0 = (int)(16u * o.ci) - (int)h;
  o.A = (uint32_t)q0 + Dl;
  o.lo = max(Sa - q0, 0);
  o.hi = min(Sb - q0, 16);
  o.in = s < T && o.hi > o.lo;
  o.slow = o.in && o.A > lim;
  return o;
}

// TX fused copy, round 4: one frame per WAVE (k_tx_wave).
//
// The lane-group kernel (k_tx_copy) keeps a frame's chain state
// -- segment starts and source deltas, the IPv4 header fields, the plan --
// in every lane of its group, ~90 VGPRs before any data, so they run at 4
// waves per SIMD with ~2 KiB of loads in flight per wave.  Here a wave owns
// one frame at a time, so all of that is wave-uniform (scalar registers,
// readlane / ballot / s_ff1 instead of group scans), and the vector registers
// hold little besides the slots: a pass is 64 U slots (U = 2: a whole 1514 B
// frame in one pass) of a piece-flat walk, one unaligned 16-byte load per
// slot: a frame's nonempty mbufs (at most kTxSeg) are PIECES, piece e = frame
// bytes [S_e, S_e+1) at source offset q + D_e, covering destination chunks
// [cf_e, cl_e); slot s is the last piece with P_e <= s and destination chunk
// cf_e + s - P_e (tx_slot).  A chunk two pieces share gets two slots, each
// with its own piece's bytes (zeros elsewhere): the fold is linear, so each
// adds its part.  (A lane-group version of this walk needed more registers
// than k_tx_copy: a frame's piece table per lane.)  The next frame's descriptors load while this
// frame's data is in flight.
//
// Every destination chunk a slot does not fill alone -- the header window
// (chunks [0, NH), where ip_sum and the L4 sum field sit), a chunk two pieces
// share, the frame's partial last chunk -- is OR-ed together in LDS (data and
// a byte mask) and stored once per frame by one lane each, after the sums are
// patched in: the pass loop itself only issues whole-chunk stores, so its
// registers stay those of the slots.
#ifndef MI_TX_WAVE_WAVES
#define MI_TX_WAVE_WAVES 6
#endif
template <int U>
__global__ __launch_bounds__(kBlock, MI_TX_WAVE_WAVES) void k_tx_wave(TxDesc t) {
  constexpr uint32_t W = 64u * U;  // slots per pass
  constexpr uint32_t NH = 8;       // header window: destination chunks [0, 8)
  constexpr uint32_t NC = NH + 4;  // LDS cells: the window, 3 piece boundaries, the last chunk
  static_assert(W >= NH + kTxSeg, "pass 0 holds every slot of the header window");
  __shared__ uint32_t s_cell[kBlock / 64][NC][5];  // 4 data dwords + byte mask
  Desc ds{}, dd{};
  ds.base = t.src;
  ds.bytes = t.src_bytes;
  dd.base = t.dst;
  dd.bytes = t.dst_bytes;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(ds), rd = rsrc_of(dd);
  const TxArrs ta = tx_arrs(t);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * (kBlock / 64);
  const uint32_t lim = t.src_bytes - 16u;
  uint32_t f = blockIdx.x * (kBlock / 64) + wv;
  // descriptors of the wave's frame (pkt_len / pkt_seg, then its segment
  // table one segment per lane), loaded a frame ahead
  uint32_t len_c = 0, k0_c = 0, k1_c = 0;
  int32_t sl_c = 0;
  uint32_t so_c = 0;
  if (f < t.n) {
    len_c = ld_u32(ta.pkt_len, f);
    k0_c = ld_u32(ta.pkt_seg, f);
    k1_c = ld_u32(ta.pkt_seg, f + 1);
    if (k0_c + lane < k1_c) {
      sl_c = (int32_t)ld_u32(ta.seg_len, k0_c + lane);
      so_c = (uint32_t)ld_u64(ta.seg_off, k0_c + lane);
    }
  }
  for (; f < t.n; f += nw) {
    const uint32_t len = __builtin_amdgcn_readfirstlane(len_c);
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(k0_c), k1 = __builtin_amdgcn_readfirstlane(k1_c);
    const int32_t sl0 = sl_c;
    const uint32_t so0 = so_c;
    const uint32_t fn = f + nw;
    uint32_t len_n = 0, k0_n = 0, k1_n = 0;
    if (fn < t.n) {
      len_n = ld_u32(ta.pkt_len, fn);
      k0_n = ld_u32(ta.pkt_seg, fn);
      k1_n = ld_u32(ta.pkt_seg, fn + 1);
    }
    bool pre2 = false;
    auto prefetch2 = [&]() {
      if (pre2) return;
      pre2 = true;
      sl_c = 0;
      so_c = 0;
      if (fn < t.n && k0_n + lane < k1_n) {
        sl_c = (int32_t)ld_u32(ta.seg_len, k0_n + lane);
        so_c = (uint32_t)ld_u64(ta.seg_off, k0_n + lane);
      }
      len_c = len_n;
      k0_c = k0_n;
      k1_c = k1_n;
    };
    const uint32_t l3 = t.l3;
    const uint32_t D = (uint32_t)(t.dst_first + (uint64_t)f * t.dst_stride);  // host-checked < 4 GiB
    const uint32_t h = D & 15u, c0 = D & ~15u;
    uint32_t st = len > t.room ? MI_TX_NOBUFS : 0u;
    // the chain, one segment per lane (chains of > 64 mbufs: walked in
    // windows of 64 for the byte count and the IP mbuf, then the generic path)
    const uint32_t nseg = k1 > k0 ? k1 - k0 : 0u;
    bool done = false;
    uint32_t ip_mlen = 0;
    if (!st && nseg > 64u) {
      uint32_t total = 0;
      for (uint32_t w = k0; w < k1; w += 64u) {
        const uint32_t k = w + lane;
        const uint32_t l = k < k1 ? (uint32_t)max(w == k0 ? sl0 : (int32_t)ld_u32(ta.seg_len, k), 0) : 0u;
        const uint32_t inc = wave_scan(l);
        const uint32_t a = total + inc - l, e = total + inc;
        const uint64_t ipb = __ballot(l != 0u && a <= l3 && l3 < e);
        if (ipb) ip_mlen = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)__builtin_ctzll(ipb)) - l3;
        total += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      }
      if (total < len) st = MI_TX_SHORT;
    }
    if (!st && nseg <= 64u) {
      const uint32_t l = lane < nseg ? (uint32_t)max(sl0, 0) : 0u;
      const uint32_t inc = wave_scan(l);
      const uint32_t a = inc - l;
      const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
      const uint64_t nz = __ballot(l != 0u);
      const uint64_t ipb = __ballot(l != 0u && a <= l3 && l3 < inc);
      if (ipb) ip_mlen = (uint32_t)__builtin_amdgcn_readlane((int)inc, (int)__builtin_ctzll(ipb)) - l3;
      if (total < len) st = MI_TX_SHORT;
      if (!st && __popcll(nz) <= (uint64_t)kTxSeg) {
        // the pieces: the first kTxSeg nonempty segments, in chain order
        const int L = (int)len;
        const uint32_t dl = so0 - a;  // source offset - frame position, per segment
        uint64_t mk = nz;
        auto take = [&](int &S, uint32_t &Dl) {
          if (mk) {
            const int j = (int)__builtin_ctzll(mk);
            mk &= mk - 1;
            S = min((int)__builtin_amdgcn_readlane((int)a, j), L);
            Dl = (uint32_t)__builtin_amdgcn_readlane((int)dl, j);
          } else {
            S = L;
            Dl = 0u;
          }
        };
        int S0, S1, S2, S3;
        uint32_t D0, D1, D2, D3;
        take(S0, D0);
        take(S1, D1);
        take(S2, D2);
        take(S3, D3);
        (void)S0;  // == 0: the frame starts with the first nonempty segment
        auto cf = [&](int S) { return (uint32_t)(S + (int)h) >> 4; };
        auto nrun = [&](int Sa, int Sb) { return Sb > Sa ? ((uint32_t)(Sb + (int)h + 15) >> 4) - cf(Sa) : 0u; };
        const uint32_t cf0 = cf(0), cf1 = cf(S1), cf2 = cf(S2), cf3 = cf(S3);
        const uint32_t P1 = nrun(0, S1), P2 = P1 + nrun(S1, S2), P3 = P2 + nrun(S2, S3), T = P3 + nrun(S3, L);
        const uint32_t npass = (T + W - 1) / W;
        const uint32_t nch = (h + len + 15u) >> 4;
        // the LDS cell of destination chunk ci: the window's own, a piece
        // boundary inside a chunk, the partial last chunk; NC = none
        auto mid = [&](int S) { return S < L && ((uint32_t)(S + (int)h) & 15u) ? cf(S) : ~0u; };
        const uint32_t b1 = mid(S1), b2 = mid(S2), b3 = mid(S3);
        const uint32_t cl = ((h + len) & 15u) ? nch - 1u : ~0u;
        auto cell_of = [&](uint32_t ci) {
          return ci < NH ? ci : ci == b1 ? NH : ci == b2 ? NH + 1 : ci == b3 ? NH + 2 : ci == cl ? NH + 3 : NC;
        };
        // a piece whose first or last slot's 16-byte load would leave the
        // source buffer (a frame at the buffer's very start or end): the
        // generic path, which reads aligned chunk pairs
        auto edge = [&](int Sa, int Sb, uint32_t Dl) {
          if (Sb <= Sa) return false;
          const uint32_t A0 = (uint32_t)((int)(16u * cf(Sa)) - (int)h) + Dl;
          const uint32_t A1 = (uint32_t)((int)(16u * (((uint32_t)(Sb + (int)h + 15) >> 4) - 1u)) - (int)h) + Dl;
          return A0 > lim || A1 > lim;
        };
        const bool edge_frame = edge(0, S1, D0) || edge(S1, S2, D1) || edge(S2, S3, D2) || edge(S3, L, D3);
        const bool odd = (h + l3) & 1u;
        IpHdr ih{};
        bool ok = false, do_ip = false, do_l4 = false, udp = false;
        uint32_t at = 0;
        int hend = 0, lend = 0;
        uint32_t acc_t = 0, acc_h = 0, acc_f = 0;
        if (!edge_frame) {
        if (lane < NC)
          s_cell[wv][lane][0] = s_cell[wv][lane][1] = s_cell[wv][lane][2] = s_cell[wv][lane][3] =
              s_cell[wv][lane][4] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t p = 0; p < npass; ++p) {
          u32x4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const TxSlot o =
                tx_slot(p * W + 64u * u + lane, P1, P2, P3, T, cf0, cf1, cf2, cf3, S1, S2, S3, L, D0, D1, D2, D3, h, lim);
            v[u] = ld16_src(rs, o.in && !o.slow ? o.A : kOOB);
          }
          if (p == 0) prefetch2();
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const TxSlot o =
                tx_slot(p * W + 64u * u + lane, P1, P2, P3, T, cf0, cf1, cf2, cf3, S1, S2, S3, L, D0, D1, D2, D3, h, lim);
            u32x4 x{0, 0, 0, 0};
            if (o.in) {
              merge_bytes(x, v[u], o.lo, o.hi);
            }
            v[u] = x;
            const uint32_t c = o.in ? cell_of(o.ci) : NC;
            if (c < NC) {
              __hip_atomic_fetch_or(&s_cell[wv][c][0], x.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_or(&s_cell[wv][c][1], x.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_or(&s_cell[wv][c][2], x.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_or(&s_cell[wv][c][3], x.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              __hip_atomic_fetch_or(&s_cell[wv][c][4], (uint32_t)((1u << o.hi) - (1u << o.lo)), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (o.in) {
              __builtin_amdgcn_raw_buffer_store_b128(x, rd, c0 + 16u * o.ci, 0, MI_TX_STORE_AUX);
            }
          }
          if (p == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            u32x4 hv{0, 0, 0, 0};
            if (lane < NH) hv = u32x4{s_cell[wv][lane][0], s_cell[wv][lane][1], s_cell[wv][lane][2], s_cell[wv][lane][3]};
            const u32x4 hw[1] = {hv};
            ih = parse_ipv4<64, 1>(hw, h + l3);
            const TxPlan pl = tx_plan(t, f, len, ih);
            ok = pl.ok;
            do_ip = pl.do_ip;
            do_l4 = pl.do_l4;
            udp = pl.udp;
            at = pl.at;
            hend = pl.hend;
            lend = pl.lend;
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const TxSlot o =
                tx_slot(p * W + 64u * u + lane, P1, P2, P3, T, cf0, cf1, cf2, cf3, S1, S2, S3, L, D0, D1, D2, D3, h, lim);
            const int q0 = (int)(16u * o.ci) - (int)h;
            if (o.in) fold_chunk(v[u], q0 - (int)l3, lend, hend, hend > 20, acc_t, acc_h, acc_f);
          }
        }
        if (npass == 0) ok = do_ip = do_l4 = false;
        const bool l4_store = do_l4 && (uint64_t)at + 2u <= ip_mlen;
        uint32_t c_ip, c_l4;
        tx_sums<64>(acc_t, acc_h, acc_f, hend, ih, odd, udp, c_ip, c_l4);
        // a sum field outside the window (csum_data far beyond the header):
        // patched into its destination chunk by byte stores once the chunk
        // has landed (rare; vmcnt(0) is this wave's own stores)
        const uint32_t pip = l3 + 10u, pl4 = l3 + at;
        const bool far = l4_store && (uint64_t)pl4 + h >= 16u * NH;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < NC) {
          // cell `lane`: its destination chunk, merged bytes and coverage
          uint32_t ci = lane;
          if (lane == NH) ci = b1;
          if (lane == NH + 1) ci = b2;
          if (lane == NH + 2) ci = b3;
          if (lane == NH + 3) ci = cl;
          // a chunk that is two cells' (a boundary chunk that is also the
          // last one, or one inside the window): stored by its first cell only
          const bool own = ci < nch && cell_of(ci) == lane;
          u32x4 x{s_cell[wv][lane][0], s_cell[wv][lane][1], s_cell[wv][lane][2], s_cell[wv][lane][3]};
          const uint32_t m = s_cell[wv][lane][4];
          if (own && m) {
            const int b0 = (int)h - (int)(16u * ci);  // frame position -> byte of the chunk
            if (do_ip) {
              if (pip < len) put_byte(x, (int)pip + b0, c_ip);
              if (pip + 1u < len) put_byte(x, (int)pip + 1 + b0, c_ip >> 8);
            }
            if (l4_store && !far) {
              if (pl4 < len) put_byte(x, (int)pl4 + b0, c_l4);
              if (pl4 + 1u < len) put_byte(x, (int)pl4 + 1 + b0, c_l4 >> 8);
            }
            store_chunk(rd, c0 + 16u * ci, x, (int)__builtin_ctz(m), 32 - (int)__builtin_clz(m));
          }
        }
        if (far && lane == 0) {
          __builtin_amdgcn_s_waitcnt(0);
          if (pl4 < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)c_l4, rd, D + pl4, 0, 0);
          if (pl4 + 1u < len) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(c_l4 >> 8), rd, D + pl4 + 1u, 0, 0);
        }
        if (lane == 0) st_u8(ta.status, f, (ok ? 0u : MI_TX_NOSUM) | (do_l4 && !l4_store ? MI_TX_L4_SKIPPED : 0u));
        done = true;
        __builtin_amdgcn_wave_barrier();  // the cells are rewritten for the wave's next frame
        }
      }
    }
    if (st) {
      if (lane == 0) st_u8(ta.status, f, st);
      done = true;
    }
    prefetch2();
    if (!done) tx_frame_generic<64, 1>(t, rs, rd, f, (int)lane, len, k0, k1, ip_mlen);
  }
}

// TX fused copy, round 6: the lane-group gather of k_tx_copy with its data
// staged through LDS (k_tx_lds, MI_CKSUM_TX_KERNEL=lds).
//
// k_tx_copy loads a pass's source chunks into VGPRs, so a wave holds one or
// two passes in flight and interleaves each pass's loads with the previous
// pass's stores.  The slot-copy probes say what the memory side wants instead
// (tools/ceiling_copy.py, profiles/r05/ceiling_copy_r05.jsonl): a lane that
// issues all its loads and then all its stores reaches 0.667 of 8 TB/s, one
// that alternates over 2-8 load/store rounds 0.56-0.62.  Here the same two
// loads per destination chunk (tx_cut: the segment holding the chunk's first
// byte at A1, the next one at A2 when the chunk straddles a boundary) go to
// LDS by `buffer_load_dwordx4 ... lds` -- gfx950 takes any byte address there
// too (tools/lds_dma_probe.hip, profiles/r06/lds_dma_probe_r06.txt) -- into a
// ring of R pass slots per wave, so R passes (R * 64 U * 16 B per wave) are in
// flight with no VGPR held for them and a 1514 B frame's loads go out at most
// two rounds apart from its stores.  A pass is built from its slot (tx_build),
// folded and stored exactly as in k_tx_copy; the slot is refilled with the
// pass R ahead once its reads have returned.
//
// Ordering (MI355X_MICROARCH.md, LDS-DMA): only the issuing wave's vmcnt
// orders a ds_read behind a DMA.  Pass p's 2U DMAs are followed by the 2U of
// each pass issued after them (gi - p - 1 of them, at most R - 1; a pass no
// lane of the wave has is not issued), so vmcnt <= 2U(gi - p - 1) retires
// them (stores and descriptor loads in between only add to the count, so the
// wait is conservative; wait_vm_ladder turns the uniform count into an
// s_waitcnt immediate).  The ring's reads are inline asm (the compiler
// would put a vmcnt(0) in front of a plain LDS read while a DMA is pending).
// One wave per workgroup: the ring is the wave's own.
#ifndef MI_TX_LDS_R
#define MI_TX_LDS_R 2  // 2 x 2 was the fastest (profiles/r06/tx_ab_r06.jsonl): deeper rings cost waves per CU
#endif
template <int U>
__device__ __forceinline__ void tx_ring_read(const u32x4 *slot, int lane, u32x4 (&xa)[U], u32x4 (&xb)[U]) {
  static_assert(U == 1 || U == 2, "ring reads for U = 1, 2");
  if constexpr (U == 1) {
    asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(xa[0]), "=&v"(xb[0])
                 : "v"(lds_addr(slot + lane)), "v"(lds_addr(slot + 64 + lane))
                 : "memory");
  } else {
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(xa[0]), "=&v"(xb[0]), "=&v"(xa[1]), "=&v"(xb[1])
        : "v"(lds_addr(slot + lane)), "v"(lds_addr(slot + 64 + lane)), "v"(lds_addr(slot + 128 + lane)),
          "v"(lds_addr(slot + 192 + lane))
        : "memory");
  }
}

#ifndef MI_TX_LDS_WAVES
#define MI_TX_LDS_WAVES 4  // waves per SIMD the register budget is held to
#endif
// (a deeper ring's LDS holds a CU below MI_TX_LDS_WAVES per SIMD anyway:
// 160 KiB / (2 U R KiB per wave) / 4 SIMDs)
constexpr int tx_lds_waves(int u, int r) {
  return 160 / (2 * u * r) / 4 < MI_TX_LDS_WAVES ? 160 / (2 * u * r) / 4 : MI_TX_LDS_WAVES;
}
// CC (cut cache): each chunk's cut (tx_cut: where its segments meet, the
// frame's ends, the slow case) is worked out once, when its pass is issued,
// and kept packed in LDS beside the ring for the build, instead of being
// computed again then (the SQ counters put the kernel's VALU ~60 % busy,
// profiles/r06/sq_counters_tx_r06.jsonl).
__device__ __forceinline__ void lds_wr32(const void *p, uint32_t x) {
  asm volatile("ds_write_b32 %0, %1" : : "v"(lds_addr(p)), "v"(x) : "memory");
}
template <int U>
__device__ __forceinline__ void lds_rd32_u(const uint32_t *row, int lane, uint32_t (&x)[U]) {
  static_assert(U == 1 || U == 2, "cut reads for U = 1, 2");
  if constexpr (U == 1) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(x[0]) : "v"(lds_addr(row + lane)) : "memory");
  } else {
    asm volatile("ds_read_b32 %0, %2\n\tds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(x[0]), "=&v"(x[1])
                 : "v"(lds_addr(row + lane)), "v"(lds_addr(row + 64 + lane))
                 : "memory");
  }
}
__device__ __forceinline__ uint32_t cut_pack(const TxCut &c) {
  return (uint32_t)(min(max(c.B, -1), 17) + 1) | (c.two ? 32u : 0u) | (c.clip ? 64u : 0u) | (c.slow ? 128u : 0u);
}
// (only what tx_build reads: q0, B and the three cases)
__device__ __forceinline__ TxCut cut_unpack(uint32_t k, int q0) {
  TxCut c;
  c.q0 = q0;
  c.B = (int)(k & 31u) - 1;
  c.A1 = c.A2 = 0;
  c.two = k & 32u;
  c.clip = k & 64u;
  c.slow = k & 128u;
  return c;
}
// (the body, shared by k_tx_lds and the AQL engine's mi_aql_tx_lds)
template <int U, int R, bool CC, int G = 8>
__device__ __forceinline__ void tx_lds_body(const TxDesc &t) {
  static_assert(G == 8 || G == 16, "8 or 16 lanes per frame (4: 0.38 of 8 TB/s, profiles/r06/tx_g4_ab_r06.jsonl)");
  constexpr uint32_t NG = 64 / G;  // frames (lane groups) per wave = per workgroup
  static_assert(R >= 2 && R <= 4, "ring depth");
  __shared__ uint32_t s_seg[NG][kTxSeg][2];
  __shared__ u32x4 s_ring[R][2 * U][64];  // pass slot q % R: chunk u's A1 loads, then its A2 loads
  __shared__ uint32_t s_cut[CC ? R : 1][CC ? U : 1][64];  // CC: pass slot q % R's packed cuts
  typedef __attribute__((address_space(3))) void *lds_ptr;
  Desc ds{}, dd{};
  ds.base = t.src;
  ds.bytes = t.src_bytes;
  dd.base = t.dst;
  dd.bytes = t.dst_bytes;
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(ds), rd = rsrc_of(dd);
  const TxArrs ta = tx_arrs(t);
  const int lane = threadIdx.x & (G - 1);
  const uint32_t grp = threadIdx.x / G;
  const uint32_t stride = gridDim.x * NG;
  uint32_t i = blockIdx.x * NG + grp;
  uint32_t len_c = 0, k0_c = 0, k1_c = 0;
  int32_t sl_c = 0;
  uint32_t so_c = 0;
  if (i < t.n) {
    len_c = ld_u32(ta.pkt_len, i);
    k0_c = ld_u32(ta.pkt_seg, i);
    k1_c = ld_u32(ta.pkt_seg, i + 1);
    if (k0_c + lane < k1_c) {
      sl_c = (int32_t)ld_u32(ta.seg_len, k0_c + lane);
      so_c = (uint32_t)ld_u64(ta.seg_off, k0_c + lane);
    }
  }
  for (; i < t.n; i += stride) {
    const uint32_t len = len_c;
    const uint32_t k0 = k0_c, k1 = k1_c;
    const int32_t sl0 = sl_c;
    const uint32_t so0 = so_c;
    const uint32_t in = i + stride;
    uint32_t len_n = 0, k0_n = 0, k1_n = 0;
    if (in < t.n) {
      len_n = ld_u32(ta.pkt_len, in);
      k0_n = ld_u32(ta.pkt_seg, in);
      k1_n = ld_u32(ta.pkt_seg, in + 1);
    }
    bool pre2 = false;
    auto prefetch2 = [&]() {
      if (pre2) return;
      pre2 = true;
      sl_c = 0;
      so_c = 0;
      if (in < t.n && k0_n + lane < k1_n) {
        sl_c = (int32_t)ld_u32(ta.seg_len, k0_n + lane);
        so_c = (uint32_t)ld_u64(ta.seg_off, k0_n + lane);
      }
      len_c = len_n;
      k0_c = k0_n;
      k1_c = k1_n;
    };
    const uint32_t l3 = t.l3;
    const uint32_t D = (uint32_t)(t.dst_first + (uint64_t)i * t.dst_stride);  // host-checked < 4 GiB
    const uint32_t h = D & 15u, c0 = D & ~15u;
    uint32_t st = len > t.room ? MI_TX_NOBUFS : 0u;
    // walk 1 (as k_tx_copy): bytes in the chain, the IP mbuf's m_len from the
    // IP header on, the first kTxSeg nonempty segments into LDS
    uint32_t total = 0, ip_mlen = 0, m = 0;
    for (uint32_t w = k0; w < k1 && !st; w += G) {
      const uint32_t k = w + lane;
      const uint32_t l = k < k1 ? (uint32_t)max(w == k0 ? sl0 : (int32_t)ld_u32(ta.seg_len, k), 0) : 0u;
      const uint32_t inc = group_scan<G>(l);
      const uint32_t a = total + inc - l, e = total + inc;
      const uint32_t nz = l ? 1u : 0u;
      const uint32_t zi = group_scan<G>(nz);
      const uint32_t idx = m + zi - nz;
      if (nz && idx < (uint32_t)kTxSeg) {
        s_seg[grp][idx][0] = a;
        s_seg[grp][idx][1] = (w == k0 ? so0 : (uint32_t)ld_u64(ta.seg_off, k)) - a;
      }
      const bool isip = l && a <= l3 && l3 < e;
      ip_mlen += group_sum<G>(isip ? e - l3 : 0u);  // leader only
      total += group_lane<G>(inc, G - 1);
      m += group_lane<G>(zi, G - 1);
    }
    if (!st && total < len) st = MI_TX_SHORT;
    if (st) {
      if (lane == 0) st_u8(ta.status, i, st);
      prefetch2();
      continue;
    }
    ip_mlen = group_lane<G>(ip_mlen, 0);
    const bool odd = (h + l3) & 1u;
    IpHdr ih{};
    bool ok = false, do_ip = false, do_l4 = false, udp = false, done = false;
    uint32_t at = 0;
    int hend = 0, lend = 0;
    uint32_t acc_t = 0, acc_h = 0, acc_f = 0;
    if (m <= (uint32_t)kTxSeg) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      static_assert(kTxSeg == 4, "segment registers S1..S3 / D0..D3");
      auto seg_start = [&](uint32_t e) { return e < m ? min((int)s_seg[grp][e][0], (int)len) : (int)len; };
      auto seg_delta = [&](uint32_t e) { return e < m ? s_seg[grp][e][1] : 0u; };
      const uint32_t nch = (h + len + 15u) >> 4;
      const uint32_t npass = (nch + G * U - 1) / (G * U);
      const int S1 = seg_start(1), S2 = seg_start(2), S3 = seg_start(3);
      const uint32_t D0 = seg_delta(0), D1 = seg_delta(1), D2 = seg_delta(2), D3 = seg_delta(3);
      const uint32_t lim = t.src_bytes - 16u;
      const TxSegs sg{S1, S2, S3, (int)len, D0, D1, D2, D3, lim};
      // pass q's 2U DMAs into ring slot q % R, if any lane of the wave has a
      // pass q (lanes past their frame's last pass, and loads a chunk does not
      // need, read nothing: offset kOOB).  gi counts the passes issued, pc
      // the passes consumed (both wave-uniform).
      uint32_t gi = 0, pc = 0;
      bool brk = false;
      auto issue = [&](uint32_t q) {
        if (!__any(q < npass)) return;
        ++gi;
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readfirstlane((int)(q % (uint32_t)R));
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const TxCut c = tx_cut(sg, q * (G * U) + u * G + lane, h);
          const bool live = q < npass && !c.slow;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)&s_ring[sl][2 * u][0], 16,
                                                  live && c.q0 < sg.L ? c.A1 : kOOB, 0, 0, MI_TX_LOAD_AUX);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)&s_ring[sl][2 * u + 1][0], 16,
                                                  live && c.two ? c.A2 : kOOB, 0, 0, MI_TX_LOAD_AUX);
          if constexpr (CC) lds_wr32(&s_cut[sl][u][threadIdx.x & 63u], cut_pack(c));
        }
      };
      u32x4 held{0, 0, 0, 0};
#pragma unroll
      for (int q = 0; q < R; ++q) issue((uint32_t)q);
      for (uint32_t p = 0; p < npass; ++p) {
        // pass p has landed: the DMAs of the gi - p - 1 passes issued after it
        // may still be in flight
        wait_vm_ladder<2 * U, R - 1>((uint32_t)__builtin_amdgcn_readfirstlane((int)(gi - pc - 1u)));
        ++pc;
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readfirstlane((int)(p % (uint32_t)R));
        u32x4 xa[U], xb[U], v[U];
        tx_ring_read<U>(&s_ring[sl][0][0], (int)threadIdx.x & 63, xa, xb);
        if constexpr (CC) {
          uint32_t pk[U];
          lds_rd32_u<U>(&s_cut[sl][0][0], (int)threadIdx.x & 63, pk);
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[u] = tx_build(sg, cut_unpack(pk[u], (int)(16u * (p * (G * U) + u * G + lane)) - (int)h), xa[u], xb[u], rs);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            v[u] = tx_build(sg, tx_cut(sg, p * (G * U) + u * G + lane, h), xa[u], xb[u], rs);
        }
        issue(p + R);  // the slot's reads have returned (lgkmcnt(0) in tx_ring_read)
        if (p == 0) {
          prefetch2();
          const u32x4 hv[1] = {v[0]};
          ih = parse_ipv4<G, 1>(hv, h + l3);
          const TxPlan pl = tx_plan(t, i, len, ih);
          ok = pl.ok;
          do_ip = pl.do_ip;
          do_l4 = pl.do_l4;
          udp = pl.udp;
          at = pl.at;
          hend = pl.hend;
          lend = pl.lend;
          const uint32_t pip = l3 + 10u, pl4 = l3 + at;
          const bool l4s = do_l4 && (uint64_t)at + 2u <= ip_mlen;
          const uint32_t need = max(do_ip ? pip + 2u : 0u, l4s ? pl4 + 2u : 0u);
          if ((uint64_t)need + h > 16ull * G) {  // a sum field beyond the held chunks: generic path
            brk = true;
            break;
          }
          done = true;
          held = v[0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t ci = p * (G * U) + u * G + lane;
          const int rel = (int)(16u * ci) - (int)(h + l3);
          fold_chunk(v[u], rel, lend, hend, hend > 20, acc_t, acc_h, acc_f);
          const int cs = (int)(16u * ci) - (int)h;
          if (ci < nch && !(p == 0 && u == 0)) store_chunk(rd, c0 + 16u * ci, v[u], -cs, (int)len - cs);
        }
      }
      if (npass == 0) {
        ok = do_ip = do_l4 = false;
        done = true;
      }
      if (done) {
        const bool l4_store = do_l4 && (uint64_t)at + 2u <= ip_mlen;
        uint32_t c_ip, c_l4;
        tx_sums<G>(acc_t, acc_h, acc_f, hend, ih, odd, udp, c_ip, c_l4);
        const uint32_t pip = l3 + 10u, pl4 = l3 + at;
        const int b0 = (int)h - (int)(16u * lane);
        if (do_ip) {
          if (pip < len) put_byte(held, (int)pip + b0, c_ip);
          if (pip + 1u < len) put_byte(held, (int)pip + 1 + b0, c_ip >> 8);
        }
        if (l4_store) {
          if (pl4 < len) put_byte(held, (int)pl4 + b0, c_l4);
          if (pl4 + 1u < len) put_byte(held, (int)pl4 + 1 + b0, c_l4 >> 8);
        }
        const uint32_t ci = lane;
        const int cs = (int)(16u * ci) - (int)h;
        if (ci < nch) store_chunk(rd, c0 + 16u * ci, held, -cs, (int)len - cs);
        if (lane == 0) st_u8(ta.status, i, (ok ? 0u : MI_TX_NOSUM) | (do_l4 && !l4_store ? MI_TX_L4_SKIPPED : 0u));
      }
      // Every pass the wave issued was below the longest frame's pass count,
      // so the groups with that frame have read them all -- unless a group
      // left for the generic path at p == 0: then passes issued for it may
      // still be in flight, and they land before the ring is written again or
      // the wave ends.  (gi / pc are equal in all lanes still in the loop,
      // stale in lanes that left it: they are not tested here.)
      if (__any(brk)) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
      __builtin_amdgcn_wave_barrier();
    }
    prefetch2();
    if (!done) tx_frame_generic<G, U>(t, rs, rd, i, lane, len, k0, k1, ip_mlen);
  }
}
template <int U, int R, int WV = tx_lds_waves(U, R), bool CC = false, int G = 8>
__global__ __launch_bounds__(64, WV) void k_tx_lds(TxDesc t) {
  tx_lds_body<U, R, CC, G>(t);
}
// Its grid: one wave (64 / G frames) per workgroup; for G = 8 the same total
// waves as k_tx_copy's 8 x 2 grid at the default cap (one frame group per
// wave at the bench's 65536 frames), for G = 16 twice as many.
inline unsigned tx_lds_grid(uint32_t n, unsigned copy_blocks, int G = 8) {
  const uint64_t ng = 64u / (unsigned)G;
  const uint64_t g = std::min<uint64_t>(((uint64_t)n + ng - 1u) / ng, 4ull * copy_blocks * (uint64_t)G / 8u);
  return g ? (unsigned)g : 1u;
}

#endif  // MI_TX_DEVICE_H
