/*
 * include/mi_cksum.h -- MI355X-native RFC 1071 Internet checksum: the C ABI.
 *
 * libmicksum.so (libunsod_amd/lib/) exports everything declared here.  Plain C,
 * plain pointers and sizes; no HIP or torch types cross the boundary (streams
 * are passed as void* hipStream_t, NULL = the default stream).
 *
 * Two levels, per SURVEY.md 8(b):
 *
 *  (b1) drop-in scalar entry points with the reference's exact names and
 *       signatures -- they replace the MACHINE_SRCS object in_cksum.o inside
 *       libuinet (src/lib/libuinet/Makefile:275-276) at link time.  They are
 *       scalar and synchronous (~0.13 us for an IPv4 header on one core), so
 *       by default they are served on the calling CPU (MI_DROPIN_HOST: the
 *       chain is folded in place by host_fold.c, no GPU, no allocation, no
 *       error) -- SURVEY.md 8(b1): "per-call GPU dispatch is not viable".
 *       MI_DROPIN_GPU (mi_cksum_set_dropin_mode, or MI_CKSUM_DROPIN=gpu in the
 *       environment) sends each call to the device's resident drop-in service
 *       instead -- one workgroup for all threads polling a mailbox slot per
 *       thread in VRAM the host writes through the PCIe BAR -- 2.7-3.3 us per
 *       in_cksum_hdr.  This level is the compatibility path;
 *       per-packet RX/TX throughput comes from (b2) at the burst /
 *       inject-ring batch points.
 *
 *  (b2) batch offload: a batch of packets that already sits in device memory
 *       (the RX burst / TX inject-ring batch points, uinet_if_dpdk.c:854-879 and
 *       :360-556) is folded by one kernel launch, asynchronously on `stream`.
 *
 * Results are bit-identical to the reference on the same bytes at the same
 * addresses (address parity matters only for in_cksum_hdr, in_cksum.c:278-285).
 * The batch calls (b2) have no CPU fallback: without a usable gfx950 device
 * they return -ENODEV.  The (b1) calls need no device in their default mode.
 */
#ifndef MI_CKSUM_H
#define MI_CKSUM_H

#include <stdint.h>

#include "mi_cksum_flags.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* (b1) drop-in entry points -- src/sys/amd64/include/in_cksum.h:44,77-83    */
/* ------------------------------------------------------------------------ */

/* Only m_next@0, m_data@16 and m_len@24 are read (src/sys/sys/mbuf.h:90-98,
 * 166-168); the chain is read-only.  struct ip is 20 bytes (netinet/ip.h). */
struct mbuf;
struct ip;

/* in_cksum.c:193-232 -- ~fold of bytes [skip, len) of the chain; a short chain
 * truncates silently; precondition 0 <= skip <= len. */
unsigned short in_cksum_skip(struct mbuf *m, int len, int skip);
#define in_cksum(m, len) in_cksum_skip((m), (len), 0)

/* in_cksum.c:241-276 -- L4 verify: pseudo-header (src, dst as loaded from the
 * header, protonum, (uint16_t)plen) + plen bytes from off0; 0 when valid.
 * Precondition: the first mbuf holds >= off0 bytes. */
uint16_t in_cksum_pseudo_header(struct mbuf *m, int plen, int off0, uint32_t src,
                                uint32_t dst, uint8_t protonum);

/* in_cksum.c:278-285 -- 20-byte IPv4 header, ABSOLUTE-address lanes: at an odd
 * address the result is byte-swapped relative to in_cksum (SURVEY KAT4). */
unsigned int in_cksum_hdr(const struct ip *ip);

/* in_cksum.c:181-191 -- non-complemented fold of three u32 (TX seed). */
unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c);

/* in_cksum.c:172-179 -- one's-complement add of two u16. */
unsigned short in_addword(unsigned short a, unsigned short b);

/* (b1) serving mode, process-wide:
 *   MI_DROPIN_HOST (default) -- folded on the calling CPU, in place over the
 *     chain (libunsod_amd/csrc/host_fold.c); never fails, needs no device;
 *   MI_DROPIN_GPU -- through the device's resident drop-in service (or one
 *     AQL dispatch per call with MI_CKSUM_DROPIN_SERVICE=0).
 * The environment's MI_CKSUM_DROPIN=gpu|host sets the initial mode.  Returns
 * the previous mode, or -EINVAL. */
#define MI_DROPIN_HOST 0
#define MI_DROPIN_GPU 1
int mi_cksum_set_dropin_mode(int mode);

/* (b1) error policy.  The reference's functions cannot fail and return only
 * the sum.  In MI_DROPIN_GPU mode a call whose GPU request fails (no device,
 * a queue error, no result within 10 s) is served by the host fold instead --
 * the same bits -- and counted (mi_cksum_dropin_degraded); a handler installed
 * here is told first, with the function name and mi_cksum_strerror().  NULL
 * removes it.  Nothing aborts.  Process-wide. */
typedef void (*mi_cksum_error_fn)(const char *what, const char *err);
void mi_cksum_set_dropin_error_handler(mi_cksum_error_fn fn);
/* GPU-mode drop-in calls an error sent to the host fold, since start. */
uint64_t mi_cksum_dropin_degraded(void);

/* ------------------------------------------------------------------------ */
/* runtime                                                                    */
/* ------------------------------------------------------------------------ */

/* Number of HIP devices visible (0 when none / no driver). */
int mi_cksum_device_count(void);
/* Bind the calling thread to `device` (hipSetDevice) and create its context.
 * 0 or -errno (-ENODEV: no such device or not gfx950). */
int mi_cksum_init(int device);
/* Text of the last error on this thread ("" if none). */
const char *mi_cksum_strerror(void);
const char *mi_cksum_version(void);
/* Diagnostics: HSA queues the library holds right now -- two (nstreams) per
 * AQL-engine repeat handle, one per thread that made a drop-in or host-burst
 * call (given back when that thread exits or moves to another device). */
int mi_cksum_hsa_queues(void);

/* Tuning knob (process-wide): force the lane-group shape -- `group` lanes per
 * packet, `chunks` 16-byte loads per lane per pass -- and cap the grid at
 * `max_blocks` workgroups.  0, 0, 0 restores the automatic choice.  Shapes
 * change speed only, never results.  -EINVAL for a shape not compiled in. */
int mi_cksum_set_shape(int group, int chunks, int max_blocks);
/* Tuning knob (process-wide): the flat-run kernel that verifies packed
 * batches with an offset array -- `chunks` = 0: the register-streaming one
 * (k_ipv4_verify_packed, the default); otherwise the LDS-DMA one
 * (k_ipv4_verify_run_dma) with `chunks` 16-byte chunks per lane per pass and
 * a ring of `slots` passes per wave (2x3, 2x4, 4x2, 4x3 are compiled in;
 * MI_CKSUM_RUN_DMA=UxR sets the initial choice).  Speed only, never results.
 * -EINVAL for a shape not compiled in. */
int mi_cksum_set_run_kernel(int chunks, int slots);

/* ------------------------------------------------------------------------ */
/* (b2) batch offload                                                         */
/* ------------------------------------------------------------------------ */

/*
 * A batch of n packets (or spans) inside one device-resident buffer.
 *   base      16-byte aligned device pointer; [base, base + roundup16(bytes))
 *             must be readable (the kernels load whole 16-byte chunks and rely
 *             on the hardware bounds check of `bytes` for anything beyond).
 *   bytes     buffer size, <= MI_BATCH_MAX_BYTES (2^32 - 8192: every byte
 *             offset and the bounds-checked tail stay 32-bit).
 *   Packet i starts at base + (offs ? offs[i] : first_off + i * stride) and is
 *   lens[i] (or fixed_len) bytes long.  offs / lens are device arrays.
 *   max_len   upper bound of lens[] (0 = unknown); sizes the lane groups.
 *   flags     MI_BATCH_PACKED: a hint that offs[] ascend and the datagrams sit
 *             back to back (gaps < 64 B), e.g. a mixed-length batch packed at
 *             8-byte offsets; verify then streams each 64-datagram range as one
 *             flat run.  Ranges that turn out not packed are still verified
 *             correctly (per-datagram fallback), only slower.
 * Spans outside [0, bytes) read as zero bytes (hardware bounds check), never
 * fault.
 */
#define MI_BATCH_MAX_BYTES 0xFFFFE000ull
/* At most this many packets (spans, chains, frames) per batch: every
 * per-packet array -- offsets (8 B each), lengths, outputs -- is read and
 * written through a buffer resource with 32-bit byte offsets (-E2BIG). */
#define MI_BATCH_MAX_N 0x1FFFFE00u
typedef struct mi_pkt_batch {
	void           *base;
	uint64_t        bytes;
	union {                         /* device (or, _host calls, host) array */
		const uint64_t *offs;   /* n u64 offsets */
		const uint32_t *offs32; /* n u32 offsets, with MI_BATCH_OFFS32 */
	};
	uint64_t        stride;
	uint64_t        first_off;
	const uint32_t *lens;
	uint32_t        fixed_len;
	uint32_t        n;
	uint32_t        max_len;
	uint32_t        flags;
} mi_pkt_batch;

#define MI_BATCH_PACKED 1u
/* MI_BATCH_DEMUX: verify / finalize take each datagram's L4 checksum the way
 * ip_input's protocol switch hands it on (the
 * small-header callers): TCP / UDP with the pseudo header, ICMP / IGMP / CARP
 * plain in_cksum, fragments and other protocols none.  See
 * mi_cksum_ipv4_verify and mi_cksum_ipv4_finalize. */
#define MI_BATCH_DEMUX  2u
/* MI_BATCH_HOST_STAGED: mi_cksum_ipv4_verify_host copies through device
 * staging even when the batch is registered (mapped) host memory. */
#define MI_BATCH_HOST_STAGED 4u
/* MI_BATCH_OFFS32: the offsets are n uint32_t at `offs32` (same storage as
 * `offs`) -- 4 descriptor bytes per packet instead of 8, which a mixed-length
 * batch of ~280 B datagrams reads beside its payload.  Any batch (<=
 * MI_BATCH_MAX_BYTES) can use it; results are identical to u64 offsets of
 * the same values.  An offset >= `bytes` is out of range either way
 * (the datagram reads as zeros and is reported MALFORMED). */
#define MI_BATCH_OFFS32 8u

/* Lane conventions for mi_cksum_span_batch. */
#define MI_SPAN_STREAM 0u  /* in_cksum_skip / in_cksum_pseudo_header: lanes
                              relative to the span start (in_cksum.c:222-225) */
#define MI_SPAN_ABS    1u  /* in_cksum_hdr: lanes by absolute address (:278-285) */

/*
 * Per span: out[i] = ~fold( seed_i + S(span i) ) & 0xffff, where
 *   seed_i = (seeds ? seeds[i] : 0)
 *          + (src ? src[i] + dst[i] + (proto[i] << 8) + bswap16(plen_i & 0xffff) : 0)
 *   plen_i = plens ? plens[i] : span length          (in_cksum.c:252-253)
 * so MI_SPAN_STREAM with no seeds == in_cksum_skip over a one-mbuf chain, and
 * with src/dst/proto == in_cksum_pseudo_header(m, plen, off0, ...) where the
 * span starts at off0.  All arrays are device pointers; out is n u16.
 */
typedef struct mi_span_seeds {
	const uint32_t *seeds;
	const uint32_t *src;
	const uint32_t *dst;
	const uint8_t  *proto;
	const uint32_t *plens;
} mi_span_seeds;

int mi_cksum_span_batch(const mi_pkt_batch *b, uint32_t lanes, const mi_span_seeds *seeds,
                        uint16_t *out, void *stream);

/*
 * Scatter-gather: checksums over mbuf chains, batched (the TX socket-buffer
 * chains of 2-4 KiB clusters, jumbo frames over several rte_mbufs).  Every
 * segment's bytes sit in one device buffer; packet i's chain is segments
 * [pkt_seg[i], pkt_seg[i+1]) -- pkt_seg has n + 1 entries -- with
 * seg_off[k] / seg_len[k] standing for m_data / m_len (mbuf.h:166-168).
 *   MI_CHAIN_SKIP:   out[i] = in_cksum_skip(chain_i, len[i], skip[i])
 *   MI_CHAIN_PSEUDO: out[i] = in_cksum_pseudo_header(chain_i, len[i] (plen),
 *                             skip[i] (off0), src[i], dst[i], proto[i])
 * with the reference's walk: leading skip across segments, zero-length mbufs
 * ignored, a short chain truncates silently (in_cksum.c:193-276).  All arrays
 * are device pointers.  max_seg: longest segment (0 = unknown).
 */
#define MI_CHAIN_SKIP   0u
#define MI_CHAIN_PSEUDO 1u
typedef struct mi_chain_batch {
	void           *base;
	uint64_t        bytes;
	const uint64_t *seg_off;
	const int32_t  *seg_len;
	const uint32_t *pkt_seg;
	uint32_t        n;
	uint32_t        mode;
	const int32_t  *len;
	const int32_t  *skip;
	const uint32_t *src;
	const uint32_t *dst;
	const uint8_t  *proto;
	uint32_t        max_seg;
	uint32_t        nseg;   /* entries of seg_off / seg_len; 0 = unknown: the
	                           allocation holding each table bounds it */
} mi_chain_batch;

int mi_cksum_chain_batch(const mi_chain_batch *b, uint16_t *out, void *stream);

/* Per-packet status bits (the observable outputs the reference counts:
 * ips_badsum ip_input.c:469, tcps_rcvbadsum tcp_input.c:717-720). */
#define MI_ST_IP_BAD    1u
#define MI_ST_L4_BAD    2u
#define MI_ST_MALFORMED 4u
#define MI_ST_L4_NONE   8u  /* MI_BATCH_DEMUX: no L4 checksum applies */

/*
 * RX verify of IPv4 datagrams (ip_input.c:459-471 + tcp_input.c:697-720 /
 * udp_usrreq.c:440-442), one pass over each datagram.  lens = bytes the NIC
 * delivered from the IP header on (frame length after Ethernet).
 *   hl = ip_hl*4, ip_len = ntohs(ip_len)
 *   flen < 20 || hl < 20 || hl > flen  -> ip = l4 = 0, MALFORMED
 *   ip = (hl == 20) ? in_cksum_hdr(ip) : in_cksum(m, hl)
 *   ip_len < hl || ip_len > flen       -> l4 = 0, MALFORMED
 *   else l4 = in_cksum_pseudo_header(m, ip_len - hl, hl, ip_src, ip_dst, ip_p)
 * With MI_BATCH_DEMUX in b->flags, l4 is instead what the protocol's input
 * routine tests (0 = accept), plen = ip_len - hl, the mbuf trimmed to ip_len
 * (ip_input.c:500-505):
 *   fragment (IP_MF or an offset)       -> l4 = 0, L4_NONE (summed after ip_reass)
 *   TCP  plen < 20 -> MALFORMED (tcps_rcvshort, tcp_input.c:688-693); else as above
 *   UDP  plen < 8 -> MALFORMED (udps_hdrops, udp_usrreq.c:375-381);
 *        uh_ulen > plen or < 8 -> MALFORMED (udps_badlen, :406-414), shorter
 *        -> trimmed to uh_ulen; uh_sum == 0 -> L4_NONE (udps_nosum, :429,451);
 *        else in_cksum_pseudo_header(m, uh_ulen, hl, src, dst, 17)   (:440-442)
 *   ICMP plen < 36 -> MALFORMED (the pullup to hl + min(icmplen,
 *        ICMP_ADVLENMIN) with icmplen = ntohs(ip_len), ip_icmp.c:336,374-378);
 *        else in_cksum(m + hl, ip_len), which the trimmed chain truncates to
 *        the plen ICMP bytes (ip_icmp.c:381-383)
 *   IGMP plen < 8 -> MALFORMED (igps_rcv_tooshort, igmp.c:1445-1452);
 *        else in_cksum(m + hl, plen)                                 (:1475-1478)
 *   CARP (112) plen < 36 -> MALFORMED (carps_badlen, ip_carp.c:600-607);
 *        else in_cksum(m + hl, 36) -- the header only                (:641-643)
 *   other protocols                     -> l4 = 0, L4_NONE
 * Any output pointer may be NULL.  bad_count (device u32, may be NULL) gains
 * one per packet with a nonzero status other than L4_NONE alone.
 */
int mi_cksum_ipv4_verify(const mi_pkt_batch *b, uint16_t *ip_sum, uint16_t *l4_sum,
                         uint8_t *status, uint32_t *bad_count, void *stream);

/*
 * mi_cksum_ipv4_verify over nb <= 16 batches in ONE launch (same semantics per
 * batch; ip / l4 / status: arrays of nb device pointers, any may be NULL;
 * bad_count one device counter for all).  For a single RX queue with several
 * bursts queued: the grid's ramp-up and drain are paid once, not per batch.
 * Batches whose plan is not the lane-group kernel (packed, 64 B slots,
 * length classes) are verified by one launch each, with the same results.
 */
int mi_cksum_ipv4_verify_multi(const mi_pkt_batch *b, uint32_t nb, uint16_t *const *ip, uint16_t *const *l4,
                               uint8_t *const *status, uint32_t *bad_count, void *stream);

/* Diagnostics: the verify kernel mi_cksum_ipv4_verify launches for this batch
 * ("k_ipv4_verify_packed<4>", "k_ipv4_verify<16,6>", ...).  Thread-local
 * string, valid until the next call.  Needs no GPU. */
const char *mi_cksum_verify_plan(const mi_pkt_batch *b);

/*
 * RX offload at the driver's batch point (uinet_if_dpdk.c:854-879, before
 * uinet_pd_deliver_to_stack): verify the burst and produce, per datagram, the
 * m_pkthdr.csum_flags / csum_data a checksumming NIC would set, so the stack's
 * unchanged call sites take the offload branch with identical accept/drop
 * decisions and counters (ip_input.c:459-460, tcp_input.c:698-709,
 * udp_usrreq.c:431-438; if_loop.c:255-276 sets the same bits):
 *   well-formed header (see mi_cksum_ipv4_verify): CSUM_IP_CHECKED, plus
 *     CSUM_IP_VALID iff the header checksum verifies;
 *   TCP, or UDP with uh_ulen == ip_len - hl, not a fragment, ip_len <= flen:
 *     CSUM_DATA_VALID | CSUM_PSEUDO_HDR, csum_data = l4 ^ 0xffff (the folded
 *     pseudo-header sum; the stack's csum_data ^ 0xffff is then exactly
 *     in_cksum_pseudo_header's result);
 *   anything else: no flags, csum_data = 0 (the stack computes as before).
 * Values are mbuf.h:281-305's.  csum_data may be NULL; bad_count as above.
 */
/* (MI_CSUM_IP_CHECKED / _IP_VALID / _DATA_VALID / _PSEUDO_HDR: mi_cksum_flags.h) */
int mi_cksum_rx_offload(const mi_pkt_batch *b, uint32_t *csum_flags, uint32_t *csum_data,
                        uint32_t *bad_count, void *stream);

/*
 * Back-to-back submission (the RX burst loop, and the bench): launch `steps`
 * verify passes, pass k over batch b[k % nb] with outputs ip/l4/status[k % nb]
 * (arrays of nb device pointers; any array may be NULL), on the k % nstreams-th
 * of nstreams (1..8) library-owned non-blocking streams, so consecutive passes
 * can overlap (a pass's ramp-up runs under its predecessor's drain).  The passes
 * start after all work already queued on the legacy default stream.
 * timing: MI_TIME_NONE; MI_TIME_REGION -- one hipEvent before the first pass
 * and one after the last pass on every stream, *span_us = GPU time of all
 * passes; MI_TIME_PER_PASS -- every pass bracketed by events on its stream,
 * kernel_us[k] = its duration (overlap included) and *span_us as above.
 * Synchronous: returns once every pass has finished.  nb <= 16.
 */
#define MI_TIME_NONE     0u
#define MI_TIME_REGION   1u
#define MI_TIME_PER_PASS 2u
/* OR'ed into timing (with NONE or REGION): submit the passes as one hipGraph
 * (stream capture of the same launches, instantiated on first use and cached
 * per launch sequence), so consecutive passes cost no host launch overhead. */
#define MI_REPEAT_GRAPH  0x100u
int mi_cksum_ipv4_verify_repeat(const mi_pkt_batch *b, uint32_t nb, uint16_t *const *ip,
                                uint16_t *const *l4, uint8_t *const *status, uint32_t steps,
                                uint32_t nstreams, uint32_t timing, float *kernel_us,
                                float *span_us);

/*
 * The same submission, prepared once (the RX queue loop that re-submits the
 * same rings): descriptors, kernel plans, nstreams (1..8) non-blocking streams
 * and events are resolved by mi_cksum_repeat_create, so mi_cksum_repeat_run
 * costs only its launches and the wait.  Run k of the handle continues the
 * batch rotation where the previous run stopped.
 *   flags  MI_TIME_REGION: events bracket the run's passes; *span_us (if not
 *            NULL) = their GPU span, or read it later with mi_cksum_repeat_span
 *            (keeps the elapsed-time queries out of a caller's timed region);
 *          MI_REPEAT_AFTER_DEFAULT: order after the work queued on the legacy
 *            default stream (otherwise the run starts at once: the caller
 *            orders earlier producers, e.g. by synchronizing);
 *          MI_REPEAT_ASYNC: return after submission (mi_cksum_repeat_span
 *            then waits and reads the span of a timed run).
 * The handle belongs to the device current at create time; one thread at a
 * time.  nb <= 1024.  Destroy waits for its streams.
 */
#define MI_REPEAT_AFTER_DEFAULT 0x200u
#define MI_REPEAT_ASYNC         0x400u
typedef struct mi_repeat mi_repeat;
int mi_cksum_repeat_create(const mi_pkt_batch *b, uint32_t nb, uint16_t *const *ip, uint16_t *const *l4,
                           uint8_t *const *status, uint32_t nstreams, mi_repeat **out);
int mi_cksum_repeat_run(mi_repeat *r, uint32_t steps, uint32_t flags, float *span_us);
int mi_cksum_repeat_span(mi_repeat *r, float *span_us);
void mi_cksum_repeat_destroy(mi_repeat *r);
/* What each pass runs: MI_REPEAT_OP_VERIFY (default, mi_cksum_ipv4_verify
 * into the outputs given at create) or MI_REPEAT_OP_FINALIZE
 * (mi_cksum_ipv4_finalize in place; outputs unused). */
#define MI_REPEAT_OP_VERIFY   0u
#define MI_REPEAT_OP_FINALIZE 1u
#define MI_REPEAT_OP_TX_COPY  2u  /* set by mi_cksum_tx_repeat_create only */
int mi_cksum_repeat_set_op(mi_repeat *r, uint32_t op);
/* How a run submits its passes.
 * MI_REPEAT_ENGINE_HIP (default): HIP launches alternating over the handle's
 *   nstreams streams.
 * MI_REPEAT_ENGINE_AQL: the kernel arguments and one AQL dispatch packet per
 *   batch are built once, here; a run copies its passes' packets into the
 *   handle's own HSA queues, rings the
 *   doorbell and spins on one completion signal.  Pass k goes to queue
 *   k % nqueues (nqueues = nstreams, 1..4); each queue runs its passes in
 *   order and the queues overlap, as the HIP engine's streams do.  Same
 *   kernels, same results.
 *   Verify passes of uniform, packed and 64-byte-slot batches (not
 *   length-class batches: -ENOTSUP).  A run does not order itself after HIP
 *   streams: complete the batches' producers first (or pass
 *   MI_REPEAT_AFTER_DEFAULT: a host-side wait on the legacy default stream).
 *   Results reach L2 and HBM with the packets' system-scope release.
 * Returns 0, -ENOTSUP / -ENOENT when the engine cannot serve the handle. */
#define MI_REPEAT_ENGINE_HIP 0u
#define MI_REPEAT_ENGINE_AQL 1u
int mi_cksum_repeat_set_engine(mi_repeat *r, uint32_t engine);

/*
 * Completion waits on the calling thread's current device busy-poll (on != 0:
 * hipDeviceScheduleSpin) or return to the runtime's default heuristic (0).
 * A polling RX loop -- like the reference's dpdk_rx kthread spinning on
 * rte_eth_rx_burst (uinet_if_dpdk.c:900-937) -- wants the wake-up latency of
 * a spin (~1 us) rather than a blocked wait's (~15-20 us on MI355X,
 * profiles/bench_regions_r02.jsonl).  Device-wide in the process.
 */
int mi_cksum_set_busy_wait(int on);

/*
 * TX finalize in place (ip_output.c:649-672 + in_delayed_cksum :958-983):
 * for TCP/UDP c = in_cksum_skip(m, ip_len, hl) over the pre-seeded L4 header
 * (UDP: 0 -> 0xffff) stored at hl + (TCP 16 | UDP 6) when inside lens[i]; then
 * ip_sum = in_cksum(m, hl) with the ip_sum field taken as 0.  Malformed
 * datagrams (as above) are left untouched.
 * With MI_BATCH_DEMUX: fragments get ip_sum only (ip_fragment sums the whole
 * datagram before cutting it and each piece's header after, ip_output.c:
 * 930,950); TCP / UDP as above; the small-header senders store a plain
 * in_cksum over their message with the sum field taken as 0:
 *   ICMP plen >= 8:  icmp_cksum at hl + 2 over plen bytes    (ip_icmp.c:889-891)
 *   IGMP plen >= 8:  igmp_cksum at hl + 2 over plen bytes    (igmp.c:2184-2185, :3483)
 *   CARP plen >= 36: carp_cksum at hl + 6 over 36 bytes      (ip_carp.c:944,985)
 * other protocols: ip_sum only.
 */
int mi_cksum_ipv4_finalize(const mi_pkt_batch *b, void *stream);

/*
 * TX checksum offload fused with the driver's copy.
 * The interface advertises if_hwassist = CSUM_IP | CSUM_TCP | CSUM_UDP, so
 * ip_output leaves ip_sum = 0 and the L4 field holding the in_pseudo seed
 * (ip_output.c:649-672, tcp_output.c:1084), and the driver's copy of every
 * outgoing frame into its rte_mbuf (m_copydata(m, 0, len, rm_data),
 * uinet_if_dpdk.c:594-597) computes and stores the sums on the way.  The
 * bytes that reach each slot are exactly what the software stack would put on
 * the wire:
 *   pkt_len[i] > room             -> MI_TX_NOBUFS, slot untouched (uinet_if_dpdk.c:585-591)
 *   chain holds < pkt_len bytes    -> MI_TX_SHORT, slot untouched (m_copydata's KASSERT)
 *   slot[0, len) = the chain's first len bytes
 *   IPv4 header at l3_off malformed (hl < 20, hl or ip_len beyond the frame,
 *   ip_len < hl)                  -> MI_TX_NOSUM, copy only
 *   csum_flags & (CSUM_TCP|CSUM_UDP): in_delayed_cksum (ip_output.c:958-983):
 *       c = in_cksum_skip(ip, ip_len, hl), CSUM_UDP: 0 -> 0xffff, stored at
 *       hl + csum_data iff those 2 bytes lie inside the IP mbuf's m_len (the
 *       segment holding frame byte l3_off, from there on), else MI_TX_L4_SKIPPED
 *   csum_flags & CSUM_IP: ip_sum = in_cksum(ip, hl) with ip_sum taken as 0
 *   (ip_output.c:667-672).  Stores beyond len never reach the slot.
 * csum_flags NULL: CSUM_IP, plus CSUM_TCP / CSUM_UDP by ip_p; csum_data NULL:
 * 16 for CSUM_TCP, 6 otherwise (tcp_output.c:1066, udp_usrreq.c:1240).
 * Segments (m_data = src + seg_off[k], m_len = seg_len[k], negative = 0) must
 * lie inside [src, src + src_bytes); frame i has segments
 * [pkt_seg[i], pkt_seg[i+1]) and lands at dst + dst_first + i * dst_stride.
 * src, dst 16-byte aligned, both <= MI_BATCH_MAX_BYTES; l3_off <= 64.  status: n bytes.
 */
/* (MI_CSUM_IP / _TCP / _UDP: mi_cksum_flags.h) */
#define MI_TX_NOBUFS     1u
#define MI_TX_SHORT      2u
#define MI_TX_NOSUM      4u
#define MI_TX_L4_SKIPPED 8u
typedef struct mi_tx_batch {
	const void     *src;
	uint64_t        src_bytes;
	const uint64_t *seg_off;
	const int32_t  *seg_len;
	const uint32_t *pkt_seg;
	const uint32_t *pkt_len;
	const uint32_t *csum_flags;
	const uint32_t *csum_data;
	void           *dst;
	uint64_t        dst_bytes;
	uint64_t        dst_stride;
	uint64_t        dst_first;
	uint32_t        room;
	uint32_t        l3_off;
	uint32_t        n;
	uint32_t        max_len;
} mi_tx_batch;

int mi_cksum_tx_copy(const mi_tx_batch *b, uint8_t *status, void *stream);

/*
 * mi_cksum_tx_copy for frames in HOST memory -- the driver's real situation:
 * the socket-buffer chains and the rte_mbuf data rooms are hugepage host
 * memory (if_dpdk_transmit, uinet_if_dpdk.c:583-597).  b->src, b->dst, every
 * descriptor array and status are host pointers; same rules, same bytes in
 * the slots, same status as mi_cksum_tx_copy.  Synchronous.
 *   zero-copy -- [src, src + src_bytes) and [dst, dst + dst_bytes) inside
 *     ranges registered with mi_cksum_host_register: the kernel gathers the
 *     chains over PCIe and writes the slots in place (descriptors and status
 *     through mapped host memory: one dispatch, one wait);
 *   staged -- otherwise, or with MI_TX_HOST_STAGED: source and slot region
 *     copied to device memory and back around the same kernel.
 */
#define MI_TX_HOST_STAGED 1u
int mi_cksum_tx_copy_host(const mi_tx_batch *b, uint8_t *status, uint32_t flags);

/*
 * mi_cksum_tx_copy prepared once for a transmit loop that re-submits the same
 * rings (the mi_cksum_repeat_* handle, op MI_REPEAT_OP_TX_COPY): pass k copies
 * batch b[k % nb] with its sums into its slots, status into status[k % nb]
 * (device arrays), over the handle's nstreams streams; run / span / destroy
 * as for a verify handle.  mi_cksum_repeat_set_engine(r, MI_REPEAT_ENGINE_AQL)
 * sends the passes as prebuilt AQL packets of the default TX kernel
 * (-ENOTSUP while MI_CKSUM_TX_KERNEL / _TX_LDS / _TX_SHAPE select another).
 * Same bytes and status as mi_cksum_tx_copy.  nb <= 1024, every batch n > 0.
 */
int mi_cksum_tx_repeat_create(const mi_tx_batch *b, uint32_t nb, uint8_t *const *status,
                              uint32_t nstreams, mi_repeat **out);

/*
 * Host-resident batch (the path's real start and end: DPDK mbufs in host
 * memory).  b->base / offs / lens are HOST pointers; outputs are host arrays.
 * Synchronous: returns when outputs are written.  Two ways across PCIe:
 *   zero-copy -- base 16-byte aligned and [base, base + roundup16(bytes))
 *     inside a range registered with mi_cksum_host_register: the verify
 *     kernel reads the datagrams in place over the link (no staging copy, no
 *     DMA engine, slot gaps never cross); descriptors go H2D once;
 *   staged -- otherwise, or with MI_BATCH_HOST_STAGED: the batch is cut into
 *     chunks copied to device staging and verified on a ring of streams
 *     (H2D || kernel || D2H; fixed slots copied pitched, envelopes only).
 */
int mi_cksum_ipv4_verify_host(const mi_pkt_batch *b, uint16_t *ip_sum, uint16_t *l4_sum,
                              uint8_t *status, uint32_t *bad_count);

/* The RX offload of mi_cksum_rx_offload for a host-resident burst -- the
 * driver-side hook at the DPDK batch point (uinet_if_dpdk.c:854-879), where
 * the burst sits in hugepage mbufs: csum_flags / csum_data are host arrays
 * of n u32 (csum_data may be NULL).  Same transport rules as
 * mi_cksum_ipv4_verify_host.  Synchronous. */
int mi_cksum_rx_offload_host(const mi_pkt_batch *b, uint32_t *csum_flags, uint32_t *csum_data,
                             uint32_t *bad_count);

/* Page-lock and map / unlock a host range for mi_cksum_ipv4_verify_host
 * (hipHostRegister, mapped + portable).  The runtime locks whole pages, so
 * a range may not share a page with another registered range (-EEXIST);
 * unregister takes the exact pointer that was registered (-ENOENT
 * otherwise) and must come before the memory is freed.  Register memory the
 * caller owns page by page -- DPDK hugepages, an mmap -- not a sub-range of a
 * malloc heap block. */
int mi_cksum_host_register(void *p, uint64_t bytes);
int mi_cksum_host_unregister(void *p);

/* ------------------------------------------------------------------------ */
/* workload generator (bench / tests; not part of the reference API)          */
/* ------------------------------------------------------------------------ */

/*
 * Fill a device batch with synthetic IPv4/TCP datagrams:
 * payload from splitmix64(seed ^ (byte_index / 8)) over the whole buffer, then
 * per packet a v4/IHL5 header (ip_len = len, TTL 64, proto 6, DF,
 * src 10.0.(i>>8).(i&255), dst 10.1.(i>>8).(i&255)) and a 20 B TCP header whose
 * th_sum holds the in_pseudo seed (tcp_output.c:1063-1085); ip_sum = 0.
 * Follow with mi_cksum_ipv4_finalize to get valid packets.
 */
int mi_cksum_synth_ipv4(const mi_pkt_batch *b, uint64_t seed, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MI_CKSUM_H */
