/*
 * oracle/batch_driver.c -- drives the scalar checksum functions over packet
 * batches the way the reference's protocol code calls them.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Compiled twice by oracle/Makefile:
 *   -DPFX=orc_  against the restatement (cksum_oracle.c)
 *   -DPFX=ref_  against the reference's own in_cksum.o (symbols renamed ref_*)
 *
 * Call patterns restated:
 *   RX  ip_input.c:459-471   hlen == 20 ? in_cksum_hdr(ip) : in_cksum(m, hlen)
 *       tcp_input.c:697,714  tlen = ntohs(ip_len) - off0;
 *                            in_cksum_pseudo_header(m, tlen, off0, src, dst, p)
 *   TX  ip_output.c:649-654 -> in_delayed_cksum (ip_output.c:958-983):
 *                            in_cksum_skip(m, ip_len, hl<<2), UDP 0 -> 0xffff,
 *                            stored at hl + csum_data (TCP 16, UDP 6) if inside m_len
 *       ip_output.c:667-672  ip_sum = 0; ip_sum = in_cksum(m, hlen)
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define F(name) CAT(PFX, name)

/* The scalar functions this build drives (orc_* or ref_*). */
uint16_t F(in_cksum_skip)(struct orc_mbuf *m, int len, int skip);
uint16_t F(in_cksum_pseudo_header)(struct orc_mbuf *m, int plen, int off0,
                                   uint32_t src, uint32_t dst, uint8_t protonum);
unsigned F(in_cksum_hdr)(const void *ip);

/* A full 256-byte mbuf, as the reference allocates (param.h:159 MSIZE). */
union drv_mbuf {
	struct orc_mbuf m;
	char pad[256];
};

static inline uint64_t pkt_off(const uint64_t *offs, uint64_t stride,
                               uint64_t first_off, uint32_t i)
{
	return offs ? offs[i] : first_off + (uint64_t)i * stride;
}

static inline uint32_t ld32(const uint8_t *p)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return v;
}

struct job {
	const uint8_t *base;
	uint8_t *wbase;
	const uint64_t *offs;
	uint64_t stride, first_off;
	const uint32_t *flen;
	uint32_t fixed_flen, lo, hi;
	uint16_t *ip_out, *l4_out;
	uint8_t *status;
	int demux;
};

static inline uint32_t be16(const uint8_t *p)
{
	return ((uint32_t)p[0] << 8) | p[1];
}

/*
 * MI_BATCH_DEMUX: the L4 value the protocol input
 * routine ip_input hands the datagram to would test, called the way that
 * routine calls the checksum.  ip_input has trimmed the mbuf to ip_len
 * (ip_input.c:500-505); the length checks are the routines' own drops.
 */
static uint16_t demux_l4(const uint8_t *ip, uint32_t hl, uint32_t iplen, uint8_t *st)
{
	union drv_mbuf mb, mp;
	const uint32_t plen = iplen - hl;
	uint32_t ulen;
	memset(&mb, 0, sizeof(mb));
	mb.m.m_data = (char *)ip;
	mb.m.m_len = (int32_t)iplen;
	/* the protocol header's mbuf view: m_data += hlen; m_len -= hlen */
	memset(&mp, 0, sizeof(mp));
	mp.m.m_data = (char *)ip + hl;
	mp.m.m_len = (int32_t)plen;
	if (be16(ip + 6) & 0x3fff) {	/* IP_MF | IP_OFFMASK: ip_reass (ip_input.c:759-770) */
		*st |= ORC_ST_L4_NONE;
		return 0;
	}
	switch (ip[9]) {
	case 6:		/* tcp_input.c:688-693 (pullup fails: tcps_rcvshort), :697-716 */
		if (plen < 20)
			break;
		return F(in_cksum_pseudo_header)(&mb.m, (int)plen, (int)hl,
		    ld32(ip + 12), ld32(ip + 16), 6);
	case 17:	/* udp_usrreq.c:375-381 (udps_hdrops), :406-414, :429-451 */
		if (plen < 8)
			break;
		ulen = be16(ip + hl + 4);
		if (ulen != plen) {
			if (ulen > plen || ulen < 8)
				break;	/* udps_badlen */
			mb.m.m_len = (int32_t)(hl + ulen);	/* m_adj(m, len - ip_len) */
		}
		if (be16(ip + hl + 6) == 0) {	/* udps_nosum */
			*st |= ORC_ST_L4_NONE;
			return 0;
		}
		return F(in_cksum_pseudo_header)(&mb.m, (int)ulen, (int)hl,
		    ld32(ip + 12), ld32(ip + 16), 17);
	case 1:		/* ip_icmp.c:336 icmplen = ntohs(ip_len); :374-378 pullup to
			   hlen + min(icmplen, ICMP_ADVLENMIN) of an ip_len-byte packet */
		if (iplen < hl + (iplen < 36 ? iplen : 36))
			break;
		return F(in_cksum_skip)(&mp.m, (int)iplen, 0);	/* :381-383, truncates */
	case 2:		/* igmp.c:1445-1452, :1475-1478 */
		if (plen < 8)
			break;
		return F(in_cksum_skip)(&mp.m, (int)plen, 0);
	case 112:	/* ip_carp.c:600-607 (carps_badlen), :641-643 */
		if (plen < 36)
			break;
		return F(in_cksum_skip)(&mp.m, 36, 0);
	default:
		*st |= ORC_ST_L4_NONE;
		return 0;
	}
	*st |= ORC_ST_MALFORMED;
	return 0;
}

static void verify_range(const struct job *j)
{
	for (uint32_t i = j->lo; i < j->hi; i++) {
		const uint8_t *ip = j->base + pkt_off(j->offs, j->stride, j->first_off, i);
		uint32_t fl = j->flen ? j->flen[i] : j->fixed_flen;
		uint16_t ipsum = 0, l4 = 0;
		uint8_t st = 0;
		union drv_mbuf mb;
		memset(&mb, 0, sizeof(mb));
		mb.m.m_data = (char *)ip;
		mb.m.m_len = (int32_t)fl;
		if (fl < 20) {
			st = ORC_ST_MALFORMED;
		} else {
			uint32_t hl = (uint32_t)(ip[0] & 0x0f) << 2;
			uint32_t iplen = ((uint32_t)ip[2] << 8) | ip[3];
			if (hl < 20 || hl > fl) {
				st = ORC_ST_MALFORMED;
			} else {
				ipsum = (hl == 20) ? (uint16_t)F(in_cksum_hdr)(ip)
				                   : F(in_cksum_skip)(&mb.m, (int)hl, 0);
				if (iplen < hl || iplen > fl)
					st |= ORC_ST_MALFORMED;
				else if (j->demux)
					l4 = demux_l4(ip, hl, iplen, &st);
				else
					l4 = F(in_cksum_pseudo_header)(&mb.m, (int)(iplen - hl),
					    (int)hl, ld32(ip + 12), ld32(ip + 16), ip[9]);
				if (ipsum)
					st |= ORC_ST_IP_BAD;
				if (l4)
					st |= ORC_ST_L4_BAD;
			}
		}
		if (j->ip_out)
			j->ip_out[i] = ipsum;
		if (j->l4_out)
			j->l4_out[i] = l4;
		if (j->status)
			j->status[i] = st;
	}
}

static void finalize_range(const struct job *j)
{
	for (uint32_t i = j->lo; i < j->hi; i++) {
		uint8_t *ip = j->wbase + pkt_off(j->offs, j->stride, j->first_off, i);
		uint32_t fl = j->flen ? j->flen[i] : j->fixed_flen;
		uint32_t hl, iplen;
		union drv_mbuf mb;
		if (fl < 20)
			continue;
		hl = (uint32_t)(ip[0] & 0x0f) << 2;
		iplen = ((uint32_t)ip[2] << 8) | ip[3];
		if (hl < 20 || hl > fl || iplen < hl || iplen > fl)
			continue;
		memset(&mb, 0, sizeof(mb));
		mb.m.m_data = (char *)ip;
		mb.m.m_len = (int32_t)fl;
		if (j->demux && (be16(ip + 6) & 0x3fff)) {
			/* a fragment: ip_fragment sums the whole datagram
			   before cutting it (ip_output.c:930,950) */
		} else if (j->demux && (ip[9] == 1 || ip[9] == 2 || ip[9] == 112)) {
			/* icmp_send ip_icmp.c:889-891, igmp.c:2184-2185 / :3483,
			   carp_send_ad ip_carp.c:944,985: field = 0, in_cksum
			   over the message from the header on */
			const uint32_t plen = iplen - hl, carp = ip[9] == 112;
			if (plen >= (carp ? 36u : 8u)) {
				union drv_mbuf mp;
				uint8_t *f = ip + hl + (carp ? 6 : 2);
				uint16_t c;
				memset(&mp, 0, sizeof(mp));
				mp.m.m_data = (char *)ip + hl;
				mp.m.m_len = (int32_t)plen;
				f[0] = f[1] = 0;
				c = F(in_cksum_skip)(&mp.m, carp ? 36 : (int)plen, 0);
				memcpy(f, &c, 2);
			}
		} else if (ip[9] == 6 || ip[9] == 17) {
			uint16_t c = F(in_cksum_skip)(&mb.m, (int)iplen, (int)hl);
			uint32_t at = hl + (ip[9] == 6 ? 16u : 6u);
			if (ip[9] == 17 && c == 0)
				c = 0xffff;
			if (at + 2 <= fl)
				memcpy(ip + at, &c, 2);
		}
		ip[10] = ip[11] = 0;
		{
			uint16_t c = F(in_cksum_skip)(&mb.m, (int)hl, 0);
			memcpy(ip + 10, &c, 2);
		}
	}
}

static void *verify_thr(void *a) { verify_range((const struct job *)a); return NULL; }
static void *finalize_thr(void *a) { finalize_range((const struct job *)a); return NULL; }

static void run_jobs(struct job *proto, uint32_t n, int nthreads, void *(*fn)(void *))
{
	enum { MAXT = 256 };
	pthread_t th[MAXT];
	struct job jobs[MAXT];
	int t, started = 0;
	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > MAXT)
		nthreads = MAXT;
	if ((uint32_t)nthreads > n)
		nthreads = n ? (int)n : 1;
	for (t = 0; t < nthreads; t++) {
		jobs[t] = *proto;
		jobs[t].lo = (uint32_t)((uint64_t)n * t / nthreads);
		jobs[t].hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
	}
	if (nthreads == 1) {
		fn(&jobs[0]);
		return;
	}
	for (t = 1; t < nthreads; t++)
		if (pthread_create(&th[t], NULL, fn, &jobs[t]) == 0)
			started = t;
		else
			break;
	fn(&jobs[0]);
	for (t = started + 1; t < nthreads; t++) /* threads that failed to start */
		fn(&jobs[t]);
	for (t = 1; t <= started; t++)
		pthread_join(th[t], NULL);
}

void F(ipv4_verify_batch)(const uint8_t *base, const uint64_t *offs,
    uint64_t stride, uint64_t first_off, const uint32_t *flen,
    uint32_t fixed_flen, uint32_t n, uint16_t *ip_out, uint16_t *l4_out,
    uint8_t *status, int nthreads)
{
	struct job j = { base, NULL, offs, stride, first_off, flen, fixed_flen,
	                 0, n, ip_out, l4_out, status, 0 };
	run_jobs(&j, n, nthreads, verify_thr);
}

void F(ipv4_finalize_batch)(uint8_t *base, const uint64_t *offs,
    uint64_t stride, uint64_t first_off, const uint32_t *flen,
    uint32_t fixed_flen, uint32_t n, int nthreads)
{
	struct job j = { base, base, offs, stride, first_off, flen, fixed_flen,
	                 0, n, NULL, NULL, NULL, 0 };
	run_jobs(&j, n, nthreads, finalize_thr);
}

void F(ipv4_demux_verify_batch)(const uint8_t *base, const uint64_t *offs,
    uint64_t stride, uint64_t first_off, const uint32_t *flen,
    uint32_t fixed_flen, uint32_t n, uint16_t *ip_out, uint16_t *l4_out,
    uint8_t *status, int nthreads)
{
	struct job j = { base, NULL, offs, stride, first_off, flen, fixed_flen,
	                 0, n, ip_out, l4_out, status, 1 };
	run_jobs(&j, n, nthreads, verify_thr);
}

void F(ipv4_demux_finalize_batch)(uint8_t *base, const uint64_t *offs,
    uint64_t stride, uint64_t first_off, const uint32_t *flen,
    uint32_t fixed_flen, uint32_t n, int nthreads)
{
	struct job j = { base, base, offs, stride, first_off, flen, fixed_flen,
	                 0, n, NULL, NULL, NULL, 1 };
	run_jobs(&j, n, nthreads, finalize_thr);
}

/* One span, in_cksum_skip(m, len, 0) repeated: the 64 KiB plumbing config. */
uint64_t F(skip_repeat)(const uint8_t *buf, int len, int iters)
{
	union drv_mbuf mb;
	uint64_t acc = 0;
	memset(&mb, 0, sizeof(mb));
	mb.m.m_data = (char *)buf;
	mb.m.m_len = len;
	for (int k = 0; k < iters; k++)
		acc += F(in_cksum_skip)(&mb.m, len, 0);
	return acc;
}

/* Build an mbuf chain over caller segments (seglen may be 0). */
static void build_chain(union drv_mbuf *mb, const uint8_t *const *seg,
                        const int32_t *seglen, int nseg)
{
	for (int k = 0; k < nseg; k++) {
		memset(&mb[k], 0, sizeof(mb[k]));
		mb[k].m.m_data = (char *)seg[k];
		mb[k].m.m_len = seglen[k];
		mb[k].m.m_next = (k + 1 < nseg) ? &mb[k + 1].m : NULL;
	}
}

#define MAX_SEGS 64

uint16_t F(chain_skip)(const uint8_t *const *seg, const int32_t *seglen,
                       int nseg, int len, int skip)
{
	union drv_mbuf mb[MAX_SEGS];
	if (nseg < 1 || nseg > MAX_SEGS)
		return 0;
	build_chain(mb, seg, seglen, nseg);
	return F(in_cksum_skip)(&mb[0].m, len, skip);
}

uint16_t F(chain_pseudo)(const uint8_t *const *seg, const int32_t *seglen,
                         int nseg, int plen, int off0, uint32_t src,
                         uint32_t dst, uint8_t proto)
{
	union drv_mbuf mb[MAX_SEGS];
	if (nseg < 1 || nseg > MAX_SEGS)
		return 0;
	build_chain(mb, seg, seglen, nseg);
	return F(in_cksum_pseudo_header)(&mb[0].m, plen, off0, src, dst, proto);
}

/*
 * TX with checksum offload, restated as the software path the device must
 * match byte for byte (see oracle.h).  Frame i is the
 * chain of segments [pkt_seg[i], pkt_seg[i+1]) (seg_off/seg_len into src =
 * m_data/m_len), pkt_len[i] bytes (m_pkthdr.len), IP header l3_off bytes in.
 *   len > room                        -> NOBUFS, nothing written  (uinet_if_dpdk.c:585-591)
 *   chain holds < len bytes           -> SHORT, nothing written   (m_copydata's KASSERT)
 *   m_copydata(m, 0, len, dst)                                     (uinet_if_dpdk.c:597)
 *   IP datagram malformed (finalize rules, flen = len - l3_off)    -> NOSUM, the copy stays
 *   flags & (CSUM_TCP|CSUM_UDP): in_delayed_cksum (ip_output.c:958-983) on the
 *       chain from the IP header: c = in_cksum_skip(m, ip_len, hl), CSUM_UDP 0 -> 0xffff,
 *       stored at hl + csum_data iff those 2 bytes lie inside the IP mbuf's m_len
 *       (else L4_SKIPPED: the "delayed m_pullup" printf, :971-981)
 *   flags & CSUM_IP: ip_sum = 0; ip_sum = in_cksum(m, hl)          (ip_output.c:667-672)
 * The sums are taken before the copy in the stack; only bytes inside the
 * frame's len reach the wire, so stores past len are dropped.  "The IP mbuf"
 * is the segment holding frame byte l3_off, from that byte on.  The chain the
 * sums walk is rebuilt over the copied bytes with the source's segmentation
 * (in_cksum_skip's result does not depend on where the bytes sit, only on the
 * walk), so the reference's chain walk runs on every case.
 */
static uint32_t tx_default_flags(uint8_t proto)
{
	return ORC_CSUM_IP | (proto == 6 ? ORC_CSUM_TCP : proto == 17 ? ORC_CSUM_UDP : 0u);
}

void F(tx_copy_batch)(const uint8_t *src, const uint64_t *seg_off,
    const int32_t *seg_len, const uint32_t *pkt_seg, const uint32_t *pkt_len,
    const uint32_t *csum_flags, const uint32_t *csum_data, uint32_t l3_off,
    uint8_t *dst, uint64_t dst_stride, uint64_t dst_first, uint32_t room,
    uint32_t n, uint8_t *status)
{
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t k0 = pkt_seg[i], k1 = pkt_seg[i + 1];
		const uint32_t len = pkt_len[i];
		uint8_t *fr = dst + dst_first + (uint64_t)i * dst_stride;
		uint8_t st = 0;
		uint64_t total = 0, pos = 0;
		int64_t ip_mlen = -1;
		uint32_t nseg = 0;
		union drv_mbuf mb[MAX_SEGS];
		if (len > room) {
			status[i] = ORC_TX_NOBUFS;
			continue;
		}
		for (uint32_t k = k0; k < k1; k++)
			total += seg_len[k] > 0 ? (uint64_t)seg_len[k] : 0;
		if (total < len) {
			status[i] = ORC_TX_SHORT;
			continue;
		}
		/* m_copydata(m, 0, len, fr) */
		for (uint32_t k = k0; k < k1 && pos < len; k++) {
			uint64_t l = seg_len[k] > 0 ? (uint64_t)seg_len[k] : 0;
			if (l > len - pos)
				l = len - pos;
			memcpy(fr + pos, src + seg_off[k], l);
			pos += l;
		}
		/* the IP datagram's chain over the copy, source segmentation */
		pos = 0;
		for (uint32_t k = k0; k < k1 && pos < len; k++) {
			uint64_t l = seg_len[k] > 0 ? (uint64_t)seg_len[k] : 0;
			uint64_t a = pos, e = pos + l;
			pos = e;
			if (e <= l3_off)
				continue;
			if (a < l3_off) {
				ip_mlen = (int64_t)(e - l3_off);
				a = l3_off;
			} else if (ip_mlen < 0) {
				ip_mlen = (int64_t)l;
			}
			if (e > len)
				e = len;
			if (nseg < MAX_SEGS) {
				memset(&mb[nseg], 0, sizeof(mb[nseg]));
				mb[nseg].m.m_data = (char *)(fr + a);
				mb[nseg].m.m_len = (int32_t)(e - a);
				if (nseg)
					mb[nseg - 1].m.m_next = &mb[nseg].m;
				nseg++;
			}
		}
		{
			const uint32_t flen = len >= l3_off ? len - l3_off : 0;
			uint8_t *ip = fr + l3_off;
			uint32_t hl = 0, iplen = 0, fl, at;
			if (flen >= 20) {
				hl = (uint32_t)(ip[0] & 0x0f) << 2;
				iplen = ((uint32_t)ip[2] << 8) | ip[3];
			}
			if (flen < 20 || hl < 20 || hl > flen || iplen < hl || iplen > flen || !nseg) {
				status[i] = ORC_TX_NOSUM;
				continue;
			}
			fl = csum_flags ? csum_flags[i] : tx_default_flags(ip[9]);
			if (fl & (ORC_CSUM_TCP | ORC_CSUM_UDP)) {
				uint16_t c = F(in_cksum_skip)(&mb[0].m, (int)iplen, (int)hl);
				uint32_t cd = csum_data ? csum_data[i] : (fl & ORC_CSUM_TCP) ? 16u : 6u;
				if ((fl & ORC_CSUM_UDP) && c == 0)
					c = 0xffff;
				at = hl + cd;
				if ((uint64_t)at + 2 > (uint64_t)ip_mlen) {
					st |= ORC_TX_L4_SKIPPED;
				} else {
					/* *(u_short *)(m_data + at) = c, of which the bytes inside len reach the wire */
					if ((uint64_t)l3_off + at < len)
						ip[at] = (uint8_t)c;
					if ((uint64_t)l3_off + at + 1 < len)
						ip[at + 1] = (uint8_t)(c >> 8);
				}
			}
			if (fl & ORC_CSUM_IP) {
				uint16_t c;
				ip[10] = ip[11] = 0;
				c = F(in_cksum_skip)(&mb[0].m, (int)hl, 0);
				memcpy(ip + 10, &c, 2);
			}
		}
		status[i] = st;
	}
}
