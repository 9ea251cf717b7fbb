/*
 * inet_dropin.c -- the (b1) drop-in entry points with the reference's names and
 * signatures (src/sys/amd64/include/in_cksum.h:77-83), in plain C.
 *
 * Each call walks the mbuf chain exactly as the reference does
 * (src/sys/amd64/amd64/in_cksum.c:193-232 and :241-276: leading skip, zero-length
 * mbufs ignored, a short chain truncates silently), packs the selected bytes
 * contiguously into the thread's page-locked staging buffer and has the GPU fold
 * them (mi__scalar_fold: a request to the thread's resident drop-in service,
 * or one AQL dispatch, and a spin on the result).  Packing preserves the checksum:
 * the reference's (clen ^ addr) & 1 swap makes every span's lanes relative to
 * the stream, and a contiguous copy starting at an even address is exactly the
 * stream.  in_cksum_hdr keeps its address mod 16 in staging because its lanes
 * are absolute (in_cksum.c:278-285).
 *
 * in_pseudo / in_addword fold two or three integers and touch no packet bytes;
 * they are computed here.  There is no CPU path for byte folding.  If the GPU
 * is unusable the call has no way to say so (the reference API has no error
 * return), so by default it aborts with a message: every value it could return
 * instead is a wrong checksum.  An embedder may install
 * mi_cksum_set_dropin_error_handler: the handler is told, and the call returns
 * 0xffff -- never the result of verifying a datagram with valid sums (those
 * verify to 0), so an RX caller drops the packet.  A TX caller (ip_output's
 * in_cksum_hdr, in_delayed_cksum's in_cksum_skip) stores it into the outgoing
 * header: with a handler installed a GPU error sends a wrong sum, so a handler
 * that must not allow that aborts itself (it runs before the value returns).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "mi_cksum.h"
#include "mi_internal.h"

/* The reference's mbuf prefix (src/sys/sys/mbuf.h:90-98). */
struct mi_mbuf_view {
	struct mi_mbuf_view *m_next;
	void                *m_nextpkt;
	char                *m_data;
	int                  m_len;
};
_Static_assert(offsetof(struct mi_mbuf_view, m_data) == 16, "m_data@16 (mbuf.h:93)");
_Static_assert(offsetof(struct mi_mbuf_view, m_len) == 24, "m_len@24 (mbuf.h:94)");

static mi_cksum_error_fn g_dropin_handler;

void mi_cksum_set_dropin_error_handler(mi_cksum_error_fn fn)
{
	__atomic_store_n(&g_dropin_handler, fn, __ATOMIC_RELEASE);
}

/* The (b1) error policy: abort, or the installed handler and 0xffff. */
static uint16_t dropin_fail(const char *what)
{
	mi_cksum_error_fn fn = __atomic_load_n(&g_dropin_handler, __ATOMIC_ACQUIRE);

	if (!fn)
		mi__fatal(what);
	fn(what, mi_cksum_strerror());
	return 0xffff;
}

/* Visit the (addr, len) spans in_cksum_skip would fold, in stream order. */
static long walk_skip(const struct mi_mbuf_view *m, long len, long skip, uint8_t *dst)
{
	long total = 0, rem = len - skip;

	for (; skip && m; m = m->m_next) {
		if (m->m_len > skip) {
			long n = m->m_len - skip;
			if (rem < n)
				n = rem;
			if (n > 0) {
				if (dst)
					memcpy(dst + total, m->m_data + skip, (size_t)n);
				total += n;
			}
			rem -= n;
			m = m->m_next;
			skip = 0;
			goto body;
		}
		skip -= m->m_len;
	}
body:
	for (; m && rem > 0; m = m->m_next) {
		long n = m->m_len;
		if (n == 0)
			continue;
		if (rem < n)
			n = rem;
		if (dst)
			memcpy(dst + total, m->m_data, (size_t)n);
		total += n;
		rem -= n;
	}
	return total;
}

/* Spans in_cksum_pseudo_header folds: first mbuf from off0, then the chain. */
static long walk_pseudo(const struct mi_mbuf_view *m, long plen, long off0, uint8_t *dst)
{
	long total = 0, rem = plen, n = (long)m->m_len - off0;
	const char *addr = m->m_data + off0;

	for (;;) {
		if (rem < n)
			n = rem;
		if (n > 0) {
			if (dst)
				memcpy(dst + total, addr, (size_t)n);
			total += n;
		}
		rem -= n;
		do {
			m = m->m_next;
		} while (m && rem && m->m_len == 0);
		if (!m || !rem)
			break;
		n = m->m_len;
		addr = m->m_data;
	}
	return total;
}

unsigned short in_cksum_skip(struct mbuf *m0, int len, int skip)
{
	const struct mi_mbuf_view *m = (const struct mi_mbuf_view *)m0;
	long total = walk_skip(m, len, skip, NULL);
	uint8_t *st = mi__scalar_staging((size_t)total + 16);
	uint16_t r;

	if (!st)
		return dropin_fail("in_cksum_skip");
	walk_skip(m, len, skip, st);
	if (mi__scalar_fold(0, (uint32_t)total, MI_SPAN_STREAM, 0, 0, 0, 0, 0, &r))
		return dropin_fail("in_cksum_skip");
	return r;
}

uint16_t in_cksum_pseudo_header(struct mbuf *m0, int plen, int off0, uint32_t src,
                                uint32_t dst, uint8_t protonum)
{
	const struct mi_mbuf_view *m = (const struct mi_mbuf_view *)m0;
	long total = walk_pseudo(m, plen, off0, NULL);
	uint8_t *st = mi__scalar_staging((size_t)total + 16);
	uint16_t r;

	if (!st)
		return dropin_fail("in_cksum_pseudo_header");
	walk_pseudo(m, plen, off0, st);
	if (mi__scalar_fold(0, (uint32_t)total, MI_SPAN_STREAM, 1, src, dst, protonum,
	                    (uint32_t)plen, &r))
		return dropin_fail("in_cksum_pseudo_header");
	return r;
}

unsigned int in_cksum_hdr(const struct ip *ip)
{
	const size_t mod = (uintptr_t)ip & 15u;
	uint8_t *st = mi__scalar_staging(64);
	uint16_t r;

	if (!st)
		return dropin_fail("in_cksum_hdr");
	memcpy(st + mod, ip, 20);
	if (mi__scalar_fold(mod, 20, MI_SPAN_ABS, 0, 0, 0, 0, 0, &r))
		return dropin_fail("in_cksum_hdr");
	return r;
}

/* in_cksum.c:181-191: (u64) a + b + c, REDUCE16 -- not complemented. */
unsigned short in_pseudo(unsigned int a, unsigned int b, unsigned int c)
{
	uint64_t s = (uint64_t)a + b + c;

	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	return (unsigned short)s;
}

/* in_cksum.c:172-179 */
unsigned short in_addword(unsigned short a, unsigned short b)
{
	unsigned int s = (unsigned int)a + b;

	return (unsigned short)(s > 65535 ? s - 65535 : s);
}
