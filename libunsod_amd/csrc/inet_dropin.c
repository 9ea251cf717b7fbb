/*
 * inet_dropin.c -- the (b1) drop-in entry points with the reference's names and
 * signatures (src/sys/amd64/include/in_cksum.h:77-83), in plain C.
 *
 * Each call walks the mbuf chain exactly as the reference does
 * (src/sys/amd64/amd64/in_cksum.c:193-232 and :241-276: leading skip, zero-length
 * mbufs ignored, a short chain truncates silently) and hands every span it
 * selects, with the span's offset in the byte stream, to a sink:
 *   MI_DROPIN_HOST (default) -- host_fold.c folds the span in place on this
 *     CPU; the spans' sums meet with the stream-parity swap (in_cksum.c:222-225);
 *   MI_DROPIN_GPU -- the span is packed into the thread's page-locked staging
 *     buffer and the GPU folds the packed bytes (mi__scalar_fold: a request to
 *     the device's resident drop-in service, or one AQL dispatch).  Packing
 *     preserves the checksum: a contiguous copy starting at an even address is
 *     exactly the stream.  in_cksum_hdr keeps its address mod 16 in staging
 *     because its lanes are absolute (in_cksum.c:278-285).
 * A GPU request that fails is served by the host fold (same bits), counted,
 * and reported to the embedder's error handler if one is installed: the
 * reference API has no error return, and the stack must not die of a GPU
 * hiccup.  in_pseudo / in_addword fold two or three integers and
 * touch no packet bytes; they are computed here in either mode.
 */
#include <errno.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cksum.h"
#include "host_fold.h"
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
static int g_dropin_mode = -1;
static uint64_t g_degraded;

void mi_cksum_set_dropin_error_handler(mi_cksum_error_fn fn)
{
	__atomic_store_n(&g_dropin_handler, fn, __ATOMIC_RELEASE);
}

uint64_t mi_cksum_dropin_degraded(void)
{
	return __atomic_load_n(&g_degraded, __ATOMIC_RELAXED);
}

static int dropin_mode(void)
{
	int v = __atomic_load_n(&g_dropin_mode, __ATOMIC_RELAXED);

	if (v < 0) {
		const char *e = getenv("MI_CKSUM_DROPIN");
		v = e && strcmp(e, "gpu") == 0 ? MI_DROPIN_GPU : MI_DROPIN_HOST;
		__atomic_store_n(&g_dropin_mode, v, __ATOMIC_RELAXED);
	}
	return v;
}

int mi_cksum_set_dropin_mode(int mode)
{
	int was;

	if (mode != MI_DROPIN_HOST && mode != MI_DROPIN_GPU)
		return -EINVAL;
	was = dropin_mode();
	__atomic_store_n(&g_dropin_mode, mode, __ATOMIC_RELAXED);
	return was;
}

/* A GPU-mode call that failed: count it and tell the embedder; the caller
 * then serves it with the host fold. */
static void dropin_degrade(const char *what)
{
	mi_cksum_error_fn fn = __atomic_load_n(&g_dropin_handler, __ATOMIC_ACQUIRE);

	__atomic_add_fetch(&g_degraded, 1, __ATOMIC_RELAXED);
	if (fn)
		fn(what, mi_cksum_strerror());
}

/* Where the spans of a walk go: packed into GPU staging, folded here, or only
 * counted (the first pass that sizes the staging). */
struct span_sink {
	uint8_t *dst;   /* pack the spans here, or NULL */
	int fold;       /* fold them on this CPU */
	long total;     /* bytes so far: the next span's offset in the stream */
	uint32_t acc;   /* the folded sum so far */
};

static void sink_span(struct span_sink *s, const char *p, long n)
{
	if (s->dst)
		memcpy(s->dst + s->total, p, (size_t)n);
	if (s->fold)
		s->acc = hf_fold_acc(s->acc, hf_span_sum(p, (size_t)n), (uint64_t)s->total);
	s->total += n;
}

/* The spans in_cksum_skip folds (in_cksum.c:203-231), in stream order. */
static void walk_skip(const struct mi_mbuf_view *m, long len, long skip, struct span_sink *s)
{
	long rem = len - skip;

	for (; skip && m; m = m->m_next) {
		if (m->m_len > skip) {
			long n = m->m_len - skip;
			if (rem < n)
				n = rem;
			if (n > 0)
				sink_span(s, m->m_data + skip, n);
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
		sink_span(s, m->m_data, n);
		rem -= n;
	}
}

/* The spans in_cksum_pseudo_header folds (in_cksum.c:254-273): the first
 * mbuf from off0, then the chain. */
static void walk_pseudo(const struct mi_mbuf_view *m, long plen, long off0, struct span_sink *s)
{
	long rem = plen, n = (long)m->m_len - off0;
	const char *addr = m->m_data + off0;

	for (;;) {
		if (rem < n)
			n = rem;
		if (n > 0)
			sink_span(s, addr, n);
		rem -= n;
		do {
			m = m->m_next;
		} while (m && rem && m->m_len == 0);
		if (!m || !rem)
			break;
		n = m->m_len;
		addr = m->m_data;
	}
}

/* in_cksum.c:252-253: the pseudo-header words, as the GPU service adds them. */
static uint64_t pseudo_seed(uint32_t src, uint32_t dst, uint8_t proto, int plen)
{
	uint32_t l = (uint32_t)plen & 0xffffu;

	return (uint64_t)(src & 0xffffu) + (src >> 16) + (dst & 0xffffu) + (dst >> 16) +
	       ((uint32_t)proto << 8) + (((l & 0xffu) << 8) | (l >> 8));
}

static uint16_t host_skip(const struct mi_mbuf_view *m, int len, int skip)
{
	struct span_sink s = { NULL, 1, 0, 0 };

	walk_skip(m, len, skip, &s);
	return (uint16_t)~s.acc;
}

static uint16_t host_pseudo(const struct mi_mbuf_view *m, int plen, int off0, uint32_t src,
                            uint32_t dst, uint8_t protonum)
{
	struct span_sink s = { NULL, 1, 0, 0 };

	walk_pseudo(m, plen, off0, &s);
	return (uint16_t)~hf_fold64(s.acc + pseudo_seed(src, dst, protonum, plen));
}

unsigned short in_cksum_skip(struct mbuf *m0, int len, int skip)
{
	const struct mi_mbuf_view *m = (const struct mi_mbuf_view *)m0;
	struct span_sink s = { NULL, 0, 0, 0 };
	uint16_t r;

	if (dropin_mode() == MI_DROPIN_HOST)
		return host_skip(m, len, skip);
	walk_skip(m, len, skip, &s);
	s.dst = mi__scalar_staging((size_t)s.total + 16);
	if (s.dst) {
		s.total = 0;
		walk_skip(m, len, skip, &s);
		if (mi__scalar_fold(0, (uint32_t)s.total, MI_SPAN_STREAM, 0, 0, 0, 0, 0, &r) == 0)
			return r;
	}
	dropin_degrade("in_cksum_skip");
	return host_skip(m, len, skip);
}

uint16_t in_cksum_pseudo_header(struct mbuf *m0, int plen, int off0, uint32_t src,
                                uint32_t dst, uint8_t protonum)
{
	const struct mi_mbuf_view *m = (const struct mi_mbuf_view *)m0;
	struct span_sink s = { NULL, 0, 0, 0 };
	uint16_t r;

	if (dropin_mode() == MI_DROPIN_HOST)
		return host_pseudo(m, plen, off0, src, dst, protonum);
	walk_pseudo(m, plen, off0, &s);
	s.dst = mi__scalar_staging((size_t)s.total + 16);
	if (s.dst) {
		s.total = 0;
		walk_pseudo(m, plen, off0, &s);
		if (mi__scalar_fold(0, (uint32_t)s.total, MI_SPAN_STREAM, 1, src, dst, protonum,
		                    (uint32_t)plen, &r) == 0)
			return r;
	}
	dropin_degrade("in_cksum_pseudo_header");
	return host_pseudo(m, plen, off0, src, dst, protonum);
}

unsigned int in_cksum_hdr(const struct ip *ip)
{
	const size_t mod = (uintptr_t)ip & 15u;
	uint8_t *st;
	uint16_t r;

	if (dropin_mode() == MI_DROPIN_HOST)
		return mi__host_cksum_hdr(ip);
	st = mi__scalar_staging(64);
	if (st) {
		memcpy(st + mod, ip, 20);
		if (mi__scalar_fold(mod, 20, MI_SPAN_ABS, 0, 0, 0, 0, 0, &r) == 0)
			return r;
	}
	dropin_degrade("in_cksum_hdr");
	return mi__host_cksum_hdr(ip);
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
