/*
 * oracle/cksum_oracle.c -- from-scratch CPU restatement of the reference's
 * RFC 1071 checksum (src/sys/amd64/amd64/in_cksum.c, the only in_cksum compiled
 * into libuinet on x86_64: src/lib/libuinet/Makefile:275-276).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Never linked into the product.
 *
 * What the reference computes, restated (SURVEY.md section 8 "Contract"):
 *   - in_cksumdata (in_cksum.c:91-170) sums aligned little-endian 32-bit words,
 *     masking the bytes outside [buf, buf+len) (in_masks, :73-79), into a u64
 *     and folds it with REDUCE32 (:60-64).  Every byte therefore lands in the
 *     16-bit lane given by its ABSOLUTE address parity: b << 8*(addr & 1)
 *     (a word's upper half is worth 2^16 == 1 mod 65535).
 *   - in_cksum_skip / in_cksum_pseudo_header (:193-232, :241-276) shift a span's
 *     sum by 8 when (bytes-so-far ^ addr) is odd (:222-225, :266-269), which
 *     turns absolute lanes into STREAM lanes, then REDUCE16 (:65-71) + ~.
 *   - REDUCE16 preserves the value mod 65535 and gives 0 only for an all-zero
 *     sum (ADDCARRY, :59), so any association order gives the same u16.
 *
 * This restatement keeps those semantics but not the reference's code shape:
 * head bytes one at a time, then aligned u64 words added with end-around carry
 * (2^64-1 is a multiple of 65535), then tail bytes.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "oracle.h"

/* u64 -> 16-bit one's-complement fold: value mod 65535, 0 only for 0. */
static inline uint32_t fold16(uint64_t s)
{
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	return (uint32_t)s;
}

static inline uint32_t swap16(uint32_t x)
{
	return ((x & 0xffu) << 8) | ((x >> 8) & 0xffu);
}

/*
 * Absolute-address-lane sum of [p, p+len), folded to 16 bits.
 * Restates in_cksumdata (in_cksum.c:91-170) + REDUCE32.  len <= 0 sums nothing.
 */
static uint32_t span_abs(const uint8_t *p, long len)
{
	uint64_t s = 0, w;
	if (len <= 0)
		return 0;
	/* head: bytes up to 8-byte alignment */
	while (len > 0 && ((uintptr_t)p & 7u)) {
		s += (uint64_t)*p << (8 * ((uintptr_t)p & 1u));
		p++;
		len--;
	}
	/* body: 32 bytes per iteration, end-around carry keeps s == sum mod 2^64-1 */
	while (len >= 32) {
		uint64_t w0, w1, w2, w3, t;
		memcpy(&w0, p, 8);
		memcpy(&w1, p + 8, 8);
		memcpy(&w2, p + 16, 8);
		memcpy(&w3, p + 24, 8);
		t = s + w0; s = t + (t < w0);
		t = s + w1; s = t + (t < w1);
		t = s + w2; s = t + (t < w2);
		t = s + w3; s = t + (t < w3);
		p += 32;
		len -= 32;
	}
	while (len >= 8) {
		uint64_t t;
		memcpy(&w, p, 8);
		t = s + w; s = t + (t < w);
		p += 8;
		len -= 8;
	}
	/* tail: p is 8-aligned here, so byte k sits in lane k & 1 */
	for (long k = 0; k < len; k++) {
		uint64_t t, v = (uint64_t)p[k] << (8 * (k & 1));
		t = s + v; s = t + (t < v);
	}
	return fold16(s);
}

/* Stream-lane contribution of a span that starts at stream offset clen. */
static inline uint32_t span_stream(const uint8_t *p, long len, long clen)
{
	uint32_t a = span_abs(p, len);
	return ((clen ^ (long)(uintptr_t)p) & 1) ? swap16(a) : a;
}

/* in_cksum.c:172-179 */
uint16_t orc_in_addword(uint16_t a, uint16_t b)
{
	uint32_t s = (uint32_t)a + b;
	return (uint16_t)(s > 65535 ? s - 65535 : s);
}

/* in_cksum.c:181-191 -- NOT complemented. */
uint16_t orc_in_pseudo(uint32_t a, uint32_t b, uint32_t c)
{
	return (uint16_t)fold16((uint64_t)a + b + c);
}

/* in_cksum.c:193-232: chain walk with skip, zero-length mbufs ignored, a short
 * chain silently truncates the sum. */
uint16_t orc_in_cksum_skip(struct orc_mbuf *m, int len, int skip)
{
	uint64_t sum = 0;
	long clen = 0;
	long rem = (long)len - skip;

	/* leading skip (:204-212) */
	for (; skip && m; m = m->m_next) {
		if (m->m_len > skip) {
			long mlen = m->m_len - skip;
			if (rem < mlen)
				mlen = rem;
			sum += span_stream((const uint8_t *)m->m_data + skip, mlen, clen);
			clen += mlen;
			rem -= mlen;
			m = m->m_next;
			skip = 0;
			goto body;
		}
		skip -= m->m_len;
	}
body:
	for (; m && rem; m = m->m_next) {
		long mlen = m->m_len;
		if (mlen == 0)
			continue;
		if (rem < mlen)
			mlen = rem;
		sum += span_stream((const uint8_t *)m->m_data, mlen, clen);
		clen += mlen;
		rem -= mlen;
	}
	return (uint16_t)(~fold16(sum) & 0xffffu);
}

/* in_cksum.c:241-276: pseudo-header seed (:252-253, plen truncated to u16 and
 * byte-swapped as htons does on little-endian), then the chain from off0. */
uint16_t orc_in_cksum_pseudo_header(struct orc_mbuf *m, int plen, int off0,
                                    uint32_t src, uint32_t dst, uint8_t protonum)
{
	uint64_t sum = (uint64_t)src + dst + ((uint32_t)protonum << 8) +
	               swap16((uint16_t)plen);
	long clen = 0, rem = plen;
	long mlen = (long)m->m_len - off0;
	const uint8_t *addr = (const uint8_t *)m->m_data + off0;

	for (;;) {
		if (rem < mlen)
			mlen = rem;
		sum += span_stream(addr, mlen, clen);
		clen += mlen;
		rem -= mlen;
		/* advance to the next non-empty mbuf while bytes remain (:258-262) */
		do {
			m = m->m_next;
		} while (m && rem && m->m_len == 0);
		if (!m || !rem)
			break;
		mlen = m->m_len;
		addr = (const uint8_t *)m->m_data;
	}
	return (uint16_t)(~fold16(sum) & 0xffffu);
}

/* in_cksum.c:278-285: 20 bytes, absolute lanes, no odd-address correction. */
unsigned orc_in_cksum_hdr(const void *ip)
{
	return ~span_abs((const uint8_t *)ip, 20) & 0xffffu;
}
