/*
 * host_fold.c -- the CPU fold that serves the (b1) drop-ins by default.
 *
 * the five in_cksum.h:77-83 functions are scalar and
 * synchronous (~0.13 us for an IPv4 header on one core), so a GPU round trip
 * per call (2.7-11 us) can never pay; the batch points
 * (b2) are the GPU's path.  This file is part of the product, written for it:
 * it is not oracle/'s restatement and links nothing under oracle/.
 *
 * Shape.  The reference sums each span in ABSOLUTE-address lanes with aligned
 * loads and a masked head (in_cksumdata, in_cksum.c:91-170), then byte-swaps
 * a span whose stream offset and address disagree in parity (:222-225).  Here
 * a span is summed in lanes counted from its own first byte, with unaligned
 * 32-bit loads (one widening add per 4 bytes, which the compiler vectorizes),
 * and swapped when its STREAM offset is odd.  Both give the stream-relative
 * sum S of SURVEY.md 8(a)'s contract, because 2^16 == 1 (mod 65535): a
 * little-endian 32-bit word is congruent to the sum of its two 16-bit lanes,
 * and a 16-bit value times 2^8 mod 65535 is its byte swap.  The fold keeps
 * "0 only for an all-zero input" (end-around carry never turns a nonzero sum
 * into 0), which is what makes the 0x0000 / 0xffff results exact.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "mi_internal.h"

/* 64 -> 16 bits, end-around carry: congruent mod 65535, 0 only if s == 0. */
uint32_t mi__host_fold64(uint64_t s)
{
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	return (uint32_t)s;
}

static uint32_t swap16(uint32_t f)
{
	return ((f & 0xffu) << 8) | (f >> 8);
}

/* The body: little-endian 32-bit words from p, widened into 64-bit sums.
 * Four independent sums so the scalar clone is not one long dependency chain;
 * 2^32 words per sum before it could carry out, far beyond any span. */
__attribute__((target_clones("avx2", "default")))
static uint64_t words_sum(const uint8_t *p, size_t nw)
{
	uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
	size_t i = 0;

	for (; i + 4 <= nw; i += 4) {
		uint32_t w[4];
		memcpy(w, p + 4 * i, 16);
		a0 += w[0];
		a1 += w[1];
		a2 += w[2];
		a3 += w[3];
	}
	for (; i < nw; ++i) {
		uint32_t w;
		memcpy(&w, p + 4 * i, 4);
		a0 += w;
	}
	return a0 + a1 + a2 + a3;
}

uint32_t mi__host_span_sum(const void *buf, size_t n)
{
	const uint8_t *p = (const uint8_t *)buf;
	uint64_t s = words_sum(p, n / 4);
	size_t i = n & ~(size_t)3;

	if (n - i >= 2) {
		s += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
		i += 2;
	}
	if (i < n) /* an odd last byte sits in an even lane of the span: low byte */
		s += p[i];
	return mi__host_fold64(s);
}

uint32_t mi__host_fold_acc(uint32_t acc, uint32_t span_sum, uint64_t stream_off)
{
	return mi__host_fold64((uint64_t)acc + ((stream_off & 1) ? swap16(span_sum) : span_sum));
}

uint16_t mi__host_cksum_hdr(const void *ip)
{
	/* in_cksum.c:278-285 sums the 20 bytes in absolute-address lanes with no
	 * odd-address correction: at an odd address that is the swapped span sum
	 * (0xb861 where in_cksum_skip gives 0x61b8). */
	uint32_t f = mi__host_span_sum(ip, 20);

	if ((uintptr_t)ip & 1)
		f = swap16(f);
	return (uint16_t)~f;
}
