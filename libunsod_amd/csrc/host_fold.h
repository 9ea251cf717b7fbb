/*
 * host_fold.h -- the (b1) drop-ins' CPU fold (MI_DROPIN_HOST), inline parts.
 * Algorithm and reasoning: host_fold.c.  Internal; not part of the C ABI.
 */
#ifndef MI_HOST_FOLD_H
#define MI_HOST_FOLD_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* host_fold.c: nb 64-byte blocks summed in 16-bit lanes (vector body). */
uint64_t mi__host_blocks_sum(const uint8_t *p, size_t nb);
/* host_fold.c: in_cksum_hdr (absolute-address lanes, in_cksum.c:278-285). */
uint16_t mi__host_cksum_hdr(const void *ip);

/* 64 -> 16 bits, end-around carry: congruent mod 65535, 0 only if s == 0. */
static inline uint32_t hf_fold64(uint64_t s)
{
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	s = (s & 0xffffu) + (s >> 16);
	return (uint32_t)s;
}

static inline uint32_t hf_swap16(uint32_t f)
{
	return ((f & 0xffu) << 8) | (f >> 8);
}

/* p[0..n) summed in 16-bit lanes counted from p[0], folded (0 only for an
 * all-zero span): 64-byte blocks by the vector body, then 32-bit words, then
 * a 16-bit and an odd last byte (an even lane of the span: the low byte). */
static inline uint32_t hf_span_sum(const void *buf, size_t n)
{
	const uint8_t *p = (const uint8_t *)buf;
	uint64_t s = 0;
	size_t i = 0;

	if (n >= 256) {
		i = n & ~(size_t)63;
		s = mi__host_blocks_sum(p, i / 64);
	}
	for (; i + 4 <= n; i += 4) {
		uint32_t w;
		memcpy(&w, p + i, 4);
		s += w;
	}
	if (n - i >= 2) {
		s += (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8);
		i += 2;
	}
	if (i < n)
		s += p[i];
	return hf_fold64(s);
}

/* acc + a span's sum, byte-swapped when the span starts at an odd offset of
 * the stream (in_cksum.c:222-225's swap, stream-relative), folded. */
static inline uint32_t hf_fold_acc(uint32_t acc, uint32_t span_sum, uint64_t stream_off)
{
	return hf_fold64((uint64_t)acc + ((stream_off & 1) ? hf_swap16(span_sum) : span_sum));
}

#endif
