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
 * a span is summed in lanes counted from its own first byte -- long spans
 * 64 bytes per step, each 32-bit word's two 16-bit halves added to 32-bit
 * vector lane sums (four ALU ops per 32 bytes), short ones word by word --
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

#include "host_fold.h"

/* The body of a long span, 64 bytes per step: every 32-bit lane is split
 * into its two 16-bit halves, each added to a 32-bit lane sum.  A lane sum
 * grows by at most 0xffff per step, so the sums are emptied into a 64-bit
 * total every 32768 steps (2 MiB).  Vector extensions, not intrinsics: the
 * AVX2 clone uses 256-bit registers, the default one 128-bit pairs. */
typedef uint32_t v8u __attribute__((vector_size(32)));

__attribute__((target_clones("avx2", "default")))
uint64_t mi__host_blocks_sum(const uint8_t *p, size_t nb)
{
	uint64_t total = 0;

	while (nb) {
		const size_t k = nb < 32768 ? nb : 32768;
		v8u a0 = {0}, b0 = {0}, a1 = {0}, b1 = {0};
		for (size_t i = 0; i < k; ++i, p += 64) {
			v8u x, y;
			memcpy(&x, p, 32);
			memcpy(&y, p + 32, 32);
			a0 += x & 0xffffu;
			b0 += x >> 16;
			a1 += y & 0xffffu;
			b1 += y >> 16;
		}
		for (int j = 0; j < 8; ++j)
			total += (uint64_t)a0[j] + b0[j] + a1[j] + b1[j];
		nb -= k;
	}
	return total;
}

uint16_t mi__host_cksum_hdr(const void *ip)
{
	/* in_cksum.c:278-285 sums the 20 bytes in absolute-address lanes with no
	 * odd-address correction: at an odd address that is the swapped span sum
	 * (0xb861 where in_cksum_skip gives 0x61b8). */
	uint32_t w[5], f;

	memcpy(w, ip, 20);
	f = hf_fold64((uint64_t)w[0] + w[1] + w[2] + w[3] + w[4]);
	if ((uintptr_t)ip & 1)
		f = hf_swap16(f);
	return (uint16_t)~f;
}
