/*
 * mi_internal.h -- bridge between the C drop-in shim (inet_dropin.c) and the
 * HIP runtime (cksum_kernels.hip).  Mirrors the reference's kernel/host split:
 * kernel-side C calls a host-compiled bridge (libuinet's *_host.c, Makefile
 * HOST_C / UINET_HOST_SRCS :30, :173-182).  Not part of the public ABI.
 */
#ifndef MI_INTERNAL_H
#define MI_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Per-thread page-locked, device-mapped staging buffer of >= need bytes,
 * 16-byte aligned.  NULL on failure (mi_cksum_strerror() says why). */
uint8_t *mi__scalar_staging(size_t need);

/* One scalar checksum on the GPU over staging[off, off + len):
 *   lanes = MI_SPAN_STREAM or MI_SPAN_ABS;
 *   pseudo != 0 adds src + dst + (proto << 8) + bswap16(plen & 0xffff).
 * Synchronous.  Returns 0 and stores the complemented u16 in *out, or -errno. */
int mi__scalar_fold(size_t off, uint32_t len, uint32_t lanes, int pseudo, uint32_t src,
                    uint32_t dst, uint8_t proto, uint32_t plen, uint16_t *out);

/* host_fold.c -- the (b1) drop-ins' CPU fold (MI_DROPIN_HOST):
 *   mi__host_span_sum: p[0..n) summed in 16-bit lanes counted from p[0],
 *     folded (0 only for an all-zero span);
 *   mi__host_fold_acc: acc + a span's sum, byte-swapped when the span starts
 *     at an odd offset of the stream, folded;
 *   mi__host_fold64: a 64-bit sum folded to 16 bits (end-around carry);
 *   mi__host_cksum_hdr: in_cksum_hdr (absolute-address lanes). */
uint32_t mi__host_span_sum(const void *p, size_t n);
uint32_t mi__host_fold_acc(uint32_t acc, uint32_t span_sum, uint64_t stream_off);
uint32_t mi__host_fold64(uint64_t s);
uint16_t mi__host_cksum_hdr(const void *ip);

#ifdef __cplusplus
}
#endif
#endif
