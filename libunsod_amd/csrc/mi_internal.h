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

/* (the CPU fold of MI_DROPIN_HOST: host_fold.h) */

#ifdef __cplusplus
}
#endif
#endif
