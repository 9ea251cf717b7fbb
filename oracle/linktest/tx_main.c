/*
 * oracle/linktest/tx_main.c -- host-side driver of tx_kernel.c (TEST
 * INFRASTRUCTURE ONLY).  One batch of outgoing frames (a file written by
 * tests/test_link_gpu.py from a tests/tx_cases.py case) goes out twice:
 *
 *   software route: if_hwassist = 0 -- ip_output's own sums with the
 *     reference's in_cksum.c, then the driver's m_copydata into the slots;
 *   offload route:  if_hwassist = CSUM_IP | CSUM_TCP | CSUM_UDP -- ip_output
 *     leaves the sums, the inject-ring hook reads the frames' descriptors out
 *     of the real struct mbufs, and mi_cksum_tx_copy_host copies and sums on
 *     the GPU (zero-copy from registered memory, then again staged).
 *
 * The slot buffers (bytes no frame may touch included) must be identical, and
 * every frame's status must be the one its route implies.  Prints one JSON
 * line; exit status 0 iff nothing differs.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cksum.h"

struct mbuf;
extern int mi_tx_mbuf_size(void);
extern int mi_tx_last_gave_up(void);
extern int mi_tx_last_udp_ffff(void);
extern int mi_tx_frame(struct mbuf *pool, char *blob, const uint64_t *seg_off, const int32_t *seg_len, uint32_t k0,
                       uint32_t k1, uint32_t pkt_len, uint32_t l3_off, int have_flags, uint32_t tflags,
                       uint32_t tdata, unsigned long hwassist, char *slot, uint32_t buf_len, uint64_t *d_off,
                       int32_t *d_len, uint32_t *d_flags, uint32_t *d_data, uint32_t *d_pkt_len);

#define TXC_IN 0
#define TXC_NOT_IP 1
#define TXC_SHORT 2
#define TXC_NOBUFS 3

static void *page_alloc(uint64_t bytes)
{
	void *p = NULL;
	if (posix_memalign(&p, 4096, (bytes + 4095) & ~4095ull))
		return NULL;
	memset(p, 0, (bytes + 4095) & ~4095ull);
	return p;
}

static int rd(void *p, size_t sz, size_t n, FILE *f)
{
	return fread(p, sz, n, f) == n;
}

int main(int argc, char **argv)
{
	FILE *f;
	uint32_t h[8];
	uint64_t g[4];
	const char *sw_out = argc == 4 && !strcmp(argv[2], "--software") ? argv[3] : NULL;
	if ((argc != 2 && !sw_out) || !(f = fopen(argv[1], "rb"))) {
		fprintf(stderr, "usage: tx_test CASE_FILE [--software OUT_FILE]\n");
		return 2;
	}
	/* u32 magic 'MITX', n, nseg, l3, room, has_flags, has_data, 0;
	 * u64 src_bytes, dst_bytes, dst_stride, dst_first; src; seg_off u64 x nseg;
	 * seg_len i32 x nseg; pkt_seg u32 x (n + 1); pkt_len u32 x n; [flags u32 x n];
	 * [data u32 x n]; dst (initial bytes) */
	if (!rd(h, 4, 8, f) || h[0] != 0x5854494du || !rd(g, 8, 4, f))
		return 2;
	const uint32_t n = h[1], nseg = h[2], l3 = h[3], room = h[4], hf = h[5], hd = h[6];
	const uint64_t sbytes = g[0], dbytes = g[1], stride = g[2], first = g[3];
	uint8_t *src = page_alloc(sbytes), *dst0 = page_alloc(dbytes);
	uint64_t *seg_off = calloc(nseg + 1, 8);
	int32_t *seg_len = calloc(nseg + 1, 4);
	uint32_t *pkt_seg = calloc(n + 1, 4), *pkt_len = calloc(n + 1, 4);
	uint32_t *tfl = calloc(n + 1, 4), *tda = calloc(n + 1, 4);
	if (!src || !dst0 || !rd(src, 1, sbytes, f) || !rd(seg_off, 8, nseg, f) || !rd(seg_len, 4, nseg, f) ||
	    !rd(pkt_seg, 4, n + 1, f) || !rd(pkt_len, 4, n, f) || (hf && !rd(tfl, 4, n, f)) ||
	    (hd && !rd(tda, 4, n, f)) || !rd(dst0, 1, dbytes, f))
		return 2;
	fclose(f);

	uint32_t maxseg = 1, maxlen = 0;
	for (uint32_t i = 0; i < n; i++) {
		if (pkt_seg[i + 1] - pkt_seg[i] > maxseg)
			maxseg = pkt_seg[i + 1] - pkt_seg[i];
		if (pkt_len[i] > maxlen)
			maxlen = pkt_len[i];
	}
	struct mbuf *pool = calloc(maxseg, (size_t)mi_tx_mbuf_size());
	uint8_t *srcA = page_alloc(sbytes), *dstA = page_alloc(dbytes);
	uint8_t *srcB = page_alloc(sbytes), *dstB = page_alloc(dbytes), *dstS = page_alloc(dbytes);
	uint64_t *d_off = calloc(nseg + 1, 8);
	int32_t *d_len = calloc(nseg + 1, 4);
	uint32_t *d_flags = calloc(n + 1, 4), *d_data = calloc(n + 1, 4), *d_plen = calloc(n + 1, 4);
	int *cls = calloc(n + 1, sizeof(int)), *gave = calloc(n + 1, sizeof(int));
	uint8_t *stZ = calloc(n + 1, 1), *stS = calloc(n + 1, 1);
	memcpy(srcA, src, sbytes);
	memcpy(srcB, src, sbytes);
	memcpy(dstA, dst0, dbytes);
	memcpy(dstB, dst0, dbytes);
	memcpy(dstS, dst0, dbytes);

	unsigned long ncls[4] = {0}, ngave = 0, nffff = 0, hw = MI_CSUM_IP | MI_CSUM_TCP | MI_CSUM_UDP;
	for (uint32_t i = 0; i < n; i++) {
		/* software route (if_hwassist = 0): the wire bytes */
		cls[i] = mi_tx_frame(pool, (char *)srcA, seg_off, seg_len, pkt_seg[i], pkt_seg[i + 1], pkt_len[i], l3,
		                     hf, tfl[i], hd ? tda[i] : 0, 0, (char *)dstA + first + i * stride, room, NULL, NULL,
		                     NULL, NULL, NULL);
		gave[i] = mi_tx_last_gave_up();
		nffff += mi_tx_last_udp_ffff();
		/* offload route: ip_output with the device's if_hwassist, descriptors for the GPU */
		int c2 = mi_tx_frame(pool, (char *)srcB, seg_off, seg_len, pkt_seg[i], pkt_seg[i + 1], pkt_len[i], l3, hf,
		                     tfl[i], hd ? tda[i] : 0, hw, NULL, room, d_off, d_len, &d_flags[i], &d_data[i],
		                     &d_plen[i]);
		if (c2 != cls[i] && !(cls[i] == TXC_SHORT || c2 == TXC_SHORT)) {
			printf("{\"error\": \"frame %u: routes classify it %d / %d\"}\n", i, cls[i], c2);
			return 1;
		}
		ncls[cls[i]]++;
		ngave += gave[i] && cls[i] == TXC_IN;
	}

	if (sw_out) {
		/* the software route alone (no GPU): slots, then per frame its class
		 * and whether in_delayed_cksum gave up (int32 each) */
		FILE *o = fopen(sw_out, "wb");
		if (!o || fwrite(dstA, 1, dbytes, o) != dbytes || fwrite(cls, sizeof(int), n, o) != n ||
		    fwrite(gave, sizeof(int), n, o) != n)
			return 2;
		fclose(o);
		printf("{\"frames\": %u, \"through_ip_output\": %lu, \"not_ip_output_input\": %lu, \"short_chain\": %lu, "
		       "\"nobufs\": %lu, \"l4_gave_up\": %lu, \"udp_zero_to_ffff\": %lu}\n",
		       n, ncls[TXC_IN], ncls[TXC_NOT_IP], ncls[TXC_SHORT], ncls[TXC_NOBUFS], ngave, nffff);
		return 0;
	}
	if (mi_cksum_init(0)) {
		printf("{\"error\": \"mi_cksum_init: %s\"}\n", mi_cksum_strerror());
		return 1;
	}
	mi_tx_batch tb;
	memset(&tb, 0, sizeof tb);
	tb.src = srcB;
	tb.src_bytes = sbytes;
	tb.seg_off = d_off;
	tb.seg_len = d_len;
	tb.pkt_seg = pkt_seg;
	tb.pkt_len = d_plen;
	tb.csum_flags = d_flags;
	tb.csum_data = d_data;
	tb.dst = dstB;
	tb.dst_bytes = dbytes;
	tb.dst_stride = stride;
	tb.dst_first = first;
	tb.room = room;
	tb.l3_off = l3;
	tb.n = n;
	tb.max_len = maxlen;
	if (mi_cksum_host_register(srcB, (sbytes + 4095) & ~4095ull) ||
	    mi_cksum_host_register(dstB, (dbytes + 4095) & ~4095ull)) {
		printf("{\"error\": \"host_register: %s\"}\n", mi_cksum_strerror());
		return 1;
	}
	int rc = mi_cksum_tx_copy_host(&tb, stZ, 0);
	mi_cksum_host_unregister(srcB);
	mi_cksum_host_unregister(dstB);
	if (rc) {
		printf("{\"error\": \"mi_cksum_tx_copy_host (zero-copy): %d %s\"}\n", rc, mi_cksum_strerror());
		return 1;
	}
	tb.dst = dstS;
	if ((rc = mi_cksum_tx_copy_host(&tb, stS, MI_TX_HOST_STAGED))) {
		printf("{\"error\": \"mi_cksum_tx_copy_host (staged): %d %s\"}\n", rc, mi_cksum_strerror());
		return 1;
	}

	/* the slots, byte for byte; each frame's status from its route */
	unsigned long bytesZ = 0, bytesS = 0, stmisZ = 0, stmisS = 0, first_bad = ~0ul;
	for (uint64_t k = 0; k < dbytes; k++) {
		if (dstB[k] != dstA[k]) {
			bytesZ++;
			if (first_bad == ~0ul)
				first_bad = k;
		}
		bytesS += dstS[k] != dstA[k];
	}
	for (uint32_t i = 0; i < n; i++) {
		uint8_t want;
		int any = 0;
		switch (cls[i]) {
		case TXC_IN: want = gave[i] ? MI_TX_L4_SKIPPED : 0; break;
		case TXC_SHORT: want = MI_TX_SHORT; break;
		case TXC_NOBUFS: want = MI_TX_NOBUFS; break;
		default: want = 0; any = 1; break;  /* no offload request: copied, NOSUM if the header is bad */
		}
		stmisZ += any ? (stZ[i] & ~MI_TX_NOSUM) != 0 : stZ[i] != want;
		stmisS += any ? (stS[i] & ~MI_TX_NOSUM) != 0 : stS[i] != want;
	}
	printf("{\"frames\": %u, \"through_ip_output\": %lu, \"not_ip_output_input\": %lu, \"short_chain\": %lu, "
	       "\"nobufs\": %lu, \"l4_gave_up\": %lu, \"udp_zero_to_ffff\": %lu, \"slot_bytes\": %llu, "
	       "\"byte_mismatch_zero_copy\": %lu, \"byte_mismatch_staged\": %lu, \"status_mismatch_zero_copy\": %lu, "
	       "\"status_mismatch_staged\": %lu, \"first_bad_byte\": %ld}\n",
	       n, ncls[TXC_IN], ncls[TXC_NOT_IP], ncls[TXC_SHORT], ncls[TXC_NOBUFS], ngave, nffff,
	       (unsigned long long)dbytes, bytesZ, bytesS, stmisZ, stmisS, first_bad == ~0ul ? -1l : (long)first_bad);
	return bytesZ || bytesS || stmisZ || stmisS;
}
