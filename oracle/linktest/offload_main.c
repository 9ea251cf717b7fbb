/*
 * oracle/linktest/offload_main.c -- host-side driver of offload_kernel.c (TEST
 * INFRASTRUCTURE ONLY).  One burst of datagrams (a file written by
 * tests/test_link_gpu.py from tests/golden/demux_golden.npz) goes through the
 * RX offload hook the way INTEGRATION.md section 2 wires it at the DPDK batch
 * point: the burst in registered host memory, mi_cksum_rx_offload_host on the
 * GPU, the flags stored into real struct mbufs (kernel-side hook).  Every
 * datagram then takes the reference's input path twice -- with the flags
 * (offload branches) and without (the reference's own in_cksum_* software
 * branches) -- and the two accept/drop decisions and tested sums must agree.
 * A second pass does the same through the staged (copy) transport.
 * Prints one JSON line; exit status 0 iff nothing differs and both offload
 * branches were taken.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cksum.h"

extern int mi_offload_decide(char *dgram, int flen, uint32_t flags, uint32_t data, int offload, uint32_t *l4_sum);
extern int mi_offload_branches(void);

#define NDEC 13

static int run(const char *tag, uint8_t *buf, uint64_t bytes, const uint64_t *offs, const uint32_t *flen,
               uint32_t n, uint32_t bflags, int last)
{
	uint32_t *fl = calloc(n, 4), *cd = calloc(n, 4);
	unsigned long dec[NDEC] = {0};
	unsigned long dmis = 0, vmis = 0, ipoff = 0, l4off = 0, l4cmp = 0;
	uint32_t i, maxl = 0;
	int rc, k;

	for (i = 0; i < n; i++)
		if (flen[i] > maxl)
			maxl = flen[i];
	mi_pkt_batch b;
	memset(&b, 0, sizeof b);
	b.base = buf;
	b.bytes = bytes;
	b.offs = offs;
	b.lens = flen;
	b.n = n;
	b.max_len = maxl;
	b.flags = bflags;
	rc = mi_cksum_rx_offload_host(&b, fl, cd, NULL);
	if (rc) {
		printf("{\"error\": \"mi_cksum_rx_offload_host: %d %s\"}\n", rc, mi_cksum_strerror());
		exit(1);
	}
	for (i = 0; i < n; i++) {
		uint32_t s1, s0;
		int d1 = mi_offload_decide((char *)buf + offs[i], (int)flen[i], fl[i], cd[i], 1, &s1);
		int br = mi_offload_branches();
		int d0 = mi_offload_decide((char *)buf + offs[i], (int)flen[i], 0, 0, 0, &s0);

		dmis += d1 != d0;
		if (s1 != 0xffffffffu || s0 != 0xffffffffu) {
			l4cmp++;
			vmis += s1 != s0;
		}
		ipoff += (br & 1) != 0;
		l4off += (br & 2) != 0 && s1 != 0xffffffffu;
		if (d0 >= 0 && d0 < NDEC)
			dec[d0]++;
	}
	printf("\"%s\": {\"datagrams\": %u, \"decision_mismatch\": %lu, \"l4_value_mismatch\": %lu, "
	       "\"l4_values_compared\": %lu, \"ip_from_flags\": %lu, \"l4_from_csum_data\": %lu, \"decisions\": [",
	       tag, n, dmis, vmis, l4cmp, ipoff, l4off);
	for (k = 0; k < NDEC; k++)
		printf("%s%lu", k ? ", " : "", dec[k]);
	printf("]}%s", last ? "" : ", ");
	free(fl);
	free(cd);
	return dmis == 0 && vmis == 0 && ipoff > 0 && l4off > 0;
}

int main(int argc, char **argv)
{
	FILE *f;
	uint32_t hdr[4], n;
	uint64_t bytes;
	uint8_t *raw, *buf;
	uint64_t *offs;
	uint32_t *flen;
	int ok;

	if (argc != 2 || !(f = fopen(argv[1], "rb"))) {
		fprintf(stderr, "usage: offload_test BURST_FILE\n");
		return 2;
	}
	/* u32 magic 'MIOB', u32 n, u64 bytes; bytes of buffer; n u64 offs; n u32 lens */
	if (fread(hdr, 4, 4, f) != 4 || hdr[0] != 0x424f494du)
		return 2;
	n = hdr[1];
	memcpy(&bytes, &hdr[2], 8);
	raw = malloc(bytes + 2 * 4096);
	buf = (uint8_t *)(((uintptr_t)raw + 4095) & ~(uintptr_t)4095);
	offs = malloc(8ull * n);
	flen = malloc(4ull * n);
	if (fread(buf, 1, bytes, f) != bytes || fread(offs, 8, n, f) != n || fread(flen, 4, n, f) != n)
		return 2;
	fclose(f);
	if (mi_cksum_init(0)) {
		printf("{\"error\": \"mi_cksum_init: %s\"}\n", mi_cksum_strerror());
		return 1;
	}
	printf("{");
	if (mi_cksum_host_register(buf, (bytes + 4095) & ~4095ull)) {
		printf("\"error\": \"host_register: %s\"}\n", mi_cksum_strerror());
		return 1;
	}
	ok = run("zero_copy", buf, bytes, offs, flen, n, 0, 0);
	mi_cksum_host_unregister(buf);
	ok &= run("staged", buf, bytes, offs, flen, n, MI_BATCH_HOST_STAGED, 1);
	printf("}\n");
	return ok ? 0 : 1;
}
