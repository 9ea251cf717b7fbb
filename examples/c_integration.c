/*
 * examples/c_integration.c -- what libunsod's C code sees of libmicksum: the
 * header and the link line, nothing else (no HIP, no Python).
 *
 *   1. (b1) the reference's drop-in symbols over real mbuf chains (struct
 *      layout of src/sys/sys/mbuf.h:90-98: m_next@0, m_data@16, m_len@24),
 *      checked against the SURVEY.md 8(a) known answers, called from several
 *      threads at once (the reference calls them from the dpdk_rx kthread, the
 *      application threads and the callout thread concurrently), folded on
 *      the CPU (the default) and through the GPU drop-in service.
 *   2. (b2) a host-memory RX burst as the DPDK driver holds it (rte_mbuf slots
 *      of 2176 B, IP header at +142): TX-finalized, registered, verified in
 *      place over PCIe, then one corrupted datagram detected.
 *
 * Built by libunsod_amd/csrc/Makefile (into libunsod_amd/lib/) with plain gcc:
 *   gcc -O2 -pthread -Iinclude examples/c_integration.c -Llibunsod_amd/lib -lmicksum
 * Prints "c_integration ok" and exits 0 when every check holds.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_cksum.h"

/* The reference's mbuf, as far as the checksum reads it (MSIZE 256). */
struct mbuf {
	struct mbuf *m_next;
	struct mbuf *m_nextpkt;
	char        *m_data;
	int          m_len;
	int          m_flags;
	char         pad[256 - 32];
};
_Static_assert(offsetof(struct mbuf, m_data) == 16, "m_data@16");
_Static_assert(offsetof(struct mbuf, m_len) == 24, "m_len@24");

static int fails;
#define CHECK(cond, ...)                                                  \
	do {                                                              \
		if (!(cond)) {                                            \
			fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
			fprintf(stderr, __VA_ARGS__);                     \
			fputc('\n', stderr);                              \
			__atomic_add_fetch(&fails, 1, __ATOMIC_RELAXED);  \
		}                                                         \
	} while (0)

static uint8_t pat[65536 + 64] __attribute__((aligned(64)));

/* KAT7 / KAT7b / KAT11 / KAT8 of SURVEY.md 8(a). */
static void *dropin_thread(void *arg)
{
	const int id = (int)(intptr_t)arg;
	for (int it = 0; it < 20; it++) {
		struct mbuf m0, m1;
		memset(&m0, 0, sizeof m0);
		memset(&m1, 0, sizeof m1);
		m0.m_data = (char *)pat;
		m0.m_len = 1500;
		CHECK(in_cksum(&m0, 1500) == 0x4e39, "thread %d KAT7 1500", id);
		m0.m_len = 9000;
		CHECK(in_cksum_skip(&m0, 9000, 0) == 0xb739, "thread %d KAT7 9000", id);
		m0.m_data = (char *)pat + 1; /* odd address: bytes (i + 1) & 0xff */
		m0.m_len = 1500;
		CHECK(in_cksum(&m0, 1500) == 0x5d4d, "thread %d KAT7b", id);
		/* KAT11: 701 + 799 chain, the second mbuf at an odd address */
		uint8_t seg2[800 + 16] __attribute__((aligned(16)));
		uint8_t *s2 = seg2 + 1;
		memcpy(s2, pat + 701, 799);
		m0.m_data = (char *)pat;
		m0.m_len = 701;
		m0.m_next = &m1;
		m1.m_data = (char *)s2;
		m1.m_len = 799;
		CHECK(in_cksum_skip(&m0, 1500, 0) == 0x4e39, "thread %d KAT11", id);
		/* KAT12: skip 20 */
		m0.m_next = NULL;
		m0.m_len = 1500;
		CHECK(in_cksum_skip(&m0, 1500, 20) == 0xb293, "thread %d KAT12", id);
		/* KAT8: TCP pseudo header, 192.168.1.1 -> 192.168.1.2 */
		const uint32_t src = 0x0101a8c0u, dst = 0x0201a8c0u; /* loaded from network order */
		CHECK(in_cksum_pseudo_header(&m0, 1480, 20, src, dst, 6) == 0x900a, "thread %d KAT8", id);
	}
	return NULL;
}

static void be16(uint8_t *p, unsigned v)
{
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}

int main(void)
{
	for (size_t i = 0; i < sizeof pat; i++)
		pat[i] = (uint8_t)i;
	if (mi_cksum_device_count() < 1 || mi_cksum_init(0) != 0) {
		fprintf(stderr, "no gfx950 device: %s\n", mi_cksum_strerror());
		return 2;
	}
	printf("%s\n", mi_cksum_version());

	/* scalar ABI: header KATs (KAT2 / KAT4) and integer helpers (KAT10) */
	static const uint8_t hdr[20] = {0x45, 0, 0, 0x73, 0, 0, 0x40, 0, 0x40, 0x11, 0, 0,
	                                0xc0, 0xa8, 0, 1, 0xc0, 0xa8, 0, 0xc7};
	static uint8_t hb[64] __attribute__((aligned(64)));
	memcpy(hb + 4, hdr, 20);
	memcpy(hb + 33, hdr, 20);
	CHECK(in_cksum_hdr((const struct ip *)(hb + 4)) == 0x61b8, "KAT2");
	CHECK(in_cksum_hdr((const struct ip *)(hb + 33)) == 0xb861, "KAT4 (odd address)");
	CHECK(in_pseudo(0x0101a8c0u, 0x0201a8c0u, 0xce050000u) == 0x2289, "KAT10");

	/* the drop-ins from 8 threads at once: folded on the calling cores (the
	 * default, MI_DROPIN_HOST), then through the GPU's drop-in service
	 * (MI_DROPIN_GPU) -- with no call answered by the host fold after a GPU
	 * error */
	const uint64_t degraded = mi_cksum_dropin_degraded();
	for (int mode = MI_DROPIN_HOST; mode <= MI_DROPIN_GPU; mode++) {
		const int was = mi_cksum_set_dropin_mode(mode);
		pthread_t th[8];
		for (int t = 0; t < 8; t++)
			pthread_create(&th[t], NULL, dropin_thread, (void *)(intptr_t)t);
		for (int t = 0; t < 8; t++)
			pthread_join(th[t], NULL);
		mi_cksum_set_dropin_mode(was);
	}
	CHECK(mi_cksum_dropin_degraded() == degraded, "GPU-mode drop-ins degraded to the host fold");

	/* a host-memory RX burst: 1024 x 1500 B datagrams in rte_mbuf slots,
	 * checksummed on the way out by the software TX path through the drop-ins
	 * (tcp_output.c:1084 seed, in_delayed_cksum ip_output.c:966, ip_sum
	 * ip_output.c:670-672) */
	const uint32_t n = 1024, L = 1500, stride = 2176, first = 142;
	const uint64_t bytes = (uint64_t)first + (uint64_t)(n - 1) * stride + L + 64;
	const uint64_t alloc = (bytes + 4095) & ~4095ull;
	uint8_t *pool = aligned_alloc(4096, alloc);
	CHECK(pool != NULL, "alloc");
	memset(pool, 0, alloc);
	for (uint32_t i = 0; i < n; i++) {
		uint8_t *ip = pool + first + (uint64_t)i * stride;
		for (uint32_t k = 40; k < L; k++)
			ip[k] = (uint8_t)(k * 7 + i);
		ip[0] = 0x45;
		be16(ip + 2, L);
		ip[6] = 0x40;
		ip[8] = 64;
		ip[9] = 6;
		ip[12] = 10; ip[13] = 0; ip[14] = (uint8_t)(i >> 8); ip[15] = (uint8_t)i;
		ip[16] = 10; ip[17] = 1; ip[18] = (uint8_t)(i >> 8); ip[19] = (uint8_t)i;
		ip[32] = 0x50; /* th_off = 5 */
		uint32_t s, d;
		memcpy(&s, ip + 12, 4);
		memcpy(&d, ip + 16, 4);
		const uint32_t tl = L - 20 + 6; /* htons(tcp length + IPPROTO_TCP) */
		uint16_t c = in_pseudo(s, d, ((tl & 0xff) << 8) | (tl >> 8));
		memcpy(ip + 36, &c, 2);
		struct mbuf m;
		memset(&m, 0, sizeof m);
		m.m_data = (char *)ip;
		m.m_len = (int)L;
		c = in_cksum_skip(&m, (int)L, 20);
		memcpy(ip + 36, &c, 2);
		c = in_cksum(&m, 20);
		memcpy(ip + 10, &c, 2);
	}
	mi_pkt_batch b;
	memset(&b, 0, sizeof b);
	b.base = pool;
	b.bytes = bytes;
	b.stride = stride;
	b.first_off = first;
	b.fixed_len = L;
	b.n = n;
	uint16_t *ip_sum = calloc(n, 2), *l4_sum = calloc(n, 2);
	uint8_t *status = calloc(n, 1);
	uint32_t bad = 0;
	/* page-lock + map the pool once: the verify kernel then reads it in place */
	CHECK(mi_cksum_host_register(pool, alloc) == 0, "register: %s", mi_cksum_strerror());
	CHECK(mi_cksum_ipv4_verify_host(&b, ip_sum, l4_sum, status, &bad) == 0, "verify_host: %s", mi_cksum_strerror());
	CHECK(bad == 0, "valid burst: %u bad", bad);
	pool[first + 777u * stride + 900] ^= 0x10;
	CHECK(mi_cksum_ipv4_verify_host(&b, ip_sum, l4_sum, status, &bad) == 0, "verify_host: %s", mi_cksum_strerror());
	CHECK(bad == 1 && status[777] == MI_ST_L4_BAD, "corrupted datagram: bad %u status %u", bad, status[777]);
	mi_cksum_host_unregister(pool);
	free(pool);
	free(ip_sum);
	free(l4_sum);
	free(status);
	if (fails) {
		fprintf(stderr, "c_integration: %d failures\n", fails);
		return 1;
	}
	printf("c_integration ok\n");
	return 0;
}
