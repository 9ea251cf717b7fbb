/*
 * oracle/linktest/kat_kernel.c -- a KERNEL-SIDE caller of the checksum ABI,
 * compiled exactly like the reference's protocol code: the reference's own
 * headers (<sys/mbuf.h>, <netinet/ip.h>, <machine/in_cksum.h>
 * src/sys/amd64/include/in_cksum.h:77-83) under its kernel flags (-nostdinc
 * -D_KERNEL -include opt_global.h ..., oracle/Makefile REF_CFLAGS, the recipe
 * of src/lib/libuinet/Makefile / src/mk/kern.mk).  It is linked against
 * libmicksum.so in place of in_cksum.o (the MACHINE_SRCS object,
 * src/lib/libuinet/Makefile:275-276), which is the substitution INTEGRATION.md
 * section 1 describes.  TEST INFRASTRUCTURE ONLY: built into oracle/_ref/.
 *
 * It runs the SURVEY.md 8(a) known-answer tests through real struct mbuf
 * chains and struct ip headers of the reference's own definitions, and stores
 * the results for the host-side driver (main.c) to check.
 */
#include <sys/cdefs.h>
#include <sys/param.h>
#include <sys/mbuf.h>
#include <sys/systm.h>
#include <netinet/in_systm.h>
#include <netinet/in.h>
#include <netinet/ip.h>
#include <machine/in_cksum.h>

#define NKAT 40

static char buf[70000 + 256] __aligned(64);
static char hdrbuf[256] __aligned(64);
static struct mbuf mb[4];

unsigned int mi_link_got[NKAT];

static void
fill_ramp(char *p, int n, int start)
{
	int i;

	for (i = 0; i < n; i++)
		p[i] = (char)((i + start) & 0xff);
}

static struct mbuf *
one_mbuf(char *data, int len)
{
	mb[0].m_next = NULL;
	mb[0].m_data = data;
	mb[0].m_len = len;
	return (&mb[0]);
}

static const unsigned char kat2_hdr[20] = {
	0x45, 0x00, 0x00, 0x73, 0x00, 0x00, 0x40, 0x00, 0x40, 0x11,
	0x00, 0x00, 0xc0, 0xa8, 0x00, 0x01, 0xc0, 0xa8, 0x00, 0xc7 };

static u_int
hdr_at(int mod)
{
	int i;

	for (i = 0; i < 20; i++)
		hdrbuf[64 + mod + i] = (char)kat2_hdr[i];
	return (in_cksum_hdr((const struct ip *)(void *)&hdrbuf[64 + mod]));
}

/* Returns the number of results stored in mi_link_got[]. */
int
mi_link_kats(void)
{
	static const unsigned char rfc[8] = { 0x00, 0x01, 0xf2, 0x03, 0xf4, 0xf5, 0xf6, 0xf7 };
	static const int lens7[10] = { 1, 2, 3, 63, 64, 1500, 1501, 9000, 65535, 65536 };
	static const int lens7b[5] = { 1, 64, 1500, 9000, 65536 };
	struct mbuf *m;
	int i, k = 0;
	uint32_t src, dst;

	/* KAT1: RFC 1071 section 3 example */
	for (i = 0; i < 8; i++)
		buf[i] = (char)rfc[i];
	mi_link_got[k++] = in_cksum(one_mbuf(buf, 8), 8);
	/* KAT2-4: in_cksum_hdr at 4-aligned, 2 mod 4, odd addresses */
	mi_link_got[k++] = hdr_at(0);
	mi_link_got[k++] = hdr_at(2);
	mi_link_got[k++] = hdr_at(1);
	/* KAT5 / KAT6: 1500 zero bytes, 1500 0xff bytes */
	for (i = 0; i < 1500; i++)
		buf[i] = 0;
	mi_link_got[k++] = in_cksum(one_mbuf(buf, 1500), 1500);
	for (i = 0; i < 1500; i++)
		buf[i] = (char)0xff;
	mi_link_got[k++] = in_cksum(one_mbuf(buf, 1500), 1500);
	/* KAT7: b[i] = i & 0xff, 64-aligned; KAT7b: read from base + 1 */
	fill_ramp(buf, 65536 + 64, 0);
	for (i = 0; i < 10; i++)
		mi_link_got[k++] = in_cksum(one_mbuf(buf, lens7[i]), lens7[i]);
	for (i = 0; i < 5; i++)
		mi_link_got[k++] = in_cksum(one_mbuf(buf + 1, lens7b[i]), lens7b[i]);
	/* KAT8 / KAT9: pseudo header, 192.168.1.1 -> 192.168.1.2, off0 = 20 */
	src = htonl(0xc0a80101);
	dst = htonl(0xc0a80102);
	m = one_mbuf(buf, 1500);
	mi_link_got[k++] = in_cksum_pseudo_header(m, 1480, 20, src, dst, IPPROTO_TCP);
	m = one_mbuf(buf, 9000);
	mi_link_got[k++] = in_cksum_pseudo_header(m, 8980, 20, src, dst, IPPROTO_UDP);
	/* KAT10: in_pseudo(src, dst, htons(20 + 6 + 1460)) */
	mi_link_got[k++] = in_pseudo(src, dst, htons(20 + IPPROTO_TCP + 1460));
	/* KAT11: the KAT7 1500 bytes as a 701 + 799 chain, 2nd mbuf at an odd address */
	for (i = 0; i < 799; i++)
		buf[20001 + i] = (char)((701 + i) & 0xff);
	mb[0].m_next = &mb[1];
	mb[0].m_data = buf;
	mb[0].m_len = 701;
	mb[1].m_next = NULL;
	mb[1].m_data = &buf[20001];
	mb[1].m_len = 799;
	mi_link_got[k++] = in_cksum(&mb[0], 1500);
	/* KAT12: KAT7 1500 bytes, skip 20 */
	mi_link_got[k++] = in_cksum_skip(one_mbuf(buf, 1500), 1500, 20);
	/* in_addword: end-around carry */
	mi_link_got[k++] = in_addword(0xffff, 0x0001);
	mi_link_got[k++] = in_addword(0x1234, 0x4321);
	return (k);
}
