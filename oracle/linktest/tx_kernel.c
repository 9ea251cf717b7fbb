/*
 * oracle/linktest/tx_kernel.c -- the TX offload contract checked against the
 * reference's own headers (TEST INFRASTRUCTURE ONLY: built into oracle/_ref/
 * by oracle/Makefile, like offload_kernel.c for RX).
 *
 * Compiled KERNEL-SIDE exactly like the reference's protocol code (REF_CFLAGS:
 * -nostdinc -D_KERNEL, the reference's <sys/mbuf.h>, <netinet/ip.h>,
 * <netinet/tcp.h>, <netinet/udp.h>), with in_cksum_* renamed to the
 * reference's own compiled in_cksum.c (ref_*, oracle/_ref/in_cksum.o):
 *
 *  1. static asserts: the csum_flags bits mi_cksum_tx_copy consumes, the
 *     CSUM_DELAY_* groupings and the csum_data defaults it assumes when none
 *     are given (include/mi_cksum_flags.h) are the reference's -- mbuf.h:
 *     281-305, offsetof(struct tcphdr, th_sum) (tcp_output.c:1066) and
 *     offsetof(struct udphdr, uh_sum) (udp_usrreq.c:1240);
 *  2. mi_tx_frame: one outgoing frame, as a chain of real struct mbufs,
 *     through the end of the stack's output path and the driver -- the
 *     transport's m_pkthdr seeding (tcp_output.c:1063-1085,
 *     udp_usrreq.c:1233-1241), ip_output's checksum decision and sums
 *     (ip_output.c:649-672, in_delayed_cksum :958-983, verbatim in shape),
 *     ether_output's M_PREPEND of the link header, and if_dpdk_transmit's
 *     buf_len check and m_copydata into the rte_mbuf (uinet_if_dpdk.c:583-597;
 *     m_copydata restated from uipc_mbuf.c:825-850).  With if_hwassist = 0 the
 *     sums are the reference's software ones (its own in_cksum_skip); with
 *     if_hwassist = CSUM_IP | CSUM_TCP | CSUM_UDP ip_output leaves them to the
 *     device and the frame's descriptors -- (m_data, m_len) of every mbuf,
 *     m_pkthdr.len / csum_flags / csum_data -- are what INTEGRATION.md section
 *     2b's inject-ring hook hands mi_cksum_tx_copy_host.
 *
 * oracle/linktest/tx_main.c runs both routes over the same frames and
 * compares the slots byte for byte (tests/test_link_gpu.py).
 */
#include <sys/cdefs.h>
#include <sys/param.h>
#include <sys/mbuf.h>
#include <sys/systm.h>
#include <netinet/in_systm.h>
#include <netinet/in.h>
#include <netinet/ip.h>
#include <netinet/tcp.h>
#include <netinet/udp.h>
#include <machine/in_cksum.h>

#include "mi_cksum_flags.h"

/* 1. the TX vocabulary of include/mi_cksum_flags.h is the reference's */
_Static_assert(MI_CSUM_IP == CSUM_IP, "CSUM_IP mbuf.h:281");
_Static_assert(MI_CSUM_TCP == CSUM_TCP, "CSUM_TCP mbuf.h:282");
_Static_assert(MI_CSUM_UDP == CSUM_UDP, "CSUM_UDP mbuf.h:283");
_Static_assert(MI_CSUM_DELAY_DATA == CSUM_DELAY_DATA, "CSUM_DELAY_DATA mbuf.h:304");
_Static_assert(MI_CSUM_DELAY_IP == CSUM_DELAY_IP, "CSUM_DELAY_IP mbuf.h:305");
_Static_assert(MI_CSUM_DATA_TCP == __offsetof(struct tcphdr, th_sum), "th_sum: tcp_output.c:1066");
_Static_assert(MI_CSUM_DATA_UDP == __offsetof(struct udphdr, uh_sum), "uh_sum: udp_usrreq.c:1240");
_Static_assert(__offsetof(struct mbuf, m_pkthdr.csum_flags) == MI_MBUF_CSUM_FLAGS_OFF, "csum_flags mbuf.h:123");
_Static_assert(__offsetof(struct mbuf, m_pkthdr.csum_data) == MI_MBUF_CSUM_DATA_OFF, "csum_data mbuf.h:124");
_Static_assert(sizeof(((struct mbuf *)0)->m_pkthdr.len) == 4, "m_pkthdr.len: the u32 pkt_len of mi_tx_batch");
_Static_assert(sizeof(((struct mbuf *)0)->m_len) == 4, "m_len: the i32 seg_len of mi_tx_batch");

/* frame classes (tx_main.c) */
#define TXC_IN		0	/* went through ip_output's checksum code */
#define TXC_NOT_IP	1	/* not a datagram ip_output takes (below) */
#define TXC_SHORT	2	/* chain holds < m_pkthdr.len bytes: m_copydata's KASSERT */
#define TXC_NOBUFS	3	/* m_pkthdr.len > buf_len: if_dpdk_transmit's ENOBUFS */

/* the one ifnet field ip_output's checksum code reads (ip_output.c:650,661) */
static struct {
	u_long	if_hwassist;
} ifnet_view;

/* what the last mi_tx_frame saw, for tx_main.c */
static int tx_gave_up;		/* in_delayed_cksum's "delayed m_pullup" return */
static int tx_udp_ffff;		/* in_delayed_cksum turned a UDP 0 into 0xffff */

int
mi_tx_mbuf_size(void)
{
	return ((int)sizeof(struct mbuf));
}

int
mi_tx_last_gave_up(void)
{
	return (tx_gave_up);
}

int
mi_tx_last_udp_ffff(void)
{
	return (tx_udp_ffff);
}

/*
 * in_delayed_cksum, ip_output.c:958-983: the software L4 sum, stored at
 * ip_hl * 4 + csum_data when that lies inside the first mbuf.  The give-up
 * branch prints in the reference; here it is counted.
 */
static void
tx_in_delayed_cksum(struct mbuf *m)
{
	struct ip *ip;
	uint16_t csum, offset, ip_len;

	ip = mtod(m, struct ip *);
	offset = ip->ip_hl << 2;
	ip_len = ntohs(ip->ip_len);
	csum = in_cksum_skip(m, ip_len, offset);
	if (m->m_pkthdr.csum_flags & CSUM_UDP && csum == 0) {
		csum = 0xffff;
		tx_udp_ffff = 1;
	}
	offset += m->m_pkthdr.csum_data;	/* checksum offset */

	if (offset + sizeof(u_short) > m->m_len) {
		tx_gave_up = 1;		/* printf("delayed m_pullup ...") */
		return;
	}
	*(u_short *)(m->m_data + offset) = csum;
}

/*
 * m_copydata, uipc_mbuf.c:825-850, restated (no M_HOLE mbufs here); the
 * KASSERT "length > size of mbuf chain" returns -1 instead of panicking.
 */
static int
tx_m_copydata(const struct mbuf *m, int off, int len, caddr_t cp)
{
	u_int count;

	while (off > 0) {
		if (m == NULL)
			return (-1);
		if (off < m->m_len)
			break;
		off -= m->m_len;
		m = m->m_next;
	}
	while (len > 0) {
		if (m == NULL)
			return (-1);
		count = min(m->m_len - off, len);
		bcopy(mtod(m, caddr_t) + off, cp, count);
		len -= count;
		cp += count;
		off = 0;
		m = m->m_next;
	}
	return (0);
}

/*
 * One outgoing frame (see the file comment).  The chain is built in `pool`
 * (k1 - k0 mbufs) over `blob`: mbuf j has m_data = blob + seg_off[k0 + j],
 * m_len = seg_len[k0 + j]; the first carries M_PKTHDR and m_pkthdr.len =
 * pkt_len.  The IP header sits l3_off bytes into the frame: the link header
 * ether_output prepends after ip_output (M_PREPEND into the IP mbuf's leading
 * space when the header mbuf holds both).
 *
 * Transport seeding (have_flags == 0): TCP csum_flags = CSUM_TCP, csum_data =
 * offsetof(struct tcphdr, th_sum) (tcp_output.c:1066,1083); UDP CSUM_UDP and
 * offsetof(struct udphdr, uh_sum) (udp_usrreq.c:1238-1240); anything else
 * none.  have_flags: the caller's (tflags, tdata) stand for what the
 * transport left in m_pkthdr.
 *
 * A frame ip_output never receives gets TXC_NOT_IP and is copied as is with
 * no offload request (csum_flags 0): its IP header does not lie whole in the
 * mbuf holding its first byte (ip = mtod(m, struct ip *), ip_output.c:
 * 225-252, tcp_output / udp_output always build it so), hl < 20, or its
 * ip_len fails rip_output's checks (raw_ip.c:494-500: ip_len > m_pkthdr.len
 * or < hl).
 *
 * slot != NULL: the driver copies the frame there (the software route's wire
 * bytes).  d_off / d_len / d_flags / d_data / d_pkt_len != NULL: the
 * offload route's descriptors, read from the mbufs after ip_output
 * (m_data - blob, m_len, m_pkthdr.len / csum_flags / csum_data).
 */
int
mi_tx_frame(struct mbuf *pool, char *blob, const uint64_t *seg_off, const int32_t *seg_len, uint32_t k0,
    uint32_t k1, uint32_t pkt_len, uint32_t l3_off, int have_flags, uint32_t tflags, uint32_t tdata,
    u_long hwassist, char *slot, uint32_t buf_len, uint64_t *d_off, int32_t *d_len, uint32_t *d_flags,
    uint32_t *d_data, uint32_t *d_pkt_len)
{
	struct mbuf *head, *m, *ipm;
	struct ip *ip;
	uint32_t j, nseg = k1 - k0;
	int64_t total = 0, pos = 0;
	int cls = TXC_IN, hlen, d, len;
	uint16_t sw_csum;

	tx_gave_up = 0;
	tx_udp_ffff = 0;
	ifnet_view.if_hwassist = hwassist;
	if (nseg == 0)
		return (TXC_SHORT);
	for (j = 0; j < nseg; j++) {
		m = &pool[j];
		bzero(m, sizeof(*m));
		m->m_data = blob + seg_off[k0 + j];
		m->m_len = seg_len[k0 + j];
		m->m_next = j + 1 < nseg ? &pool[j + 1] : NULL;
		total += m->m_len;
	}
	head = &pool[0];
	head->m_flags = M_PKTHDR;
	head->m_pkthdr.len = (int)pkt_len;
	if (total < (int64_t)pkt_len)
		cls = TXC_SHORT;

	/* the mbuf holding frame byte l3_off: the IP mbuf before M_PREPEND */
	ipm = NULL;
	d = 0;
	for (m = head; m != NULL && cls == TXC_IN; m = m->m_next) {
		if (m->m_len > 0 && pos <= l3_off && l3_off < pos + m->m_len) {
			ipm = m;
			d = (int)(l3_off - pos);
			break;
		}
		pos += m->m_len;
	}
	if (cls == TXC_IN) {
		ip = ipm != NULL ? (struct ip *)(ipm->m_data + d) : NULL;
		if (ip == NULL || ipm->m_len - d < (int)sizeof(struct ip) ||
		    (ip->ip_hl << 2) < (int)sizeof(struct ip) || (ip->ip_hl << 2) > ipm->m_len - d ||
		    ntohs(ip->ip_len) > (int)pkt_len - (int)l3_off || ntohs(ip->ip_len) < (ip->ip_hl << 2))
			cls = TXC_NOT_IP;
	}

	if (cls == TXC_IN) {
		/* the chain as ip_output gets it: from the IP header on, the
		 * packet header on its first mbuf with the transport's seeding */
		ipm->m_data += d;
		ipm->m_len -= d;
		ipm->m_flags |= M_PKTHDR;
		ipm->m_pkthdr.len = (int)(pkt_len - l3_off);
		ip = mtod(ipm, struct ip *);
		if (have_flags) {
			ipm->m_pkthdr.csum_flags = tflags;
			ipm->m_pkthdr.csum_data = tdata;
		} else if (ip->ip_p == IPPROTO_TCP) {
			ipm->m_pkthdr.csum_flags = CSUM_TCP;
			ipm->m_pkthdr.csum_data = offsetof(struct tcphdr, th_sum);
		} else if (ip->ip_p == IPPROTO_UDP) {
			ipm->m_pkthdr.csum_flags = CSUM_UDP;
			ipm->m_pkthdr.csum_data = offsetof(struct udphdr, uh_sum);
		}
		m = ipm;
		hlen = ip->ip_hl << 2;

		/* ip_output.c:649-654, 661 */
		m->m_pkthdr.csum_flags |= CSUM_IP;
		sw_csum = m->m_pkthdr.csum_flags & ~ifnet_view.if_hwassist;
		if (sw_csum & CSUM_DELAY_DATA) {
			tx_in_delayed_cksum(m);
			sw_csum &= ~CSUM_DELAY_DATA;
		}
		m->m_pkthdr.csum_flags &= ifnet_view.if_hwassist;
		/* ip_output.c:666-672, the frame fits the interface (ip_len <= mtu) */
		ip->ip_sum = 0;
		if (sw_csum & CSUM_DELAY_IP)
			ip->ip_sum = in_cksum(m, hlen);

		/* ether_output's M_PREPEND (into the leading space when the IP
		 * mbuf holds the link header too); M_MOVE_PKTHDR to the head */
		ipm->m_data -= d;
		ipm->m_len += d;
		if (ipm != head) {
			head->m_pkthdr.csum_flags = ipm->m_pkthdr.csum_flags;
			head->m_pkthdr.csum_data = ipm->m_pkthdr.csum_data;
			ipm->m_flags &= ~M_PKTHDR;
		}
		head->m_pkthdr.len = ipm->m_pkthdr.len + (int)l3_off;
	}

	/* if_dpdk_transmit, uinet_if_dpdk.c:583-597 */
	len = head->m_pkthdr.len;
	if (len > (int)buf_len)
		cls = TXC_NOBUFS;
	if (slot != NULL && cls != TXC_NOBUFS && cls != TXC_SHORT)
		if (tx_m_copydata(head, 0, len, slot) != 0)
			cls = TXC_SHORT;
	if (d_off != NULL) {
		/* the inject-ring hook: per mbuf m_data /
		 * m_len, per frame the packet header's fields */
		for (m = head, j = k0; m != NULL; m = m->m_next, j++) {
			d_off[j] = (uint64_t)(m->m_data - blob);
			d_len[j] = m->m_len;
		}
		*d_flags = cls == TXC_NOT_IP ? 0 : head->m_pkthdr.csum_flags;
		*d_data = cls == TXC_NOT_IP ? 0 : head->m_pkthdr.csum_data;
		*d_pkt_len = (uint32_t)head->m_pkthdr.len;
	}
	return (cls);
}
