/*
 * oracle/linktest/offload_kernel.c -- the RX offload contract checked against
 * the reference's own headers (TEST INFRASTRUCTURE ONLY: built into
 * oracle/_ref/ by oracle/Makefile, like kat_kernel.c).
 *
 * Compiled KERNEL-SIDE exactly like the reference's protocol code (REF_CFLAGS:
 * -nostdinc -D_KERNEL, the reference's <sys/mbuf.h>, <netinet/ip.h>,
 * <netinet/tcp.h>, <netinet/udp.h>), with in_cksum_* renamed to the
 * reference's own compiled in_cksum.c (ref_*, oracle/_ref/in_cksum.o):
 *
 *  1. static asserts: the flag values mi_cksum_rx_offload produces and the
 *     m_pkthdr field offsets of include/mi_cksum_flags.h are the reference's
 *     (src/sys/sys/mbuf.h:123-124, 281-293);
 *  2. mi_offload_hook: INTEGRATION.md section 2's per-burst hook, as written
 *     there, storing a GPU burst's flags into real struct mbufs;
 *  3. mi_offload_decide: the accept/drop path a datagram takes through
 *     ip_input (src/sys/netinet/ip_input.c:421-505), tcp_input
 *     (tcp_input.c:688-720) and udp_input (udp_usrreq.c:375-451), restated
 *     step by step with the reference's field names -- their checksum
 *     branches (ip_input.c:459-471, tcp_input.c:698-716, udp_usrreq.c:429-450)
 *     verbatim in shape: with the hook's flags the offload branches
 *     (th_sum = csum_data ^ 0xffff), without them the software branches
 *     (the reference's in_cksum_hdr / in_cksum / in_cksum_pseudo_header).
 *
 * oracle/linktest/offload_main.c runs one GPU burst of the demux golden
 * datagrams through mi_cksum_rx_offload_host and compares the two paths per
 * datagram (tests/test_link_gpu.py).
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

/* 1. the vocabulary of include/mi_cksum_flags.h is the reference's */
_Static_assert(MI_CSUM_IP == CSUM_IP, "CSUM_IP mbuf.h:281");
_Static_assert(MI_CSUM_TCP == CSUM_TCP, "CSUM_TCP mbuf.h:282");
_Static_assert(MI_CSUM_UDP == CSUM_UDP, "CSUM_UDP mbuf.h:283");
_Static_assert(MI_CSUM_IP_CHECKED == CSUM_IP_CHECKED, "CSUM_IP_CHECKED mbuf.h:290");
_Static_assert(MI_CSUM_IP_VALID == CSUM_IP_VALID, "CSUM_IP_VALID mbuf.h:291");
_Static_assert(MI_CSUM_DATA_VALID == CSUM_DATA_VALID, "CSUM_DATA_VALID mbuf.h:292");
_Static_assert(MI_CSUM_PSEUDO_HDR == CSUM_PSEUDO_HDR, "CSUM_PSEUDO_HDR mbuf.h:293");
_Static_assert(__offsetof(struct mbuf, m_pkthdr) == MI_MBUF_PKTHDR_OFF, "m_pkthdr");
_Static_assert(__offsetof(struct mbuf, m_pkthdr.csum_flags) == MI_MBUF_CSUM_FLAGS_OFF, "csum_flags mbuf.h:123");
_Static_assert(__offsetof(struct mbuf, m_pkthdr.csum_data) == MI_MBUF_CSUM_DATA_OFF, "csum_data mbuf.h:124");
_Static_assert(sizeof(((struct mbuf *)0)->m_pkthdr.csum_flags) == 4, "csum_flags is a 32-bit int");
_Static_assert(sizeof(((struct mbuf *)0)->m_pkthdr.csum_data) == 4, "csum_data is a 32-bit int");

/* decisions (the counter each drop increments in the reference) */
#define D_ACCEPT	0	/* handed to the protocol's socket layer */
#define D_TOOSHORT	1	/* ips_tooshort / ips_toosmall */
#define D_BADVERS	2	/* ips_badvers */
#define D_BADHLEN	3	/* ips_badhlen */
#define D_IP_BADSUM	4	/* ips_badsum */
#define D_BADLEN	5	/* ips_badlen / ips_tooshort (ip_len) */
#define D_REASS		6	/* fragment: to ip_reass, no L4 check here */
#define D_L4_SHORT	7	/* tcps_rcvshort / udps_hdrops */
#define D_L4_BADSUM	8	/* tcps_rcvbadsum / udps_badsum */
#define D_UDP_BADLEN	9	/* udps_badlen */
#define D_UDP_NOSUM	10	/* udps_nosum: accepted without a check */
#define D_UDP_PORT0	11	/* uh_dport == 0 */
#define D_OTHER		12	/* another protocol: no checksum on this path */

static struct mbuf mb;

/*
 * 2. INTEGRATION.md section 2's hook (per datagram of a burst):
 *	m->m_pkthdr.csum_flags |= csum_flags[i];
 *	m->m_pkthdr.csum_data = csum_data[i];
 */
static void
mi_offload_hook(struct mbuf *m, uint32_t csum_flags, uint32_t csum_data)
{
	m->m_pkthdr.csum_flags |= csum_flags;
	m->m_pkthdr.csum_data = csum_data;
}

/*
 * 3. One datagram (IP header at `dgram`, `flen` bytes delivered) through the
 * input path.  offload != 0: the hook stored (flags, data) first, as
 * if_dpdk_batch_receive would before uinet_pd_deliver_to_stack.  *l4_sum gets
 * the value the transport tested (th_sum / uh_sum; 0xffffffff if none).
 */
int
mi_offload_decide(char *dgram, int flen, uint32_t flags, uint32_t data, int offload, uint32_t *l4_sum)
{
	struct mbuf *m = &mb;
	struct ip *ip;
	int hlen, off0, tlen, len, uip_len;
	uint16_t sum, ip_len;

	*l4_sum = 0xffffffffu;
	bzero(m, sizeof(*m));
	m->m_next = NULL;
	m->m_data = dgram;
	m->m_len = flen;
	m->m_flags = M_PKTHDR;
	m->m_pkthdr.len = flen;
	if (offload)
		mi_offload_hook(m, flags, data);

	/* ip_input.c:421-449 */
	if (m->m_pkthdr.len < (int)sizeof(struct ip))
		return (D_TOOSHORT);
	ip = mtod(m, struct ip *);
	if (ip->ip_v != IPVERSION)
		return (D_BADVERS);
	hlen = ip->ip_hl << 2;
	if (hlen < (int)sizeof(struct ip))
		return (D_BADHLEN);
	if (hlen > m->m_len)		/* m_pullup(m, hlen) fails: not that many bytes */
		return (D_BADHLEN);

	/* ip_input.c:459-471 */
	if (m->m_pkthdr.csum_flags & CSUM_IP_CHECKED) {
		sum = !(m->m_pkthdr.csum_flags & CSUM_IP_VALID);
	} else {
		if (hlen == sizeof(struct ip)) {
			sum = in_cksum_hdr(ip);
		} else {
			sum = in_cksum(m, hlen);
		}
	}
	if (sum)
		return (D_IP_BADSUM);

	/* ip_input.c:482-505 */
	ip_len = ntohs(ip->ip_len);
	if (ip_len < hlen)
		return (D_BADLEN);
	if (m->m_pkthdr.len < ip_len)
		return (D_BADLEN);
	if (m->m_pkthdr.len > ip_len) {
		m->m_len = ip_len;
		m->m_pkthdr.len = ip_len;
	}
	/* ip_input.c: fragments go to ip_reass before the protocol switch */
	if (ip->ip_off & htons(IP_MF | IP_OFFMASK))
		return (D_REASS);

	if (ip->ip_p == IPPROTO_TCP) {
		u_short th_sum;

		/* tcp_input.c:688-696 */
		off0 = hlen;
		if (m->m_len < off0 + (int)sizeof(struct tcphdr))
			return (D_L4_SHORT);
		tlen = ntohs(ip->ip_len) - off0;
		/* tcp_input.c:698-716 */
		if (m->m_pkthdr.csum_flags & CSUM_DATA_VALID) {
			if (m->m_pkthdr.csum_flags & CSUM_PSEUDO_HDR)
				th_sum = m->m_pkthdr.csum_data;
			else
				th_sum = in_pseudo(ip->ip_src.s_addr,
						ip->ip_dst.s_addr,
						htonl(m->m_pkthdr.csum_data +
							tlen +
							IPPROTO_TCP));
			th_sum ^= 0xffff;
		} else {
			th_sum = in_cksum_pseudo_header(m, tlen, off0,
					ip->ip_src.s_addr, ip->ip_dst.s_addr,
					IPPROTO_TCP);
		}
		*l4_sum = th_sum;
		/* tcp_input.c:717-720 */
		return (th_sum ? D_L4_BADSUM : D_ACCEPT);
	}
	if (ip->ip_p == IPPROTO_UDP) {
		struct udphdr *uh;
		int iphlen = hlen;

		/* udp_usrreq.c:375-388 */
		if (m->m_len < iphlen + (int)sizeof(struct udphdr))
			return (D_L4_SHORT);
		uh = (struct udphdr *)((caddr_t)ip + iphlen);
		if (uh->uh_dport == 0)
			return (D_UDP_PORT0);
		/* udp_usrreq.c:404-414 */
		len = ntohs((u_short)uh->uh_ulen);
		uip_len = ntohs(ip->ip_len) - iphlen;
		if (uip_len != len) {
			if (len > uip_len || len < (int)sizeof(struct udphdr))
				return (D_UDP_BADLEN);
			m->m_len -= uip_len - len;	/* m_adj(m, len - ip_len) */
			m->m_pkthdr.len -= uip_len - len;
		}
		/* udp_usrreq.c:426-451 */
		if (uh->uh_sum) {
			u_short uh_sum;

			if (m->m_pkthdr.csum_flags & CSUM_DATA_VALID) {
				if (m->m_pkthdr.csum_flags & CSUM_PSEUDO_HDR)
					uh_sum = m->m_pkthdr.csum_data;
				else
					uh_sum = in_pseudo(ip->ip_src.s_addr,
					    ip->ip_dst.s_addr, htonl((u_short)len +
					    m->m_pkthdr.csum_data + IPPROTO_UDP));
				uh_sum ^= 0xffff;
			} else {
				uh_sum = in_cksum_pseudo_header(m, len, iphlen,
					      ip->ip_src.s_addr, ip->ip_dst.s_addr,
					      IPPROTO_UDP);
			}
			*l4_sum = uh_sum;
			return (uh_sum ? D_L4_BADSUM : D_ACCEPT);
		}
		return (D_UDP_NOSUM);
	}
	return (D_OTHER);
}

/* Which branch the last mi_offload_decide took for each sum (bit 0: the IP
 * header from the flags, bit 1: the L4 sum from csum_data). */
int
mi_offload_branches(void)
{
	return (((mb.m_pkthdr.csum_flags & CSUM_IP_CHECKED) ? 1 : 0) |
	    ((mb.m_pkthdr.csum_flags & CSUM_DATA_VALID) ? 2 : 0));
}
