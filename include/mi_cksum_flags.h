/*
 * include/mi_cksum_flags.h -- the m_pkthdr checksum-offload vocabulary the
 * library produces and consumes, as plain macros (no includes), so that code
 * compiled kernel-side with the reference's own headers and -nostdinc -- the
 * driver glue of src/lib/libuinet/uinet_if_dpdk.c, where INTEGRATION.md
 * section 2's hook sits -- can include it beside <sys/mbuf.h>.
 *
 * oracle/linktest/offload_kernel.c (RX) and tx_kernel.c (TX) static-assert
 * every value below against the reference's definitions (src/sys/sys/mbuf.h:
 * 123-124, 281-305; netinet/tcp.h, netinet/udp.h) under the reference's
 * kernel flags; mi_cksum.h includes this file.
 */
#ifndef MI_CKSUM_FLAGS_H
#define MI_CKSUM_FLAGS_H

/* m_pkthdr.csum_flags bits (mbuf.h:281-293) */
#define MI_CSUM_IP         0x0001u  /* TX: will csum IP            (CSUM_IP) */
#define MI_CSUM_TCP        0x0002u  /* TX: will csum TCP           (CSUM_TCP) */
#define MI_CSUM_UDP        0x0004u  /* TX: will csum UDP           (CSUM_UDP) */
#define MI_CSUM_IP_CHECKED 0x0100u  /* RX: did csum IP             (CSUM_IP_CHECKED) */
#define MI_CSUM_IP_VALID   0x0200u  /* RX:   ... the csum is valid (CSUM_IP_VALID) */
#define MI_CSUM_DATA_VALID 0x0400u  /* RX: csum_data field valid   (CSUM_DATA_VALID) */
#define MI_CSUM_PSEUDO_HDR 0x0800u  /* RX: csum_data has pseudo hdr (CSUM_PSEUDO_HDR) */

/* TX combinations (mbuf.h:304-305): the sums ip_output leaves to
 * in_delayed_cksum / the device, and the IP header sum */
#define MI_CSUM_DELAY_DATA (MI_CSUM_TCP | MI_CSUM_UDP)
#define MI_CSUM_DELAY_IP   MI_CSUM_IP

/* TX m_pkthdr.csum_data: where the L4 sum field sits in the L4 header, as
 * the transports set it -- offsetof(struct tcphdr, th_sum) (tcp_output.c:1066)
 * and offsetof(struct udphdr, uh_sum) (udp_usrreq.c:1240); in_delayed_cksum
 * stores at ip_hl * 4 + csum_data (ip_output.c:969-982).  Static-asserted
 * against <netinet/tcp.h> / <netinet/udp.h> by oracle/linktest/tx_kernel.c. */
#define MI_CSUM_DATA_TCP 16u
#define MI_CSUM_DATA_UDP 6u

/* Where the two fields sit in the reference's amd64 struct mbuf (M_PKTHDR
 * mbufs; mbuf.h:123-124 inside struct pkthdr at m_pkthdr, :166-168), both
 * 4-byte ints -- for callers that fill mbufs without the reference's headers
 * (the Python MbufChain, tools). */
#define MI_MBUF_PKTHDR_OFF      40
#define MI_MBUF_CSUM_FLAGS_OFF  64
#define MI_MBUF_CSUM_DATA_OFF   68

#endif /* MI_CKSUM_FLAGS_H */
