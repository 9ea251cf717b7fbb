/*
 * oracle/oracle.h -- CPU oracle for the RFC 1071 checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (libunsod_amd/, include/)
 * may include, link or call this.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker / the timed CPU
 * baseline.
 *
 * Two builds share these declarations:
 *   oracle/_build/liboracle.so  -- the from-scratch restatement (orc_* symbols,
 *                                  cksum_oracle.c) + the batch driver
 *                                  (batch_driver.c compiled with PFX=orc_).
 *   oracle/_ref/libref.so       -- the reference's own in_cksum.c compiled from
 *                                  /root/reference (symbols renamed ref_*) + the
 *                                  same batch driver compiled with PFX=ref_.
 *
 * Parity is pinned: tests/golden/ holds vectors produced by libref.so (the
 * reference itself) and the restatement must reproduce every one of them.
 */
#ifndef ORACLE_ORACLE_H
#define ORACLE_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/*
 * The mbuf fields the checksum reads.  Reference: src/sys/sys/mbuf.h:90-98
 * (struct m_hdr) and :166-168 (m_next / m_data / m_len).  Offsets on LP64:
 * m_next@0, m_data@16, m_len@24.  The real struct is 256 B (MSIZE, param.h:159);
 * the checksum never touches anything past m_len.
 */
struct orc_mbuf {
	struct orc_mbuf *m_next;
	struct orc_mbuf *m_nextpkt;
	char            *m_data;
	int32_t          m_len;
	int32_t          m_flags;
	int16_t          m_type;
};

/* Restated reference entry points (src/sys/amd64/include/in_cksum.h:77-83). */
uint16_t orc_in_cksum_skip(struct orc_mbuf *m, int len, int skip);
uint16_t orc_in_cksum_pseudo_header(struct orc_mbuf *m, int plen, int off0,
                                    uint32_t src, uint32_t dst, uint8_t protonum);
unsigned orc_in_cksum_hdr(const void *ip);
uint16_t orc_in_pseudo(uint32_t a, uint32_t b, uint32_t c);
uint16_t orc_in_addword(uint16_t a, uint16_t b);

/*
 * Batch drivers (batch_driver.c).  They build one-mbuf chains over packets that
 * sit in a flat buffer and call the scalar functions exactly the way the
 * reference's protocol code does; PFX is orc_ or ref_.
 *
 * Packet i's IPv4 datagram starts at base + (offs ? offs[i] : first_off + i*stride)
 * and has flen[i] (or fixed_flen) bytes available (the frame length after the
 * Ethernet header, i.e. what the NIC delivered).
 *
 * ipv4_verify (RX: ip_input.c:459-471 + tcp_input.c:698-720):
 *   hl = ip_hl*4, ip_len = ntohs(ip_len)
 *   if flen < 20 || hl < 20 || hl > flen:     ip=l4=0, status = MALFORMED
 *   else ip = (hl == 20) ? in_cksum_hdr(ip) : in_cksum(m, hl)
 *        if ip_len < hl || ip_len > flen:     l4 = 0, status |= MALFORMED
 *        else l4 = in_cksum_pseudo_header(m, ip_len-hl, hl, src, dst, ip_p)
 *   status |= (ip != 0) * IP_BAD | (l4 != 0) * L4_BAD
 *
 * ipv4_finalize (TX: ip_output.c:649-672 + in_delayed_cksum ip_output.c:958-983),
 * in place:
 *   skipped (nothing written) when the datagram is malformed as above
 *   if ip_p is TCP or UDP: c = in_cksum_skip(m, ip_len, hl); UDP: c==0 -> 0xffff;
 *        stored at hl + (TCP ? 16 : 6) if that u16 lies inside flen
 *   ip_sum = 0; ip_sum = in_cksum(m, hl)
 */
#define ORC_ST_IP_BAD    1u
#define ORC_ST_L4_BAD    2u
#define ORC_ST_MALFORMED 4u
#define ORC_ST_L4_NONE   8u	/* demux: no L4 checksum applies */

/*
 * tx_copy_batch (TX checksum offload fused with the driver's copy,
 * uinet_if_dpdk.c:561-606 + ip_output.c:649-672,958-983): see batch_driver.c.
 * csum_flags (m_pkthdr.csum_flags, mbuf.h:281-288; NULL -> CSUM_IP plus
 * CSUM_TCP / CSUM_UDP by ip_p) and csum_data (offset of the L4 sum field, NULL
 * -> 16 TCP / 6 UDP, tcp_output.c:1066, udp_usrreq.c:1240).
 */
#define ORC_CSUM_IP  0x1u
#define ORC_CSUM_TCP 0x2u
#define ORC_CSUM_UDP 0x4u
#define ORC_TX_NOBUFS     1u
#define ORC_TX_SHORT      2u
#define ORC_TX_NOSUM      4u
#define ORC_TX_L4_SKIPPED 8u

#define ORC_DECL_BATCH(PFX)                                                     \
	void PFX##ipv4_verify_batch(const uint8_t *base, const uint64_t *offs,     \
	    uint64_t stride, uint64_t first_off, const uint32_t *flen,              \
	    uint32_t fixed_flen, uint32_t n, uint16_t *ip_out, uint16_t *l4_out,    \
	    uint8_t *status, int nthreads);                                         \
	void PFX##ipv4_finalize_batch(uint8_t *base, const uint64_t *offs,         \
	    uint64_t stride, uint64_t first_off, const uint32_t *flen,              \
	    uint32_t fixed_flen, uint32_t n, int nthreads);                         \
	void PFX##ipv4_demux_verify_batch(const uint8_t *base,                      \
	    const uint64_t *offs, uint64_t stride, uint64_t first_off,              \
	    const uint32_t *flen, uint32_t fixed_flen, uint32_t n,                  \
	    uint16_t *ip_out, uint16_t *l4_out, uint8_t *status, int nthreads);     \
	void PFX##ipv4_demux_finalize_batch(uint8_t *base, const uint64_t *offs,   \
	    uint64_t stride, uint64_t first_off, const uint32_t *flen,              \
	    uint32_t fixed_flen, uint32_t n, int nthreads);                         \
	uint64_t PFX##skip_repeat(const uint8_t *buf, int len, int iters);          \
	uint16_t PFX##chain_skip(const uint8_t *const *seg, const int32_t *seglen,  \
	    int nseg, int len, int skip);                                           \
	uint16_t PFX##chain_pseudo(const uint8_t *const *seg,                       \
	    const int32_t *seglen, int nseg, int plen, int off0, uint32_t src,      \
	    uint32_t dst, uint8_t proto);                                           \
	void PFX##tx_copy_batch(const uint8_t *src, const uint64_t *seg_off,       \
	    const int32_t *seg_len, const uint32_t *pkt_seg,                        \
	    const uint32_t *pkt_len, const uint32_t *csum_flags,                    \
	    const uint32_t *csum_data, uint32_t l3_off, uint8_t *dst,               \
	    uint64_t dst_stride, uint64_t dst_first, uint32_t room, uint32_t n,     \
	    uint8_t *status);

ORC_DECL_BATCH(orc_)
ORC_DECL_BATCH(ref_)

#ifdef __cplusplus
}
#endif
#endif /* ORACLE_ORACLE_H */
