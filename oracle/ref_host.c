/*
 * ref_host.c - exports the reference's own host-side pieces of the rx path
 * that are header-only or build standalone, so the product's host C
 * (caladan_amd/csrc/gcl_host.c) and the oracle can be checked against them:
 *
 *  - lrpc_send (inc/base/lrpc.h:48-63, static inline) over __lrpc_send,
 *    lrpc_init_out and lrpc_init_in (base/lrpc.c, linked unmodified), lrpc_recv
 *    (inc/base/lrpc.h:121-140) for the consumer side, and the layouts of
 *    struct lrpc_msg / lrpc_chan_out;
 *  - union rxq_cmd and the RX_NET_RECV / CHECKSUM_TYPE_* values
 *    (inc/iokernel/queue.h:10-65) that rx_make_cmd (rx.c:24-38) fills;
 *  - the loopback hint payload helpers (inc/iokernel/queue.h:120-134) and
 *    TXFLAG_LOCAL_HINT;
 *  - NCPU (inc/base/limits.h:7);
 *  - frames written through the reference's own wire-format structs
 *    (inc/net/ethernet.h:67-71, ip.h:59-81, arp.h:11-32, udp.h:9-14,
 *    tcp.h:17-40) and ETHTYPE_* / ARP_OP_* values, so the parse offsets of
 *    the classifier are checked against them rather than against our own
 *    idea of the layout.
 *
 * Test infrastructure only; compiled only when /root/reference is mounted
 * (oracle/Makefile, target ref).
 */
#include <stddef.h>
#include <stdint.h>

#include <string.h>

#include <base/limits.h>
#include <base/lrpc.h>
#include <iokernel/queue.h>
#include <net/arp.h>
#include <net/ethernet.h>
#include <net/ip.h>
#include <net/tcp.h>
#include <net/udp.h>

bool ref_lrpc_send(struct lrpc_chan_out *chan, uint64_t cmd, unsigned long payload)
{
	return lrpc_send(chan, cmd, payload);
}

bool ref_lrpc_recv(struct lrpc_chan_in *chan, uint64_t *cmd, unsigned long *payload)
{
	return lrpc_recv(chan, cmd, payload);
}

/* out[]: sizeof(lrpc_msg), offsetof cmd, payload, sizeof(lrpc_chan_out),
 * offsetof send_head, send_tail, tbl, recv_head_wb, size, pad */
void ref_lrpc_layout(uint64_t out[10])
{
	out[0] = sizeof(struct lrpc_msg);
	out[1] = offsetof(struct lrpc_msg, cmd);
	out[2] = offsetof(struct lrpc_msg, payload);
	out[3] = sizeof(struct lrpc_chan_out);
	out[4] = offsetof(struct lrpc_chan_out, send_head);
	out[5] = offsetof(struct lrpc_chan_out, send_tail);
	out[6] = offsetof(struct lrpc_chan_out, tbl);
	out[7] = offsetof(struct lrpc_chan_out, recv_head_wb);
	out[8] = offsetof(struct lrpc_chan_out, size);
	out[9] = offsetof(struct lrpc_chan_out, pad);
}

/* rx_make_cmd's assignments (rx.c:28-35) into the reference's union; the
 * reference leaves .pad uninitialised, here it is 0 */
uint64_t ref_rxq_cmd(uint16_t len, int csum_good)
{
	union rxq_cmd cmd;

	cmd.lrpc_cmd = 0;
	cmd.len = len;
	cmd.rxcmd = RX_NET_RECV;
	cmd.csum_type = csum_good ? CHECKSUM_TYPE_UNNECESSARY : CHECKSUM_TYPE_NEEDED;
	return cmd.lrpc_cmd;
}

uint64_t ref_rss_from_txpkt_payload(uint64_t payload)
{
	return rss_from_txpkt_payload(payload);
}

uint64_t ref_txpkt_to_payload(uint64_t ptr, uint16_t rss)
{
	return txpkt_to_payload(ptr, rss);
}

uint32_t ref_txflag_local_hint(void)
{
	return TXFLAG_LOCAL_HINT;
}

uint32_t ref_ncpu(void)
{
	return NCPU;
}

/*
 * ref_build_frame - 64 bytes of one frame into @out (zero-filled):
 *   kind 0: Ethernet / IPv4 (header_len @ihl, fragment field @ip_off) / UDP
 *   kind 1: Ethernet / IPv4 / TCP
 *   kind 2: Ethernet / ARP for IPv4 with opcode @arp_op, sender @saddr,
 *           target @daddr (ports ignored)
 * Addresses and ports are host order, as rx.c sees them after
 * rte_be_to_cpu_* (rx.c:159, :166).  Returns 0, or -1 for a layout past 64 B.
 */
int ref_build_frame(uint8_t *out, int kind, uint32_t saddr, uint32_t daddr, uint16_t sport,
                    uint16_t dport, uint8_t ihl, uint16_t ip_off, uint16_t arp_op)
{
	struct eth_hdr *eth = (struct eth_hdr *)out;

	memset(out, 0, 64);
	if (kind == 2) {
		struct arp_hdr *arp = (struct arp_hdr *)(eth + 1);
		struct arp_hdr_ethip *body = (struct arp_hdr_ethip *)(arp + 1);
		eth->type = cpu_to_be16(ETHTYPE_ARP);
		arp->htype = cpu_to_be16(ARP_HTYPE_ETHER);
		arp->ptype = cpu_to_be16(ETHTYPE_IP);
		arp->hlen = sizeof(struct eth_addr);
		arp->plen = sizeof(uint32_t);
		arp->op = cpu_to_be16(arp_op);
		body->sender_ip = cpu_to_be32(saddr);
		body->target_ip = cpu_to_be32(daddr);
		return 0;
	}
	if (ihl < 5 || sizeof(struct eth_hdr) + ihl * 4u + 4 > 64)
		return -1;
	struct ip_hdr *ip = (struct ip_hdr *)(eth + 1);
	eth->type = cpu_to_be16(ETHTYPE_IP);
	ip->version = 4;
	ip->header_len = ihl;
	ip->len = cpu_to_be16(46);
	ip->off = cpu_to_be16(ip_off);
	ip->ttl = 64;
	ip->proto = kind == 1 ? IPPROTO_TCP : IPPROTO_UDP;
	ip->saddr = cpu_to_be32(saddr);
	ip->daddr = cpu_to_be32(daddr);
	uint8_t *l4 = (uint8_t *)ip + ihl * 4u;
	if (kind == 1) {
		struct tcp_hdr th;
		memset(&th, 0, sizeof(th));
		th.sport = cpu_to_be16(sport);
		th.dport = cpu_to_be16(dport);
		memcpy(l4, &th, 4); /* the ports; the rest of the header may pass 64 B */
	} else {
		struct udp_hdr uh;
		memset(&uh, 0, sizeof(uh));
		uh.src_port = cpu_to_be16(sport);
		uh.dst_port = cpu_to_be16(dport);
		memcpy(l4, &uh, 4);
	}
	return 0;
}

/* values the classifier compares against (ethernet.h:88,94,300, arp.h:42-43,
 * ip.h:74-75) */
void ref_net_consts(uint32_t out[6])
{
	out[0] = ETHTYPE_IP;
	out[1] = ETHTYPE_ARP;
	out[2] = ETHTYPE_IPV6;
	out[3] = ARP_OP_REQUEST;
	out[4] = ARP_OP_REPLY;
	out[5] = IP_MF | IP_OFFMASK;
}
