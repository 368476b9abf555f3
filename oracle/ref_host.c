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
 *  - NCPU (inc/base/limits.h:7).
 *
 * Test infrastructure only; compiled only when /root/reference is mounted
 * (oracle/Makefile, target ref).
 */
#include <stddef.h>
#include <stdint.h>

#include <base/limits.h>
#include <base/lrpc.h>
#include <iokernel/queue.h>

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
