/*
 * gcl_host.h - host (CPU, C) side of the rx path that stays on the dataplane
 * core: turning GPU verdicts into lrpc messages for the runtimes.
 *
 * This is the part of rx_one_pkt that cannot run on the GPU
 * (iokernel/rx.c:50-92, :171-233): lrpc_send into the runtime's shared-memory
 * ring (inc/base/lrpc.h:48-63, base/lrpc.c:10-27), ownership bookkeeping of
 * the mbuf (rx.c:86-90), the sched_add_core wake path for runtimes with no
 * active kthread (rx.c:62-72), the Azure ARP broadcast/response, and the
 * ring-full counters RX_UNICAST_FAIL / RX_BROADCAST_FAIL.  Verdicts are
 * consumed in packet order and every DELIVER / WAKE verdict's flow_tbl slot
 * is resolved against p->flow_tbl and p->active_thread_count as they stand
 * when that packet is delivered (rx.c:55-72): a wake earlier in the batch
 * whose sched_add_core activated a kthread, or disabled another runtime's
 * (sched.c:208-216), steers the later packets exactly as in the reference.
 */
#ifndef GCL_HOST_H
#define GCL_HOST_H

#include <stdbool.h>
#include <stdint.h>

#include "gclassify.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as struct lrpc_msg / struct lrpc_chan_out
 * (inc/base/lrpc.h:15-35), so a reference thread's &th->rxq can be passed. */
struct gcl_lrpc_msg {
	uint64_t cmd;
	unsigned long payload;
};

struct gcl_lrpc_chan_out {
	uint32_t send_head;
	uint32_t send_tail;
	struct gcl_lrpc_msg *tbl;
	uint32_t *recv_head_wb;
	uint32_t size;
	uint32_t pad;
};

#define GCL_LRPC_DONE_PARITY (1ULL << 63)

/* lrpc_init_out (base/lrpc.c:38-52): -EINVAL unless @size is a power of 2 */
int gcl_lrpc_init_out(struct gcl_lrpc_chan_out *chan, struct gcl_lrpc_msg *tbl,
                      unsigned int size, uint32_t *recv_head_wb);
/* lrpc_send / __lrpc_send: false when the ring is full */
bool gcl_lrpc_send(struct gcl_lrpc_chan_out *chan, uint64_t cmd, unsigned long payload);

/* The slice of struct proc (iokernel/defs.h:187-251) the rx path touches. */
struct gcl_host_proc {
	uint16_t uniqid;
	uint16_t thread_count;
	uint16_t active_thread_count;
	int16_t  idle_top;                 /* list_top(&p->idle_threads), -1 if empty */
	uint16_t flow_tbl[GCL_NCPU];
	struct gcl_lrpc_chan_out *rxq[GCL_NCPU]; /* &p->threads[i].rxq */
};

/* Callbacks into the surrounding dataplane (all optional). */
struct gcl_host_ops {
	void *arg;
	/* sched_add_core(p) (sched.c:870-878): may activate threads and rewrite
	 * p->flow_tbl / active_thread_count / idle_top before returning. */
	void (*sched_add_core)(void *arg, struct gcl_host_proc *p);
	/* thread_enable_sched_poll(th) (rx.c:58, :71) */
	void (*enable_poll)(void *arg, struct gcl_host_proc *p, unsigned int thread);
	/* rte_pktmbuf_free(buf) of packet i (rx.c:231) */
	void (*free_pkt)(void *arg, uint64_t i);
	/* pdata->owner = p; list_add_tail(&p->owned_rx_bufs) (rx.c:86-90) */
	void (*owned)(void *arg, struct gcl_host_proc *p, uint64_t i);
	/* rte_mbuf_refcnt_update(buf, delta) (rx.c:188) */
	void (*refcnt_update)(void *arg, uint64_t i, int delta);
	/* azure_arp_response(buf) (rx.c:94-114): true if transmitted */
	bool (*arp_respond)(void *arg, uint64_t i);
};

/* rx_make_cmd (rx.c:24-38): RX_NET_RECV | len << 16 | csum_type << 48 */
uint64_t gcl_rx_make_cmd(uint16_t pkt_len, uint8_t olflags);

/*
 * gcl_host_deliver - consume @n verdicts in order.
 * @clients_by_id  dp.clients_by_id (iokernel/defs.h:386), @max_runtimes long
 * @clients        dp.clients[0..nr_clients) (broadcast order, rx.c:175)
 * @pkt_len/@olflags per-packet mbuf metadata (olflags NULL: @default_olflags)
 * @shmptr         per-packet ptr_to_shmptr(ingress region, data) (rx.c:82)
 * @stats          u64[GCL_NR_STATS], accumulated (host-side counters only)
 * Returns the number of packets handed to a runtime.
 */
uint64_t gcl_host_deliver(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                          struct gcl_host_proc *const *clients, int nr_clients,
                          const struct gcl_verdict *v, const uint16_t *pkt_len,
                          const uint8_t *olflags, uint8_t default_olflags,
                          const uint64_t *shmptr, uint64_t n,
                          const struct gcl_host_ops *ops, uint64_t *stats);

/*
 * gcl_host_deliver4 - the same over compact verdicts (GCL_CFG_VERDICT4), whose
 * @thread is the flow_tbl slot (hash % thread_count) like gcl_verdict's.
 * @bcast_hash     per-packet hash for GCL_ACT_BROADCAST fan-out: in
 *                 GCL_HASH_NIC mode the mbuf hash.rss array the batch was
 *                 classified with (masked to 16 bits under GCL_CFG_HASH16);
 *                 NULL in the computed modes, where ARP hashes to 0.
 */
uint64_t gcl_host_deliver4(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const struct gcl_verdict4 *v, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats);

/* gcl_verdict2_to4 - widen a GCL_CFG_VERDICT2 verdict of a context opened
 * with @thread_bits to the gcl_verdict4 the same packet gets under
 * GCL_CFG_VERDICT4 (GCL_ACT_F_FDIR aside, which the 2-byte form drops). */
struct gcl_verdict4 gcl_verdict2_to4(uint16_t v, uint8_t thread_bits);

/*
 * gcl_host_deliver2 - gcl_host_deliver4 over 2-byte verdicts: the same
 * replay of rx_send_pkt_to_runtime / rx_send_to_runtime (rx.c:50-92),
 * packet by packet, of @v widened by gcl_verdict2_to4.  The DELIVER
 * fast path reads flow_tbl[slot] of the runtime the queue index names.
 */
uint64_t gcl_host_deliver2(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const uint16_t *v, uint8_t thread_bits, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats);

/* gcl_verdict1_to4 - widen a GCL_CFG_VERDICT1 verdict of a context opened
 * with @thread_bits: a queue verdict becomes DELIVER of that flow_tbl slot
 * (the post-pass takes rx.c's wake path itself when the runtime has no
 * active kthread), any other its action. */
struct gcl_verdict4 gcl_verdict1_to4(uint8_t v, uint8_t thread_bits);

/*
 * gcl_host_deliver1 - gcl_host_deliver2 over 1-byte verdicts (GCL_CFG_VERDICT1),
 * with the same outcome packet by packet.
 */
uint64_t gcl_host_deliver1(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const uint8_t *v, uint8_t thread_bits, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats);

/*
 * gcl_host_deliver_recs - the same post-pass straight over a burst's verdict
 * records in the persistent loop's ring slot (gcl_rxloop_peek), without
 * copying them out: @vbytes is the context's verdict width (1, 2, 4 or 8)
 * and @thread_bits its GclCfg.thread_bits (1- and 2-byte verdicts).
 * Returns 0 for a bad @vbytes / @thread_bits.
 */
uint64_t gcl_host_deliver_recs(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                               struct gcl_host_proc *const *clients, int nr_clients,
                               const struct gcl_loop_rec *recs, uint8_t vbytes,
                               uint8_t thread_bits, const uint32_t *bcast_hash,
                               const uint16_t *pkt_len, const uint8_t *olflags,
                               uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                               const struct gcl_host_ops *ops, uint64_t *stats);

/*
 * gcl_host_prefetch_rxq - a hint for a dataplane thread with time to spare
 * (waiting for a burst's verdicts): the ring slot each kthread's next message
 * lands in, and the channel state, taken for writing, so that the post-pass
 * after the wait writes lines it owns.  No effect on results.
 */
void gcl_host_prefetch_rxq(struct gcl_host_proc *const *clients, int nr_clients);

#ifdef __cplusplus
}
#endif

#endif
