/*
 * gcl_host.c - host-side C of the rx classify path: table helpers, the CPU
 * forms of the two hashes, and the verdict post-pass that feeds lrpc rings.
 */
#include <errno.h>
#include <math.h>
#include <string.h>

#include "../../include/gcl_host.h"
#include "../../include/gclassify.h"

#define ROT(x, k) (((x) << (k)) | ((x) >> (32 - (k))))

/*
 * gcl_jenkins_hash - lookup3 hashlittle, initval 0 (base/jenkins_hash.c:
 * 126-297), the function rte_jhash(key, len, 0) applies to the ip_to_proc
 * keys.  Reads 12-byte blocks as little-endian words (memcpy, any alignment).
 */
uint32_t gcl_jenkins_hash(const void *key, size_t length)
{
	const uint8_t *k = key;
	uint32_t a, b, c, w[3];

	a = b = c = 0xdeadbeefu + (uint32_t)length;
	while (length > 12) {
		memcpy(w, k, 12);
		a += w[0];
		b += w[1];
		c += w[2];
		a -= c; a ^= ROT(c, 4);  c += b;
		b -= a; b ^= ROT(a, 6);  a += c;
		c -= b; c ^= ROT(b, 8);  b += a;
		a -= c; a ^= ROT(c, 16); c += b;
		b -= a; b ^= ROT(a, 19); a += c;
		c -= b; c ^= ROT(b, 4);  b += a;
		length -= 12;
		k += 12;
	}
	if (length == 0)
		return c;
	w[0] = w[1] = w[2] = 0;
	memcpy(w, k, length); /* the masked tail of the aligned path, :166-181 */
	a += w[0];
	b += w[1];
	c += w[2];
	c ^= b; c -= ROT(b, 14);
	a ^= c; a -= ROT(c, 11);
	b ^= a; b -= ROT(a, 25);
	c ^= b; c -= ROT(b, 16);
	a ^= c; a -= ROT(c, 4);
	b ^= a; b -= ROT(a, 14);
	c ^= b; c -= ROT(b, 24);
	return c;
}

/*
 * gcl_toeplitz - Toeplitz hash of @input under @key, bit i of the input
 * (MSB first) selecting the 32-bit key window starting at bit i.  For the
 * 12-byte IPv4 tuple this equals do_toeplitz (runtime/net/core.c:120-139).
 */
uint32_t gcl_toeplitz(const uint8_t *key, size_t keylen, const uint8_t *input, size_t len)
{
	uint32_t ret = 0;
	uint64_t window = 0;
	size_t kb = 0;

	/* 64-bit sliding window over the key bits */
	for (; kb < 8; kb++)
		window = window << 8 | (kb < keylen ? key[kb] : 0);
	for (size_t i = 0; i < len; i++) {
		for (int bit = 7; bit >= 0; bit--) {
			int shift = 7 - bit; /* bits consumed from this byte so far */
			if (input[i] & (1u << bit))
				ret ^= (uint32_t)(window >> (32 - shift));
		}
		window = window << 8 | (kb < keylen ? key[kb] : 0);
		kb++;
	}
	return ret;
}

/* sched_steer_flows rule (iokernel/sched.c:122-147) */
int gcl_steer_flows(uint16_t thread_count, const uint16_t *active_idx,
                    uint16_t active_count, uint16_t *flow_tbl)
{
	unsigned int rr = 0;

	if (thread_count == 0 || thread_count > GCL_NCPU || active_count > thread_count ||
	    !flow_tbl || (active_count && !active_idx))
		return -EINVAL;
	if (active_count == 0)
		return 0; /* "don't do anything if zero threads are active" */
	for (unsigned int i = 0; i < active_count; i++)
		if (active_idx[i] >= thread_count)
			return -EINVAL;
	for (unsigned int i = 0; i < thread_count; i++)
		flow_tbl[i] = UINT16_MAX;
	for (unsigned int i = 0; i < active_count; i++)
		flow_tbl[active_idx[i]] = active_idx[i];
	for (unsigned int i = 0; i < thread_count; i++)
		if (flow_tbl[i] == UINT16_MAX)
			flow_tbl[i] = active_idx[rr++ % active_count];
	return 0;
}

/* tx_prepare_tx_mbuf (tx.c:81) + copy_batch (dma.c:182-185) */
uint8_t gcl_loopback_olflags(uint8_t tx_olflags)
{
	const uint8_t TXFLAG_LOCAL_HINT = 1u << 6; /* inc/iokernel/queue.h:42 */
	return (uint8_t)(((tx_olflags & TXFLAG_LOCAL_HINT) ? GCL_F_RSS_HASH : 0) |
	                 GCL_F_IP_CKSUM_GOOD);
}

/* rss_from_txpkt_payload, inc/iokernel/queue.h:131-134 */
uint32_t gcl_txpkt_rss(uint64_t payload)
{
	return (uint32_t)(payload >> 48);
}

/* CRC32C (Castagnoli, reflected 0x82F63B78) over the 8 little-endian bytes of
 * @val starting from @crc with no inversion: the crc32q instruction that
 * hash_crc32c_one/two use (inc/base/hash.h:23-40, inc/asm/ops.h:77-80). */
uint32_t gcl_crc32c_u64(uint32_t crc, uint64_t val)
{
	for (int i = 0; i < 8; i++) {
		crc ^= (uint8_t)(val >> (8 * i));
		for (int b = 0; b < 8; b++)
			crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1)));
	}
	return crc;
}

/* trans_hash_5tuple / trans_hash_3tuple, runtime/net/transport.c:29-42 */
void gcl_trans_hash(uint32_t seed, uint8_t proto, uint32_t lip, uint16_t lport, uint32_t rip,
                    uint16_t rport, struct gcl_trans *out)
{
	uint64_t l = (uint64_t)lip | (uint64_t)lport << 32;
	uint64_t r = (uint64_t)rip | (uint64_t)rport << 32 | (uint64_t)proto << 48;
	out->h5 = gcl_crc32c_u64(gcl_crc32c_u64(seed, l), r);
	out->h3 = gcl_crc32c_u64(seed, l | (uint64_t)proto << 48);
}

uint32_t gcl_runtime_ip(uint32_t r)
{
	return 0x0A000000u + r + 1;
}

int gcl_zipf_cdf(uint32_t nflows, double s, uint64_t *cdf_out)
{
	double h = 0.0, acc = 0.0;

	if (!nflows || !cdf_out)
		return -EINVAL;
	for (uint32_t k = 0; k < nflows; k++)
		h += pow((double)k + 1.0, -s);
	for (uint32_t k = 0; k < nflows; k++) {
		double x;
		acc += pow((double)k + 1.0, -s);
		x = ldexp(acc / h, 64);
		cdf_out[k] = x >= 18446744073709551615.0 ? UINT64_MAX : (uint64_t)x;
	}
	cdf_out[nflows - 1] = UINT64_MAX;
	return 0;
}

/* ---------------------------------------------------------------------- */

int gcl_lrpc_init_out(struct gcl_lrpc_chan_out *chan, struct gcl_lrpc_msg *tbl,
                      unsigned int size, uint32_t *recv_head_wb)
{
	if (!size || (size & (size - 1)))
		return -EINVAL;
	memset(chan, 0, sizeof(*chan));
	chan->tbl = tbl;
	chan->size = size;
	chan->recv_head_wb = recv_head_wb;
	return 0;
}

bool gcl_lrpc_send(struct gcl_lrpc_chan_out *chan, uint64_t cmd, unsigned long payload)
{
	struct gcl_lrpc_msg *dst;

	if (chan->send_head - chan->send_tail >= chan->size) {
		/* __lrpc_send: refresh the consumer position (base/lrpc.c:16-19) */
		chan->send_tail = __atomic_load_n(chan->recv_head_wb, __ATOMIC_ACQUIRE);
		if (chan->send_head - chan->send_tail == chan->size)
			return false;
	}
	dst = &chan->tbl[chan->send_head & (chan->size - 1)];
	cmd |= (chan->send_head++ & chan->size) ? 0 : GCL_LRPC_DONE_PARITY;
	dst->payload = payload;
	__atomic_store_n(&dst->cmd, cmd, __ATOMIC_RELEASE);
	return true;
}

uint64_t gcl_rx_make_cmd(uint16_t pkt_len, uint8_t olflags)
{
	uint64_t csum = (olflags & GCL_F_IP_CKSUM_MASK) == GCL_F_IP_CKSUM_GOOD ? 1 : 0;
	return 0 /* RX_NET_RECV */ | (uint64_t)pkt_len << 16 | csum << 48;
}

/* rx_send_to_runtime (rx.c:50-73) for the flow_tbl slot @slot of runtime @p
 * (hash % thread_count: every DELIVER or WAKE verdict carries it), or, when
 * @slot < 0, the slot of @hash.  The flow_tbl and the active count are read
 * here, at delivery time, like rx.c:55-72: a sched_add_core earlier in the
 * same batch that re-steered @p (or took its last core) is seen. */
static bool send_to_runtime(struct gcl_host_proc *p, uint32_t hash, int slot,
                            uint64_t cmd, unsigned long payload,
                            const struct gcl_host_ops *ops)
{
	int th;

	/* verdicts come from device memory: a flow_tbl slot outside the
	 * runtime's thread_count (a stale or corrupted verdict) is refused
	 * like a full ring, never used as an index */
	if (p->thread_count == 0 || p->thread_count > GCL_NCPU)
		return false;
	if (slot < 0)
		slot = (int)(hash % p->thread_count);
	else if (slot >= p->thread_count)
		return false;
	if (p->active_thread_count > 0) {
		th = p->flow_tbl[slot];
	} else {
		if (ops && ops->sched_add_core)
			ops->sched_add_core(ops->arg, p);
		if (p->active_thread_count == 0)
			th = p->idle_top;
		else
			th = p->flow_tbl[slot];
	}
	if (th < 0 || th >= p->thread_count || !p->rxq[th])
		return false;
	if (ops && ops->enable_poll)
		ops->enable_poll(ops->arg, p, (unsigned int)th);
	return gcl_lrpc_send(p->rxq[th], cmd, payload);
}

/* One verdict stream, either format: @v8 (gcl_verdict) or @v4 (gcl_verdict4,
 * whose broadcast hashes come from @bcast_hash).  Callbacks see packet
 * index @base + i. */
static uint64_t deliver(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                        struct gcl_host_proc *const *clients, int nr_clients,
                        const struct gcl_verdict *v8, const struct gcl_verdict4 *v4,
                        const uint32_t *bcast_hash, const uint16_t *pkt_len,
                        const uint8_t *olflags, uint8_t default_olflags,
                        const uint64_t *shmptr, uint64_t n,
                        const struct gcl_host_ops *ops, uint64_t base, uint64_t *stats)
{
	uint64_t delivered = 0;

	for (uint64_t i = 0; i < n; i++) {
		const uint16_t uniqid = v8 ? v8[i].uniqid : v4[i].uniqid;
		const uint8_t thread = v8 ? v8[i].thread : v4[i].thread;
		const uint8_t act = (v8 ? v8[i].action : v4[i].action) & GCL_ACT_MASK;
		const uint32_t hash = v8 ? v8[i].hash : (bcast_hash ? bcast_hash[i] : 0);
		uint8_t fl = olflags ? olflags[i] : default_olflags;
		uint64_t cmd = gcl_rx_make_cmd(pkt_len ? pkt_len[i] : 0, fl);
		unsigned long payload = shmptr ? shmptr[i] : 0;
		struct gcl_host_proc *p = NULL;
		bool ok;

		if (act == GCL_ACT_DELIVER || act == GCL_ACT_WAKE) {
			if (uniqid < max_runtimes)
				p = clients_by_id[uniqid];
			ok = p && send_to_runtime(p, hash, (int)thread, cmd, payload, ops);
			if (ok) {
				delivered++;
				if (ops && ops->owned)
					ops->owned(ops->arg, p, base + i);
				continue;
			}
			stats[GCL_RX_UNICAST_FAIL]++; /* rx.c:140-142, :213-215 */
		} else if (act == GCL_ACT_BROADCAST) {
			int n_sent = 0;
			for (int c = 0; c < nr_clients; c++) {
				if (send_to_runtime(clients[c], hash, -1, cmd, payload, ops)) {
					n_sent++;
					if (ops && ops->owned)
						ops->owned(ops->arg, clients[c], base + i);
				} else {
					stats[GCL_RX_BROADCAST_FAIL]++;
				}
			}
			if (n_sent == 0) {
				if (ops && ops->free_pkt)
					ops->free_pkt(ops->arg, base + i);
			} else {
				delivered++;
				if (ops && ops->refcnt_update)
					ops->refcnt_update(ops->arg, base + i, n_sent - 1);
			}
			continue; /* rx.c:185-189: no RX_UNHANDLED */
		} else if (act == GCL_ACT_ARP_RESPOND) {
			if (ops && ops->arp_respond && ops->arp_respond(ops->arg, base + i))
				continue;
			stats[GCL_RX_UNREGISTERED_MAC]++; /* rx.c:205 */
		} else {
			/* DROP_*: the device already counted them */
			if (ops && ops->free_pkt)
				ops->free_pkt(ops->arg, base + i);
			continue;
		}
		/* fail_free, rx.c:225-232 */
		if (ops && ops->free_pkt)
			ops->free_pkt(ops->arg, base + i);
		stats[GCL_RX_UNHANDLED]++;
	}
	return delivered;
}

uint64_t gcl_host_deliver(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                          struct gcl_host_proc *const *clients, int nr_clients,
                          const struct gcl_verdict *v, const uint16_t *pkt_len,
                          const uint8_t *olflags, uint8_t default_olflags,
                          const uint64_t *shmptr, uint64_t n,
                          const struct gcl_host_ops *ops, uint64_t *stats)
{
	return deliver(clients_by_id, max_runtimes, clients, nr_clients, v, NULL, NULL, pkt_len,
	               olflags, default_olflags, shmptr, n, ops, 0, stats);
}

struct gcl_verdict4 gcl_verdict2_to4(uint16_t v, uint8_t thread_bits)
{
	struct gcl_verdict4 o;
	const uint16_t kind = v & GCL_V2_KIND, q = v & GCL_V2_Q_MASK;

	if (kind == GCL_V2_DELIVER || kind == GCL_V2_WAKE) {
		o.uniqid = (uint16_t)(q >> thread_bits);
		o.thread = (uint8_t)(q & ((1u << thread_bits) - 1));
		o.action = kind == GCL_V2_WAKE ? GCL_ACT_WAKE : GCL_ACT_DELIVER;
	} else {
		o.uniqid = GCL_NO_RUNTIME;
		o.thread = GCL_NO_THREAD;
		o.action = (uint8_t)(v & GCL_ACT_MASK);
	}
	return o;
}

struct gcl_verdict4 gcl_verdict1_to4(uint8_t v, uint8_t thread_bits)
{
	struct gcl_verdict4 o;

	if (!(v & GCL_V1_OTHER)) {
		o.uniqid = (uint16_t)((v & GCL_V1_Q_MASK) >> thread_bits);
		o.thread = (uint8_t)(v & ((1u << thread_bits) - 1));
		o.action = GCL_ACT_DELIVER;
	} else {
		o.uniqid = GCL_NO_RUNTIME;
		o.thread = GCL_NO_THREAD;
		o.action = (uint8_t)(v & GCL_ACT_MASK);
	}
	return o;
}

/* deliver() for compact verdicts, with the common case inlined: a DELIVER
 * verdict for a runtime that still has an active kthread goes straight into
 * the ring of flow_tbl[slot] as it stands now (rx.c:55-59, then :76-92),
 * with the two per-delivery callbacks of the reference,
 * thread_enable_sched_poll and the ownership record.  Everything else (WAKE,
 * a runtime whose last core a scheduler side effect of this batch took,
 * broadcast, drops, a full ring) takes deliver() for that one packet, in
 * order, so the outcome is the same packet by packet.  A write prefetch of
 * the ring slot 8-32 packets ahead made it slower (profiles/archive/r01_deliver.txt).
 * Verdicts are @v2 (2-byte, of a context with @thread_bits), @v1 (1-byte) or
 * @v4; always inlined with constant NULLs for the two absent forms. */
static inline __attribute__((always_inline)) uint64_t
deliver_compact(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                struct gcl_host_proc *const *clients, int nr_clients,
                const struct gcl_verdict4 *v4, const uint16_t *v2, const uint8_t *v1,
                uint8_t thread_bits,
                const uint32_t *bcast_hash, const uint16_t *pkt_len, const uint8_t *olflags,
                uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                const struct gcl_host_ops *ops, uint64_t *stats, size_t vstride)
{
	const uint64_t csum_def = (default_olflags & GCL_F_IP_CKSUM_MASK) == GCL_F_IP_CKSUM_GOOD;
	void (*const enable_poll)(void *, struct gcl_host_proc *, unsigned int) =
		ops ? ops->enable_poll : NULL;
	void (*const owned)(void *, struct gcl_host_proc *, uint64_t) = ops ? ops->owned : NULL;
	const uint32_t tmask = (1u << thread_bits) - 1;
	uint64_t delivered = 0;

	for (uint64_t i = 0; i < n; i++) {
		struct gcl_host_proc *p;
		struct gcl_lrpc_chan_out *chan;
		uint32_t uniqid, slot, th;
		bool fast;

		/* verdict i sits @vstride bytes after verdict i - 1: packed
		 * arrays, or the rx loop's 16-B records read in place */
		const uint16_t *v2i = v2 ? (const uint16_t *)((const char *)v2 + i * vstride) : NULL;
		const uint8_t *v1i = v1 ? (const uint8_t *)v1 + i * vstride : NULL;
		const struct gcl_verdict4 *v4i =
			v4 ? (const struct gcl_verdict4 *)((const char *)v4 + i * vstride) : NULL;
		if (v1) { /* no WAKE mark: the active count below decides, as rx.c:59 */
			const uint8_t x = *v1i;
			uniqid = (x & GCL_V1_Q_MASK) >> thread_bits;
			slot = x & tmask;
			fast = !(x & GCL_V1_OTHER);
		} else if (v2) {
			const uint16_t x = *v2i;
			uniqid = (x & GCL_V2_Q_MASK) >> thread_bits;
			slot = x & tmask;
			fast = (x & GCL_V2_KIND) == GCL_V2_DELIVER;
		} else {
			const struct gcl_verdict4 x = *v4i;
			uniqid = x.uniqid;
			slot = x.thread;
			fast = (x.action & GCL_ACT_MASK) == GCL_ACT_DELIVER;
		}
		if (!fast || uniqid >= max_runtimes || !(p = clients_by_id[uniqid]) ||
		    slot >= p->thread_count || p->active_thread_count == 0 ||
		    (th = p->flow_tbl[slot]) >= p->thread_count || !(chan = p->rxq[th]) ||
		    chan->send_head - chan->send_tail >= chan->size) {
			const struct gcl_verdict4 w = v1 ? gcl_verdict1_to4(*v1i, thread_bits)
			                            : v2 ? gcl_verdict2_to4(*v2i, thread_bits) : *v4i;
			delivered += deliver(clients_by_id, max_runtimes, clients, nr_clients, NULL, &w,
			                     bcast_hash ? bcast_hash + i : NULL, pkt_len ? pkt_len + i : NULL,
			                     olflags ? olflags + i : NULL, default_olflags,
			                     shmptr ? shmptr + i : NULL, 1, ops, i, stats);
			continue;
		}
		if (enable_poll)
			enable_poll(ops->arg, p, th);
		const uint64_t csum = olflags ?
			(olflags[i] & GCL_F_IP_CKSUM_MASK) == GCL_F_IP_CKSUM_GOOD : csum_def;
		const uint32_t h = chan->send_head++;
		struct gcl_lrpc_msg *dst = &chan->tbl[h & (chan->size - 1)];
		dst->payload = shmptr ? shmptr[i] : 0;
		__atomic_store_n(&dst->cmd, (uint64_t)(pkt_len ? pkt_len[i] : 0) << 16 | csum << 48 |
		                            ((h & chan->size) ? 0 : GCL_LRPC_DONE_PARITY),
		                 __ATOMIC_RELEASE);
		if (owned)
			owned(ops->arg, p, i);
		delivered++;
	}
	return delivered;
}

uint64_t gcl_host_deliver4(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const struct gcl_verdict4 *v, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats)
{
	return deliver_compact(clients_by_id, max_runtimes, clients, nr_clients, v, NULL, NULL, 0,
	                       bcast_hash, pkt_len, olflags, default_olflags, shmptr, n, ops, stats,
	                       sizeof(*v));
}

uint64_t gcl_host_deliver2(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const uint16_t *v, uint8_t thread_bits, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats)
{
	if (thread_bits > 8 || !v)
		return 0;
	return deliver_compact(clients_by_id, max_runtimes, clients, nr_clients, NULL, v, NULL,
	                       thread_bits, bcast_hash, pkt_len, olflags, default_olflags, shmptr,
	                       n, ops, stats, sizeof(*v));
}

uint64_t gcl_host_deliver1(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                           struct gcl_host_proc *const *clients, int nr_clients,
                           const uint8_t *v, uint8_t thread_bits, const uint32_t *bcast_hash,
                           const uint16_t *pkt_len, const uint8_t *olflags,
                           uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                           const struct gcl_host_ops *ops, uint64_t *stats)
{
	if (thread_bits > 7 || !v)
		return 0;
	return deliver_compact(clients_by_id, max_runtimes, clients, nr_clients, NULL, NULL, v,
	                       thread_bits, bcast_hash, pkt_len, olflags, default_olflags, shmptr,
	                       n, ops, stats, sizeof(*v));
}

void gcl_host_prefetch_rxq(struct gcl_host_proc *const *clients, int nr_clients)
{
	for (int c = 0; c < nr_clients; c++) {
		const struct gcl_host_proc *p = clients[c];
		if (!p)
			continue;
		const unsigned int nt = p->thread_count <= GCL_NCPU ? p->thread_count : GCL_NCPU;
		for (unsigned int t = 0; t < nt; t++) {
			struct gcl_lrpc_chan_out *ch = p->rxq[t];
			if (!ch || !ch->tbl || !ch->size)
				continue;
			__builtin_prefetch(ch, 1, 3);
			__builtin_prefetch(&ch->tbl[ch->send_head & (ch->size - 1)], 1, 3);
		}
	}
}

uint64_t gcl_host_deliver_recs(struct gcl_host_proc *const *clients_by_id, uint32_t max_runtimes,
                               struct gcl_host_proc *const *clients, int nr_clients,
                               const struct gcl_loop_rec *recs, uint8_t vbytes,
                               uint8_t thread_bits, const uint32_t *bcast_hash,
                               const uint16_t *pkt_len, const uint8_t *olflags,
                               uint8_t default_olflags, const uint64_t *shmptr, uint64_t n,
                               const struct gcl_host_ops *ops, uint64_t *stats)
{
	uint64_t delivered = 0;

	if (!recs || thread_bits > 8)
		return 0;
	if (vbytes == 4)
		return deliver_compact(clients_by_id, max_runtimes, clients, nr_clients,
		                       (const struct gcl_verdict4 *)&recs[0].verdict, NULL, NULL, 0,
		                       bcast_hash, pkt_len, olflags, default_olflags, shmptr, n, ops, stats,
		                       sizeof(*recs));
	if (vbytes == 2)
		return deliver_compact(clients_by_id, max_runtimes, clients, nr_clients, NULL,
		                       (const uint16_t *)&recs[0].verdict, NULL, thread_bits, bcast_hash,
		                       pkt_len, olflags, default_olflags, shmptr, n, ops, stats,
		                       sizeof(*recs));
	if (vbytes == 1)
		return thread_bits > 7 ? 0
		                       : deliver_compact(clients_by_id, max_runtimes, clients, nr_clients,
		                                         NULL, NULL, (const uint8_t *)&recs[0].verdict,
		                                         thread_bits, bcast_hash, pkt_len, olflags,
		                                         default_olflags, shmptr, n, ops, stats,
		                                         sizeof(*recs));
	if (vbytes != 8)
		return 0;
	/* 8-byte contexts: a record's first 8 bytes are the struct gcl_verdict */
	for (uint64_t i = 0; i < n; i++) {
		struct gcl_verdict v;
		memcpy(&v, &recs[i], sizeof(v));
		delivered += deliver(clients_by_id, max_runtimes, clients, nr_clients, &v, NULL, NULL,
		                     pkt_len ? pkt_len + i : NULL, olflags ? olflags + i : NULL,
		                     default_olflags, shmptr ? shmptr + i : NULL, 1, ops, i, stats);
	}
	return delivered;
}
