/*
 * gclassify.h - C ABI of the MI355X (gfx950) rx packet classifier.
 *
 * This library replaces the per-packet work that Caladan's IOKernel does in
 * rx_burst()/rx_one_pkt() (iokernel/rx.c:116-233, :270-290): parse the
 * Ethernet/IPv4/ARP header, look the destination IP up in the IP->runtime
 * table (dp.ip_to_proc, an rte_hash keyed by rte_jhash, iokernel/dp_clients.c:
 * 349-363), and steer the packet to a runtime kthread through that runtime's
 * flow table (rx_send_to_runtime, iokernel/rx.c:50-73).  The GPU emits one
 * 8-byte verdict per packet; the host (one dataplane thread, as in the
 * reference) turns verdicts into lrpc_send() calls (see gcl_host.h).
 *
 * Conventions follow the reference: every function returns 0 or -errno
 * (rx_init iokernel/rx.c:398-415, lrpc_init_out base/lrpc.c:38-52), nothing is
 * thread-safe, and one context serves one GPU the way one dataplane core
 * serves one NIC queue (iokernel/dpdk.c:276-280).  There are no per-packet
 * error returns: outcomes are verdict actions plus counters, exactly like the
 * reference's STAT_INC counters (iokernel/defs.h:417-460).
 *
 * All pointers passed to gcl_classify() are DEVICE pointers (HBM); table
 * setters take host pointers.  Table updates are applied on the stream of the
 * next gcl_classify() call, before its kernel, giving the snapshot semantics
 * of the reference's single-threaded dataplane (tables only change between
 * bursts, iokernel/main.c:144-176).
 */
#ifndef GCLASSIFY_H
#define GCLASSIFY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Limits of the reference data model. */
#define GCL_MAX_PROC      4096  /* IOKERNEL_MAX_PROC, iokernel/defs.h:69 */
#define GCL_NCPU          256   /* NCPU, inc/base/limits.h:7: max threads per proc */
#define GCL_RX_BURST_SIZE 64    /* IOKERNEL_RX_BURST_SIZE, iokernel/defs.h:75 */

/* Header constants parsed on the path (inc/net/ethernet.h, inc/net/arp.h). */
#define GCL_ETHTYPE_IP    0x0800
#define GCL_ETHTYPE_ARP   0x0806
#define GCL_ETHTYPE_IPV6  0x86DD
#define GCL_ARP_OP_REQUEST 1
#define GCL_ARP_OP_REPLY   2
#define GCL_HDR_GRANULE   64    /* bytes of each frame the kernel stages */

/*
 * Per-packet offload flags: one byte that carries the rte_mbuf ol_flags bits
 * rx.c reads (RTE_MBUF_F_RX_RSS_HASH at rx.c:132/:160, RTE_MBUF_F_RX_FDIR_ID at
 * rx.c:131, RTE_MBUF_F_RX_IP_CKSUM_MASK at rx.c:31-35).
 */
#define GCL_F_RSS_HASH           0x01
#define GCL_F_FDIR_ID            0x02
#define GCL_F_IP_CKSUM_MASK      0x0C
#define GCL_F_IP_CKSUM_UNKNOWN   0x00
#define GCL_F_IP_CKSUM_BAD       0x04
#define GCL_F_IP_CKSUM_GOOD      0x08
#define GCL_F_IP_CKSUM_NONE      0x0C

/*
 * Steering-hash source.  The reference steers with buf->hash.rss (rx.c:83),
 * i.e. the NIC's Toeplitz RSS over IPv4 TCP/UDP (iokernel/dpdk.c:67-82).
 *  NIC      - use the per-packet rss[] array, exactly like rx.c.
 *  JENKINS  - compute lookup3 (base/jenkins_hash.c:126-297) over the 13-byte
 *             key {saddr, daddr, dport, sport, proto} (host-order fields).
 *  TOEPLITZ - compute the NIC's Toeplitz hash in software, bit-exact with
 *             do_toeplitz (runtime/net/core.c:120-139) for the configured key.
 * In the two computed modes the hash is 0 unless the frame is IPv4 with
 * IHL >= 5, not a fragment (MF clear, offset 0) and protocol TCP or UDP
 * (the NIC's RTE_ETH_RSS_NONFRAG_IPV4_TCP|UDP, dpdk.c:79).
 */
enum gcl_hash_mode {
	GCL_HASH_NIC = 0,
	GCL_HASH_JENKINS = 1,
	GCL_HASH_TOEPLITZ = 2,
};

/* gcl_cfg.flags */
#define GCL_CFG_AZURE_ARP  0x1  /* cfg.azure_arp_mode: rx.c:171-190, :200-203 */
#define GCL_CFG_HASH16     0x2  /* truncate the steering hash to 16 bits, as the
                                   loopback hint does (runtime/net/core.c:524,
                                   iokernel/tx.c:81-83, inc/iokernel/queue.h:120-134) */
#define GCL_CFG_PROFILE    0x4  /* record HIP events around every classify kernel */
#define GCL_CFG_TRANS_HASH 0x8  /* also compute the destination runtime's transport
                                   demux hashes (gcl_classify_ex, struct gcl_trans) */
#define GCL_CFG_VERDICT4   0x10 /* write 4-byte struct gcl_verdict4 instead of
                                   struct gcl_verdict (see there) */
#define GCL_CFG_VERDICT2   0x20 /* write 2-byte queue verdicts (gcl_verdict2 below);
                                   needs cfg.thread_bits, excludes VERDICT4 and
                                   TRANS_HASH */
#define GCL_CFG_VERDICT1   0x40 /* write 1-byte queue verdicts (gcl_verdict1 below):
                                   needs cfg.thread_bits with max_runtimes <<
                                   thread_bits <= GCL_V1_QUEUES, excludes VERDICT2,
                                   VERDICT4 and TRANS_HASH */

struct gcl_cfg {
	uint32_t max_runtimes;    /* uniqids must be < max_runtimes (<= GCL_MAX_PROC) */
	uint32_t hash_mode;       /* enum gcl_hash_mode */
	uint32_t flags;           /* GCL_CFG_* */
	uint8_t  default_olflags; /* flags of every packet when gcl_batch.olflags == NULL */
	uint8_t  rss_key[40];     /* Toeplitz key (NIC key, dpdk.c:219-228) */
	uint8_t  thread_bits;     /* GCL_CFG_VERDICT2 / VERDICT1: kthread queues per runtime
	                             are 1 << thread_bits (thread_count may not exceed it),
	                             and max_runtimes << thread_bits <= GCL_V2_QUEUES
	                             (GCL_V1_QUEUES) */
	uint8_t  pad[2];
};

/* One batch of received frames, resident in device memory. */
struct gcl_batch {
	const uint8_t  *frames;     /* frame bytes (mbuf data) */
	uint64_t        frames_len; /* readable bytes at frames (< 2^64 - 1, else -EINVAL);
	                               reads past it see 0, at any offset */
	uint64_t        stride;     /* slot stride when offs == NULL (multiple of 16) */
	const uint64_t *offs;       /* optional u64[n] frame start offsets, any alignment:
	                               a 4-B-aligned frame (16-B aligned, or the
	                               reference's mbuf data at element + 344,
	                               iokernel/defs.h:503-506) is staged as the
	                               16-B-aligned 64-B window starting up to 12 B
	                               before it (four 16-B loads), cut at the first
	                               128-B line end when that line holds frame
	                               bytes 0-39; any other alignment is read byte
	                               by byte */
	const uint8_t  *olflags;    /* optional u8[n]  GCL_F_* per packet */
	const uint32_t *rss;        /* optional u32[n] buf->hash.rss (NIC mode) */
	const uint32_t *fdir_hi;    /* optional u32[n] buf->hash.fdir.hi (FDIR mark) */
	const uint16_t *pkt_len;    /* optional u16[n] rte_pktmbuf_pkt_len; NOT read by
	                               the kernel, only by the host post-pass that
	                               builds rxq_cmd (rx_make_cmd, rx.c:24-38) */
	uint64_t        n;          /* packets in the batch */
	const uint32_t *dst_hint;   /* optional u32[n] loopback hint: tx_pktmbuf_priv.dst_ip
	                               (host order, 0 = none).  A hint found in ip_to_proc
	                               marks the packet FDIR with hash.fdir.hi = uniqid
	                               before classification, as rx_loopback does
	                               (iokernel/rx.c:249-262); it overrides fdir_hi[] */
};

/*
 * Verdict actions.  Each is one exit of rx_one_pkt (rx.c:116-233).
 * GCL_ACT_F_FDIR is or-ed in when the runtime was found by the FDIR mark.
 */
enum gcl_action {
	GCL_ACT_DELIVER = 0,       /* rx_send_pkt_to_runtime(p) -> threads[thread] */
	GCL_ACT_WAKE = 1,          /* runtime has no active thread: the host must
	                              replay rx_send_to_runtime (sched_add_core,
	                              rx.c:62-72) in packet order */
	GCL_ACT_DROP_ETHERTYPE = 2,/* rx.c:191-194 -> fail_free, RX_UNHANDLED */
	GCL_ACT_DROP_UNREG = 3,    /* rx.c:198-207: RX_UNREGISTERED_MAC, RX_UNHANDLED */
	GCL_ACT_BROADCAST = 4,     /* azure ARP reply, rx.c:171-190 (host fans out) */
	GCL_ACT_ARP_RESPOND = 5,   /* azure ARP request miss, rx.c:200-203 (host) */
};
#define GCL_ACT_MASK    0x3F
#define GCL_ACT_F_FDIR  0x80
#define GCL_ACT_F_TRANS 0x40  /* struct gcl_trans of this packet is valid */
#define GCL_NO_RUNTIME  0xFFFF
#define GCL_NO_THREAD   0xFF

/*
 * DELIVER and WAKE verdicts name the runtime and its flow-table SLOT,
 * hash % thread_count (rx.c:57, :68), not the kthread: the host post-pass
 * (gcl_host.h) reads p->flow_tbl[slot] and p->active_thread_count when it
 * delivers the packet, as rx_send_to_runtime does (rx.c:55-72), so a
 * scheduler change earlier in the same batch is seen by the later packets.
 * DELIVER means the runtime had an active kthread in the classify snapshot,
 * WAKE that it had none; the post-pass re-checks either way.
 *
 * BREAKING in ABI 4 (round 4): before it, .thread held the kthread
 * (flow_tbl[slot]) in the same layout.  A direct consumer of the verdicts
 * that indexes kthread rings with .thread must check gcl_abi_version() >= 4
 * and read flow_tbl[.thread] itself (or use the gcl_host_deliver* post-pass).
 */
#define GCL_ABI_VERSION 6
/* GCL_ABI_VERSION of the library actually loaded: 4 = verdict .thread is
 * the flow-table slot; 5 = gcl_group_open_v2 and struct gcl_group_cfg.size;
 * 6 = struct gcl_tune / gcl_ctx_tune (the library reads no environment) */
int gcl_abi_version(void);
struct gcl_verdict {
	uint32_t hash;    /* steering hash (hash.rss, or the computed flow hash) */
	uint16_t uniqid;  /* proc->uniqid of the destination, GCL_NO_RUNTIME if none */
	uint8_t  thread;  /* the flow_tbl slot hash % thread_count, GCL_NO_THREAD if none */
	uint8_t  action;  /* enum gcl_action | GCL_ACT_F_FDIR */
};

/*
 * Compact verdict (GCL_CFG_VERDICT4): the last four bytes of gcl_verdict,
 * without the hash.  rx_send_to_runtime uses the hash only as
 * hash % thread_count (rx.c:57, :68), and thread_count is fixed per runtime,
 * so the slot in @thread is all the post-pass needs.  The only other use of
 * the hash is the Azure ARP broadcast fan-out, where it is the mbuf's
 * hash.rss in GCL_HASH_NIC mode and 0 in the computed modes (ARP is not
 * hashed): gcl_host_deliver4 takes it from the caller.
 */
struct gcl_verdict4 {
	uint16_t uniqid;  /* as gcl_verdict */
	uint8_t  thread;  /* DELIVER, WAKE: the flow_tbl slot hash % thread_count;
	                     otherwise GCL_NO_THREAD */
	uint8_t  action;  /* as gcl_verdict */
};

/*
 * 2-byte verdict (GCL_CFG_VERDICT2): a u16 per packet naming a runtime's
 * flow-table slot q = uniqid << thread_bits | slot, one flat index over
 * every runtime's flow_tbl (defs.h:244), slot = hash % thread_count.
 *   DELIVER (any flags)  q
 *   WAKE                 GCL_V2_WAKE | q
 *   every other action   GCL_V2_OTHER | action (DROP_*, BROADCAST, ARP_RESPOND)
 * It drops what gcl_verdict4 keeps beyond that: GCL_ACT_F_FDIR, which the
 * host never reads (RX_FLOW_TAG_MATCH is counted on the device).  Half the
 * verdict stores of the 4-byte form; gcl_verdict2_to4 (gcl_host.h) widens one.
 */
#define GCL_V2_QUEUES   0x4000
#define GCL_V2_Q_MASK   0x3FFF
#define GCL_V2_KIND     0xC000
#define GCL_V2_DELIVER  0x0000
#define GCL_V2_WAKE     0x4000
#define GCL_V2_OTHER    0xC000

/*
 * 1-byte verdict (GCL_CFG_VERDICT1), for contexts whose queues fit 7 bits
 * (max_runtimes << thread_bits <= 128: config 2's 16 runtimes x 8 kthreads):
 *   DELIVER or WAKE      q = uniqid << thread_bits | slot
 *   every other action   GCL_V1_OTHER | action (DROP_*, BROADCAST, ARP_RESPOND)
 * A WAKE is not marked: the post-pass reads the runtime's live
 * active_thread_count at delivery anyway and takes rx.c's wake path when it
 * is 0 (rx.c:55-72), so the mark carried nothing the host uses.  Half the
 * verdict bytes of the 2-byte form; gcl_verdict1_to4 (gcl_host.h) widens one.
 */
#define GCL_V1_QUEUES   0x80
#define GCL_V1_Q_MASK   0x7F
#define GCL_V1_OTHER    0x80

/*
 * Counter slots; indices 0..5 keep the order of the reference enum
 * (iokernel/defs.h:421-426).  The device adds RX_PULLED, RX_FLOW_TAG_MATCH,
 * RX_HASH_MISSING, RX_UNREGISTERED_MAC and RX_UNHANDLED (for its drops); the
 * host adds RX_UNICAST_FAIL / RX_BROADCAST_FAIL (ring full) and the UNHANDLED
 * that goes with them.
 */
enum {
	GCL_RX_UNREGISTERED_MAC = 0,
	GCL_RX_UNICAST_FAIL,
	GCL_RX_BROADCAST_FAIL,
	GCL_RX_FLOW_TAG_MATCH,
	GCL_RX_UNHANDLED,
	GCL_RX_HASH_MISSING,
	GCL_RX_PULLED,
	GCL_NR_STATS = 8, /* padded */
};

struct gcl_ctx;

/*
 * gcl_open - create a classifier context on HIP device @hip_device.
 * Replaces the ip_to_proc creation in dp_clients_init (dp_clients.c:349-363)
 * and the flow tables held in struct proc (defs.h:244).
 * Returns 0, -EINVAL (bad cfg), -ENODEV (no such device) or -ENOMEM.
 */
int gcl_open(int hip_device, const struct gcl_cfg *cfg, struct gcl_ctx **out);
void gcl_close(struct gcl_ctx *ctx);

/*
 * gcl_runtime_set - add or update a runtime (proc).
 * Mirrors dp_clients_add_client (dp_clients.c:156-185: clients_by_id[uniqid],
 * rte_hash_add_key_data(ip)) plus the flow table that sched_steer_flows writes
 * (sched.c:122-147).  @flow_tbl holds @thread_count entries (ignored when
 * @active_count == 0).  Returns -EEXIST if another runtime owns @ip_host
 * (dp_clients.c:174-179), -EINVAL on out-of-range arguments.
 */
int gcl_runtime_set(struct gcl_ctx *ctx, uint16_t uniqid, uint32_t ip_host,
                    uint16_t thread_count, uint16_t active_count,
                    const uint16_t *flow_tbl);

/* gcl_runtime_del - remove a runtime (dp_clients_remove_client,
 * dp_clients.c:230-250).  Returns -ENOENT if @uniqid is not present. */
int gcl_runtime_del(struct gcl_ctx *ctx, uint16_t uniqid);

/*
 * gcl_steer_flows - the flow_tbl rule of sched_steer_flows (sched.c:122-147):
 * identity for the active threads, the rest round-robin over them.  Host-only
 * helper; leaves @flow_tbl untouched when @active_count == 0, like the
 * reference.  @active_idx lists the active thread indices in activation order.
 */
int gcl_steer_flows(uint16_t thread_count, const uint16_t *active_idx,
                    uint16_t active_count, uint16_t *flow_tbl);

/*
 * gcl_classify - classify @b->n packets on @hip_stream (NULL = null stream).
 * @verdicts       device gcl_verdict[n] (gcl_verdict4[n] with GCL_CFG_VERDICT4,
 *                 u16[n] with GCL_CFG_VERDICT2)
 * @runtime_counts device u64[max_runtimes], ACCUMULATED: packets steered to
 *                 each runtime (DELIVER + WAKE), may be NULL
 * @stats          device u64[GCL_NR_STATS], ACCUMULATED, may be NULL
 * Asynchronous; returns -EINVAL for malformed batches (including n > 2^40),
 * -EIO when the table
 * upload fails, -ENOSPC when the IP table cannot place every key (cuckoo
 * placement failed for all 256 seeds: not seen at the table's load <= 1/2).
 * Replaces the rx_one_pkt loop of rx_burst (rx.c:281-287).
 */
int gcl_classify(struct gcl_ctx *ctx, const struct gcl_batch *b,
                 void *verdicts, uint64_t *runtime_counts,
                 uint64_t *stats, void *hip_stream);

/*
 * End-to-end classification of a batch whose frames are in HOST memory (the
 * NIC's mbufs in the iokernel's ingress region), verdicts returned to host
 * memory; synchronous.  Two transports:
 *  GCL_E2E_COPY     the 64-B header granule of every fixed-stride slot is
 *                   DMA-gathered into HBM (hipMemcpy2DAsync), classified, and
 *                   the verdicts copied back; chunks pipelined over nstreams.
 *  GCL_E2E_ZEROCOPY the kernel reads the headers directly from pinned or
 *                   registered host memory over PCIe (gcl_host_register) and
 *                   writes the verdicts directly into host memory.
 * @host_counts / @host_stats are accumulated (may be NULL).
 * Returns -EFAULT when a ZEROCOPY buffer is not pinned/registered.
 */
enum gcl_e2e_mode {
	GCL_E2E_COPY = 0,
	GCL_E2E_ZEROCOPY = 1,
};

struct gcl_e2e_opts {
	uint32_t mode;      /* enum gcl_e2e_mode */
	uint32_t nstreams;  /* COPY: chunks in flight (1..4, 0 = 2) */
	uint64_t chunk;     /* COPY: packets per chunk (0 = 1 Mi) */
};

int gcl_classify_host(struct gcl_ctx *ctx, const struct gcl_batch *host_batch,
                      void *host_verdicts, uint64_t *host_counts,
                      uint64_t *host_stats, const struct gcl_e2e_opts *opts);

/*
 * gcl_header_gather - the COPY transport's gather step over per-packet
 * offsets, as gcl_classify_host uses it (and gcl_group_classify_host, per
 * GPU): on the current HIP device's @hip_stream, row i of @rows (device
 * memory, @n x GCL_GATHER_ROW bytes) gets frame bytes [0, GCL_GATHER_ROW)
 * of the frame at @frames + offs[i], bytes at or past @frames_len reading 0
 * (offsets clamped as gcl_batch's).  @frames and @offs are device-visible
 * pointers (a registered region's mapped address, or HBM).  The rows hold
 * everything rx_one_pkt reads (ports end at byte 78 for IHL 15), so a
 * classify over @rows with stride GCL_GATHER_ROW equals one over the
 * frames.  Asynchronous; 0, -EINVAL or -EIO.
 */
#define GCL_GATHER_ROW 80
int gcl_header_gather(const uint8_t *frames, uint64_t frames_len, const uint64_t *offs, uint64_t n,
                      uint8_t *rows, void *hip_stream);

/* Pin + map host memory for ZEROCOPY / async copies (hipHostRegister). */
int gcl_host_register(void *p, size_t len);
int gcl_host_unregister(void *p);

/*
 * Transport demux pre-hash (runtime/net/transport.c:29-42, :355-398).  For a
 * packet delivered to runtime p that the runtime will hand to trans_lookup
 * -- IPv4, version 4, IHL 5, the MF test of ip_hdr_supported as written
 * (runtime/net/core.c:203-209: IP_MF applied to the network-order field),
 * TCP or UDP -- the GPU computes, with p's trans_seed:
 *   h5 = hash_crc32c_two(seed, laddr.ip | laddr.port << 32,
 *                        raddr.ip | raddr.port << 32 | proto << 48)
 *   h3 = hash_crc32c_one(seed, laddr.ip | laddr.port << 32 | proto << 48)
 * with laddr = (daddr, dport), raddr = (saddr, sport) in host order, i.e.
 * trans_hash_5tuple / trans_hash_3tuple; the runtime's table buckets are
 * h % TRANS_TBL_SIZE.  GCL_ACT_F_TRANS marks valid entries.
 */
struct gcl_trans {
	uint32_t h5;
	uint32_t h3;
};

/* gcl_runtime_set_trans_seed - the runtime's trans_seed (transport.c:27,
 * :459); needs GCL_CFG_TRANS_HASH.  -ENOENT if @uniqid is not present. */
int gcl_runtime_set_trans_seed(struct gcl_ctx *ctx, uint16_t uniqid, uint32_t seed);

/* All outputs of one classify launch (device pointers; NULL = not wanted). */
struct gcl_out {
	void *verdicts;                  /* required: gcl_verdict[n] or gcl_verdict4[n] */
	uint64_t *runtime_counts;        /* accumulated */
	uint64_t *stats;                 /* accumulated */
	struct gcl_trans *trans;         /* GCL_CFG_TRANS_HASH only */
};

int gcl_classify_ex(struct gcl_ctx *ctx, const struct gcl_batch *b, const struct gcl_out *out,
                    void *hip_stream);

/*
 * gcl_access_probe - a measurement aid beside the classify kernel's roofline
 * (bench.py roofline.ceiling_ms), not part of the rx path.  Asynchronous on
 * @hip_stream; 0, -EINVAL or -EIO.  @out receives @vbytes (1, 2, 4 or 8)
 * bytes per packet (not verdicts: a fold of the loaded bytes).
 *
 * At the context's own verdict width: the gcl_classify launch itself -- the
 * same kernel and geometry, its loads (tiles staged through LDS with their
 * drains and barriers for a dense batch; lane-pair header loads, offsets and
 * side arrays for a batch with offsets), and the same verdict writes
 * (deferred where the context defers them) -- with rx_one_pkt replaced by a
 * fold of the header words it reads (and the batch's ol_flags, and hash.rss
 * in a NIC-mode context).  So its time is the kernel's memory shape with
 * nothing computed: the kernel's own ceiling.
 *
 * At another width, or with GCL_PROBE_MIN or'ed into @vbytes: the memory requests
 * one launch over @b cannot do without, and nothing else -- the ceiling the
 * frame layout itself sets (e.g. one 128-B line fetched per 64-B header of a
 * 1536-B slot).  One 16-B load per packet of the line holding frame byte 0
 * (plus one of the next line when frame bytes [0, 40) cross into it), @b's
 * offs, olflags and rss when given, and one write-through store per packet.
 */
#define GCL_PROBE_MIN 0x100
int gcl_access_probe(struct gcl_ctx *ctx, const struct gcl_batch *b, void *out, uint32_t vbytes,
                     void *hip_stream);

/*
 * Test and A/B overrides of the library's measured defaults.  A dataplane
 * never needs them: with every field GCL_TUNE_AUTO (gcl_tune_init) the
 * library makes its own choice, and no environment variable changes it.  The
 * parity tests use them to drive every launch shape and loop form through
 * the same code, tools/ for its A/Bs.
 *
 * gcl_tune_init  - every field GCL_TUNE_AUTO, loop_t0 and debug 0, size set.
 * gcl_ctx_tune   - copy @t into @ctx (NULL: back to the defaults); 0, or
 *                  -EINVAL for a wrong size or a field out of its range.  The
 *                  batch fields apply from the next gcl_classify*, the loop
 *                  fields from the next gcl_rxloop_start.
 */
#define GCL_TUNE_AUTO (-1)
struct gcl_tune {
	uint32_t size;           /* sizeof(struct gcl_tune) */
	/* batch kernels */
	int32_t tables;          /* 0: tables in LDS when they fit, 1: in HBM */
	int32_t depth;           /* tiles in flight per block: 1 or 2 */
	int32_t threads;         /* lanes (packets) per block: 256, 512 or 1024 */
	int32_t grid;            /* blocks per launch (default: the persistent grid) */
	int32_t blocks_per_cu;   /* cap on blocks per CU */
	int32_t defer;           /* dense 1-/2-B verdicts: 0 stored per packet, 1 kept in LDS +
	                            registers and written after the reads where that takes
	                            <= 2 writes per block (default), 2 always */
	int32_t pair_lean;       /* classify_pair_kernel: plain-IPv4 waves on the lean path (1) */
	int32_t tile_lean;       /* classify_kernel: plain-IPv4 waves on the lean path (1) */
	/* the persistent loop */
	int32_t loop64;          /* 0: bursts <= 64 through the general loop kernel */
	int32_t loop_lean;       /* plain-IPv4 bursts on the lean path (1) */
	int32_t loop_spec;       /* speculative window in 10-ns ticks (400; 1 ms with <= 2 workers) */
	int32_t loop_phase_max;  /* poll-phase delay: ceiling in ticks (0 off), set with the two below */
	int32_t loop_phase_up;   /* its step up (> 0) */
	int32_t loop_phase_down; /* its step down (<= up) */
	int32_t loop_prefetch;   /* the next ticket's poll during classification (0 / 1) */
	uint32_t debug;          /* 1: loop diagnostics to stderr */
	int32_t rec_prefetch;    /* GCL_LOOP_HDR_RECORDS: frame headers gcl_rxloop_submit keeps
	                            in flight while it writes the records, 0..64 (64) */
	int32_t slot_prefetch;   /* a wait with no later ticket submitted takes the next
	                            ticket's slot lines for writing while it spins (0 / 1; 1) */
	int32_t vstage;          /* deferred verdicts: the register-held part of the last write
	                            staged through LDS and stored 16 B per lane (1, default) or
	                            stored a verdict per lane per tile (0) */
	int32_t pair_i32;        /* classify_pair_kernel: batches within 2 GiB in 32-bit
	                            arithmetic through buffer descriptors (1) */
	int32_t tile_order;      /* classify_kernel: tiles dealt round-robin over the blocks (0)
	                            or one contiguous run of tiles per block (1) */
	uint64_t loop_t0;        /* tickets start after loop_t0 (rounded down to a multiple of the
	                            ring's slots): tests of the stamps' wrap */
};
void gcl_tune_init(struct gcl_tune *t);
int gcl_ctx_tune(struct gcl_ctx *ctx, const struct gcl_tune *t);

/* Host CRC32C step with the crc32q contract (no inversion, inc/asm/ops.h:77-80)
 * and the two transport hashes, for the runtime side. */
uint32_t gcl_crc32c_u64(uint32_t crc, uint64_t val);
void gcl_trans_hash(uint32_t seed, uint8_t proto, uint32_t lip, uint16_t lport, uint32_t rip,
                    uint16_t rport, struct gcl_trans *out);

/* Synchronise the context's last stream. */
int gcl_sync(struct gcl_ctx *ctx);

/*
 * gcl_kernel_time - with GCL_CFG_PROFILE: total milliseconds the classify
 * kernel ran (HIP events around each launch, on its own stream) and the
 * number of launches since the last reset.  Synchronises.
 */
int gcl_kernel_time(struct gcl_ctx *ctx, double *ms, uint64_t *launches, int reset);

/*
 * gcl_profile_sample - with GCL_CFG_PROFILE, time only one classify launch in
 * @every (the first of each run of @every); gcl_kernel_time then reports the
 * timed launches.  A timed HIP event pair costs the stream ~10 us per launch
 * on MI355X; sampling keeps that out of the throughput it measures.
 * Default 1 (every launch).  -EINVAL for @every == 0.
 */
int gcl_profile_sample(struct gcl_ctx *ctx, uint32_t every);

/*
 * Synthetic rx traffic generator (device).  Counter-based: packet g of the
 * global stream depends only on (seed, g), so every rank and the CPU oracle
 * produce identical bytes.  Packet j of this call is global packet
 * ((j / shard_block) * world + rank) * shard_block + j % shard_block
 * (round-robin block sharding across ranks).
 */
enum gcl_workload {
	GCL_WL_UDP64 = 0,       /* 64-B Eth/IPv4/UDP, uniform 5-tuples */
	GCL_WL_TCP1500_ZIPF = 1,/* 1500-B Eth/IPv4/TCP, Zipf flow ranks */
	GCL_WL_MIXED = 2,       /* IPv4 TCP/UDP + IPv6 + ARP, jumbo lengths */
};

struct gcl_gen_params {
	uint32_t workload;      /* enum gcl_workload */
	uint32_t nruntimes;     /* R: destination IPs are gcl_runtime_ip(r), r < R */
	uint64_t seed;
	uint64_t n;             /* packets to generate */
	uint64_t stride;        /* slot stride (>= 64, multiple of 16) */
	uint32_t rank, world;   /* shard position */
	uint64_t shard_block;   /* packets per round-robin block (0 = no sharding) */
	const uint64_t *zipf_cdf; /* device u64[nflows] (TCP1500_ZIPF only) */
	uint32_t nflows;
	uint32_t pad;
	uint16_t *pkt_len;      /* optional device u16[n]: frame length on the wire
	                           (64, 1500, or the mixed stream's IP/ARP length) */
};

/* Write the first GCL_HDR_GRANULE bytes of every slot of @frames (n * stride
 * bytes; the rest of each slot is left as the caller initialised it), and
 * optionally olflags[n] (what the NIC would report) and rss[n] (an arbitrary
 * 32-bit NIC hash value, so NIC mode can be exercised). */
int gcl_generate(const struct gcl_gen_params *p, uint8_t *frames,
                 uint8_t *olflags, uint32_t *rss, void *hip_stream);

/* IP address of runtime r in the synthetic workloads: 10.0.0.0 + r + 1. */
uint32_t gcl_runtime_ip(uint32_t r);

/* Host helper: Zipf(s) CDF over @nflows ranks as u64 fixed point
 * (cdf[k] = floor(P(rank <= k) * 2^64), last entry saturated). */
int gcl_zipf_cdf(uint32_t nflows, double s, uint64_t *cdf_out);

/*
 * Loopback feed helpers (iokernel/tx.c:81-83, iokernel/dma.c:182-185): the rx
 * olflags of a looped-back tx packet (RSS_HASH iff the runtime set
 * TXFLAG_LOCAL_HINT; IP checksum always good after copy_batch), and the 16-bit
 * steering hint carried in bits 48..63 of the txpkt payload
 * (inc/iokernel/queue.h:120-134).
 */
uint8_t gcl_loopback_olflags(uint8_t tx_olflags);
uint32_t gcl_txpkt_rss(uint64_t payload);

/* Host reference of the two hashes the kernel computes (for callers that
 * need the same value on the CPU, e.g. the loopback hint). */
uint32_t gcl_jenkins_hash(const void *key, size_t len);
uint32_t gcl_toeplitz(const uint8_t *key, size_t keylen, const uint8_t *input,
                      size_t len);

/* Device memory for batches (hipMalloc on @hip_device): 0, -ENODEV, -ENOMEM. */
int gcl_dev_alloc(int hip_device, size_t bytes, void **out);
int gcl_dev_free(void *p);

/*
 * Placement-aware device allocation for the two long-lived classify buffers
 * (the frame pool and the verdict ring, the GPU-side counterparts of the
 * iokernel's ingress region and rxq rings, shm.h:14-15, ioqueues.c:31-40).
 * On MI355X the header read stream and the verdict write stream run ~15%
 * slower when the two buffers fall in the same physical placement class
 * (measured: DESIGN.md §4 "Buffer placement", profiles/archive/r01_pair_*.jsonl).
 * The class cannot be read from a virtual address, so this allocates a
 * candidate, times a read+write probe of the classify kernel's access shape
 * over the whole of both buffers (up to 4 GiB read, 256 MiB written) against
 * @partner, and keeps the first candidate whose probe differs from an
 * earlier one by more than the class gap (the faster of the two), trying at
 * most GCL_PAIR_TRIES candidates; losers are freed.  Classes come in runs of
 * consecutive allocations (4-34 GiB of 2-GiB pools in a row were measured,
 * profiles/archive/r02_classmap.jsonl), so after every GCL_PAIR_RUN candidates of one
 * class a spacer of 2, 4, 8, then 16 x @bytes is allocated to step past the
 * run.  Candidates and spacers together hold at most 60% of the free device
 * memory; all but the kept buffer are freed before returning.  When no second
 * class shows up the fastest candidate is kept, @info->classes is 1 and a
 * warning goes to stderr (the GCL_PAIR_QUIET flag silences it;
 * GCL_PAIR_VERBOSE prints every candidate's probe).
 *
 * GCL_PAIR_NEW_READS: the new buffer is the one stream-read (frames) and
 *                     @partner the one written (verdicts);
 * GCL_PAIR_NEW_WRITES: the reverse.
 * OR in GCL_PAIR_VBYTES(1|2|4|8), the verdict width the kernel will write
 * (default 4): the probe stores the same width, so its time tracks the
 * kernel's for every format.
 * The probe WRITES to the written side's first min(bytes, 256 MiB), rounded
 * down to whole 256-verdict tiles (@info->probe_write_bytes), and nothing past it: call it before that buffer
 * holds data.  @info may be NULL.
 * Returns 0, -EINVAL, -ENODEV, -ENOMEM or -EIO.
 */
#define GCL_PAIR_NEW_READS  0x1
#define GCL_PAIR_NEW_WRITES 0x2
#define GCL_PAIR_VBYTES(b)  ((uint32_t)(b) << 8)
#define GCL_PAIR_VBYTES_OF(f) (((f) >> 8) & 0xFF)
#define GCL_PAIR_QUIET      0x10000
#define GCL_PAIR_VERBOSE    0x20000
#define GCL_PAIR_TRIES      24
#define GCL_PAIR_RUN        2
struct gcl_pair_info {
	double   chosen_us;         /* probe time of the buffer kept */
	double   worst_us;          /* slowest candidate probed */
	uint32_t candidates;        /* candidates probed */
	uint32_t classes;           /* placement classes seen: 2, or 1 (kept one may be slow) */
	uint64_t spacer_bytes;      /* spacer memory held during the search */
	uint64_t probe_write_bytes; /* bytes of the written side the probe stored to */
};
int gcl_dev_alloc_paired(int hip_device, size_t bytes, const void *partner, size_t partner_bytes,
                         uint32_t flags, void **out, struct gcl_pair_info *info);

/*
 * Persistent rx loop: the classifier at the reference's own granularity, one
 * rx_burst of <= IOKERNEL_RX_BURST_SIZE mbufs at a time (iokernel/rx.c:270-290,
 * defs.h:75), with microsecond latency instead of batch latency.  A
 * persistent kernel polls a ring of burst slots in coherent host memory,
 * classifies each burst straight from the registered ingress region (the 2
 * GiB mbuf pool, shm.h:14-15) and writes the verdicts back into the slot.
 *
 * gcl_rxloop_start - launch the loop for @ctx.  @cfg->region must be
 *   registered with gcl_host_register; frames are addressed by byte offsets
 *   into it (mbuf data pointer - region base, like ptr_to_shmptr, shm.h:40-47).
 *   The kernel leaves by itself after @cfg->lifetime_ms.  Tables must fit in
 *   LDS (-E2BIG otherwise); with GCL_CFG_TRANS_HASH each burst's transport
 *   demux hashes come back beside its verdicts (gcl_rxloop_trans);
 *   one loop per context (-EBUSY); the region must be shorter than 2^40 - 64
 *   bytes (-EINVAL: offsets share their slot entry with a stamp, so a burst
 *   of <= 64 packets has its offsets with the poll that finds it; offsets at
 *   or past the region's end still read as frames of zeros).  Table changes
 *   made with gcl_runtime_set /
 *   _del apply from the next submitted burst on (snapshot semantics).
 * gcl_rxloop_submit - publish one burst; returns its ticket (> 0), -EAGAIN
 *   when the ring is full (a slot is reused only after gcl_rxloop_wait has
 *   collected the burst it held, as an lrpc ring's consumer frees a slot), -EINVAL, -E2BIG (tables grew past LDS) or
 *   -ESHUTDOWN when the kernel has left.  The arrays are copied; the side
 *   arrays (olflags, rss, fdir_hi, dst_hint) are optional, as in gcl_batch.
 * gcl_rxloop_wait - spin up to @spin_ns for @ticket; 0 and the burst's
 *   verdicts (gcl_verdict or gcl_verdict4 per the context) copied to
 *   @verdicts_out (may be NULL), -EAGAIN if not done yet, -ESTALE if the slot
 *   was already reused, -ESHUTDOWN if the kernel left first.
 * gcl_rxloop_stop - raise the stop flag, wait for the kernel, free the loop.
 * gcl_rxloop_drive - measurement helper: @iters bursts of the same @n offsets
 *   with @depth bursts in flight; lat_ns[i] = submit -> verdicts seen of
 *   burst i, *elapsed_ns the whole run.
 */
struct gcl_rxloop;
struct gcl_rxloop_cfg {
	uint32_t slots;        /* ring depth: power of two, 2..1024 */
	uint32_t max_burst;    /* packets per burst: 1..4096 */
	uint32_t workers;      /* polling workgroups: 1..64 */
	uint32_t lifetime_ms;  /* kernel lifetime bound: 1..600000 */
	const void *region;    /* registered host region holding the frames */
	uint64_t region_len;
	uint64_t *counts;      /* device u64[max_runtimes] (optional), accumulated; the loop
	                          runs on a stream of its own: gcl_rxloop_start waits for the
	                          default stream's work (e.g. their zeroing), work on other
	                          streams must be complete before the call */
	uint64_t *stats;       /* device u64[GCL_NR_STATS] (optional), accumulated, as counts */
	uint32_t flags;        /* GCL_LOOP_INLINE_HDRS or GCL_LOOP_HDR_RECORDS */
	uint32_t pad;
};
/* gcl_rxloop_submit copies each frame's first 64-B header granule into the
 * ring slot (the dataplane core reads the headers, as rx_one_pkt does), so
 * the kernel fetches them with the burst's side arrays instead of one PCIe
 * round trip later from the region.  Since the offsets arrive with the poll
 * the two forms take the same time for one burst; inlining saves the GPU's
 * reads of the region when many workers keep PCIe busy. */
#define GCL_LOOP_INLINE_HDRS 0x1
/* gcl_rxloop_submit writes each packet as one 64-B header record in the
 * slot: the header words rx_one_pkt reads (frame bytes 12-15 and 20-43), its
 * offset and its side fields, every 16-B chunk led by the slot's use count
 * and written with one 16-B store (the four chunks of a record in four
 * planes, so the GPU reads each plane contiguously).  A worker polling a burst of <= 64
 * packets reads the records with the slot word and, when every chunk carries
 * the current count, classifies at once: one PCIe round trip per burst
 * instead of two.  Ports past byte 43 (IHL >= 7) are read from the region.
 * Exclusive with GCL_LOOP_INLINE_HDRS (-EINVAL).  A worker polls the records
 * (or, without this flag, the stamped offsets) during the first 4 us of a
 * wait, or the first 1 ms in a loop of 1 or 2 workers (gcl_tune.loop_spec);
 * a burst found later is read after its word.  In a loop of 1 or 2 workers
 * with bursts of <= 64 a worker issues the first poll of each ticket a
 * little after its last verdict records, the delay following the host's
 * turnaround (up to 1.2 us; gcl_tune.loop_phase_*): a dataplane core that
 * submits once it has seen the last verdicts is sampled just after its
 * submit rather than a round trip later.  In a loop of more than 2 workers
 * without this flag (stamped offsets), a worker whose burst was already
 * there at its first poll issues the next ticket's poll while it classifies
 * that burst (gcl_tune.loop_prefetch). */
#define GCL_LOOP_HDR_RECORDS 0x2
/* Measurement: lane 0 of the worker stores each burst's stage times into
 * the slot header after its records (gcl_rxloop_stamps). */
#define GCL_LOOP_STAMPS 0x4
int gcl_rxloop_start(struct gcl_ctx *ctx, const struct gcl_rxloop_cfg *cfg,
                     struct gcl_rxloop **out);
int64_t gcl_rxloop_submit(struct gcl_rxloop *loop, uint32_t n, const uint64_t *offs,
                          const uint8_t *olflags, const uint32_t *rss, const uint32_t *fdir_hi,
                          const uint32_t *dst_hint);
int gcl_rxloop_wait(struct gcl_rxloop *loop, int64_t ticket, void *verdicts_out, uint64_t spin_ns);
/*
 * gcl_rxloop_peek - gcl_rxloop_wait without the copy: on 0, *@recs points at
 * the burst's @*n verdict records in the ring slot itself (one 16-B record per
 * packet, written by the kernel with one store; @verdict holds the verdict in
 * the context's width -- gcl_verdict4 bytes, the 2-byte queue verdict in the
 * low half, or with 8-byte verdicts {hash, verdict} is the struct gcl_verdict).
 * The records stay valid, and the slot is not reused, until
 * gcl_rxloop_release(@ticket): the post-pass (gcl_host_deliver_recs) reads
 * them in place.  Errors as gcl_rxloop_wait.
 */
struct gcl_loop_rec {
	uint32_t hash;
	uint32_t verdict;
	uint64_t ticket;
};
int gcl_rxloop_peek(struct gcl_rxloop *loop, int64_t ticket, uint64_t spin_ns,
                    const struct gcl_loop_rec **recs, uint32_t *n);
int gcl_rxloop_release(struct gcl_rxloop *loop, int64_t ticket);
/* gcl_rxloop_poll_stats - how the loop's bursts have arrived so far, summed
 * over its workers: @out[0] with the poll that found the burst (offsets or
 * header records already current: one PCIe round trip), @out[1] eligible
 * for that (<= 64 packets, in the speculative window) but an entry still
 * stale, so read after the word, @out[2] read after the word (the window
 * over, a longer burst, or inline granules).  Before gcl_rxloop_stop.
 * The burst-of-64 kernel's writer wave posts these counters (and the lean
 * count below) after the burst's verdict records, so both can lag the bursts
 * a gcl_rxloop_wait has seen complete by up to a few microseconds: poll. */
int gcl_rxloop_poll_stats(struct gcl_rxloop *loop, uint64_t out[3]);
/* gcl_rxloop_lean_bursts - how many of the loop's bursts so far were
 * classified by the burst-of-64 kernel's lean path (every packet plain IPv4:
 * IHL 5, no FDIR mark, no dst_ip hint, no transport pre-hash; the verdicts and
 * counters are classify_core's), summed over its workers, into @out.  Before
 * gcl_rxloop_stop. */
int gcl_rxloop_lean_bursts(struct gcl_rxloop *loop, uint64_t *out);
/* gcl_rxloop_trans - a GCL_CFG_TRANS_HASH context's transport demux hashes
 * of @ticket's burst (struct gcl_trans per packet, as gcl_classify_ex writes
 * them), copied to @out once the burst is complete: after gcl_rxloop_wait
 * and before the slot's next submit, or between gcl_rxloop_peek and
 * _release.  -EINVAL (no transport hashes), -EAGAIN (not complete yet),
 * -ESTALE (the slot was reused). */
int gcl_rxloop_trans(struct gcl_rxloop *loop, int64_t ticket, struct gcl_trans *out);
/* gcl_rxloop_stamps - with GCL_LOOP_STAMPS: @ticket's stage times in ns
 * (s_memrealtime, 10-ns ticks): @out[0] the round trip of the poll that
 * found the burst (its issue to its return), @out[1] from that return to
 * the packets classified, @out[2] to the last verdict record's store issued,
 * @out[3] the polls of that wait, @out[4..6] from the return to past the
 * worker's first, second and third barriers (burst header shared, tables
 * and histogram ready, tile ready), @out[7] 0; with the kernel for bursts of
 * <= 64 (max_burst <= 64), @out[4..6] from the return to the packets in
 * registers, the burst posted to the writer wave, the writer taking it,
 * and @out[7] 1.  -EAGAIN until they land
 * (they are posted after the records), -ESTALE once the slot is reused,
 * -EINVAL without the flag. */
int gcl_rxloop_stamps(struct gcl_rxloop *loop, int64_t ticket, uint64_t out[8]);
int gcl_rxloop_stop(struct gcl_rxloop *loop);
int gcl_rxloop_drive(struct gcl_rxloop *loop, uint32_t n, const uint64_t *offs, uint32_t iters,
                     uint32_t depth, uint64_t *lat_ns, uint64_t *elapsed_ns);

/* Library version string. */
const char *gcl_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GCLASSIFY_H */
