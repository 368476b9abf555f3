/*
 * gcl_group.h - the multi-GPU step of the rx classifier behind the C ABI
 * (libgclgroup.so, links libgclassify.so and RCCL).
 *
 * The iokernel is ONE process with ONE dataplane thread on one lcore
 * (iokernel/dpdk.c:276-280, iokernel/main.c:144-150), so the form of the
 * multi-GPU step it can link is one process driving every GPU: a group of
 * one gcl_ctx per GPU with replicated tables, each batch split round-robin
 * in blocks of packets over the GPUs (packets are independent, rx.c:116-233
 * reads nothing across packets), and one RCCL all-gather of every GPU's
 * per-runtime counts and rx counters (u64[max_runtimes + GCL_NR_STATS]) over
 * xGMI, on a communicator made by ncclCommInitAll.  The only cross-packet
 * output of rx_burst is those counters (the per-proc steering is per packet
 * and the STAT_INC counters are global, iokernel/defs.h:417-460), so that is
 * the whole exchange.
 *
 * Conventions are gclassify.h's: 0 or -errno, not thread-safe, one group per
 * dataplane thread.
 */
#ifndef GCL_GROUP_H
#define GCL_GROUP_H

#include <stdint.h>

#include "gclassify.h"

#ifdef __cplusplus
extern "C" {
#endif

#define GCL_GROUP_MAX_DEV     16
#define GCL_GROUP_BLOCK       (64u << 10)  /* default packets per round-robin block */
#define GCL_GROUP_MAX_STREAMS 4

/* How gcl_group_exchange combines the GPUs' counters. */
enum gcl_group_xchg {
	GCL_XCHG_RCCL = 0, /* one ncclAllGather per GPU (ncclGroupStart/End) + a sum kernel */
	GCL_XCHG_HOST = 1, /* copy each GPU's vector to the host and sum there: only for a
	                      group whose contexts share a GPU (rehearsals on a one-GPU box;
	                      RCCL refuses two ranks of one communicator on one device) */
};

struct gcl_group_cfg {
	uint64_t block;    /* packets per round-robin block, multiple of 256; 0 = GCL_GROUP_BLOCK */
	uint32_t exchange; /* enum gcl_group_xchg */
	uint32_t nstreams; /* work streams per GPU for gcl_group_classify_host, 1..4 (0 = 2) */
	uint32_t init_timeout_ms; /* GCL_XCHG_RCCL: bound on communicator init, and on an
	                             exchange's RCCL enqueue (0 = GCL_GROUP_INIT_TIMEOUT_MS) */
	uint32_t size;     /* sizeof(struct gcl_group_cfg): GCL_GROUP_CFG_INIT sets it;
	                      gcl_group_open refuses another value (-EINVAL) */
};
/* The struct's history: rounds 1-3, 16 B (block, exchange, nstreams) through
 * the symbol gcl_group_open; round 4, 24 B (+ init_timeout_ms and a pad word)
 * through the same symbol; round 5 (GCL_GROUP_ABI 2, library ABI 5), the pad
 * word became `size` and the entry point gcl_group_open_v2, to which this
 * header maps the name.  The exported gcl_group_open reads only the 16-B
 * fields: a binary built against the round-4 header loses init_timeout_ms
 * (the default bound applies) until it is rebuilt against this header. */
#define GCL_GROUP_ABI 2
#define GCL_GROUP_CFG_INIT { 0, GCL_XCHG_RCCL, 0, 0, sizeof(struct gcl_group_cfg) }
#define GCL_GROUP_INIT_TIMEOUT_MS 60000

struct gcl_group;

/*
 * gcl_group_open - one context per entry of @devs (HIP device ids, distinct
 * for GCL_XCHG_RCCL), all with @cfg, and the RCCL communicator over them.
 * @gcfg may be NULL (64 Ki blocks, RCCL, 2 streams).
 * The communicators are created non-blocking (ncclCommInitRankConfig with
 * blocking = 0) and polled: a bootstrap that does not finish within
 * init_timeout_ms is aborted and gives -ETIMEDOUT instead of blocking the
 * caller.
 * @gcfg->size must be sizeof(struct gcl_group_cfg) (GCL_GROUP_CFG_INIT).
 * Returns 0, -EINVAL, -ENODEV, -ENOMEM, -ETIMEDOUT, or -EIO when RCCL init fails.
 */
int gcl_group_open_v2(int ndev, const int *devs, const struct gcl_cfg *cfg,
                      const struct gcl_group_cfg *gcfg, struct gcl_group **out);
#define gcl_group_open gcl_group_open_v2
void gcl_group_close(struct gcl_group *g);

/* Number of GPUs (contexts), and context @i (NULL if out of range): the
 * per-GPU calls of gclassify.h (gcl_kernel_time, gcl_rxloop_*) work on it. */
int gcl_group_size(const struct gcl_group *g);
struct gcl_ctx *gcl_group_ctx(struct gcl_group *g, int i);
/* HIP stream (hipStream_t) of GPU @i's device-resident classify launches. */
void *gcl_group_stream(struct gcl_group *g, int i);

/* Table changes fanned out to every context (dp_clients_add_client /
 * _remove_client + sched_steer_flows, as gcl_runtime_set / _del): the first
 * context decides the result (-EEXIST, -EINVAL, -ENOENT) and the others are
 * only changed when it succeeds, so the replicas never diverge. */
int gcl_group_runtime_set(struct gcl_group *g, uint16_t uniqid, uint32_t ip_host,
                          uint16_t thread_count, uint16_t active_count,
                          const uint16_t *flow_tbl);
int gcl_group_runtime_del(struct gcl_group *g, uint16_t uniqid);
int gcl_group_runtime_set_trans_seed(struct gcl_group *g, uint16_t uniqid, uint32_t seed);

/*
 * Round-robin shard math (host-only): block b of @block packets goes to GPU
 * b mod @world.  gcl_shard_count - packets GPU @rank holds of an @n-packet
 * batch; gcl_shard_global - the batch index of GPU @rank's local packet @j
 * (the mapping gcl_generate's rank/world/shard_block reproduces).
 */
uint64_t gcl_shard_count(uint64_t n, uint32_t world, uint32_t rank, uint64_t block);
uint64_t gcl_shard_global(uint64_t j, uint32_t world, uint32_t rank, uint64_t block);

/*
 * gcl_group_classify - every GPU classifies its own shard, already resident
 * in its HBM (@shards[i], @verdicts[i]: device pointers on GPU i, e.g. filled
 * by the NIC or by gcl_generate with rank i of world n), on its group stream.
 * Counts accumulate on each GPU.  Asynchronous.
 */
int gcl_group_classify(struct gcl_group *g, const struct gcl_batch *shards,
                       void *const *verdicts);

/*
 * gcl_group_classify_host - one batch in HOST memory (the ingress mbufs),
 * split round-robin in blocks over the GPUs; each GPU classifies its blocks
 * (GCL_E2E_ZEROCOPY: straight from registered memory; GCL_E2E_COPY: the
 * blocks' 64-B header granules DMA-gathered into HBM, fixed-stride slots
 * only) and writes their verdicts at their batch positions of
 * @host_verdicts.  All GPUs run at once from this one thread; synchronous.
 * @o->chunk is ignored (the block is the unit); @o->nstreams (1..4) overrides
 * the group's streams per GPU when non-zero.  Counts accumulate on the GPUs as with
 * gcl_group_classify.  -EFAULT when a ZEROCOPY buffer is not registered.
 */
int gcl_group_classify_host(struct gcl_group *g, const struct gcl_batch *hb,
                            void *host_verdicts, const struct gcl_e2e_opts *o);

/*
 * gcl_group_exchange - snapshot every GPU's accumulated [counts | stats]
 * after the work enqueued so far, then all-gather the snapshots (RCCL on a
 * side stream per GPU, so later classify launches overlap it) and sum them
 * into the node-wide vector on every GPU.  Asynchronous; up to 4 exchanges
 * may be in flight.
 * gcl_group_read - wait for the last exchange and return the node-wide
 * per-runtime counts (u64[max_runtimes]) and rx counters (u64[GCL_NR_STATS]),
 * totals since open or the last reset, and optionally the gathered
 * per-GPU vectors (u64[n][max_runtimes + GCL_NR_STATS]).  Any output may be
 * NULL.  -ENODATA before the first exchange.
 * An exchange whose RCCL enqueue fails (-EIO) or does not complete within
 * init_timeout_ms (-ETIMEDOUT) aborts every communicator (ncclCommAbort) and
 * leaves the group failed: every later call except close returns -EIO (the
 * all-gather may still hold the exchange's buffers, and the communicators
 * are in an unknown state).  gcl_group_test_fault makes every RCCL
 * exchange fail that way (tests).
 */
int gcl_group_exchange(struct gcl_group *g);
int gcl_group_read(struct gcl_group *g, uint64_t *node_counts, uint64_t *node_stats,
                   uint64_t *per_gpu);
/* Zero every GPU's accumulated counters (synchronises); -EIO on a failed group. */
int gcl_group_reset(struct gcl_group *g);
/* Wait for everything enqueued on every GPU; a failed group's streams are
 * still drained, and the call returns -EIO. */
int gcl_group_sync(struct gcl_group *g);

/* The rank count of the group's RCCL communicators as RCCL reports it
 * (ncclCommCount; every GPU's communicator must agree), into @ranks: the
 * number of GPUs the exchange really spans.  0 for GCL_XCHG_HOST; -EIO on a
 * failed group or a disagreement. */
int gcl_group_rccl_ranks(const struct gcl_group *g, int *ranks);

/* Test hook: make every later RCCL exchange of @g fail as a timed-out
 * enqueue would (GCL_GROUP_FAULT_EXCHANGE), to exercise the sticky failure
 * above; 0 clears it.  0 or -EINVAL.  Not for production use. */
#define GCL_GROUP_FAULT_EXCHANGE 0x1
int gcl_group_test_fault(struct gcl_group *g, uint32_t what);

#ifdef __cplusplus
}
#endif

#endif /* GCL_GROUP_H */
