/*
 * orc.h - CPU oracle for the rx classify path.  TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference algorithm, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker and
 * as the timed CPU baseline.  The product (caladan_amd/) never links, loads or
 * calls anything in oracle/.
 *
 * What it restates (each function cites its reference lines):
 *   orc_jhash         base/jenkins_hash.c:126-297 (lookup3 hashlittle, initval 0)
 *   orc_do_toeplitz   runtime/net/core.c:120-139
 *   orc_steer_flows   iokernel/sched.c:122-147
 *   orc_rx_burst      iokernel/rx.c:270-290 (bursts of 64, prefetch stride 2)
 *   orc_rx_one_pkt    iokernel/rx.c:116-233 (+ rx_send_to_runtime :50-73)
 *   rx_one_pkt_direct the same, as the CPU baseline: rx.c's direct header
 *                     struct loads and the NIC hash (orc_bench_ex DIRECT)
 *   orc_crc32c_u64    crc32q, inc/asm/ops.h:77-80 (hash_crc32c_one/two)
 *   orc_trans         trans_hash_5tuple/3tuple, runtime/net/transport.c:29-42
 *   orc_iptab_*       the ip_to_proc rte_hash (iokernel/dp_clients.c:349-363),
 *                     keyed by jhash of the 4-byte host-order IP like rte_jhash
 *
 * Pinning: orc_jhash is checked against base/jenkins_hash.c compiled from the
 * reference tree (oracle/_ref, see oracle/Makefile) and the published lookup3
 * KATs; orc_do_toeplitz against the reference's own do_toeplitz, compiled in
 * place (oracle/ref_core.c, tests/golden/toeplitz_ref.json), and the
 * Microsoft RSS verification vectors; orc_rx_one_pkt against
 * hand-derived scenario fixtures (tests/golden/rx_scenarios.json) that cite
 * rx.c line by line.  iokernel/rx.c itself needs DPDK headers that are not in
 * this image, so it is not compiled here, and the reference ships no tests or
 * fixtures for it: the decision tree of orc_rx_one_pkt is PARITY UNPINNED by
 * reference outputs (pinned only by those hand-derived fixtures); the hashes
 * it calls are pinned (see DESIGN.md "Oracle").  The host post-pass's lrpc
 * ring and rxq_cmd encoding are pinned against base/lrpc.c and
 * inc/iokernel/queue.h built from the reference (oracle/ref_host.c,
 * tests/test_ref_host.py).
 */
#ifndef ORC_H
#define ORC_H

#include <stddef.h>
#include <stdint.h>

#include "../include/gclassify.h"

#ifdef __cplusplus
extern "C" {
#endif

uint32_t orc_jhash(const void *key, size_t len);
uint32_t orc_do_toeplitz(const uint8_t *key, uint32_t saddr, uint32_t daddr,
                         uint16_t sport, uint16_t dport);
/* generic Toeplitz over a byte string (MSB-first), for the KAT vectors */
uint32_t orc_toeplitz_bytes(const uint8_t *key, size_t keylen,
                            const uint8_t *in, size_t len);
uint32_t orc_crc32c_u64(uint32_t crc, uint64_t val);
void orc_steer_flows(uint16_t thread_count, const uint16_t *active_idx,
                     uint16_t active_count, uint16_t *flow_tbl);

struct orc_runtime {
	int      present;
	uint32_t ip;
	uint16_t thread_count;
	uint16_t active;
	uint16_t flow_tbl[GCL_NCPU];
};

struct orc_tables;

struct orc_tables *orc_tables_new(uint32_t max_runtimes, uint32_t hash_mode,
                                  uint32_t flags, uint8_t default_olflags,
                                  const uint8_t *rss_key40);
void orc_tables_free(struct orc_tables *t);
/* 0, -EEXIST (duplicate ip), -EINVAL */
int orc_runtime_set(struct orc_tables *t, uint16_t uniqid, uint32_t ip,
                    uint16_t thread_count, uint16_t active,
                    const uint16_t *flow_tbl);
int orc_runtime_del(struct orc_tables *t, uint16_t uniqid);
int orc_runtime_set_trans_seed(struct orc_tables *t, uint16_t uniqid, uint32_t seed);

/* Classify a host batch (gcl_batch with host pointers), accumulating counts
 * and stats.  Processes bursts of 64 with the rx.c prefetch stride. */
void orc_classify(const struct orc_tables *t, const struct gcl_batch *b,
                  struct gcl_verdict *v, uint64_t *counts, uint64_t *stats);

/* Same, plus the runtime-side transport demux hashes when the tables were
 * created with GCL_CFG_TRANS_HASH (trans may be NULL). */
void orc_classify_ex(const struct orc_tables *t, const struct gcl_batch *b,
                     struct gcl_verdict *v, uint64_t *counts, uint64_t *stats,
                     struct gcl_trans *tr);

/* Same, plus lrpc_send of a 16-B message per delivered packet into
 * 4096-deep per-(runtime, thread) rings that are drained after every burst
 * (inc/base/lrpc.h:48-63, runtime/ioqueues.c:31-40). */
void orc_classify_lrpc(const struct orc_tables *t, const struct gcl_batch *b,
                       struct gcl_verdict *v, uint64_t *counts, uint64_t *stats);

/* CPU baseline timer: classify the batch @passes times on @threads threads
 * (each thread a contiguous shard, its own verdict/count buffers).  Returns
 * wall seconds. */
double orc_bench(const struct orc_tables *t, const struct gcl_batch *b,
                 int threads, int passes, int with_lrpc);

/* orc_bench with options: ORC_BENCH_LRPC adds the lrpc_send of every
 * delivered packet; ORC_BENCH_DIRECT classifies with rx.c's direct header
 * loads (no bounds test: every frame's first 54 bytes must be in range). */
#define ORC_BENCH_LRPC   0x1
#define ORC_BENCH_DIRECT 0x2
/* the ORC_BENCH_LRPC loop (command, flow_tbl[slot]) without the ring write:
 * isolates lrpc_send's own cost from the loop's shape */
#define ORC_BENCH_NOSEND 0x4
double orc_bench_ex(const struct orc_tables *t, const struct gcl_batch *b,
                    int threads, int passes, unsigned int flags);
/* orc_bench_ex with thread i pinned to CPU @cpus[i] (a -1 entry, or a NULL
 * @cpus, leaves a thread unpinned) */
double orc_bench_pinned(const struct orc_tables *t, const struct gcl_batch *b,
                        int threads, int passes, unsigned int flags, const int *cpus);

/* A CPU dataplane for the pipeline baseline (tools/cpupipe): the lrpc rings
 * of orc_classify_lrpc kept across bursts, so one rx_burst at a time --
 * rx_one_pkt with rx.c's direct header loads and prefetch stride 2, plus
 * (@send) rx_make_cmd + lrpc_send of every delivered packet -- runs as the
 * reference's dataplane loop does (rx.c:270-290). */
struct orc_dataplane;
struct orc_dataplane *orc_dataplane_new(const struct orc_tables *t);
void orc_dataplane_free(struct orc_dataplane *d);
void orc_dataplane_burst(struct orc_dataplane *d, const struct gcl_batch *b, struct gcl_verdict *v,
                         uint64_t *counts, uint64_t *stats, int send);

/* orc_classify through the CPU-baseline form (direct header loads, same
 * preconditions as ORC_BENCH_DIRECT; dst_hint is ignored). */
void orc_classify_direct(const struct orc_tables *t, const struct gcl_batch *b,
                         struct gcl_verdict *v, uint64_t *counts, uint64_t *stats);

/* Synthetic generator: the same streams as gcl_generate, written on the CPU.
 * frames must hold n*stride bytes (pre-zeroed by the caller). */
int orc_generate(const struct gcl_gen_params *p, const uint64_t *zipf_cdf,
                 uint8_t *frames, uint8_t *olflags, uint32_t *rss);
uint32_t orc_runtime_ip(uint32_t r);
int orc_zipf_cdf(uint32_t nflows, double s, uint64_t *cdf);

#ifdef __cplusplus
}
#endif

#endif
