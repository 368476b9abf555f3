/* deliver_bench.c - the lrpc post-pass alone on one host core: compact
 * verdicts of a udp64-like stream (16 runtimes x 8 kthreads, every packet
 * DELIVER) through gcl_host_deliver4 into 4096-deep rings, the runtimes
 * emulated as infinitely fast consumers as in tools/rxpipe.
 *
 *   deliver_bench <burst> <packets> [ops]   -> one JSON line
 *
 * With "ops" the two per-delivery callbacks of the reference are wired in:
 * thread_enable_sched_poll as a bit set in a per-runtime poll mask, and the
 * ownership record (rx.c:86-90) as an append to a per-runtime list threaded
 * through a per-mbuf next array.
 *
 * Build: gcc -std=gnu11 -O3 -Iinclude -o tools/deliver_bench tools/deliver_bench.c \
 *          caladan_amd/csrc/gcl_host.c -lm
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "gcl_host.h"

static uint64_t poll_mask[16][4];
static uint32_t *own_next, own_tail[16];

static void enable_poll(void *arg, struct gcl_host_proc *p, unsigned int th)
{
	(void)arg;
	poll_mask[p->uniqid][th >> 6] |= 1ull << (th & 63);
}

static void owned(void *arg, struct gcl_host_proc *p, uint64_t i)
{
	const uint32_t base = *(const uint32_t *)arg;
	own_next[own_tail[p->uniqid]] = base + (uint32_t)i;
	own_tail[p->uniqid] = base + (uint32_t)i;
}

static uint64_t now_ns(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int main(int argc, char **argv)
{
	const uint32_t burst = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
	const uint64_t npkts = argc > 2 ? strtoull(argv[2], NULL, 0) : 1 << 26;
	const uint32_t R = 16, T = 8, RING = 4096, NV = 1 << 16;
	static struct gcl_host_proc procs[16];
	struct gcl_host_proc *by_id[16];
	static struct gcl_lrpc_chan_out chans[16 * 8];
	static uint32_t heads[16 * 8];
	struct gcl_lrpc_msg *msgs = aligned_alloc(64, sizeof(*msgs) * R * T * RING);
	struct gcl_verdict4 *v = malloc(sizeof(*v) * NV);
	uint16_t *len = malloc(2 * NV);
	uint64_t *shm = malloc(8 * NV), stats[GCL_NR_STATS] = {0};
	uint64_t x = 0x9E3779B97F4A7C15ull, delivered = 0;
	const int with_ops = argc > 3 && !strcmp(argv[3], "ops");
	uint32_t at_base = 0;
	struct gcl_host_ops ops = {.arg = &at_base, .enable_poll = enable_poll, .owned = owned};

	own_next = calloc(NV, sizeof(*own_next));

	if (!burst || burst > NV || !msgs || !v || !len || !shm || !own_next)
		return 1;
	for (uint32_t r = 0; r < R; r++) {
		uint16_t act[GCL_NCPU];
		const uint16_t na = (uint16_t)(r % T + 1);
		for (uint16_t i = 0; i < na; i++)
			act[i] = i;
		memset(&procs[r], 0, sizeof(procs[r]));
		procs[r].uniqid = (uint16_t)r;
		procs[r].thread_count = (uint16_t)T;
		procs[r].active_thread_count = na;
		procs[r].idle_top = -1;
		gcl_steer_flows((uint16_t)T, act, na, procs[r].flow_tbl);
		for (uint32_t t = 0; t < T; t++) {
			gcl_lrpc_init_out(&chans[r * T + t], &msgs[(size_t)(r * T + t) * RING], RING,
			                  &heads[r * T + t]);
			procs[r].rxq[t] = &chans[r * T + t];
		}
		by_id[r] = &procs[r];
	}
	for (uint32_t i = 0; i < NV; i++) {
		x ^= x << 13, x ^= x >> 7, x ^= x << 17;
		const uint32_t r = (uint32_t)(x % R);
		v[i].uniqid = (uint16_t)r;
		v[i].thread = (uint8_t)((x >> 32) % T); /* the flow_tbl slot */
		v[i].action = GCL_ACT_DELIVER;
		len[i] = 60;
		shm[i] = (uint64_t)i * 64;
	}
	uint64_t best = ~0ull;
	for (int rep = 0; rep < 5; rep++) {
		const uint64_t t0 = now_ns();
		for (uint64_t done = 0; done < npkts; done += burst) {
			const uint32_t at = (uint32_t)(done % (NV - NV % burst));
			at_base = at;
			delivered += gcl_host_deliver4(by_id, R, by_id, (int)R, v + at, NULL, len + at, NULL,
			                               GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD, shm + at, burst,
			                               with_ops ? &ops : NULL, stats);
			for (uint32_t i = 0; i < R * T; i++)
				heads[i] = chans[i].send_head;
		}
		const uint64_t el = now_ns() - t0;
		best = el < best ? el : best;
	}
	printf("{\"burst\": %u, \"ops\": %d, \"packets\": %llu, \"ns_per_pkt\": %.2f, \"mpps\": %.1f, "
	       "\"check\": \"%s\"}\n", burst, with_ops, (unsigned long long)npkts, (double)best / npkts,
	       npkts * 1e3 / best, delivered == 5 * ((npkts + burst - 1) / burst) * burst &&
	       !stats[GCL_RX_UNICAST_FAIL] ? "ok" : "MISMATCH");
	return 0;
}
