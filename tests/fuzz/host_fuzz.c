/*
 * host_fuzz.c - CPU fuzz driver for the host C that parses untrusted input,
 * built with AddressSanitizer + UndefinedBehaviorSanitizer by
 * caladan_amd/build.py --sanitize (tests/test_sanitize.py runs it).
 *
 *   host_fuzz pcap FILE...        gcl_pcap_load each file; print its return
 *                                 code, packet and skipped counts, and touch every
 *                                 captured byte it reports
 *   host_fuzz deliver SEED ITERS  random verdict streams (8-, 4- and 2-byte)
 *                                 through gcl_host_deliver{,4,2}: uniqids past
 *                                 max_runtimes, NULL clients, threads and
 *                                 flow_tbl slots past thread_count, NULL rings,
 *                                 one-slot rings that fill, every action code,
 *                                 a sched_add_core that rewrites the tables
 *   host_fuzz oracle SEED ITERS   random bytes at random offsets (straddling
 *                                 frames_len) through the oracle's bounds-
 *                                 checked classifier in every mode
 *
 * Exit 0 when every call returned; a sanitizer report aborts with non-zero.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/gcl_host.h"
#include "../../include/gcl_pcap.h"
#include "../../oracle/orc.h"

static uint64_t rng_state;

static uint64_t rnd(void)
{
	uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

static int fuzz_pcap(int argc, char **argv)
{
	for (int i = 0; i < argc; i++) {
		struct gcl_trace t;
		int r = gcl_pcap_load(argv[i], &t, 0);
		uint64_t sum = 0;
		if (r == 0) {
			for (uint64_t k = 0; k < t.n; k++) {
				if (t.offs[k] + t.pkt_len[k] > t.frames_len) {
					printf("%s BAD_BOUNDS %llu\n", argv[i], (unsigned long long)k);
					return 2;
				}
				for (uint32_t b = 0; b < t.pkt_len[k]; b++)
					sum += t.frames[t.offs[k] + b];
			}
		}
		printf("%s %d %llu %llu %llu\n", argv[i], r, (unsigned long long)(r ? 0 : t.n),
		       (unsigned long long)(r ? 0 : t.skipped), (unsigned long long)sum);
		if (r == 0)
			gcl_pcap_free(&t);
	}
	return 0;
}

/* ---------------------------------------------------------------------- */

#define NPROC 8
#define MAXR 12 /* max_runtimes given to the post-pass: ids 8..11 have no client */

struct world {
	struct gcl_host_proc procs[NPROC];
	struct gcl_host_proc *by_id[MAXR];
	struct gcl_host_proc *clients[NPROC];
	struct gcl_lrpc_chan_out chans[NPROC][GCL_NCPU];
	struct gcl_lrpc_msg *tbl[NPROC][GCL_NCPU];
	uint32_t head_wb[NPROC][GCL_NCPU];
	uint64_t owned, freed, polls;
};

static void w_free(struct world *w)
{
	for (int p = 0; p < NPROC; p++)
		for (int t = 0; t < GCL_NCPU; t++)
			free(w->tbl[p][t]);
}

static void w_init(struct world *w)
{
	memset(w, 0, sizeof(*w));
	for (int p = 0; p < NPROC; p++) {
		struct gcl_host_proc *pr = &w->procs[p];
		uint16_t tc = (uint16_t)(1 + rnd() % (p == 7 ? GCL_NCPU : 8));
		uint16_t act = (uint16_t)(rnd() % (tc + 1));
		uint16_t idx[GCL_NCPU];
		pr->uniqid = (uint16_t)p;
		pr->thread_count = tc;
		pr->active_thread_count = act;
		pr->idle_top = (int16_t)((rnd() & 3) ? (int)(rnd() % tc) : -1);
		for (uint16_t i = 0; i < act; i++)
			idx[i] = i;
		if (act)
			gcl_steer_flows(tc, idx, act, pr->flow_tbl);
		for (int t = 0; t < tc; t++) {
			unsigned size = 1u << (rnd() % 4); /* 1..8 slots: rings fill */
			if ((rnd() & 7) == 0)
				continue;                       /* no ring for this thread */
			w->tbl[p][t] = calloc(size, sizeof(struct gcl_lrpc_msg));
			gcl_lrpc_init_out(&w->chans[p][t], w->tbl[p][t], size, &w->head_wb[p][t]);
			pr->rxq[t] = &w->chans[p][t];
		}
		w->clients[p] = pr;
		if (p != 3) /* a registered id whose client is gone */
			w->by_id[p] = pr;
	}
}

static void cb_add_core(void *arg, struct gcl_host_proc *p)
{
	(void)arg;
	if (rnd() & 1) { /* activate everything; flow_tbl by the reference rule */
		uint16_t idx[GCL_NCPU];
		for (uint16_t i = 0; i < p->thread_count; i++)
			idx[i] = i;
		gcl_steer_flows(p->thread_count, idx, p->thread_count, p->flow_tbl);
		p->active_thread_count = p->thread_count;
	}
}
static void cb_poll(void *arg, struct gcl_host_proc *p, unsigned th)
{
	struct world *w = arg;
	if (th >= p->thread_count)
		abort();
	w->polls++;
}
static void cb_free(void *arg, uint64_t i) { ((struct world *)arg)->freed++; (void)i; }
static void cb_owned(void *arg, struct gcl_host_proc *p, uint64_t i)
{
	(void)p;
	(void)i;
	((struct world *)arg)->owned++;
}
static void cb_refcnt(void *arg, uint64_t i, int d) { (void)arg; (void)i; (void)d; }
static bool cb_arp(void *arg, uint64_t i) { (void)arg; return (i & 1) != 0; }

static void drain(struct world *w)
{
	for (int p = 0; p < NPROC; p++)
		for (int t = 0; t < GCL_NCPU; t++)
			if ((rnd() & 1) && w->procs[p].rxq[t])
				w->head_wb[p][t] = w->chans[p][t].send_head; /* the runtime caught up */
}

static int fuzz_deliver(uint64_t iters)
{
	enum { N = 512 };
	static struct gcl_verdict v8[N];
	static struct gcl_verdict4 v4[N];
	static uint16_t v2[N], plen[N];
	static uint8_t olf[N];
	static uint32_t bh[N];
	static uint64_t shm[N];
	uint64_t stats[GCL_NR_STATS] = { 0 };

	for (uint64_t it = 0; it < iters; it++) {
		struct world *w = calloc(1, sizeof(*w));
		struct gcl_host_ops ops = { w, cb_add_core, cb_poll, cb_free, cb_owned, cb_refcnt, cb_arp };
		const struct gcl_host_ops *o = (rnd() & 3) ? &ops : NULL;
		const uint64_t n = rnd() % N;
		const uint8_t tb = (uint8_t)(rnd() % 10); /* 9: refused */
		w_init(w);
		for (uint64_t i = 0; i < n; i++) {
			const uint64_t r = rnd();
			v8[i].hash = (uint32_t)r;
			v8[i].uniqid = (uint16_t)((r >> 32) % 16 == 0 ? r >> 40 : (r >> 40) % MAXR);
			v8[i].thread = (uint8_t)(r >> 56);
			v8[i].action = (uint8_t)((r >> 12) & 0xC7); /* actions 0..7 + flag bits */
			v4[i].uniqid = v8[i].uniqid;
			v4[i].thread = v8[i].thread;
			v4[i].action = v8[i].action;
			v2[i] = (uint16_t)(r >> 20);
			plen[i] = (uint16_t)(r >> 3);
			olf[i] = (uint8_t)(r >> 44);
			bh[i] = (uint32_t)(r >> 17);
			shm[i] = r;
		}
		switch (rnd() % 3) {
		case 0:
			gcl_host_deliver(w->by_id, MAXR, w->clients, NPROC, v8, (rnd() & 1) ? plen : NULL,
			                 (rnd() & 1) ? olf : NULL, 0x09, (rnd() & 1) ? shm : NULL, n, o, stats);
			break;
		case 1:
			gcl_host_deliver4(w->by_id, MAXR, w->clients, NPROC, v4, (rnd() & 1) ? bh : NULL,
			                  (rnd() & 1) ? plen : NULL, (rnd() & 1) ? olf : NULL, 0x09,
			                  (rnd() & 1) ? shm : NULL, n, o, stats);
			break;
		default:
			gcl_host_deliver2(w->by_id, MAXR, w->clients, NPROC, v2, tb, (rnd() & 1) ? bh : NULL,
			                  (rnd() & 1) ? plen : NULL, (rnd() & 1) ? olf : NULL, 0x09,
			                  (rnd() & 1) ? shm : NULL, n, o, stats);
			break;
		}
		drain(w);
		w_free(w);
		free(w);
	}
	printf("deliver ok %llu %llu\n", (unsigned long long)stats[GCL_RX_UNICAST_FAIL],
	       (unsigned long long)stats[GCL_RX_UNHANDLED]);
	return 0;
}

/* ---------------------------------------------------------------------- */

static int fuzz_oracle(uint64_t iters)
{
	for (uint64_t it = 0; it < iters; it++) {
		const uint32_t R = (rnd() & 1) ? 16 : 1024;
		const uint32_t mode = (uint32_t)(rnd() % 3);
		const uint32_t flags = (uint32_t)(rnd() & (GCL_CFG_AZURE_ARP | GCL_CFG_HASH16 | GCL_CFG_TRANS_HASH));
		uint8_t key[40];
		for (int i = 0; i < 40; i++)
			key[i] = (uint8_t)rnd();
		struct orc_tables *t = orc_tables_new(R, mode, flags, (uint8_t)rnd(), key);
		for (uint32_t r = 0; r < R; r += 1 + (uint32_t)(rnd() % 7)) {
			uint16_t tc = (uint16_t)(1 + rnd() % 16), act = (uint16_t)(rnd() % (tc + 1));
			uint16_t idx[GCL_NCPU], fl[GCL_NCPU];
			for (uint16_t i = 0; i < act; i++)
				idx[i] = i;
			if (act)
				orc_steer_flows(tc, idx, act, fl);
			orc_runtime_set(t, (uint16_t)r, (rnd() & 1) ? 0x0A000000u + r + 1 : (uint32_t)rnd(), tc, act,
			                act ? fl : NULL);
		}
		const uint64_t n = 1 + rnd() % 300, flen = 1 + rnd() % 8192;
		uint8_t *frames = malloc(flen);
		uint64_t *offs = malloc(n * 8);
		uint8_t *olf = malloc(n);
		uint32_t *rss = malloc(n * 4), *fdir = malloc(n * 4), *hint = malloc(n * 4);
		struct gcl_verdict *v = malloc(n * sizeof(*v));
		struct gcl_trans *tr = malloc(n * sizeof(*tr));
		uint64_t *counts = calloc(R, 8), stats[GCL_NR_STATS] = { 0 };
		for (uint64_t i = 0; i < flen; i++)
			frames[i] = (uint8_t)rnd();
		for (uint64_t i = 0; i + 14 < flen; i += 64) { /* plausible ethertypes */
			static const uint16_t et[] = { 0x0800, 0x0806, 0x86DD, 0x8100 };
			uint16_t e = et[rnd() % 4];
			frames[i + 12] = (uint8_t)(e >> 8);
			frames[i + 13] = (uint8_t)e;
		}
		for (uint64_t i = 0; i < n; i++) {
			const uint64_t r = rnd();
			offs[i] = (r & 3) == 0 ? flen - (r >> 8) % 80 : (r >> 8) % (flen + 100);
			olf[i] = (uint8_t)(r >> 40);
			rss[i] = (uint32_t)(r >> 3);
			fdir[i] = (uint32_t)((r >> 50) % (R + 8));
			hint[i] = (r >> 61) ? 0 : 0x0A000000u + (uint32_t)((r >> 20) % (R + 4));
		}
		struct gcl_batch b = { 0 };
		b.frames = frames;
		b.frames_len = flen;
		b.offs = offs;
		b.olflags = (rnd() & 1) ? olf : NULL;
		b.rss = (rnd() & 1) ? rss : NULL;
		b.fdir_hi = (rnd() & 1) ? fdir : NULL;
		b.dst_hint = (rnd() & 1) ? hint : NULL;
		b.n = n;
		orc_classify_ex(t, &b, v, counts, stats, tr);
		if (stats[GCL_RX_PULLED] != n) {
			printf("oracle RX_PULLED %llu != %llu\n", (unsigned long long)stats[GCL_RX_PULLED],
			       (unsigned long long)n);
			return 2;
		}
		free(frames);
		free(offs);
		free(olf);
		free(rss);
		free(fdir);
		free(hint);
		free(v);
		free(tr);
		free(counts);
		orc_tables_free(t);
	}
	printf("oracle ok\n");
	return 0;
}

int main(int argc, char **argv)
{
	if (argc < 2)
		return 64;
	if (!strcmp(argv[1], "pcap"))
		return fuzz_pcap(argc - 2, argv + 2);
	if (argc < 4)
		return 64;
	rng_state = strtoull(argv[2], NULL, 0);
	if (!strcmp(argv[1], "deliver"))
		return fuzz_deliver(strtoull(argv[3], NULL, 0));
	if (!strcmp(argv[1], "oracle"))
		return fuzz_oracle(strtoull(argv[3], NULL, 0));
	return 64;
}
