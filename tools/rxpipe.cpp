// rxpipe.cpp - the whole rx_burst replacement on one dataplane core: bursts
// of mbufs from a registered host ingress region go through the persistent
// GPU loop (gcl_rxloop_*), and every verdict through the lrpc post-pass
// (gcl_host_deliver4) into per-kthread rings, as INTEGRATION.md §4b wires it
// into iokernel/rx.c:270-290.  The measured rate is what one host core
// sustains with the GPU classifying, to set beside the reference's own
// classify + lrpc_send rate on one core (bench.py cpu_baseline.lrpc_1core_mpps).
//
//   rxpipe <burst> <workers> <depth> <bursts> [copy|inline|records]   -> one JSON line
//
// Each burst's verdicts are read in place in the loop's ring slot
// (gcl_rxloop_peek + gcl_host_deliver_recs, then gcl_rxloop_release); with
// the fifth argument `copy` they are copied out first (gcl_rxloop_wait +
// gcl_host_deliver4), the round-2 form; with `inline` the submitting core
// copies each frame's 64-B header granule into the slot
// (GCL_LOOP_INLINE_HDRS: the core reads the headers, as rx_one_pkt does, and
// the kernel saves a PCIe round trip); with `records` it writes one stamped
// 64-B header record per packet (GCL_LOOP_HDR_RECORDS), which a worker reads
// with its poll: one PCIe round trip per burst of <= 64.
// Runtime consumers are emulated as infinitely fast and are never touched by
// the dataplane loop: each ring's recv_head_wb points at its own send_head,
// so when a ring looks full the producer's refresh (__lrpc_send,
// base/lrpc.c:16-19) finds it drained -- the reference's own path, taken
// once per 4096 messages per ring, as in the CPU baseline's lrpc variant.
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/rxpipe tools/rxpipe.cpp
//         -Lcaladan_amd -lgclassify -Wl,-rpath,'$ORIGIN/../caladan_amd'
#include <hip/hip_runtime.h>
#include <ctype.h>
#include <errno.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "gcl_host.h"
#include "gclassify.h"
#include "nicsim.h"
#include "pinning.h"
#include "tune_env.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

static uint64_t now_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* The per-burst clock: the TSC (a few ns) rather than clock_gettime (~20
 * ns, five calls a burst were ~1.6 ns per packet of a 64-packet burst),
 * converted with the rate measured over the run. */
static inline uint64_t ticks()
{
	/* rdtscp: after every earlier instruction has executed, so the wait /
	 * deliver split does not move a load still in flight (the last records'
	 * miss) into the deliver side */
	unsigned int aux;
	return __builtin_ia32_rdtscp(&aux);
}

int main(int argc, char **argv)
{
	const uint32_t burst = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
	const uint32_t workers = argc > 2 ? (uint32_t)atoi(argv[2]) : 1;
	const uint32_t depth = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
	const uint32_t nbursts = argc > 4 ? (uint32_t)atoi(argv[4]) : 20000;
	const bool copy_out = argc > 5 && !strcmp(argv[5], "copy");
	const bool inline_hdrs = argc > 5 && !strcmp(argv[5], "inline");
	const bool hdr_records = argc > 5 && !strcmp(argv[5], "records");
	const uint32_t R = 16, T = 8, RING = 4096;
	const uint64_t nframes = 1 << 16, stride = 64;
	if (!burst || burst > 4096 || !workers || workers > 64 || !depth || depth > 64) {
		fprintf(stderr, "bad arguments\n");
		return 1;
	}

	/* RXPIPE_HASH=nic: the flow hash is the mbuf's hash.rss, as rx.c:83 passes
	 * it (GCL_HASH_NIC, rss[] submitted with the offsets); default: JENKINS, the
	 * 5-tuple lookup3 computed on the GPU (no NIC in the loop) */
	const bool nic_hash = getenv("RXPIPE_HASH") && !strcmp(getenv("RXPIPE_HASH"), "nic");
	/* ingress region: udp64 frames generated on the GPU, copied to pinned host memory */
	uint8_t *dfr, *region;
	uint32_t *drss;
	CHECK(hipMalloc(&dfr, nframes * stride));
	CHECK(hipMalloc(&drss, nframes * 4));
	CHECK(hipMemset(dfr, 0, nframes * stride));
	struct gcl_gen_params gp = {};
	gp.workload = GCL_WL_UDP64;
	gp.nruntimes = R;
	gp.seed = 0xCA1ADA4;
	gp.n = nframes;
	gp.stride = stride;
	gp.world = 1;
	if (gcl_generate(&gp, dfr, nullptr, drss, nullptr))
		return 1;
	std::vector<uint32_t> rss(nframes);
	CHECK(hipMemcpy(rss.data(), drss, nframes * 4, hipMemcpyDeviceToHost));
	CHECK(hipFree(drss));
	CHECK(hipHostMalloc((void **)&region, nframes * stride, hipHostMallocMapped));
	CHECK(hipMemcpy(region, dfr, nframes * stride, hipMemcpyDeviceToHost));
	CHECK(hipFree(dfr));

	struct gcl_cfg cfg = {};
	cfg.max_runtimes = R;
	cfg.hash_mode = nic_hash ? GCL_HASH_NIC : GCL_HASH_JENKINS;
	cfg.flags = GCL_CFG_VERDICT4;
	cfg.default_olflags = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	struct gcl_ctx *ctx;
	if (gcl_open(0, &cfg, &ctx) || tune_from_env(ctx))
		return 1;

	/* RXPIPE_POOL=ingress: the bursts come from the emulated NIC
	 * (tools/nicsim.h) -- mbufs of the reference's pool geometry (data at
	 * element + 344 of 9408-B elements), recycled through a mempool, each
	 * frame freshly written with non-temporal stores so that no CPU cache
	 * holds its header, as behind a NIC without DDIO -- instead of a static
	 * 4 MiB region of 64-B slots walked in order (cache-hot headers).
	 * tools/cpupipe runs the CPU baseline on the same emulation. */
	const bool ingress = getenv("RXPIPE_POOL") && !strcmp(getenv("RXPIPE_POOL"), "ingress");
	const uint32_t nic_threads = getenv("RXPIPE_NIC_THREADS") ? (uint32_t)atoi(getenv("RXPIPE_NIC_THREADS")) : 4;
	const uint32_t pool_mbufs = getenv("RXPIPE_POOL_MBUFS") ? (uint32_t)atoi(getenv("RXPIPE_POOL_MBUFS")) : 16384;
	nicsim::NicSim nic;
	if (ingress) {
		if (!nic.init(pool_mbufs, nic_threads, burst, region, rss.data(), (uint32_t)nframes) ||
		    gcl_host_register(nic.region, nic.region_len)) {
			fprintf(stderr, "nicsim init failed\n");
			return 1;
		}
	}

	/* host side of the runtimes: struct proc slices with one lrpc ring per kthread */
	std::vector<gcl_host_proc> procs(R);
	std::vector<gcl_host_proc *> by_id(R), clients(R);
	std::vector<gcl_lrpc_chan_out> chans(R * T);
	std::vector<gcl_lrpc_msg> msgs((size_t)R * T * RING);

	for (uint32_t r = 0; r < R; r++) {
		const uint16_t na = (uint16_t)(r % T + 1);
		uint16_t act[GCL_NCPU];
		for (uint16_t i = 0; i < na; i++)
			act[i] = i;
		gcl_host_proc &p = procs[r];
		memset(&p, 0, sizeof(p));
		p.uniqid = (uint16_t)r;
		p.thread_count = (uint16_t)T;
		p.active_thread_count = na;
		p.idle_top = -1;
		gcl_steer_flows((uint16_t)T, act, na, p.flow_tbl);
		for (uint32_t t = 0; t < T; t++) {
			gcl_lrpc_chan_out *ch = &chans[r * T + t];
			gcl_lrpc_init_out(ch, &msgs[(size_t)(r * T + t) * RING], RING, &ch->send_head);
			p.rxq[t] = &chans[r * T + t];
		}
		by_id[r] = clients[r] = &p;
		gcl_runtime_set(ctx, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, p.flow_tbl);
	}

	struct gcl_rxloop_cfg lc = {};
	lc.slots = 64; /* RXPIPE_SLOTS overrides (a power of two >= 2 * depth) */
	if (const char *e = getenv("RXPIPE_SLOTS"))
		lc.slots = (uint32_t)atoi(e);
	lc.max_burst = burst;
	lc.workers = workers;
	lc.lifetime_ms = 60000;
	lc.region = ingress ? nic.region : region;
	lc.region_len = ingress ? nic.region_len : nframes * stride;
	lc.flags = inline_hdrs ? GCL_LOOP_INLINE_HDRS : hdr_records ? GCL_LOOP_HDR_RECORDS : 0;
	/* RXPIPE_STAMPS=1: the lone-burst breakdown (depth 1): host submit and
	 * submit -> records seen on the TSC, the worker's stage times
	 * (GCL_LOOP_STAMPS) per burst */
	const bool stamps = getenv("RXPIPE_STAMPS") && atoi(getenv("RXPIPE_STAMPS")) && depth == 1;
	if (stamps)
		lc.flags |= GCL_LOOP_STAMPS;
	std::vector<uint64_t> st_sub, st_seen, st_rtt, st_cls, st_store, st_polls, st_b1, st_b2, st_b3;
	uint64_t st_kernel = 0; /* gcl_rxloop_stamps out[7]: 1 = the loop64 kernel */
	struct gcl_rxloop *loop;
	int ret = gcl_rxloop_start(ctx, &lc, &loop);
	if (ret) {
		fprintf(stderr, "gcl_rxloop_start: %d\n", ret);
		return 1;
	}

	/* bursts walk the region in order, like mbufs handed out by a mempool */
	const uint32_t nb = (uint32_t)(nframes / burst);
	std::vector<uint64_t> offs(nframes);
	for (uint64_t i = 0; i < nframes; i++)
		offs[i] = i * stride;
	std::vector<uint16_t> len(burst, 60);
	std::vector<nicsim::Burst> inflight(ingress ? depth : 0); /* the bursts' descriptors until delivered */
	std::vector<gcl_verdict4> v(burst);
	uint64_t stats[GCL_NR_STATS] = {0};
	std::vector<int64_t> tk(depth);
	std::vector<uint64_t> t_sub(depth), lat;
	lat.reserve(nbursts);
	/* the submit / wait / deliver split is sampled on every 8th burst; the
	 * latency (submit -> delivered) is taken on every one */
	uint64_t delivered = 0, t_deliver = 0, t_submit = 0, t_wait = 0, seq = 0, n_sub = 0, n_tail = 0;
	/* RXPIPE_GAP_NS (depth 1): spin this long after a burst's delivery before
	 * the next submit, or "rand": a uniform [0, 2000) ns per burst, so that
	 * the submit lands at any phase of the worker's polls (which start when
	 * it has stored the previous burst's records) as bursts from a NIC do;
	 * "rand:N": uniform [0, N) ns (sparser traffic) */
	/* while a lone burst (depth 1) is awaited, the rings' next slots are taken
	 * for writing (gcl_host_prefetch_rxq); six
	 * interleaved rounds, cache-hot lone burst NIC: p50 medians 3.27 -> 3.09
	 * us, submit + deliver 7.2 -> 6.0 ns/pkt (profiles/r06_ring_prefetch_ab.jsonl).
	 * RXPIPE_RING_PREFETCH=0 leaves it out */
	const bool ring_pf = depth == 1 && !(getenv("RXPIPE_RING_PREFETCH") && !atoi(getenv("RXPIPE_RING_PREFETCH")));
	const char *gap_env = getenv("RXPIPE_GAP_NS");
	const bool gap_rand = gap_env && !strncmp(gap_env, "rand", 4);
	const uint64_t gap_span = gap_rand && gap_env[4] == ':' ? strtoull(gap_env + 5, nullptr, 0) : 2000;
	const uint64_t gap_fixed = gap_env && !gap_rand ? strtoull(gap_env, nullptr, 0) : 0;
	double ticks_per_ns = 1.0;
	{
		const uint64_t n0 = now_ns(), k0 = ticks();
		while (now_ns() - n0 < 20000000ull)
			;
		ticks_per_ns = (double)(ticks() - k0) / (double)(now_ns() - n0);
	}
	uint64_t gap_state = 0x9E3779B97F4A7C15ull;
	auto gap_spin = [&]() {
		if (depth != 1 || (!gap_rand && !gap_fixed))
			return;
		uint64_t g = gap_fixed;
		if (gap_rand) {
			gap_state ^= gap_state << 13;
			gap_state ^= gap_state >> 7;
			gap_state ^= gap_state << 17;
			g = gap_state % (gap_span ? gap_span : 1);
		}
		const uint64_t end = ticks() + (uint64_t)(g * ticks_per_ns);
		while (ticks() < end)
			__builtin_ia32_pause();
	};
	/* @count bursts with up to @depth in flight, in ticket order */
	auto pump = [&](uint32_t count, bool timed) {
		uint32_t head = 0, tail = 0;
		while (tail < count) {
			while (head < count && head - tail < depth) {
				const uint32_t b = (uint32_t)((seq + head) % nb);
				gap_spin();
				const uint64_t *so = &offs[(size_t)b * burst];
				const uint32_t *sr = &rss[(size_t)b * burst];
				if (ingress) { /* rte_eth_rx_burst: the next burst of descriptors */
					nicsim::Burst &nb_ = nic.pull();
					nicsim::Burst &f = inflight[head % depth];
					f.n = nb_.n;
					f.owner = nb_.owner;
					memcpy(f.mbuf, nb_.mbuf, 4 * nb_.n);
					memcpy(f.off, nb_.off, 8 * nb_.n);
					memcpy(f.rss, nb_.rss, 4 * nb_.n);
					nic.consumed(nb_);
					so = f.off;
					sr = f.rss;
				}
				const uint64_t ts = ticks();
				t_sub[head % depth] = ts;
				const int64_t r = gcl_rxloop_submit(loop, burst, so, nullptr, nic_hash ? sr : nullptr, nullptr,
				                                    nullptr);
				if (timed && (head & 7) == 0) {
					t_submit += ticks() - ts;
					n_sub++;
				}
				if (stamps && timed)
					st_sub.push_back(ticks() - ts);
				if (r < 0) {
					fprintf(stderr, "submit: %lld\n", (long long)r);
					exit(1);
				}
				tk[head % depth] = r;
				head++;
			}
			const uint32_t b = (uint32_t)((seq + tail) % nb);
			const uint64_t *doffs = ingress ? inflight[tail % depth].off : &offs[(size_t)b * burst];
			const int64_t t = tk[tail % depth];
			const bool samp = timed && (tail & 7) == 0;
			const uint64_t tw = samp ? ticks() : 0;
			uint64_t d0 = 0, d1;
			if (copy_out) {
				const int w = gcl_rxloop_wait(loop, t, v.data(), 1000000000ull);
				if (w) {
					fprintf(stderr, "wait: %d\n", w);
					exit(1);
				}
				if (samp)
					d0 = ticks();
				delivered += gcl_host_deliver4(by_id.data(), R, clients.data(), (int)R, v.data(),
				                               nullptr, len.data(), nullptr, cfg.default_olflags,
				                               doffs, burst, nullptr, stats);
				d1 = ticks();
			} else {
				const gcl_loop_rec *recs;
				uint32_t n = 0;
				if (ring_pf)
					gcl_host_prefetch_rxq(clients.data(), (int)R);
				const int w = gcl_rxloop_peek(loop, t, 1000000000ull, &recs, &n);
				if (w || n != burst) {
					fprintf(stderr, "peek: %d (n %u)\n", w, n);
					exit(1);
				}
				if (samp)
					d0 = ticks();
				delivered += gcl_host_deliver_recs(by_id.data(), R, clients.data(), (int)R, recs, 4, 0,
				                                   nullptr, len.data(), nullptr, cfg.default_olflags,
				                                   doffs, burst, nullptr, stats);
				d1 = ticks();
				gcl_rxloop_release(loop, t);
			}
			if (ingress) { /* delivered: the mbufs go back to the mempool */
				const nicsim::Burst &f = inflight[tail % depth];
				nic.recycle(f.owner, f.mbuf, f.n);
			}
			if (samp) {
				t_deliver += d1 - d0;
				t_wait += d0 - tw;
				n_tail++;
			}
			if (stamps && timed) {
				/* d0 is the peek's return when sampled; re-take it otherwise */
				uint64_t g[8];
				while (gcl_rxloop_stamps(loop, t, g) == -EAGAIN)
					__builtin_ia32_pause();
				st_seen.push_back(samp ? d0 - t_sub[tail % depth] : 0);
				st_rtt.push_back(g[0]);
				st_cls.push_back(g[1]);
				st_store.push_back(g[2]);
				st_polls.push_back(g[3]);
				st_b1.push_back(g[4]);
				st_b2.push_back(g[5]);
				st_b3.push_back(g[6]);
				st_kernel = g[7];
			}
			if (timed)
				lat.push_back(d1 - t_sub[tail % depth]);
			tail++;
		}
		seq += count;
	};
	/* pinned after the runtime's own threads exist (they keep their masks) */
	const int cpu = pin_near_gpu(0);
	if (ingress)
		nic.launch(pick_other_cpus(nic_threads, cpu));
	const uint32_t warm = 200;
	pump(warm, false);
	const uint64_t nic_w0 = nic.wait_ns;
	const uint64_t t0 = now_ns(), k0 = ticks();
	pump(nbursts, true);
	const uint64_t el = now_ns() - t0;
	const uint64_t nic_waited = nic.wait_ns - nic_w0;
	const double ns_tick = (double)el / (double)(ticks() - k0);
	uint64_t ps[3] = {0, 0, 0};
	gcl_rxloop_poll_stats(loop, ps);
	gcl_rxloop_stop(loop);
	const double huge_frac = ingress && nic.region_len ? (double)nic.huge_bytes() / nic.region_len : 0.0;
	if (ingress) {
		gcl_host_unregister(nic.region);
		nic.shutdown();
	}
	std::sort(lat.begin(), lat.end());
	const double pkts = (double)burst * nbursts;
	const double sub_pkts = (double)burst * (n_sub ? n_sub : 1), tail_pkts = (double)burst * (n_tail ? n_tail : 1);
	printf("{\"burst\": %u, \"workers\": %u, \"depth\": %u, \"bursts\": %u, \"hash\": \"%s\", "
	       "\"gap_ns\": \"%s\", \"verdicts\": \"%s\", "
	       "\"mpps_one_core\": %.2f, "
	       "\"burst_latency_p50_us\": %.2f, \"burst_latency_p99_us\": %.2f, "
	       "\"deliver_ns_per_pkt\": %.2f, \"submit_ns_per_pkt\": %.2f, \"wait_ns_per_pkt\": %.2f, "
	       "\"delivered_check\": \"%s\", \"unicast_fail\": %llu, \"host_cpu\": %d, "
	       "\"bursts_early\": %llu, \"bursts_stale\": %llu, \"bursts_late\": %llu, \"pool\": \"%s\", "
	       "\"nic_wait_frac\": %.4f, \"pool_huge_frac\": %.3f}\n",
	       burst, workers, depth, nbursts, nic_hash ? "nic (hash.rss, rx.c:83)" : "jenkins",
	       gap_rand ? (gap_span == 2000 ? "rand [0, 2000)" : gap_env) : gap_env ? gap_env : "0",
	       copy_out ? "copied out" : inline_hdrs ? "read in place, headers inlined in the slot"
	       : hdr_records ? "read in place, stamped header records in the slot" : "read in place",
	       pkts / (el * 1e-3), lat[lat.size() / 2] * ns_tick * 1e-3,
	       lat[lat.size() * 99 / 100] * ns_tick * 1e-3, t_deliver * ns_tick / tail_pkts,
	       t_submit * ns_tick / sub_pkts, t_wait * ns_tick / tail_pkts,
	       delivered == (uint64_t)burst * (nbursts + warm) ? "ok" : "MISMATCH",
	       (unsigned long long)stats[GCL_RX_UNICAST_FAIL], cpu, (unsigned long long)ps[0],
	       (unsigned long long)ps[1], (unsigned long long)ps[2],
	       ingress ? "ingress: mbuf pool at element + 344 of 9408-B elements, frames written by NIC threads "
	                 "with non-temporal stores (cold headers)"
	               : "static 64-B slots walked in order (cache-hot headers)",
	       (double)nic_waited / el, huge_frac);
	if (stamps) {
		/* medians; the submit -> seen split only on the sampled bursts */
		auto med = [](std::vector<uint64_t> v, bool drop0) {
			if (drop0)
				v.erase(std::remove(v.begin(), v.end(), 0ull), v.end());
			if (v.empty())
				return 0.0;
			std::sort(v.begin(), v.end());
			return (double)v[v.size() / 2];
		};
		const double sub = med(st_sub, false) * ns_tick, seen = med(st_seen, true) * ns_tick;
		const double rtt = med(st_rtt, false), cls = med(st_cls, false), sto = med(st_store, false);
		static const char *const b64[] = {"gpu_hit_to_data_in_registers", "gpu_hit_to_posted_to_writer",
		                                  "gpu_hit_to_writer_start"};
		static const char *const bar[] = {"gpu_hit_to_barrier1", "gpu_hit_to_barrier2", "gpu_hit_to_barrier3"};
		const char *const *b = st_kernel ? b64 : bar;
		printf("{\"lone_burst_stages_ns\": {\"host_submit\": %.0f, \"submit_to_records_seen\": %.0f, "
		       "\"gpu_hit_poll_round_trip\": %.0f, \"gpu_hit_to_classified\": %.0f, "
		       "\"gpu_hit_to_last_record_issued\": %.0f, \"polls_per_wait\": %.0f, "
		       "\"residual_word_to_hit_plus_writeback\": %.0f, \"%s\": %.0f, "
		       "\"%s\": %.0f, \"%s\": %.0f}, \"burst\": %u, \"flags\": \"%s\", \"kernel\": \"%s\"}\n",
		       sub, seen, rtt, cls, sto, med(st_polls, false), seen - sub - sto, b[0], med(st_b1, false),
		       b[1], med(st_b2, false), b[2], med(st_b3, false), burst,
		       hdr_records ? "records" : inline_hdrs ? "inline" : "offsets",
		       st_kernel ? "rxloop64" : "rxloop");
	}
	gcl_close(ctx);
	CHECK(hipHostFree(region));
	return 0;
}
