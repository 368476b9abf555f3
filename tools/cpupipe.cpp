// cpupipe.cpp - the CPU baseline of the rx_burst pipeline on the same inputs
// as tools/rxpipe's ingress mode: the reference's own per-packet work on ONE
// dataplane core -- rx_burst's bursts of 64 through rx_one_pkt with rx.c's
// direct header loads and prefetch stride 2, plus rx_make_cmd + lrpc_send of
// every delivered packet (iokernel/rx.c:76-92, :116-233, :270-290; the
// oracle's restatement, oracle/orc.c) -- over frames the emulated NIC
// (tools/nicsim.h) has just written into the reference's mbuf pool geometry
// with non-temporal stores, so every header read misses to DRAM as it does
// behind a real NIC on a host without DDIO.  The CPU baseline leg of
// bench.py's pipeline rows; test infrastructure, not the product.
//
//   cpupipe <bursts> [classify|lrpc] [prefetch]   -> one JSON line
//
// `prefetch`: before each burst, prefetch every frame's header (the records
// submit's own trick, gcl_tune.rec_prefetch) on top of rx.c's stride 2 -- not
// the reference's code, the CPU path given the same help as the GPU's host side.
//
// RXPIPE_HASH=nic: NIC mode (hash.rss from the descriptor, rx.c:83); default
// JENKINS.  RXPIPE_NIC_THREADS (4), RXPIPE_POOL_MBUFS (16384) as in rxpipe.
// Build: hipcc --offload-arch=gfx950 -O3 -march=native -Iinclude -o tools/cpupipe
//        tools/cpupipe.cpp oracle/orc.c (bench.py builds it on the box, like
//        the native oracle of cpu_baseline)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../oracle/orc.h"
#include "nicsim.h"
#include "pinning.h"

int main(int argc, char **argv)
{
	const uint32_t nbursts = argc > 1 ? (uint32_t)atoi(argv[1]) : 200000;
	const bool send = !(argc > 2 && !strcmp(argv[2], "classify"));
	const bool deep = argc > 3 && !strcmp(argv[3], "prefetch");
	const uint32_t burst = 64, R = 16, T = 8;
	const bool nic_hash = getenv("RXPIPE_HASH") && !strcmp(getenv("RXPIPE_HASH"), "nic");
	const uint32_t nthreads = getenv("RXPIPE_NIC_THREADS") ? (uint32_t)atoi(getenv("RXPIPE_NIC_THREADS")) : 4;
	const uint32_t nmbufs = getenv("RXPIPE_POOL_MBUFS") ? (uint32_t)atoi(getenv("RXPIPE_POOL_MBUFS")) : 16384;

	/* the template stream: the udp64 frames rxpipe generates on the GPU, the
	 * same bytes (orc_generate = gcl_generate), with the NIC's hash.rss */
	const uint32_t ntmpl = 1 << 16;
	std::vector<uint8_t> tmpl((size_t)ntmpl * 64, 0);
	std::vector<uint32_t> trss(ntmpl);
	struct gcl_gen_params gp = {};
	gp.workload = GCL_WL_UDP64;
	gp.nruntimes = R;
	gp.seed = 0xCA1ADA4;
	gp.n = ntmpl;
	gp.stride = 64;
	gp.world = 1;
	if (orc_generate(&gp, nullptr, tmpl.data(), nullptr, trss.data()))
		return 1;

	struct orc_tables *t = orc_tables_new(R, nic_hash ? GCL_HASH_NIC : GCL_HASH_JENKINS, 0,
	                                      GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD, nullptr);
	for (uint32_t r = 0; r < R; r++) { /* rxpipe's runtimes: r % T + 1 active kthreads */
		const uint16_t na = (uint16_t)(r % T + 1);
		uint16_t act[GCL_NCPU], flow[GCL_NCPU];
		for (uint16_t i = 0; i < na; i++)
			act[i] = i;
		orc_steer_flows((uint16_t)T, act, na, flow);
		orc_runtime_set(t, (uint16_t)r, orc_runtime_ip(r), (uint16_t)T, na, flow);
	}
	struct orc_dataplane *d = orc_dataplane_new(t);

	const int cpu = pin_near_gpu(0);
	nicsim::NicSim nic;
	if (!nic.start(nmbufs, nthreads, burst, tmpl.data(), trss.data(), ntmpl, pick_other_cpus(nthreads, cpu))) {
		fprintf(stderr, "nicsim start failed\n");
		return 1;
	}
	std::vector<gcl_verdict> v(burst);
	uint64_t counts[16] = {0}, stats[GCL_NR_STATS] = {0};
	nicsim::Burst cur;
	auto one = [&]() {
		nicsim::Burst &b = nic.pull();
		cur.n = b.n;
		cur.owner = b.owner;
		memcpy(cur.mbuf, b.mbuf, 4 * b.n);
		memcpy(cur.off, b.off, 8 * b.n);
		memcpy(cur.rss, b.rss, 4 * b.n);
		nic.consumed(b);
		struct gcl_batch gb = {};
		gb.frames = nic.region;
		gb.frames_len = nic.region_len;
		gb.offs = cur.off;
		gb.rss = nic_hash ? cur.rss : nullptr;
		gb.n = cur.n;
		if (deep)
			for (uint32_t i = 0; i < cur.n; i++)
				__builtin_prefetch(nic.region + cur.off[i] + 12, 0, 3);
		orc_dataplane_burst(d, &gb, v.data(), counts, stats, send);
		nic.recycle(cur.owner, cur.mbuf, cur.n);
	};
	for (uint32_t i = 0; i < 2000; i++)
		one();
	const uint64_t w0 = nic.wait_ns;
	memset(counts, 0, sizeof(counts));
	memset(stats, 0, sizeof(stats));
	const uint64_t t0 = nicsim::mono_ns();
	for (uint32_t i = 0; i < nbursts; i++)
		one();
	const uint64_t el = nicsim::mono_ns() - t0;
	const uint64_t waited = nic.wait_ns - w0;
	const double huge_frac = (double)nic.huge_bytes() / nic.region_len;
	nic.shutdown();
	uint64_t delivered = 0;
	for (uint32_t r = 0; r < R; r++)
		delivered += counts[r];
	const double pkts = (double)burst * nbursts;
	printf("{\"pipeline\": \"cpu\", \"burst\": %u, \"bursts\": %u, \"hash\": \"%s\", \"post\": \"%s\", "
	       "\"prefetch\": \"%s\", \"pool\": \"ingress: %u mbufs, data at element + 344 of 9408-B elements, frames written by %u NIC "
	       "threads with non-temporal stores\", "
	       "\"mpps_one_core\": %.2f, \"ns_per_pkt\": %.2f, \"nic_wait_frac\": %.4f, "
	       "\"delivered_check\": \"%s\", \"unicast_fail\": %llu, \"host_cpu\": %d, \"pool_huge_frac\": %.3f}\n",
	       burst, nbursts, nic_hash ? "nic (hash.rss, rx.c:83)" : "jenkins",
	       send ? "classify + rx_make_cmd + lrpc_send" : "classify only",
	       deep ? "the burst's 64 headers, then rx.c's stride 2" : "rx.c's stride 2", nmbufs, nthreads,
	       pkts / (el * 1e-3), el / pkts, (double)waited / el,
	       delivered == (uint64_t)pkts && stats[GCL_RX_PULLED] == (uint64_t)pkts ? "ok" : "MISMATCH",
	       (unsigned long long)stats[GCL_RX_UNICAST_FAIL], cpu, huge_frac);
	orc_dataplane_free(d);
	orc_tables_free(t);
	return 0;
}
