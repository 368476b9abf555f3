/*
 * nicsim.h - tools only: the NIC side of an rx_burst pipeline, for the host
 * pipeline tools (tools/rxpipe: the GPU loop; tools/cpupipe: the CPU
 * baseline), so that both see identical frames in the same cache state.
 *
 * The ingress pool has the reference's geometry: 9408-B elements packed in
 * 2 MiB pages, frame data at element + 344 (iokernel/defs.h:503-523; the
 * mbuf header and headroom before it).  NIC threads play the hardware: each
 * takes free mbufs from its own share of the pool, writes the next frame of
 * a template stream into each with NON-TEMPORAL stores -- a NIC's DMA write,
 * which on EPYC (no DDIO) leaves no copy of the line in any CPU cache, so
 * the dataplane core's first read of a header misses to DRAM as rx_one_pkt's
 * does (rx.c:281-285 prefetches two frames ahead for exactly that) -- and
 * publishes a burst of descriptors {mbuf, data offset, hash.rss} into its rx
 * ring (SPSC).  The dataplane thread pulls bursts round-robin from the NIC
 * threads' rings, like rte_eth_rx_burst (rx.c:277), and recycles each
 * burst's mbufs to their owner once it has delivered them, as the mempool
 * does when the runtime frees them (dpdk.c:50-54, :127-131).
 *
 * NicSim::wait_ns counts the time the dataplane found no burst ready: a
 * pipeline rate with a large share of it measures the emulated NIC, not the
 * dataplane.
 */
#pragma once

#include <immintrin.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <atomic>
#include <thread>
#include <vector>

namespace nicsim {

constexpr uint64_t kPage = 2ull << 20;     /* PGSIZE_2MB */
constexpr uint64_t kEltSize = 9408;        /* RX_ELT_SIZE, iokernel/defs.h:504 */
constexpr uint64_t kEltPerPage = kPage / kEltSize;
constexpr uint64_t kDataOff = 64 + 128 + 24 + 128; /* mbuf data from element start */
constexpr uint32_t kMaxBurst = 64;         /* IOKERNEL_RX_BURST_SIZE */
constexpr uint32_t kRxRingBursts = 32;     /* 2048 descriptors (MLX5_RX_RING_SIZE, dpdk.c:53)
                                              as 32 bursts of 64, split over the NIC threads */

/* data offset of mbuf @i from the region base */
inline uint64_t mbuf_off(uint64_t i)
{
	return (i / kEltPerPage) * kPage + (i % kEltPerPage) * kEltSize + kDataOff;
}

inline uint64_t region_bytes(uint64_t nmbufs)
{
	return (nmbufs + kEltPerPage - 1) / kEltPerPage * kPage;
}

struct Burst {
	uint32_t n;
	uint32_t owner;               /* NIC thread whose share the mbufs belong to */
	uint32_t mbuf[kMaxBurst];
	uint64_t off[kMaxBurst];      /* frame data offset (mbuf data pointer - region base) */
	uint32_t rss[kMaxBurst];      /* hash.rss the NIC reported */
};

/* single-producer single-consumer ring of T, power-of-two capacity */
template <typename T>
struct Spsc {
	std::vector<T> buf;
	uint32_t mask = 0;
	alignas(64) std::atomic<uint32_t> head{0}; /* producer */
	alignas(64) std::atomic<uint32_t> tail{0}; /* consumer */
	void init(uint32_t cap)
	{
		uint32_t c = 1;
		while (c < cap)
			c <<= 1;
		buf.assign(c, T());
		mask = c - 1;
	}
	uint32_t size() const { return head.load(std::memory_order_acquire) - tail.load(std::memory_order_acquire); }
	bool full() const { return head.load(std::memory_order_relaxed) - tail.load(std::memory_order_acquire) > mask; }
	T &slot_at_head() { return buf[head.load(std::memory_order_relaxed) & mask]; }
	void push_commit() { head.store(head.load(std::memory_order_relaxed) + 1, std::memory_order_release); }
	bool empty() const { return head.load(std::memory_order_acquire) == tail.load(std::memory_order_relaxed); }
	T &front() { return buf[tail.load(std::memory_order_relaxed) & mask]; }
	void pop_commit() { tail.store(tail.load(std::memory_order_relaxed) + 1, std::memory_order_release); }
};

/* a 64-B frame written with non-temporal 8-B stores (frame data is 8-B
 * aligned at element + 344), as DMA leaves it: in DRAM, in no CPU cache */
inline void nt_write64(uint8_t *dst, const uint8_t *src)
{
	for (int i = 0; i < 8; i++) {
		long long v;
		memcpy(&v, src + 8 * i, 8);
		_mm_stream_si64((long long *)(dst + 8 * i), v);
	}
}

inline uint64_t mono_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

struct NicSim {
	uint8_t *region = nullptr;
	uint64_t region_len = 0;
	uint32_t nmbufs = 0, nthreads = 0, burst = 0;
	const uint8_t *tmpl = nullptr;     /* ntmpl frames of 64 B */
	const uint32_t *tmpl_rss = nullptr;
	uint32_t ntmpl = 0;
	struct Lane {
		Spsc<Burst> rx;
		Spsc<uint32_t> free;
		std::thread th;
		uint64_t seq = 0;
		int cpu = -1;
	};
	std::vector<Lane> lanes;
	std::atomic<bool> stop{false};
	uint64_t next = 0;         /* dataplane: next burst's lane (round-robin) */
	uint64_t wait_ns = 0;      /* dataplane: time spent on empty rx rings */

	/* the pool, its region and the rings (launch() starts the NIC threads) */
	bool init(uint32_t nmbufs_, uint32_t nthreads_, uint32_t burst_, const uint8_t *tmpl_,
	          const uint32_t *tmpl_rss_, uint32_t ntmpl_)
	{
		nmbufs = nmbufs_;
		nthreads = nthreads_;
		burst = burst_;
		tmpl = tmpl_;
		tmpl_rss = tmpl_rss_;
		ntmpl = ntmpl_;
		if (!nthreads || !burst || burst > kMaxBurst || nmbufs < nthreads * burst * (kRxRingBursts + 4))
			return false;
		region_len = region_bytes(nmbufs);
		region = (uint8_t *)aligned_alloc(kPage, region_len);
		if (!region)
			return false;
		memset(region, 0, region_len);
		lanes = std::vector<Lane>(nthreads);
		for (uint32_t k = 0; k < nthreads; k++) {
			Lane &L = lanes[k];
			L.rx.init(kRxRingBursts / nthreads ? kRxRingBursts / nthreads : 1);
			L.free.init(nmbufs / nthreads + 1);
			for (uint32_t i = k; i < nmbufs; i += nthreads) { /* this thread's share of the pool */
				L.free.slot_at_head() = i;
				L.free.push_commit();
			}
			L.seq = k;
		}
		return true;
	}

	/* the NIC threads, thread i pinned to @cpus[i] (absent or -1: not pinned) */
	void launch(const std::vector<int> &cpus)
	{
		for (uint32_t k = 0; k < nthreads; k++) {
			lanes[k].cpu = k < cpus.size() ? cpus[k] : -1;
			lanes[k].th = std::thread([this, k]() { run(k); });
		}
	}

	bool start(uint32_t nmbufs_, uint32_t nthreads_, uint32_t burst_, const uint8_t *tmpl_,
	           const uint32_t *tmpl_rss_, uint32_t ntmpl_, const std::vector<int> &cpus)
	{
		if (!init(nmbufs_, nthreads_, burst_, tmpl_, tmpl_rss_, ntmpl_))
			return false;
		launch(cpus);
		return true;
	}

	void run(uint32_t k)
	{
		Lane &L = lanes[k];
		if (L.cpu >= 0) {
			cpu_set_t one;
			CPU_ZERO(&one);
			CPU_SET(L.cpu, &one);
			(void)sched_setaffinity(0, sizeof(one), &one);
		}
		while (!stop.load(std::memory_order_relaxed)) {
			if (L.rx.full() || L.free.size() < burst) {
				_mm_pause();
				continue;
			}
			Burst &b = L.rx.slot_at_head();
			b.n = burst;
			b.owner = k;
			for (uint32_t i = 0; i < burst; i++) {
				const uint32_t id = L.free.front();
				L.free.pop_commit();
				const uint64_t f = L.seq % ntmpl;
				L.seq += nthreads;
				b.mbuf[i] = id;
				b.off[i] = mbuf_off(id);
				b.rss[i] = tmpl_rss ? tmpl_rss[f] : 0;
				nt_write64(region + b.off[i], tmpl + 64 * f);
			}
			_mm_sfence(); /* the frames are in memory before the descriptors say so */
			L.rx.push_commit();
		}
	}

	/* the next burst (round-robin over the NIC threads' rings), spinning
	 * until it is ready */
	Burst &pull()
	{
		Lane &L = lanes[next % nthreads];
		if (L.rx.empty()) {
			const uint64_t t0 = mono_ns();
			while (L.rx.empty())
				_mm_pause();
			wait_ns += mono_ns() - t0;
		}
		next++;
		return L.rx.front();
	}

	/* the pulled burst @b is off the rx ring (its descriptors copied or done
	 * with): the ring slot goes back to the NIC */
	void consumed(Burst &b) { lanes[b.owner].rx.pop_commit(); }

	/* mbufs delivered: back to their NIC thread's free list (the mempool) */
	void recycle(uint32_t owner, const uint32_t *mbuf, uint32_t n)
	{
		Spsc<uint32_t> &F = lanes[owner].free;
		for (uint32_t i = 0; i < n; i++) {
			F.slot_at_head() = mbuf[i];
			F.push_commit();
		}
	}

	void shutdown()
	{
		stop.store(true);
		for (Lane &L : lanes)
			if (L.th.joinable())
				L.th.join();
		free(region);
		region = nullptr;
	}
};

} // namespace nicsim
