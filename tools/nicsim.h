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
#include <sys/mman.h>
#include <stdint.h>
#include <stdio.h>
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
	/* @n elements at once, one index update (the caller checked size() / room) */
	void push_n(const T *v, uint32_t n)
	{
		const uint32_t h = head.load(std::memory_order_relaxed);
		for (uint32_t i = 0; i < n; i++)
			buf[(h + i) & mask] = v[i];
		head.store(h + n, std::memory_order_release);
	}
	void pop_n(T *v, uint32_t n)
	{
		const uint32_t t = tail.load(std::memory_order_relaxed);
		for (uint32_t i = 0; i < n; i++)
			v[i] = buf[(t + i) & mask];
		tail.store(t + n, std::memory_order_release);
	}
};

/* Frame data sits kDataOff % 64 = 24 B into a cache line (elements are
 * 64-B multiples in 2 MiB pages), so a 64-B frame spans two lines.  DMA
 * leaves it in DRAM and in no CPU cache: both lines are written WHOLE with
 * non-temporal 16-B stores from a pre-built 128-B image (the frame's bytes,
 * zeros around them: the headroom before element + 344 and the rest of the
 * second line), since a partly written write-combining line drains as a slow
 * partial write (8-B stores at element + 344 ran ~130 ns per frame) */
constexpr uint64_t kLineHead = kDataOff % 64;
static_assert(kEltSize % 64 == 0 && kPage % 64 == 0, "frame data at a fixed offset in its line");

inline void nt_write_lines(uint8_t *line0, const uint8_t *img128)
{
	for (int i = 0; i < 8; i++)
		_mm_stream_si128((__m128i *)(line0 + 16 * i), _mm_loadu_si128((const __m128i *)(img128 + 16 * i)));
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
	bool huge = false;         /* madvise(MADV_HUGEPAGE) took */
	uint32_t nmbufs = 0, nthreads = 0, burst = 0;
	const uint32_t *tmpl_rss = nullptr;
	uint32_t ntmpl = 0;
	std::vector<uint8_t> img;          /* the template frames as 128-B line images */
	std::vector<uint64_t> offs;        /* mbuf data offsets (mbuf_off) */
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
		tmpl_rss = tmpl_rss_;
		ntmpl = ntmpl_;
		const uint32_t ring = rx_bursts_per_thread();
		if (!nthreads || !burst || burst > kMaxBurst || nmbufs < nthreads * burst * (ring + 4))
			return false;
		img.assign((size_t)ntmpl * 128 + 64, 0);
		for (uint32_t f = 0; f < ntmpl; f++)
			memcpy(&img[(size_t)f * 128 + kLineHead], tmpl_ + (size_t)f * 64, 64);
		offs.resize(nmbufs);
		for (uint32_t i = 0; i < nmbufs; i++)
			offs[i] = mbuf_off(i);
		region_len = region_bytes(nmbufs);
		region = (uint8_t *)aligned_alloc(kPage, region_len);
		if (!region)
			return false;
		/* the pool sits in 2 MiB pages, as the reference's (mempool memory
		 * from PGSIZE_2MB mappings, defs.h:503-506): one TLB entry per
		 * 222 mbufs for the dataplane core and the GPU alike */
		huge = madvise(region, region_len, MADV_HUGEPAGE) == 0;
		memset(region, 0, region_len);
		lanes = std::vector<Lane>(nthreads);
		for (uint32_t k = 0; k < nthreads; k++) {
			Lane &L = lanes[k];
			L.rx.init(ring);
			L.free.init(nmbufs / nthreads + 1);
			for (uint32_t i = k; i < nmbufs; i += nthreads) { /* this thread's share of the pool */
				L.free.slot_at_head() = i;
				L.free.push_commit();
			}
			L.seq = k;
		}
		return true;
	}

	/* bytes of the pool region backed by transparent huge pages (smaps) */
	uint64_t huge_bytes() const
	{
		FILE *f = fopen("/proc/self/smaps", "r");
		if (!f)
			return 0;
		char line[512];
		bool in = false;
		uint64_t kb = 0;
		const uintptr_t a = (uintptr_t)region, e = a + region_len;
		while (fgets(line, sizeof(line), f)) {
			unsigned long lo, hi;
			if (sscanf(line, "%lx-%lx ", &lo, &hi) == 2 && strchr(line, '-') < strchr(line, ' '))
				in = lo < e && hi > a;
			else if (in && !strncmp(line, "AnonHugePages:", 14))
				kb += strtoull(line + 14, nullptr, 10);
		}
		fclose(f);
		return kb << 10;
	}

	uint32_t rx_bursts_per_thread() const
	{
		return kRxRingBursts / nthreads >= 4 ? kRxRingBursts / nthreads : 4;
	}

	cpu_set_t any_cpus;
	bool any_cpus_set = false;

	/* the NIC threads, thread i pinned to @cpus[i]; threads past the list run
	 * on any of @cpus (none: unpinned) */
	void launch(const std::vector<int> &cpus)
	{
		CPU_ZERO(&any_cpus);
		for (int c : cpus)
			if (c >= 0) {
				CPU_SET(c, &any_cpus);
				any_cpus_set = true;
			}
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
		} else if (any_cpus_set) { /* not the dataplane's core (the mask it inherited) */
			(void)sched_setaffinity(0, sizeof(any_cpus), &any_cpus);
		}
		while (!stop.load(std::memory_order_relaxed)) {
			if (L.rx.full() || L.free.size() < burst) {
				_mm_pause();
				continue;
			}
			Burst &b = L.rx.slot_at_head();
			b.n = burst;
			b.owner = k;
			L.free.pop_n(b.mbuf, burst);
			for (uint32_t i = 0; i < burst; i++) {
				const uint64_t f = L.seq % ntmpl;
				L.seq += nthreads;
				b.off[i] = offs[b.mbuf[i]];
				b.rss[i] = tmpl_rss ? tmpl_rss[f] : 0;
				nt_write_lines(region + b.off[i] - kLineHead, &img[f * 128]);
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
		lanes[owner].free.push_n(mbuf, n);
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
