/*
 * gcl_loop.hip - the persistent rx loop (gcl_rxloop_*): rx_burst at its own
 * granularity, <= 64 mbufs a burst (iokernel/rx.c:270-290, defs.h:75), with
 * microsecond latency.  A persistent kernel polls a ring of burst slots in
 * coherent host memory and classifies each burst straight out of the
 * registered ingress region (rxloop64_kernel for bursts <= 64, rxloop_kernel
 * for longer ones); the host side publishes bursts and collects the verdict
 * records.
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/gclassify.h"
#include "gcl_ctx.h"

namespace gclk {

/* ------------------------------------------------------------------------
 * Persistent rx loop (gcl_rxloop_*): a burst-at-a-time classifier for the
 * reference's own granularity, rx_burst's <= 64 mbufs (iokernel/rx.c:270-290).
 * Each of `workers` 256-lane blocks owns tickets w+1, w+1+W, ...: it polls
 * the ticket's ring slot in host memory, classifies the burst straight out of
 * the registered ingress region, writes the verdicts back into the slot and
 * publishes the ticket.  Everything the CPU writes is read with system-scope
 * loads, so recycled mbufs and reused slots are never served from a stale
 * cache line.  Every block leaves on the stop flag or at its own deadline
 * (s_memrealtime, 100 MHz), so the grid always drains.
 */
struct LoopSlotHdr {       /* first 64 B of a ring slot */
	uint64_t word;          /* host: the published burst, one load for the poller:
	                           ticket[63:24] n[23:11] flags[10:7] img[6] img_seq%64[5:0] */
	uint32_t pad[14];
};

/* One verdict record per packet of a burst, written by the kernel with ONE
 * 16-B system-scope store: the verdict in the gcl_verdict layout plus the
 * ticket.  The record is its own completion flag: the host polls the
 * tickets, so the kernel neither waits for its stores nor raises a flag. */
struct LoopRec {
	uint32_t hash, vlo;
	uint64_t ticket;
};
static_assert(sizeof(LoopRec) == 16 && sizeof(LoopRec) == sizeof(gcl_loop_rec), "LoopRec");
__host__ __device__ constexpr uint64_t loop_word(uint64_t t, uint32_t n, uint32_t fl, uint32_t img,
                                                 uint32_t iseq)
{
	return (t & ((1ull << 40) - 1)) << 24 | (uint64_t)(n & 0x1FFF) << 11 | (fl & 0xF) << 7 |
	       (img & 1) << 6 | (iseq & 63);
}
static_assert(sizeof(LoopSlotHdr) == 64, "LoopSlotHdr");

/* Offsets in a ring slot carry a stamp of the slot's use count in their top 24 bits
 * (offsets themselves are < 2^40: the ingress region is bounded at start).
 * An 8-B entry is written and read whole, so a lane that reads its entry
 * while polling knows by the stamp whether it holds this burst's offset or a
 * stale one: the offsets arrive with the poll that sees the burst, one PCIe
 * round trip sooner.  Entries past a burst's n keep older stamps; every
 * kLoopRefresh uses of a slot the host rewrites all of them, so no entry is
 * ever 2^23 uses stale (the stamp's period) and a stamp never aliases. */
constexpr int kLoopStampShift = 40;
constexpr uint64_t kLoopOffMask = (1ull << kLoopStampShift) - 1;
constexpr uint64_t kLoopRefresh = 256;
/* s_memrealtime ticks (100 MHz) a wait polls the offsets or header records
 * with the word: a burst that arrives later costs their round trip after the
 * word.  Loops of 1 or 2 workers keep polling them for kLoopSpecIdle (1 ms):
 * sparse lone bursts (random gaps of [0, 20) us) 4.50-4.73 -> 3.76-3.81 us
 * p50 for ~3 GB/s of idle PCIe reads per worker; with more workers that
 * traffic costs the pipeline more than the late bursts do (8 x 16 records
 * 139-142 -> 122-132 Mpkt/s), so they keep 4 us
 * (profiles/r05_spec_ab.jsonl) */
constexpr uint64_t kLoopSpecTicks = 400;
constexpr uint64_t kLoopSpecIdle = 100000;
constexpr uint32_t kLoopSpecIdleWorkers = 2;
/* gcl_tune.loop_lean default: bursts whose every packet is plain IPv4 (IHL 5,
 * no FDIR mark, no hint) classified by classify_lean */
constexpr uint32_t kDefaultLoopLean = 1;
/* gcl_tune.loop_phase_* default (max, up, down in ticks; loops of up to
 * kLoopSpecIdleWorkers workers): the poll-phase delay's ceiling and steps.
 * 1 x 1 header records, NIC hash, three fresh processes per form
 * (profiles/r05_phase_ab.jsonl, r05_phase_sweep.jsonl): back to back
 * 3.94-3.98 -> 3.11-3.19 us p50, random phase 3.61-3.90 -> 3.49-3.57, sparse
 * lone bursts unchanged (3.64-4.02 / 3.76-3.79), 2 workers x 2 in flight
 * 3.99-4.01 -> 3.14-3.45; a 200-tick ceiling let the delay outgrow the host's
 * turnaround at a random phase (3.86-4.05) */
constexpr uint32_t kDefaultLoopPhaseMax = 120, kDefaultLoopPhaseUp = 16, kDefaultLoopPhaseDown = 1;
/* gcl_tune.loop_prefetch default (loops of more than kLoopSpecIdleWorkers
 * workers over stamped offsets, whose bursts take a second round trip for
 * the headers that the next poll overlaps): 4 x 8 offsets 58.2-59.8 ->
 * 72.1-76.3 Mpkt/s in fresh processes (profiles/r05_prefetch_ab.jsonl,
 * r05_prefetch_gated_ab.jsonl); with header records only the ~0.6-us
 * classification is left to overlap and the gated form measured no gain
 * (4 x 8 JENKINS 90.8-93.7 -> 82.2-95.1) */
constexpr uint32_t kDefaultLoopPrefetch = 1;
/* how a worker's bursts arrived (gcl_rxloop_poll_stats): with the poll that
 * found the word; eligible for that, but an entry or record still stale so
 * read after it; or after the word, the speculative window over or the
 * burst too long for it */
enum { kLoopPollEarly = 0, kLoopPollStale = 1, kLoopPollLate = 2 };
/* never 0 (bit 23 of the stamp is always set, the slot's use count in bits
 * 0-22), so an entry that was never loaded, or never written since the loop
 * started, cannot pass for a current one; host and device compute it the same
 * way.  Shifts and masks only (nslots is a power of two): the poller computes
 * it per ticket. */
__host__ __device__ constexpr uint64_t loop_stamp(uint64_t t, uint32_t nslots)
{
	return ((((t - 1) >> __builtin_ctz(nslots)) & 0x7FFFFFull) | 0x800000ull) << kLoopStampShift;
}
/* gcl_tune.rec_prefetch default: frame headers in flight while the submitting
 * core writes header records -- a whole 64-packet burst's, issued before the
 * first record.  Six interleaved rounds (profiles/r06_rec_prefetch_ab2.jsonl),
 * medians for distances 2 / 16 / 64: cold headers 4 x 8 34.5 / 35.5 / 44.0
 * Mpkt/s (submit 12.8 / 12.4 / 9.5 ns per packet), cold 1 x 1 submit 16.7 /
 * 12.3 / 8.2, cache-hot lone burst 3.31 / 3.27 / 3.19 us p50 */
constexpr uint32_t kRecPrefetch = 64;
/* gcl_tune.slot_prefetch default.  Six interleaved rounds of fresh processes
 * (profiles/r06_slot_prefetch_ab.jsonl), p50 medians off -> on: cache-hot
 * lone burst, NIC hash 3.35 -> 3.24 us (5 of 6 rounds faster, one equal),
 * 2 x 2 3.22 -> 3.09; JENKINS 3.30 -> 3.32 and cold headers 4.20 -> 4.21,
 * within their noise */
constexpr uint32_t kDefaultSlotPrefetch = 1;

struct LoopImgHdr {        /* first 64 B of a table image buffer */
	uint32_t bytes, ipt_mask, off_rt, off_flow, off_toep, ipt_seed, off_seed, off_crc, pad[8];
};
static_assert(sizeof(LoopImgHdr) == 64, "LoopImgHdr");

#define GCL_LOOP_F_OLF  0x1
#define GCL_LOOP_F_RSS  0x2
#define GCL_LOOP_F_FDIR 0x4
#define GCL_LOOP_F_HINT 0x8

struct LoopParams {
	uint8_t *slots;            /* device view of the slot ring */
	uint64_t slot_bytes;
	uint32_t nslots, workers;
	uint32_t off_offs, off_olf, off_rss, off_fdir, off_hint, off_verd;
	const uint8_t *img[2];     /* device views of the two image buffers */
	const uint32_t *stop;
	uint32_t *where;           /* host words: XCC_ID + 1 of worker b at [b] (b < 8) */
	uint32_t *exited;          /* host word: set by a worker that leaves */
	uint32_t *polls;           /* host words: worker b's bursts at [4b + k] by how they
	                              arrived (kLoopPollEarly / Stale / Late) */
	uint64_t lifetime_ticks;   /* s_memrealtime ticks each block may run */
	const uint8_t *frames;     /* device view of the registered region */
	uint64_t frames_len;
	unsigned long long *counts, *stats;
	uint32_t max_rt, cflags, default_flags;
	uint32_t off_hdr;          /* GCL_LOOP_INLINE_HDRS: 64-B granules in the slot,
	                              GCL_LOOP_HDR_RECORDS: 64-B header records; else 0 */
	uint32_t spec;             /* bursts <= 64: poll the stamped offsets (or records) too */
	uint32_t hdr_rec;          /* off_hdr holds header records (GCL_LOOP_HDR_RECORDS) */
	uint32_t spec_ticks;       /* how long a wait polls them (s_memrealtime ticks) */
	uint32_t off_trans;        /* GCL_CFG_TRANS_HASH: 16-B {h5, h3, ticket} per packet; else 0 */
	uint64_t t0;               /* tickets start after t0 (0; gcl_tune.loop_t0 tests the
	                              stamps' wrap), a multiple of nslots */
	uint32_t stamps;           /* GCL_LOOP_STAMPS: per-burst stage times into the slot header */
	uint32_t rec_plane;        /* GCL_LOOP_HDR_RECORDS: bytes between the records' chunk
	                              planes (chunk j of packet i at off_hdr + j * rec_plane + 16 i) */
	uint32_t lean;             /* rxloop64_kernel: plain-IPv4 bursts on classify_lean
	                              (gcl_tune.loop_lean 0: always classify_core) */
	uint32_t phase_max;        /* rxloop64_kernel: the poll-phase delay's ceiling in ticks
	                              (0: off; gcl_tune.loop_phase_*), and its steps */
	uint32_t phase_up, phase_down;
	uint32_t prefetch;         /* rxloop64_kernel: the next ticket's poll issued before a
	                              burst is classified (gcl_tune.loop_prefetch) */
};

/* GCL_LOOP_HDR_RECORDS: the submitting core writes each packet as one 64-B
 * record of four 16-B chunks, each stored whole and led by the slot's use
 * count, so that a lane reading them while it polls knows whether all four
 * are this burst's.  Together they carry everything rx_one_pkt reads:
 *   q0 {stamp, d3, d5, d6}      frame dwords: bytes 12-15, 20-27
 *   q1 {stamp, d7, d8, d9}      bytes 28-39
 *   q2 {stamp, d10, rss, fdir}  bytes 40-43, hash.rss, hash.fdir.hi
 *   q3 {stamp, off[31:0], off[39:32] | ol_flags << 8, dst_hint}
 * (d4, total length and IP id, and the MAC addresses are never read.)  A burst
 * of <= 64 packets then arrives whole with the poll that finds its word: one
 * PCIe round trip per burst.  Ports past byte 43 (IHL >= 7) are read from the
 * frame at the record's offset.  The chunks lie in four planes (q_j of packet
 * i at off_hdr + j * rec_plane + 16 i), so each of a poll's four loads reads
 * 1 KiB contiguous across the wave: 64 PCIe read requests of 64 B for a
 * 64-packet burst instead of 256 of 16 B with 64-B records. */
__host__ __device__ constexpr uint32_t loop_rec_stamp(uint64_t t, uint32_t nslots)
{
	/* never 0, as loop_stamp: bit 31 set, the use count in bits 0-30 */
	return (uint32_t)(((t - 1) >> __builtin_ctz(nslots)) & 0x7FFFFFFFull) | 0x80000000u;
}

/* the value lane 0 of the wave holds, in scalar registers: the poll's word
 * and stop flag are loaded by lane 0 only, and a uniform broadcast keeps
 * the loops they end uniform (a __shfl broadcast is an LDS round trip, and
 * its VGPR result makes the compiler treat the slot address, and with it the
 * buffer descriptors, as divergent: waterfall loops around every load) */
__device__ __forceinline__ uint64_t lane0_u64(uint64_t v)
{
	return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32 |
	       (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}

/* a record's four chunks -> the packet's tile row and side-array entries */
__device__ __forceinline__ void rec_to_row(const uint4 *q, uint4 *tile, int p, uint64_t *offs,
                                           uint8_t *olf, uint32_t *rss, uint32_t *fdir,
                                           uint32_t *hint)
{
	tile[tile_slot(p, 0)] = make_uint4(0, 0, 0, q[0].y);
	tile[tile_slot(p, 1)] = make_uint4(0, q[0].z, q[0].w, q[1].y);
	tile[tile_slot(p, 2)] = make_uint4(q[1].z, q[1].w, q[2].y, 0);
	offs[p] = (uint64_t)(q[3].z & 0xFF) << 32 | q[3].y;
	olf[p] = (uint8_t)(q[3].z >> 8);
	rss[p] = q[2].z;
	fdir[p] = q[2].w;
	hint[p] = q[3].w;
}

/* header tile + 2 x side arrays (offs, rss, fdir, hint, olflags) + verdicts +
 * transport hashes + ctl */
constexpr uint32_t kLoopSide = 256 * 8 + 3 * 256 * 4 + 256;
constexpr uint32_t kLoopFixedLds = 256 * 64 + 2 * kLoopSide + 2 * 256 * 8 + 64;

/* Side arrays of one 256-packet chunk, double-buffered in LDS so the next
 * chunk's arrive while the current one is classified. */
struct LoopSide {
	uint64_t *offs;
	uint32_t *rss, *fdir, *hint;
	uint8_t *olf;
	__device__ LoopSide(uint8_t *b)
	    : offs((uint64_t *)b), rss((uint32_t *)(b + 2048)), fdir(rss + 256), hint(fdir + 256),
	      olf((uint8_t *)(hint + 256)) {}
	/* packets [base, base + m) of the burst in @slot, one per lane (the
	 * offsets too unless the poll already brought them) */
	__device__ void load(const uint8_t *slot, const LoopParams &L, uint32_t fl, uint32_t base,
	                     uint32_t m, int tid, bool with_offs = true)
	{
		if ((uint32_t)tid >= m)
			return;
		const uint32_t i = base + tid;
		if (with_offs)
			offs[tid] = gcl::ld_sys64(slot + L.off_offs + 8 * i) & kLoopOffMask;
		if (fl & GCL_LOOP_F_OLF)
			olf[tid] = (uint8_t)(gcl::ld_sys32(slot + L.off_olf + (i & ~3u)) >> (8 * (i & 3)));
		if (fl & GCL_LOOP_F_RSS)
			rss[tid] = gcl::ld_sys32(slot + L.off_rss + 4 * i);
		if (fl & GCL_LOOP_F_FDIR)
			fdir[tid] = gcl::ld_sys32(slot + L.off_fdir + 4 * i);
		if (fl & GCL_LOOP_F_HINT)
			hint[tid] = gcl::ld_sys32(slot + L.off_hint + 4 * i);
	}
};


template <int MODE>
__global__ void __launch_bounds__(256) rxloop_kernel(LoopParams L)
{
	extern __shared__ uint4 smem[];
	uint4 *tile = smem;
	uint8_t *side_mem = (uint8_t *)(tile + 1024);
	/* the two side-array buffers, picked by arithmetic (an array of
	 * LoopSide indexed by chunk parity would live in scratch) */
	auto side = [&](uint32_t b) { return LoopSide(side_mem + (b & 1) * kLoopSide); };
	uint2 *s_verd = (uint2 *)(side_mem + 2 * kLoopSide);
	uint2 *s_trans = s_verd + 256;
	uint32_t *s_ctl = (uint32_t *)(s_trans + 256);
	uint32_t *hist = s_ctl + 16;
	uint8_t *lds_tab = (uint8_t *)(hist + ((L.max_rt + 3) & ~3u));
	const int tid = threadIdx.x;
	const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + L.lifetime_ticks;
	/* the poll's clock (s_memrealtime, 100 MHz: the stamps' 10-ns ticks) */
	auto sclk = []() -> uint64_t { return __builtin_amdgcn_s_memrealtime(); };
	auto to10 = [](uint64_t d) -> uint32_t { return (uint32_t)d; };
	const __amdgpu_buffer_rsrc_t frs = gcl::host_rsrc(L.frames, L.frames_len);
	if (tid == 0 && blockIdx.x < 8) /* which XCD this worker runs on */
		gcl::st_sys32(&L.where[blockIdx.x], __builtin_amdgcn_s_getreg((3 << 11) | 20) + 1);

	KParams k = {};
	k.frames = L.frames;
	k.frames_len = L.frames_len;
	k.verdicts = s_verd;
	k.max_rt = L.max_rt;
	k.cflags = L.cflags; /* with thread_bits in [31:24] */
	k.default_flags = L.default_flags;
	k.trans = L.off_trans ? s_trans : nullptr; /* classify_core's per-packet pair */
	Tables tb = {};
	uint32_t cur_seq = 0xFF; /* no image yet (versions are taken mod 64) */
	uint32_t polls[3] = {0, 0, 0};
	int poll_kind = 0; /* tid 0: how this burst arrived */

	for (uint64_t t = L.t0 + blockIdx.x + 1;; t += L.workers) {
		uint8_t *slot = L.slots + ((t - 1) % L.nslots) * L.slot_bytes;
		LoopSlotHdr *h = (LoopSlotHdr *)slot;
		const __amdgpu_buffer_rsrc_t srs = gcl::host_rsrc(slot, L.slot_bytes);
		if (tid < 64) {
			/* wave 0 polls.  One system-scope load of the slot word carries
			 * the whole burst header, and without inline headers each lane
			 * also reads its stamped offset entry (with header records, its
			 * packet's four stamped chunks), so a burst of <= 64 packets has
			 * its offsets (or all it needs) when the word shows it.  (The
			 * stop flag is read beside every 8th poll, never after one: that
			 * made each poll two round trips.)  The offsets or records are
			 * polled only for the first L.spec_ticks of a wait:
			 * a worker that waits longer (many workers, deep queues) polls
			 * the word alone, so idle polls do not crowd the PCIe requests
			 * of the workers that are reading frames */
			const bool spec = L.spec, rec = L.hdr_rec;
			const uint64_t stamp = loop_stamp(t, L.nslots);
			const uint32_t rstamp = loop_rec_stamp(t, L.nslots);
			const uint64_t spec_end = __builtin_amdgcn_s_memrealtime() + L.spec_ticks;
			uint64_t w = 0, e = 0;
			bool rok = false, sp_hit = false;
			uint4 q[4], qv[4] = {}; /* header records: the lane's packet's chunks */
			uint64_t t_issue = 0;   /* GCL_LOOP_STAMPS: this poll's issue time */
			uint32_t npoll = 0;
			for (uint32_t k = 0;; k++) {
				if (L.stamps)
					t_issue = sclk();
				npoll = k + 1;
				const bool sp = spec && __builtin_amdgcn_s_memrealtime() < spec_end;
				const uint64_t ev = sp && !rec ? gcl::ld_sys64(slot + L.off_offs + 8 * tid) : 0;
				if (sp && rec) {
#pragma unroll
					for (int j = 0; j < 4; j++) {
						const auto v = __builtin_amdgcn_raw_buffer_load_b128(
						        srs, (int)(L.off_hdr + L.rec_plane * j + 16 * tid), 0, gcl::kSysAux);
						qv[j] = make_uint4(v[0], v[1], v[2], v[3]);
					}
				}
				uint64_t wv = 0;
				uint32_t sv = 0;
				if (tid == 0) {
					wv = gcl::ld_sys64(&h->word);
					if ((k & 7) == 7) /* a stop waits for up to 8 polls */
						sv = gcl::ld_sys32(L.stop);
				}
				wv = lane0_u64(wv);
				sv = (uint32_t)__builtin_amdgcn_readfirstlane((int)sv);
				if ((wv >> 24) == (t & ((1ull << 40) - 1))) {
					w = wv;
					e = ev;
					sp_hit = sp;
					rok = sp && qv[0].x == rstamp && qv[1].x == rstamp && qv[2].x == rstamp &&
					      qv[3].x == rstamp;
#pragma unroll
					for (int j = 0; j < 4; j++)
						q[j] = qv[j];
					break;
				}
				if (sv || __builtin_amdgcn_s_memrealtime() > t_end)
					break;
				__builtin_amdgcn_s_sleep(1);
			}
			const uint32_t nw = (uint32_t)(w >> 11) & 0x1FFF;
			/* an entry counts only if it was loaded with the poll that found
			 * the word (sp_hit): e is 0 otherwise */
			const bool fresh = (uint32_t)tid >= nw ||
			                   (rec ? rok : sp_hit && (e & ~kLoopOffMask) == stamp);
			const bool early = spec && w && nw <= 64 && __all(fresh);
			if (early && (uint32_t)tid < nw) {
				const LoopSide s0 = side(0);
				if (rec)
					rec_to_row(q, tile, tid, s0.offs, s0.olf, s0.rss, s0.fdir, s0.hint);
				else
					s0.offs[tid] = e & kLoopOffMask;
			}
			if (tid == 0 && w) {
				/* counted now, published after the burst's records: on gfx9
				 * stores share vmcnt with loads, and any vmcnt(0) between
				 * the hit and the records (the classify path has several)
				 * would wait for this store's PCIe round trip, ~1.2 us
				 * (GCL_LOOP_STAMPS, profiles/r04_stages.jsonl) */
				poll_kind = early ? kLoopPollEarly
				          : (sp_hit && nw <= 64) ? kLoopPollStale : kLoopPollLate;
				polls[poll_kind]++;
			}
			if (tid == 0) {
				s_ctl[0] = w != 0;
				s_ctl[1] = nw;
				s_ctl[2] = (uint32_t)(w >> 7) & 0xF;
				s_ctl[3] = (uint32_t)(w >> 6) & 1;
				s_ctl[4] = (uint32_t)w & 63;
				s_ctl[5] = early;
				if (L.stamps) { /* hit time, the hitting poll's round trip, polls */
					const uint64_t now = sclk();
					s_ctl[6] = (uint32_t)now;
					s_ctl[7] = (uint32_t)(now >> 32);
					s_ctl[8] = to10(now - t_issue);
					s_ctl[9] = npoll;
				}
			}
		}
		__syncthreads();
		uint32_t st_b1 = 0, st_b2 = 0, st_b3 = 0; /* GCL_LOOP_STAMPS: past each barrier */
		if (L.stamps && tid == 0)
			st_b1 = (uint32_t)sclk();
		if (!s_ctl[0]) {
			/* the host stops publishing on this (one word it can read
			 * without asking the HIP runtime per burst) */
			if (tid == 0)
				gcl::st_sys32(L.exited, 1);
			break;
		}
		const uint32_t n = s_ctl[1], fl = s_ctl[2], img = s_ctl[3], img_seq = s_ctl[4];
		const bool early_offs = s_ctl[5];
		if (img_seq != cur_seq) { /* a new table snapshot: copy it into LDS */
			const uint8_t *ib = L.img[img];
			const uint32_t bytes = gcl::ld_sys32(ib);
			for (uint32_t i = tid; i < bytes / 4; i += 256)
				((uint32_t *)lds_tab)[i] = gcl::ld_sys32(ib + 64 + 4 * i);
			k.ipt_mask = gcl::ld_sys32(ib + 4);
			k.ipt_seed = gcl::ld_sys32(ib + 20);
			tb.ipt = (const uint2 *)lds_tab;
			tb.rtab = (const RtEntry *)(lds_tab + gcl::ld_sys32(ib + 8));
			tb.flow = lds_tab + gcl::ld_sys32(ib + 12);
			tb.toep = (const uint32_t *)(lds_tab + gcl::ld_sys32(ib + 16));
			tb.seed = (const uint32_t *)(lds_tab + gcl::ld_sys32(ib + 24));
			tb.crc = (const uint32_t *)(lds_tab + gcl::ld_sys32(ib + 28));
			cur_seq = img_seq;
		}
		for (uint32_t i = tid; i < L.max_rt; i += 256)
			hist[i] = 0;
		Counters cnt = {0, 0, 0, 0};
		__syncthreads(); /* s_ctl consumed, tables and hist ready */
		if (L.stamps && tid == 0)
			st_b2 = (uint32_t)sclk();
		/* chunk pipeline: the side arrays of chunk c+1 and the frames of
		 * chunk c are in flight together, and chunk c+1's frame loads are
		 * issued before chunk c is classified */
		const uint32_t nch = (n + 255) / 256;
		uint4 r[4];
		auto chunk_m = [&](uint32_t c) { return n - 256 * c < 256 ? n - 256 * c : 256u; };
		const bool rec = L.hdr_rec;
		auto load_frames = [&](const LoopSide &sd, uint32_t c0, uint32_t m) {
			if (rec) { /* one packet per lane: its record's four chunks */
#pragma unroll
				for (int j = 0; j < 4; j++) {
					if ((uint32_t)tid >= m) {
						r[j] = make_uint4(0, 0, 0, 0);
					} else {
						const auto v = __builtin_amdgcn_raw_buffer_load_b128(
						        srs, (int)(L.off_hdr + L.rec_plane * j + 16 * (256 * c0 + tid)), 0, gcl::kSysAux);
						r[j] = make_uint4(v[0], v[1], v[2], v[3]);
					}
				}
				return;
			}
#pragma unroll
			for (int j = 0; j < 4; j++) {
				const int c = j * 256 + tid, p = c >> 2, q = c & 3;
				if ((uint32_t)p >= m) {
					r[j] = make_uint4(0, 0, 0, 0);
				} else if (L.off_hdr) { /* granules inlined in the slot by the host */
					const auto v = __builtin_amdgcn_raw_buffer_load_b128(
					        srs, (int)(L.off_hdr + 64 * (256 * c0 + p) + 16 * q), 0, gcl::kSysAux);
					r[j] = make_uint4(v[0], v[1], v[2], v[3]);
				} else {
					r[j] = gcl::load16_host(frs, L.frames, L.frames_len, sd.offs[p] + 16 * (uint64_t)q);
				}
			}
		};
		/* the granules do not wait for the offsets, nor do frames whose
		 * offsets came with the poll */
		if (rec) {
			/* the records carry the side arrays too; a burst that came
			 * with the poll is already in the tile */
			if (!early_offs)
				load_frames(side(0), 0, chunk_m(0));
		} else {
			if (L.off_hdr || early_offs)
				load_frames(side(0), 0, chunk_m(0));
			side(0).load(slot, L, fl, 0, chunk_m(0), tid, !early_offs);
			__syncthreads();
			if (!L.off_hdr && !early_offs)
				load_frames(side(0), 0, chunk_m(0));
		}
		for (uint32_t c = 0; c < nch; c++) {
			const uint32_t m = chunk_m(c), base = 256 * c;
			const LoopSide cur = side(c);
			if (rec) {
				if ((c || !early_offs) && (uint32_t)tid < m)
					rec_to_row(r, tile, tid, cur.offs, cur.olf, cur.rss, cur.fdir, cur.hint);
			} else {
				if (c + 1 < nch)
					side(c + 1).load(slot, L, fl, base + 256, chunk_m(c + 1), tid);
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const int cc = j * 256 + tid;
					tile[tile_slot(cc >> 2, cc & 3)] = r[j];
				}
			}
			__syncthreads(); /* tile of c and side arrays of c + 1 in LDS */
			if (L.stamps && tid == 0)
				st_b3 = (uint32_t)sclk();
			if (c + 1 < nch)
				load_frames(side(c + 1), c + 1, chunk_m(c + 1));
			k.n = m;
			k.offs = cur.offs;
			k.olflags = (fl & GCL_LOOP_F_OLF) ? cur.olf : nullptr;
			k.rss = (fl & GCL_LOOP_F_RSS) ? cur.rss : nullptr;
			k.fdir = (fl & GCL_LOOP_F_FDIR) ? cur.fdir : nullptr;
			k.dst_hint = (fl & GCL_LOOP_F_HINT) ? cur.hint : nullptr;
			if ((uint32_t)tid < m) {
				put_verdict(k, (uint64_t)tid,
				            classify_one<MODE, true, true>(k, tile, tid, (uint64_t)tid, tb, hist, cnt,
				                                           rec ? kSpanRec : kSpanFull));
				const bool v4 = L.cflags & GCL_CFG_VERDICT4, v2 = L.cflags & GCL_CFG_VERDICT2;
				const bool v1 = L.cflags & GCL_CFG_VERDICT1;
				const uint32_t hsh = v4 || v2 || v1 ? 0u : s_verd[tid].x;
				const uint32_t vlo = v1 ? ((const uint8_t *)s_verd)[tid]
				                   : v2 ? ((const uint16_t *)s_verd)[tid]
				                   : v4 ? ((const uint32_t *)s_verd)[tid] : s_verd[tid].y;
				if (L.off_trans) { /* before the record: the host checks both tickets */
					const gcl::u32x4 tr = {s_trans[tid].x, s_trans[tid].y, (uint32_t)t, (uint32_t)(t >> 32)};
					__builtin_amdgcn_raw_buffer_store_b128(tr, srs, (int)(L.off_trans + 16 * (base + tid)),
					                                       0, gcl::kSysAux);
				}
				const uint64_t t_cls = L.stamps ? sclk() : 0;
				const gcl::u32x4 rec = {hsh, vlo, (uint32_t)t, (uint32_t)(t >> 32)};
				__builtin_amdgcn_raw_buffer_store_b128(
				        rec, srs, (int)(L.off_verd + sizeof(LoopRec) * (base + tid)), 0, gcl::kSysAux);
				if (L.stamps && tid == 0 && c + 1 == nch) {
					/* stage times of this burst (10-ns ticks from the hit):
					 * {ticket, hit's round trip, classified, record stored}
					 * {ticket, polls, hit time lo, hi} */
					const uint64_t hit = (uint64_t)s_ctl[7] << 32 | s_ctl[6];
					const uint64_t t_st = sclk();
					const gcl::u32x4 a = {(uint32_t)t, s_ctl[8], to10(t_cls - hit), to10(t_st - hit)};
					const gcl::u32x4 b2 = {(uint32_t)t, s_ctl[9], s_ctl[6], s_ctl[7]};
					const gcl::u32x4 c3 = {(uint32_t)t, to10(st_b1 - (uint32_t)hit),
					                       to10(st_b2 - (uint32_t)hit), to10(st_b3 - (uint32_t)hit)};
					__builtin_amdgcn_raw_buffer_store_b128(a, srs, 16, 0, gcl::kSysAux);
					__builtin_amdgcn_raw_buffer_store_b128(b2, srs, 32, 0, gcl::kSysAux);
					__builtin_amdgcn_raw_buffer_store_b128(c3, srs, 48, 0, gcl::kSysAux);
				}
			}
			__syncthreads(); /* tile and side(c) free again */
		}
		/* counters of this burst */
		for (uint32_t i = tid; i < L.max_rt; i += 256)
			if (hist[i] && L.counts)
				atomicAdd(&L.counts[i], (unsigned long long)hist[i]);
		if (L.stats) {
			for (int off = 32; off > 0; off >>= 1) {
				cnt.flowtag += __shfl_xor(cnt.flowtag, off);
				cnt.hashmiss += __shfl_xor(cnt.hashmiss, off);
				cnt.unreg += __shfl_xor(cnt.unreg, off);
				cnt.unhandled += __shfl_xor(cnt.unhandled, off);
			}
			if ((tid & 63) == 0) {
				if (cnt.flowtag)
					atomicAdd(&L.stats[GCL_RX_FLOW_TAG_MATCH], (unsigned long long)cnt.flowtag);
				if (cnt.hashmiss)
					atomicAdd(&L.stats[GCL_RX_HASH_MISSING], (unsigned long long)cnt.hashmiss);
				if (cnt.unreg)
					atomicAdd(&L.stats[GCL_RX_UNREGISTERED_MAC], (unsigned long long)cnt.unreg);
				if (cnt.unhandled)
					atomicAdd(&L.stats[GCL_RX_UNHANDLED], (unsigned long long)cnt.unhandled);
			}
			if (tid == 0)
				atomicAdd(&L.stats[GCL_RX_PULLED], (unsigned long long)n);
		}
		if (tid == 0)
			gcl::st_sys32(&L.polls[4 * blockIdx.x + poll_kind], polls[poll_kind]);
	}
}

/* ------------------------------------------------------------------------
 * rxloop64_kernel<MODE>: the loop at the reference's own burst size (<= 64
 * mbufs, IOKERNEL_RX_BURST_SIZE, defs.h:75), chosen by gcl_rxloop_start
 * whenever max_burst <= 64.  A burst that size is one packet per lane of ONE
 * wave, so a wave takes it from the poll to the verdicts alone, from
 * registers, with no barrier: rxloop_kernel's three barriers and its LDS tile
 * cost 0.7 us of a lone burst (GCL_LOOP_STAMPS, profiles/r04_stages_reentry.jsonl).
 *
 * Two waves per worker.  The poller polls the worker's next ticket,
 * classifies the burst and stores its verdict records.  The writer adds the
 * counts and the counters (device atomics) and the poll counters, so their
 * retirement never holds the poller's vmcnt (on gfx9 stores and loads share
 * vmcnt and retire in order); bursts reach it through two LDS mailboxes,
 * ordered by LDS-only fences (lgkmcnt, never vmcnt).
 *
 * A second poller sharing the ticket sequence through LDS (each slot sampled
 * twice per poll round trip, the burst claimed by an LDS compare-and-swap)
 * lost the round-5 A/B on header records: lone bursts 3.84 -> 3.9-4.06 us p50,
 * 4 workers x 8 deep 103 -> 92 Mpkt/s (profiles/r05_pollers_ab.jsonl); it
 * won only on stamped offsets, the slower form, and was removed.
 *
 * The poll-phase delay (round 5, L.phase_max, loops of 1-2 workers): a host
 * that submits once it has seen the last burst's verdicts cannot land before
 * its own turnaround, so a ticket's first poll waits dly ticks after the last
 * records, dly stepping down after a burst found whole by the first poll and
 * up after one found by the second.  Round 4's form (a knob since removed)
 * delayed only after a burst that needed more than one poll, so a
 * back-to-back stream alternated delayed and undelayed polls and never
 * locked on.
 */
struct Mbox64 {
	uint32_t p[64];   /* each packet's runtime (~0: none): the counts */
	uint64_t t;       /* ticket */
	uint32_t n, kind; /* packets; how the burst arrived (kLoopPollEarly ...) */
	uint32_t cnt[4];  /* flowtag, hashmiss, unreg, unhandled */
	uint32_t st[8];   /* GCL_LOOP_STAMPS: hit lo, hit hi, the hitting poll's round
	                     trip, polls, hit -> packets in registers, hit -> posted,
	                     hit -> classified, hit -> records issued */
	uint32_t flag;    /* 1: posted by the poller, 0: free */
	uint32_t lean;    /* classified by classify_lean */
	uint32_t pad[2];
};
static_assert(sizeof(Mbox64) % 16 == 0, "Mbox64");

/* one classifying wave's LDS: its mailboxes and the side arrays classify_core
 * reads through KParams */
struct Wave64 {
	Mbox64 mbox[2];
	uint64_t offs[64];
	uint32_t fdir[64], hint[64];
	uint2 trans[64];
};
static_assert(sizeof(Wave64) % 16 == 0, "Wave64");

/* the worker's shared words */
struct Ctl64 {
	uint32_t exited; /* the poller has left */
	uint32_t pad[3];
};
static_assert(sizeof(Ctl64) % 16 == 0, "Ctl64");

/* LDS of rxloop64_kernel with @copy bytes for the table copy (a 64-B image
 * header + the image) */
__host__ __device__ constexpr uint32_t loop64_lds(uint32_t copy)
{
	return (uint32_t)sizeof(Ctl64) + (uint32_t)sizeof(Wave64) + copy;
}

/* rxloop64_kernel's writer wave: each posted burst's counts and counters,
 * the poll counters, the stage stamps; leaves once the poller has left and
 * its mailboxes are drained. */
__device__ __forceinline__ void rxloop64_writer(const LoopParams &L, Wave64 *wv, Ctl64 *ctl, int lane)
{
	uint32_t pe = 0, ps = 0, pl = 0; /* bursts by how they arrived (no indexed array: scratch) */
	uint32_t pn = 0;                 /* bursts on classify_lean (gcl_rxloop_lean_bursts) */
	for (uint32_t b = 0;; b ^= 1) {
		Mbox64 &m = wv->mbox[b];
		/* one producer, in order: wait on this mailbox */
		for (;;) {
			if (__hip_atomic_load(&m.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
				break;
			if (__hip_atomic_load(&ctl->exited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
			    !__hip_atomic_load(&m.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
				return;
			__builtin_amdgcn_s_sleep(1);
		}
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
		const uint64_t t_w = L.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
		const uint64_t t = m.t;
		const uint32_t n = m.n, kind = m.kind, lean = m.lean;
		const uint32_t p = m.p[lane];
		if ((uint32_t)lane < n && p != ~0u && L.counts)
			atomicAdd(&L.counts[p], 1ull);
		uint32_t c[4] = {m.cnt[0], m.cnt[1], m.cnt[2], m.cnt[3]};
		uint32_t st[8];
		if (L.stamps)
			for (int i = 0; i < 8; i++)
				st[i] = m.st[i];
		/* every LDS read of the mailbox is done: hand it back */
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
		if (lane == 0)
			__hip_atomic_store(&m.flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		if (lane == 0) {
			if (L.stats) {
				if (c[0])
					atomicAdd(&L.stats[GCL_RX_FLOW_TAG_MATCH], (unsigned long long)c[0]);
				if (c[1])
					atomicAdd(&L.stats[GCL_RX_HASH_MISSING], (unsigned long long)c[1]);
				if (c[2])
					atomicAdd(&L.stats[GCL_RX_UNREGISTERED_MAC], (unsigned long long)c[2]);
				if (c[3])
					atomicAdd(&L.stats[GCL_RX_UNHANDLED], (unsigned long long)c[3]);
				atomicAdd(&L.stats[GCL_RX_PULLED], (unsigned long long)n);
			}
			pe += kind == kLoopPollEarly;
			ps += kind == kLoopPollStale;
			pl += kind == kLoopPollLate;
			gcl::st_sys32(&L.polls[4 * blockIdx.x + kind],
			              kind == kLoopPollEarly ? pe : kind == kLoopPollStale ? ps : pl);
			if (lean)
				gcl::st_sys32(&L.polls[4 * blockIdx.x + 3], ++pn);
			if (L.stamps) {
				/* {ticket, hit's round trip, hit -> classified, hit -> records issued}
				 * {ticket, polls, hit lo, hi}
				 * {ticket, hit -> packets in registers, hit -> posted, hit -> writer} */
				const __amdgpu_buffer_rsrc_t srs =
				        gcl::host_rsrc(L.slots + ((t - 1) & (L.nslots - 1)) * (uint64_t)L.slot_bytes, L.slot_bytes);
				const uint64_t hit = (uint64_t)st[1] << 32 | st[0];
				const gcl::u32x4 a = {(uint32_t)t, st[2], st[6], st[7]};
				const gcl::u32x4 b2 = {(uint32_t)t, st[3], st[0], st[1]};
				const gcl::u32x4 c3 = {(uint32_t)t, st[4], st[5], (uint32_t)(t_w - hit)};
				__builtin_amdgcn_raw_buffer_store_b128(a, srs, 16, 0, gcl::kSysAux);
				__builtin_amdgcn_raw_buffer_store_b128(b2, srs, 32, 0, gcl::kSysAux);
				__builtin_amdgcn_raw_buffer_store_b128(c3, srs, 48, 0, gcl::kSysAux);
			}
		}
	}
}

/* a value of lane 0, uniform (scalar) */
__device__ __forceinline__ uint32_t lane0_u32(uint32_t v)
{
	return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

template <int MODE>
__global__ void __launch_bounds__(128) rxloop64_kernel(LoopParams L)
{
	extern __shared__ uint4 smem[];
	Ctl64 *ctl = (Ctl64 *)smem;
	Wave64 *wv = (Wave64 *)(ctl + 1);
	uint8_t *cb = (uint8_t *)(wv + 1); /* the table copy: a LoopImgHdr + the image */
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	if (threadIdx.x == 0) {
		wv->mbox[0].flag = wv->mbox[1].flag = 0;
		ctl->exited = 0;
	}
	__syncthreads(); /* the only barrier */
	if (w == 1) {
		rxloop64_writer(L, wv, ctl, lane);
		return;
	}
	Wave64 &me = *wv;
	const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + L.lifetime_ticks;
	const __amdgpu_buffer_rsrc_t frs = gcl::host_rsrc(L.frames, L.frames_len);
	if (lane == 0 && w == 0 && blockIdx.x < 8) /* which XCD this worker runs on */
		gcl::st_sys32(&L.where[blockIdx.x], __builtin_amdgcn_s_getreg((3 << 11) | 20) + 1);
	KParams k = {};
	k.frames = L.frames;
	k.frames_len = L.frames_len;
	k.max_rt = L.max_rt;
	k.cflags = L.cflags; /* with thread_bits in [31:24] */
	k.default_flags = L.default_flags;
	k.offs = me.offs;
	k.trans = L.off_trans ? me.trans : nullptr;
	Tables tb = {};
	uint32_t cur_seq = 0xFF; /* the image tb points at (0xFF: none) */
	uint32_t mb = 0;
	const bool spec = L.spec, rec = L.hdr_rec;
	uint64_t kt = 0; /* this worker's next ticket index */
	uint64_t spec_end = __builtin_amdgcn_s_memrealtime() + L.spec_ticks;
	uint32_t npoll = 0; /* polls of this ticket */
	/* the poll-phase delay (L.phase_max): a ticket's first poll waits dly
	 * ticks after the last burst's records went out */
	uint32_t dly = 0;
	uint64_t t_done = 0;
	uint32_t ph_max = L.phase_max, ph_up = L.phase_up, ph_dn = L.phase_down;
	/* the next ticket's poll, issued while this burst is classified
	 * (L.prefetch): its word, offsets or records, issue time and window */
	bool pf = false, psp = false;
	uint64_t pw = 0, pev = 0, pis = 0;
	uint4 pq[4] = {};

	for (uint32_t kk = 0;; kk++) {
		/* the ticket and its slot, uniform: a slot address the compiler
		 * thinks divergent puts every buffer load in a waterfall loop
		 * (nslots is a power of two: a mask, not a 64-bit modulo) */
		kt = lane0_u64(kt);
		/* the context flags and the delay's parameters opaque here, so that
		 * the compiler keeps them in registers rather than re-reading the
		 * kernel arguments (a scalar load and its wait) between a hit and
		 * the classification, or between the store and the next poll */
		asm volatile("" : "+s"(k.cflags), "+s"(k.default_flags), "+s"(ph_max), "+s"(ph_up), "+s"(ph_dn));
		const uint64_t t = lane0_u64(L.t0 + blockIdx.x + 1 + kt * L.workers);
		uint8_t *slot = L.slots + ((t - 1) & (L.nslots - 1)) * (uint64_t)L.slot_bytes;
		LoopSlotHdr *h = (LoopSlotHdr *)slot;
		const __amdgpu_buffer_rsrc_t srs = gcl::host_rsrc(slot, L.slot_bytes);
		const uint64_t stamp = loop_stamp(t, L.nslots);
		const uint32_t rstamp = loop_rec_stamp(t, L.nslots);
		/* the poll: the slot word, and for the first L.spec_ticks of a wait
		 * each lane's stamped offset or header record.  The word goes out
		 * first: the host writes the records before the word, so records
		 * read after a word that shows the burst are current unless the
		 * fabric reorders the two (the other order made nearly every lone
		 * burst's records stale).  Every lane loads the word and the stop
		 * flag (one address: one request), so no divergent branch lets the
		 * compiler consume the records before the word is even issued. */
		uint64_t t_issue, wv0, ev;
		uint32_t sv0;
		bool sp;
		uint4 q[4];
		if (pf) { /* issued while the last burst was classified */
			pf = false;
			t_issue = pis;
			sp = psp;
			wv0 = pw;
			ev = pev;
			sv0 = 0;
#pragma unroll
			for (int j = 0; j < 4; j++)
				q[j] = pq[j];
		} else {
			if (npoll == 0 && dly) {
				/* A host that submits once it has seen the last records (a
				 * closed loop) cannot land before its turnaround: a poll
				 * issued at once samples the slot too early, and every
				 * later sample is a round trip apart from it.  The first
				 * poll waits instead; dly tracks that turnaround (below). */
				const uint64_t until = t_done + dly;
				while (__builtin_amdgcn_s_memrealtime() < until)
					__builtin_amdgcn_s_sleep(1);
				spec_end = __builtin_amdgcn_s_memrealtime() + L.spec_ticks;
			}
			t_issue = __builtin_amdgcn_s_memrealtime();
			sp = spec && t_issue < spec_end;
			wv0 = gcl::ld_sys64(&h->word);
			sv0 = (kk & 7) == 7 ? gcl::ld_sys32(L.stop) : 0u; /* a stop waits <= 8 polls */
			ev = sp && !rec ? gcl::ld_sys64(slot + L.off_offs + 8 * lane) : 0;
#pragma unroll
			for (int j = 0; j < 4; j++)
				q[j] = make_uint4(0, 0, 0, 0);
			if (sp && rec) {
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const auto v = __builtin_amdgcn_raw_buffer_load_b128(
					        srs, (int)(L.off_hdr + L.rec_plane * j + 16 * lane), 0, gcl::kSysAux);
					q[j] = make_uint4(v[0], v[1], v[2], v[3]);
				}
			}
		}
		npoll++;
		const uint64_t w_word = lane0_u64(wv0);
		const uint32_t sv = lane0_u32(sv0);
		const bool found = (w_word >> 24) == (t & ((1ull << 40) - 1));
		if (!found) {
			if (sv || __builtin_amdgcn_s_memrealtime() > t_end)
				break; /* stopped, or the lifetime is over */
			__builtin_amdgcn_s_sleep(1);
			continue;
		}
		const uint32_t nw = (uint32_t)(w_word >> 11) & 0x1FFF, fl = (uint32_t)(w_word >> 7) & 0xF;
		const uint32_t img = (uint32_t)(w_word >> 6) & 1, img_seq = (uint32_t)w_word & 63;
		const bool live = (uint32_t)lane < nw;
		const bool rok = sp && q[0].x == rstamp && q[1].x == rstamp && q[2].x == rstamp && q[3].x == rstamp;
		const bool fresh = !live || (rec ? rok : sp && (ev & ~kLoopOffMask) == stamp);
		const bool early = spec && nw <= 64 && __all(fresh);
		const uint64_t hit = L.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
		const uint32_t kind = early ? kLoopPollEarly : (sp && nw <= 64) ? kLoopPollStale : kLoopPollLate;
		const uint32_t polls_used = npoll;
		Mbox64 &m = me.mbox[mb]; /* free: waited for after the last post */
		if (img_seq != cur_seq) { /* this burst's table snapshot: copied into LDS */
			const uint8_t *ib = L.img[img];
			const uint32_t bytes = gcl::ld_sys32(ib);
			const __amdgpu_buffer_rsrc_t irs = gcl::host_rsrc(ib, 64 + (uint64_t)bytes);
			uint32_t *t32 = (uint32_t *)cb;
			for (uint32_t o = 16 * lane; o < 64 + bytes; o += 4 * 16 * 64) {
				gcl::u32x4 x[4];
#pragma unroll
				for (int j = 0; j < 4; j++)
					x[j] = __builtin_amdgcn_raw_buffer_load_b128(irs, (int)(o + 1024 * j), 0, gcl::kSysAux);
#pragma unroll
				for (int j = 0; j < 4; j++)
#pragma unroll
					for (int d = 0; d < 4; d++)
						if (o + 1024 * j + 4 * d < 64 + bytes)
							t32[(o + 1024 * j) / 4 + d] = x[j][d];
			}
			/* the copy before its reads */
			__builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup", "local");
			const LoopImgHdr *ih = (const LoopImgHdr *)cb;
			const uint8_t *tab = cb + 64;
			k.ipt_mask = lane0_u32(ih->ipt_mask);
			k.ipt_seed = lane0_u32(ih->ipt_seed);
			tb.ipt = (const uint2 *)tab;
			tb.rtab = (const RtEntry *)(tab + lane0_u32(ih->off_rt));
			tb.flow = tab + lane0_u32(ih->off_flow);
			tb.toep = (const uint32_t *)(tab + lane0_u32(ih->off_toep));
			tb.seed = (const uint32_t *)(tab + lane0_u32(ih->off_seed));
			tb.crc = (const uint32_t *)(tab + lane0_u32(ih->off_crc));
			cur_seq = img_seq;
		}
		/* this lane's packet in registers: its header words and side fields */
		HdrWords hw;
		uint64_t off = 0;
		uint32_t olf = 0, rss = 0, fdir = 0, hint = 0;
		if (rec) {
			if (!early && live) { /* the records after the word: a second round trip */
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const auto v = __builtin_amdgcn_raw_buffer_load_b128(
					        srs, (int)(L.off_hdr + L.rec_plane * j + 16 * lane), 0, gcl::kSysAux);
					q[j] = make_uint4(v[0], v[1], v[2], v[3]);
				}
			}
			hw.d3 = q[0].y, hw.d5 = q[0].z, hw.d6 = q[0].w, hw.d7 = q[1].y;
			hw.d8 = q[1].z, hw.d9 = q[1].w, hw.d10 = q[2].y;
			off = (uint64_t)(q[3].z & 0xFF) << 32 | q[3].y;
			olf = (q[3].z >> 8) & 0xFF;
			rss = q[2].z;
			fdir = q[2].w;
			hint = q[3].w;
		} else {
			uint4 r[4] = {};
			uint32_t olw = 0;
			if (live) {
				/* the offset first (a late burst's own round trip); then the
				 * side arrays and the frames, all in flight together.  The
				 * side loads issued between the offset's load and its use
				 * made that use wait for them as well (vmcnt counts in
				 * order, and the early path shares the use): two round trips */
				const uint64_t ent = early ? ev : gcl::ld_sys64(slot + L.off_offs + 8 * lane);
				off = ent & kLoopOffMask;
				/* keeps the side loads below the offset's use (the scheduler
				 * would hoist them above it, and its wait with them) */
				asm volatile("" : : "v"((uint32_t)off), "v"((uint32_t)(off >> 32)) : "memory");
				if (fl & GCL_LOOP_F_OLF)
					olw = gcl::ld_sys32(slot + L.off_olf + (lane & ~3));
				if (fl & GCL_LOOP_F_RSS)
					rss = gcl::ld_sys32(slot + L.off_rss + 4 * lane);
				if (fl & GCL_LOOP_F_FDIR)
					fdir = gcl::ld_sys32(slot + L.off_fdir + 4 * lane);
				if (fl & GCL_LOOP_F_HINT)
					hint = gcl::ld_sys32(slot + L.off_hint + 4 * lane);
#pragma unroll
				for (int j = 0; j < 4; j++) {
					if (L.off_hdr) { /* granules inlined in the slot by the host */
						const auto v = __builtin_amdgcn_raw_buffer_load_b128(
						        srs, (int)(L.off_hdr + 64 * lane + 16 * j), 0, gcl::kSysAux);
						r[j] = make_uint4(v[0], v[1], v[2], v[3]);
					} else {
						r[j] = gcl::load16_host(frs, L.frames, L.frames_len, off + 16 * (uint64_t)j);
					}
				}
			}
			olf = (olw >> (8 * (lane & 3))) & 0xFF;
			hw.d3 = r[0].w, hw.d5 = r[1].y, hw.d6 = r[1].z, hw.d7 = r[1].w;
			hw.d8 = r[2].x, hw.d9 = r[2].y, hw.d10 = r[2].z;
		}
		if (L.prefetch && polls_used == 1) {
			/* The next ticket's poll now, with this burst's fields in
			 * registers: its round trip runs while this burst is
			 * classified and its records stored, rather than after.
			 * Nothing below waits on memory loads (the lean path reads
			 * LDS), so the poll's loads hold no wait here; it is used,
			 * whatever it finds, as the next ticket's first poll.  Only
			 * while the host is ahead (this burst was there at the first
			 * poll): a worker that has caught up would sample the next
			 * slot too early and set every later sample a round trip
			 * off (8 x 16 records 139-155 -> 93-112 Mpkt/s without this
			 * condition, profiles/r05_prefetch_ab.jsonl). */
			const uint64_t t2 = lane0_u64(L.t0 + blockIdx.x + 1 + (kt + 1) * L.workers);
			uint8_t *slot2 = L.slots + ((t2 - 1) & (L.nslots - 1)) * (uint64_t)L.slot_bytes;
			const __amdgpu_buffer_rsrc_t srs2 = gcl::host_rsrc(slot2, L.slot_bytes);
			pis = __builtin_amdgcn_s_memrealtime();
			psp = spec;
			pw = gcl::ld_sys64(&((LoopSlotHdr *)slot2)->word);
			pev = psp && !rec ? gcl::ld_sys64(slot2 + L.off_offs + 8 * lane) : 0;
#pragma unroll
			for (int j = 0; j < 4; j++)
				pq[j] = make_uint4(0, 0, 0, 0);
			if (psp && rec) {
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const auto v = __builtin_amdgcn_raw_buffer_load_b128(
					        srs2, (int)(L.off_hdr + L.rec_plane * j + 16 * lane), 0, gcl::kSysAux);
					pq[j] = make_uint4(v[0], v[1], v[2], v[3]);
				}
			}
			pf = true;
		}
		const uint64_t t_data = L.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
		me.offs[lane] = off;
		me.fdir[lane] = fdir;
		me.hint[lane] = hint;
		k.olflags = (fl & GCL_LOOP_F_OLF) ? (const uint8_t *)me.hint : nullptr; /* read via pre */
		k.rss = (fl & GCL_LOOP_F_RSS) ? me.hint : nullptr;                      /* read via pre */
		k.fdir = (fl & GCL_LOOP_F_FDIR) ? me.fdir : nullptr;
		k.dst_hint = (fl & GCL_LOOP_F_HINT) ? me.hint : nullptr;
		const uint32_t pre[2] = {olf, rss};
		Counters cnt = {0, 0, 0, 0};
		uint64_t t_cls = 0, t_st = 0;
		/* plain IPv4 only (and nothing that needs the general path): lean */
		const uint32_t lflags = (fl & GCL_LOOP_F_OLF) ? olf : k.default_flags;
		const bool plain = !live || ((hw.d3 & 0x000FFFFF) == 0x00050008 && !(lflags & GCL_F_FDIR_ID));
		const bool lean = L.lean && !(fl & GCL_LOOP_F_HINT) && !L.off_trans && __all(plain);
		if (live) {
			const uint64_t v = lean ? classify_lean<MODE>(k, hw, tb, lflags, rss, m.p, lane, cnt)
			                        : classify_core<MODE, true, true, true, 0, false>(
			                                  k, hw, nullptr, lane, (uint64_t)lane, tb, m.p, cnt, 0, 64, pre);
			if (L.stamps)
				t_cls = __builtin_amdgcn_s_memrealtime();
			const bool v4 = k.cflags & GCL_CFG_VERDICT4, v2 = k.cflags & GCL_CFG_VERDICT2;
			const bool v1 = k.cflags & GCL_CFG_VERDICT1;
			const uint32_t hsh = v4 || v2 || v1 ? 0u : (uint32_t)v;
			const uint32_t vlo = v1 ? (uint32_t)(uint8_t)v : v2 ? (uint32_t)(uint16_t)v
			                   : v4 ? (uint32_t)v : (uint32_t)(v >> 32);
			if (L.off_trans) { /* before the record: the host checks both tickets */
				const uint2 tr = me.trans[lane];
				const gcl::u32x4 x = {tr.x, tr.y, (uint32_t)t, (uint32_t)(t >> 32)};
				__builtin_amdgcn_raw_buffer_store_b128(x, srs, (int)(L.off_trans + 16 * lane), 0,
				                                       gcl::kSysAux);
			}
			const gcl::u32x4 x = {hsh, vlo, (uint32_t)t, (uint32_t)(t >> 32)};
			__builtin_amdgcn_raw_buffer_store_b128(x, srs, (int)(L.off_verd + sizeof(LoopRec) * lane), 0,
			                                       gcl::kSysAux);
			if (L.stamps)
				t_st = __builtin_amdgcn_s_memrealtime();
		}
		/* one packet per lane: each counter is 0 or 1 per lane, a ballot
		 * (no cross-lane shuffles, which are LDS round trips) */
		const uint32_t c_ft = (uint32_t)__popcll(__ballot(cnt.flowtag != 0));
		const uint32_t c_hm = (uint32_t)__popcll(__ballot(cnt.hashmiss != 0));
		const uint32_t c_ur = (uint32_t)__popcll(__ballot(cnt.unreg != 0));
		const uint32_t c_uh = (uint32_t)__popcll(__ballot(cnt.unhandled != 0));
		if (lane == 0) {
			m.t = t;
			m.n = nw;
			m.kind = kind;
			m.lean = lean;
			m.cnt[0] = c_ft;
			m.cnt[1] = c_hm;
			m.cnt[2] = c_ur;
			m.cnt[3] = c_uh;
			if (L.stamps) {
				m.st[0] = (uint32_t)hit;
				m.st[1] = (uint32_t)(hit >> 32);
				m.st[2] = (uint32_t)(hit - t_issue);
				m.st[3] = polls_used;
				m.st[4] = (uint32_t)(t_data - hit);
				m.st[5] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - hit);
				m.st[6] = (uint32_t)(t_cls - hit);
				m.st[7] = (uint32_t)(t_st - hit);
			}
		}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
		if (lane == 0)
			__hip_atomic_store(&m.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		mb ^= 1;
		/* the mailbox the next burst will be posted to, freed by the writer
		 * long before: waited for here, not after the next hit */
		while (__hip_atomic_load(&me.mbox[mb].flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
			__builtin_amdgcn_s_sleep(1);
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
		if (ph_max) {
			/* The poll-phase delay, updated here, after the records went
			 * out: its LoopParams reads are scalar loads the compiler
			 * re-issues from the kernel arguments, which right after the
			 * hit cost the burst ~0.1 us (profiles/r05_stages_phase.jsonl).
			 * Found whole by the first poll: it may have waited longer
			 * than needed, so wait a step less next time; found by the
			 * second, or with its records still being written: the first
			 * poll was early, a step more.  Later finds are sparse
			 * traffic, whose phase is its own: no change.  The steps are
			 * asymmetric, so about phase_down / (phase_up + phase_down)
			 * of closed-loop bursts pay the round trip a miss costs.  (A
			 * loop without the speculative window -- inline headers,
			 * gcl_tune.loop_spec 0 -- finds every burst "late": on time
			 * when at the first poll.) */
			if (polls_used == 1 && kind != kLoopPollStale)
				dly = dly > ph_dn ? dly - ph_dn : 0;
			else if (polls_used <= 2)
				dly = dly + ph_up < ph_max ? dly + ph_up : ph_max;
		}
		/* the next ticket, its own spec window */
		kt++;
		npoll = 0;
		t_done = __builtin_amdgcn_s_memrealtime();
		spec_end = (pf ? pis : t_done) + L.spec_ticks;
	}
	/* the writer drains what was posted, then leaves; the host stops
	 * publishing on this word (one it reads without a HIP call per burst) */
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
	if (lane == 0) {
		__hip_atomic_fetch_add(&ctl->exited, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
		gcl::st_sys32(L.exited, 1);
	}
}

} // namespace gclk

using namespace gclk;

/* ==========================================================================
 * Persistent rx loop (host side).  Ring slots and table images live in
 * coherent, mapped host memory; the CPU publishes a slot with a release store
 * of its ticket word, the kernel answers with one 16-B record per packet that
 * carries the ticket.
 */

/* NUMA node of the page holding @p (move_pages with no target nodes only
 * reports), -1 if unknown */
static int page_node(const void *p)
{
	void *pg = (void *)((uintptr_t)p & ~(uintptr_t)4095);
	int status = -1;
	if (!p || syscall(SYS_move_pages, 0, 1ul, &pg, nullptr, &status, 0) != 0)
		return -1;
	return status;
}

/* the loop's control page: [0] stop, [1] exited, [8, 16) where, then 4
 * poll counters per worker (gcl_rxloop_poll_stats) */
constexpr uint32_t kLoopCtlPolls = 64;
constexpr size_t kLoopCtlBytes = 4 * (kLoopCtlPolls + 4 * 64);

struct gcl_rxloop {
	gcl_ctx *c;
	hipStream_t st;
	uint8_t *slots;          /* host view */
	uint8_t *img[2];         /* host views: LoopImgHdr + image */
	uint32_t *ctl;           /* stop flag */
	LoopParams lp;
	uint32_t max_burst, vbytes;
	uint64_t next;           /* last ticket issued */
	uint32_t cur_img, img_seq;
	uint64_t img_last[2];    /* last ticket that read image i */
	std::vector<uint64_t> retired; /* per slot: last ticket the host collected */
	const uint8_t *region;         /* host view, for GCL_LOOP_INLINE_HDRS */
	uint64_t region_len;
	bool ended;              /* the kernel has finished (hipStreamQuery) */
	bool left;               /* some worker has left: submit no more */
	bool k64;                /* rxloop64_kernel (bursts <= 64) */
	bool debug;              /* gcl_tune.debug at start */
	uint32_t rec_pf;         /* header prefetch distance of loop_write_records */
	bool slot_pf;            /* loop_await prefetches the next slot for writing */
	uint64_t slot_pf_t;      /* ... once per ticket: the last ticket it did so for */
};

static uint64_t now_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static LoopSlotHdr *loop_slot(gcl_rxloop *L, uint64_t t)
{
	return (LoopSlotHdr *)(L->slots + ((t - 1) % L->lp.nslots) * L->lp.slot_bytes);
}

static bool loop_ended(gcl_rxloop *L)
{
	if (!L->ended && hipStreamQuery(L->st) != hipErrorNotReady)
		L->ended = true;
	return L->ended;
}

/* The submit path's check, without a HIP call (hipStreamQuery cost ~100 ns
 * per burst): a worker that leaves raises ctl[1], and no burst is published
 * after that.  Bursts already published may still be classified by the
 * other workers, so only loop_ended (the kernel finished) lets a wait give
 * up with -ESHUTDOWN; a kernel that died without raising ctl[1] is caught by
 * loop_await's periodic loop_ended. */
static bool loop_left(gcl_rxloop *L)
{
	if (!L->left && (L->ended || __atomic_load_n(&L->ctl[1], __ATOMIC_ACQUIRE)))
		L->left = true;
	return L->left;
}

static const LoopRec *loop_recs(gcl_rxloop *L, LoopSlotHdr *h)
{
	return (const LoopRec *)((const uint8_t *)h + L->lp.off_verd);
}

/* Every verdict record of ticket @t's burst carries @t (its slot must still
 * hold @t).  The last records usually land last, so scan backwards. */
static bool burst_complete(gcl_rxloop *L, uint64_t t)
{
	LoopSlotHdr *h = loop_slot(L, t);
	const uint32_t n = (uint32_t)(h->word >> 11) & 0x1FFF;
	const LoopRec *r = loop_recs(L, h);
	for (uint32_t i = n; i-- > 0;)
		if (__atomic_load_n(&r[i].ticket, __ATOMIC_ACQUIRE) != t)
			return false;
	if (L->lp.off_trans) { /* the transport hashes land by stores of their own */
		const LoopRec *tr = (const LoopRec *)((const uint8_t *)h + L->lp.off_trans);
		for (uint32_t i = n; i-- > 0;)
			if (__atomic_load_n(&tr[i].ticket, __ATOMIC_ACQUIRE) != t)
				return false;
	}
	return true;
}

static bool ticket_done(gcl_rxloop *L, uint64_t t)
{
	if (t == 0 || t + L->lp.nslots <= L->next)
		return true; /* never issued, or its slot has been reused since */
	return burst_complete(L, t);
}

/* Build the current tables into image buffer @i (host memory). */
static int loop_write_image(gcl_rxloop *L, int i)
{
	gcl_ctx *c = L->c;
	if (hipEventSynchronize(c->staging_free) != hipSuccess)
		return -EIO;
	const uint32_t bytes = build_image(c);
	if (!bytes)
		return -ENOSPC;
	if (bytes > kLdsTableBudget)
		return -E2BIG;
	LoopImgHdr hdr = {};
	hdr.bytes = bytes;
	hdr.ipt_mask = c->ipt_slots / 2 - 1;
	hdr.ipt_seed = c->ipt_seed;
	hdr.off_rt = c->off_rt;
	hdr.off_flow = c->off_flow;
	hdr.off_toep = c->off_toep;
	hdr.off_seed = c->off_seed;
	hdr.off_crc = c->off_crc;
	memcpy(L->img[i] + 64, c->staging, bytes);
	memcpy(L->img[i], &hdr, sizeof(hdr));
	c->loop_dirty = false;
	return 0;
}

/* bursts of <= 64 packets (@k64): rxloop64_kernel, a poller wave and the
 * writer, no barrier; else the general loop (bursts past 64, or
 * gcl_tune.loop64 0: the tests' way to run short bursts through it) */
template <int MODE>
static hipError_t loop_launch(const LoopParams &lp, bool k64, hipStream_t s)
{
	const void *fn = k64 ? (const void *)rxloop64_kernel<MODE> : (const void *)rxloop_kernel<MODE>;
	const uint32_t lds = k64 ? loop64_lds(64 + kLdsTableBudget)
	                         : kLoopFixedLds + ((lp.max_rt + 3) & ~3u) * 4 + kLdsTableBudget;
	if (lds > 64 * 1024) {
		const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
		                                         160 * 1024);
		if (e != hipSuccess)
			return e;
	}
	if (k64)
		hipLaunchKernelGGL(rxloop64_kernel<MODE>, dim3(lp.workers), dim3(128), lds, s, lp);
	else
		hipLaunchKernelGGL(rxloop_kernel<MODE>, dim3(lp.workers), dim3(256), lds, s, lp);
	return hipGetLastError();
}

extern "C" int gcl_rxloop_start(struct gcl_ctx *c, const struct gcl_rxloop_cfg *cfg,
                                struct gcl_rxloop **out)
{
	if (!c || !cfg || !out || !cfg->region || !cfg->region_len || cfg->slots < 2 ||
	    cfg->slots > 1024 || (cfg->slots & (cfg->slots - 1)) || !cfg->max_burst ||
	    cfg->max_burst > 4096 || !cfg->workers || cfg->workers > 64 || !cfg->lifetime_ms ||
	    cfg->lifetime_ms > 600000)
		return -EINVAL;
	if ((cfg->flags & ~(uint32_t)(GCL_LOOP_INLINE_HDRS | GCL_LOOP_HDR_RECORDS | GCL_LOOP_STAMPS)) ||
	    (cfg->flags & GCL_LOOP_INLINE_HDRS && cfg->flags & GCL_LOOP_HDR_RECORDS))
		return -EINVAL;
	if (cfg->region_len > kLoopOffMask - GCL_HDR_GRANULE)
		return -EINVAL; /* offsets share their slot entry with a stamp */
	if (c->loop)
		return -EBUSY;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	void *frames_d = mapped(cfg->region);
	if (!frames_d)
		return -EINVAL; /* not registered */
	gcl_rxloop *L = new (std::nothrow) gcl_rxloop();
	if (!L)
		return -ENOMEM;
	L->c = c;
	L->region = (const uint8_t *)cfg->region;
	L->region_len = cfg->region_len;
	const struct gcl_tune &tu = c->tune;
	{
		const uint64_t t0 = tu.loop_t0 / cfg->slots * cfg->slots; /* tests: start near a stamp wrap */
		L->lp.t0 = t0;
		L->next = t0;
		L->retired.assign(cfg->slots, t0);
	}
	L->max_burst = cfg->max_burst;
	L->debug = tu.debug != 0;
	L->rec_pf = (uint32_t)tuned(tu.rec_prefetch, (int32_t)kRecPrefetch);
	L->slot_pf = tuned(tu.slot_prefetch, (int32_t)kDefaultSlotPrefetch) != 0;
	L->vbytes = verdict_bytes(c);
	const uint64_t mb = align16(cfg->max_burst);
	LoopParams &lp = L->lp;
	lp.off_offs = 64;
	lp.off_olf = lp.off_offs + 8 * mb;
	lp.off_rss = lp.off_olf + mb;
	lp.off_fdir = lp.off_rss + 4 * mb;
	lp.off_hint = lp.off_fdir + 4 * mb;
	lp.off_verd = lp.off_hint + 4 * mb;
	lp.hdr_rec = (cfg->flags & GCL_LOOP_HDR_RECORDS) != 0;
	lp.stamps = (cfg->flags & GCL_LOOP_STAMPS) != 0;
	lp.lean = (uint32_t)tuned(tu.loop_lean, kDefaultLoopLean);
	lp.off_hdr = (cfg->flags & (GCL_LOOP_INLINE_HDRS | GCL_LOOP_HDR_RECORDS))
	                     ? lp.off_verd + sizeof(LoopRec) * mb : 0;
	lp.rec_plane = (uint32_t)(16 * mb);
	lp.spec = (!lp.off_hdr || lp.hdr_rec) && cfg->max_burst <= 64;
	lp.spec_ticks = cfg->workers <= kLoopSpecIdleWorkers ? kLoopSpecIdle : kLoopSpecTicks;
	L->k64 = cfg->max_burst <= 64 && tuned(tu.loop64, 1); /* 0: tests, the general loop */
	lp.spec_ticks = (uint32_t)tuned(tu.loop_spec, (int32_t)lp.spec_ticks);
	/* the poll-phase delay: closed-loop submitters are the few-worker case;
	 * a deep pipeline finds its bursts queued */
	lp.phase_max = cfg->workers <= kLoopSpecIdleWorkers ? kDefaultLoopPhaseMax : 0;
	lp.phase_up = kDefaultLoopPhaseUp;
	lp.phase_down = kDefaultLoopPhaseDown;
	if (tu.loop_phase_max != GCL_TUNE_AUTO) { /* all three set (gcl_ctx_tune) */
		lp.phase_max = (uint32_t)tu.loop_phase_max;
		lp.phase_up = (uint32_t)tu.loop_phase_up;
		lp.phase_down = (uint32_t)tu.loop_phase_down;
	}
	/* the next ticket's poll during classification: for workers that find
	 * their bursts queued (more than the closed-loop few) */
	lp.prefetch = (uint32_t)tuned(tu.loop_prefetch,
	                              cfg->workers > kLoopSpecIdleWorkers && !lp.hdr_rec ? kDefaultLoopPrefetch : 0);
	{
		const uint64_t end = lp.off_verd + sizeof(LoopRec) * mb + (lp.off_hdr ? GCL_HDR_GRANULE * mb : 0);
		lp.off_trans = (c->cfg.flags & GCL_CFG_TRANS_HASH) ? (uint32_t)end : 0;
		lp.slot_bytes = (end + (lp.off_trans ? 16 * mb : 0) + 255) & ~255ull;
	}
	lp.nslots = cfg->slots;
	lp.workers = cfg->workers;
	lp.lifetime_ticks = (uint64_t)cfg->lifetime_ms * 100000ull;
	lp.frames = (const uint8_t *)frames_d;
	lp.frames_len = cfg->region_len;
	lp.counts = (unsigned long long *)cfg->counts;
	lp.stats = (unsigned long long *)cfg->stats;
	lp.max_rt = c->cfg.max_runtimes;
	lp.cflags = kernel_cflags(c);
	lp.default_flags = c->cfg.default_olflags;
	const unsigned hf = hipHostMallocCoherent | hipHostMallocMapped;
	int ret = -ENOMEM;
	void *d;
	if (hipHostMalloc((void **)&L->slots, lp.nslots * lp.slot_bytes, hf) != hipSuccess ||
	    hipHostMalloc((void **)&L->img[0], 64 + c->image_cap, hf) != hipSuccess ||
	    hipHostMalloc((void **)&L->img[1], 64 + c->image_cap, hf) != hipSuccess ||
	    hipHostMalloc((void **)&L->ctl, kLoopCtlBytes, hf) != hipSuccess)
		goto fail;
	memset(L->slots, 0, lp.nslots * lp.slot_bytes);
	memset(L->ctl, 0, kLoopCtlBytes);
	if (tu.debug)
		fprintf(stderr, "gcl_rxloop_start: NUMA node of slots %d, image %d, ctl %d, region %d\n",
		        page_node(L->slots), page_node(L->img[0]), page_node(L->ctl),
		        page_node(cfg->region));
	ret = loop_write_image(L, 0);
	if (ret)
		goto fail;
	L->cur_img = 0;
	L->img_seq = 1;
	ret = -EIO;
	if (hipHostGetDevicePointer(&d, L->slots, 0) != hipSuccess)
		goto fail;
	lp.slots = (uint8_t *)d;
	for (int i = 0; i < 2; i++) {
		if (hipHostGetDevicePointer(&d, L->img[i], 0) != hipSuccess)
			goto fail;
		lp.img[i] = (const uint8_t *)d;
	}
	if (hipHostGetDevicePointer(&d, L->ctl, 0) != hipSuccess)
		goto fail;
	lp.stop = (const uint32_t *)d;
	lp.where = (uint32_t *)d + 8;
	lp.exited = (uint32_t *)d + 1;
	lp.polls = (uint32_t *)d + kLoopCtlPolls;
	/* the caller's counts / stats are typically zeroed on the default stream
	 * just before (a hipMemsetAsync, torch.zeros): the loop runs on a
	 * non-blocking stream of its own, so that work is waited for here, or the
	 * first bursts' counts could land before the zeroing (the loop's rx_burst
	 * counters read short) */
	if (hipStreamSynchronize(nullptr) != hipSuccess)
		goto fail;
	if (hipStreamCreateWithFlags(&L->st, hipStreamNonBlocking) != hipSuccess)
		goto fail;
	{
		hipError_t e = c->cfg.hash_mode == GCL_HASH_NIC ? loop_launch<GCL_HASH_NIC>(lp, L->k64, L->st)
		             : c->cfg.hash_mode == GCL_HASH_JENKINS ? loop_launch<GCL_HASH_JENKINS>(lp, L->k64, L->st)
		             : loop_launch<GCL_HASH_TOEPLITZ>(lp, L->k64, L->st);
		if (e != hipSuccess) {
			(void)hipStreamDestroy(L->st);
			L->st = nullptr;
			goto fail;
		}
	}
	c->loop = L;
	*out = L;
	return 0;
fail:
	(void)hipHostFree(L->slots);
	(void)hipHostFree(L->img[0]);
	(void)hipHostFree(L->img[1]);
	(void)hipHostFree(L->ctl);
	delete L;
	return ret;
}

/* GCL_LOOP_HDR_RECORDS: packet i of ticket @t's burst as one stamped 64-B
 * record (the layout above loop_rec_stamp), every 16-B chunk written by one aligned
 * 16-B store so the GPU never sees a chunk half-written.  The core reads the
 * header bytes rx_one_pkt reads, prefetching two frames ahead as rx_burst
 * does (rx.c:281-285); bytes past the region read 0. */
typedef uint32_t u32x4_h __attribute__((vector_size(16), aligned(16)));

static void loop_write_records(gcl_rxloop *L, uint64_t t, uint8_t *dst, uint32_t n,
                               const uint64_t *offs, const uint8_t *olflags, const uint32_t *rss,
                               const uint32_t *fdir_hi, const uint32_t *dst_hint)
{
	const uint32_t S = loop_rec_stamp(t, L->lp.nslots);
	/* four planes of 16-B chunks, chunk j of packet i at j * plane + 16 i: a
	 * poll's 64 lanes read each plane as one contiguous 1 KiB (16 64-B PCIe
	 * reads a plane, not 64 16-B ones) */
	const size_t P = L->lp.rec_plane / sizeof(u32x4_h);
	volatile u32x4_h *q = (volatile u32x4_h *)dst;
	/* Headers a NIC has just written miss to DRAM: the core keeps
	 * L->rec_pf of them in flight (bytes 12 and 39, the two ends of what
	 * every packet reads; gcl_tune.rec_prefetch, kRecPrefetch by default)
	 * instead of rx.c's two, which pays one DRAM latency per two packets.
	 * (With cache-hot headers distances 2 and 6 measured the same:
	 * profiles/r03_hdr_records_prefetch_ab.jsonl.) */
	auto prefetch_hdr = [&](uint32_t i) {
		if (offs[i] < L->region_len && L->region_len - offs[i] >= 40) {
			__builtin_prefetch(L->region + offs[i] + 12, 0, 3);
			__builtin_prefetch(L->region + offs[i] + 39, 0, 3);
		}
	};
	const uint32_t pf = L->rec_pf;
	for (uint32_t i = 0; i < n && i < pf; i++)
		prefetch_hdr(i);
	for (uint32_t i = 0; i < n; i++, q++) {
		if (i + pf < n)
			prefetch_hdr(i + pf);
		const uint64_t o = offs[i];
		/* frame dwords 3-6 and 7-10 (bytes 12-43) in two registers, shuffled
		 * into the chunks without a trip through memory */
		u32x4_h v0, v1;
		if (o < L->region_len && L->region_len - o >= 44) {
			memcpy(&v0, L->region + o + 12, 16);
			uint32_t w[4];
			memcpy(w, L->region + o + 28, 12);
			/* d10 (bytes 40-43) is read for ARP's target IP (rx.c:165-167)
			 * and the ports behind IPv4 options; a plain IPv4 header (IHL 5,
			 * the kernels' own test) never reads it, so neither does the
			 * core: in the reference's pool (data at element + 344,
			 * defs.h:503-506) byte 40 starts the next cache line, a second
			 * DRAM miss per packet once the NIC has written the frame */
			w[3] = (v0[0] & 0x000FFFFFu) == 0x00050008u ? 0u : ({
				uint32_t d;
				memcpy(&d, L->region + o + 40, 4);
				d;
			});
			memcpy(&v1, w, 16);
		} else {
			uint8_t b[32] = {0};
			if (o < L->region_len && L->region_len - o > 12)
				memcpy(b, L->region + o + 12, L->region_len - o - 12);
			memcpy(&v0, b, 16);
			memcpy(&v1, b + 16, 16);
		}
		const uint64_t off = std::min<uint64_t>(o, kLoopOffMask);
		const uint32_t olf = olflags ? olflags[i] : 0;
		const u32x4_h sv = {S, S, S, S};
		const u32x4_h side = {S, 0, rss ? rss[i] : 0u, fdir_hi ? fdir_hi[i] : 0u};
		const u32x4_h c0 = __builtin_shufflevector(v0, sv, 4, 0, 2, 3);   /* S d3 d5 d6 */
		const u32x4_h c1 = __builtin_shufflevector(v1, sv, 4, 0, 1, 2);   /* S d7 d8 d9 */
		const u32x4_h c2 = __builtin_shufflevector(side, v1, 0, 7, 2, 3); /* S d10 rss fdir */
		const u32x4_h c3 = u32x4_h{S, (uint32_t)off, (uint32_t)(off >> 32) | olf << 8,
		                           dst_hint ? dst_hint[i] : 0u};
		/* (non-temporal stores, past the core's caches, measured no
		 * different: profiles/r04_loop_nt_ab.jsonl) */
		q[0] = c0;
		q[P] = c1;
		q[2 * P] = c2;
		q[3 * P] = c3;
	}
	/* records past n keep older stamps; rewrite them now and then so that
	 * none is ever 2^31 uses stale (loop_stamp's rule for the offsets) */
	if (((t - 1) / L->lp.nslots) % kLoopRefresh == kLoopRefresh - 1)
		for (uint32_t i = n; i < L->max_burst; i++, q++)
			for (int j = 0; j < 4; j++)
				q[j * P] = u32x4_h{S, 0, 0, 0};
}

/* Ticket @t's burst into slot @s as stamped offsets, the optional header
 * granules (GCL_LOOP_INLINE_HDRS) and the side arrays. */
static void loop_write_arrays(gcl_rxloop *L, uint64_t t, uint8_t *s, uint32_t n,
                              const uint64_t *offs, const uint8_t *olflags, const uint32_t *rss,
                              const uint32_t *fdir_hi, const uint32_t *dst_hint)
{
	{ /* offsets stamped with the slot's use count (loop_stamp) */
		uint64_t *so = (uint64_t *)(s + L->lp.off_offs);
		const uint64_t st = loop_stamp(t, L->lp.nslots);
		for (uint32_t i = 0; i < n; i++) /* past the region either way: reads 0 */
			so[i] = std::min<uint64_t>(offs[i], kLoopOffMask) | st;
		if ((((t - 1) / L->lp.nslots) % kLoopRefresh) == kLoopRefresh - 1)
			for (uint32_t i = n; i < L->max_burst; i++)
				so[i] = st;
	}
	if (L->lp.off_hdr) { /* the header granules ride in the slot; past the region: 0 */
		uint8_t *hd = s + L->lp.off_hdr;
		for (uint32_t i = 0; i < n; i++, hd += GCL_HDR_GRANULE) {
			const uint64_t o = offs[i];
			/* no o + granule: an offset near UINT64_MAX must not wrap past the check */
			const uint64_t k = o < L->region_len ? std::min<uint64_t>(L->region_len - o, GCL_HDR_GRANULE) : 0;
			if (k)
				memcpy(hd, L->region + o, k);
			if (k < GCL_HDR_GRANULE)
				memset(hd + k, 0, GCL_HDR_GRANULE - k);
		}
	}
	if (olflags)
		memcpy(s + L->lp.off_olf, olflags, n);
	if (rss)
		memcpy(s + L->lp.off_rss, rss, 4ull * n);
	if (fdir_hi)
		memcpy(s + L->lp.off_fdir, fdir_hi, 4ull * n);
	if (dst_hint)
		memcpy(s + L->lp.off_hint, dst_hint, 4ull * n);
}

extern "C" int64_t gcl_rxloop_submit(struct gcl_rxloop *L, uint32_t n, const uint64_t *offs,
                                     const uint8_t *olflags, const uint32_t *rss,
                                     const uint32_t *fdir_hi, const uint32_t *dst_hint)
{
	if (!L || !n || n > L->max_burst || !offs)
		return -EINVAL;
	if (loop_left(L))
		return -ESHUTDOWN;
	const uint64_t t = L->next + 1;
	/* a slot is reused only after the host collected its previous burst */
	if (t > L->lp.nslots && L->retired[(t - 1) % L->lp.nslots] < t - L->lp.nslots)
		return -EAGAIN;
	if (L->c->loop_dirty) {
		/* the other image buffer: wait for the last burst that read it */
		const int x = L->cur_img ^ 1;
		while (!ticket_done(L, L->img_last[x]))
			if (loop_ended(L))
				return -ESHUTDOWN;
		const int ret = loop_write_image(L, x);
		if (ret)
			return ret;
		L->cur_img = x;
		L->img_seq++;
	}
	LoopSlotHdr *h = loop_slot(L, t);
	uint8_t *s = (uint8_t *)h;
	const uint32_t fl = (olflags ? GCL_LOOP_F_OLF : 0) | (rss ? GCL_LOOP_F_RSS : 0) |
	                    (fdir_hi ? GCL_LOOP_F_FDIR : 0) | (dst_hint ? GCL_LOOP_F_HINT : 0);
	if (L->lp.hdr_rec) /* everything rides in the records */
		loop_write_records(L, t, s + L->lp.off_hdr, n, offs, olflags, rss, fdir_hi, dst_hint);
	else
		loop_write_arrays(L, t, s, n, offs, olflags, rss, fdir_hi, dst_hint);
	__atomic_store_n(&h->word, loop_word(t, n, fl, L->cur_img, L->img_seq), __ATOMIC_RELEASE);
	L->img_last[L->cur_img] = t;
	L->next = t;
	return (int64_t)t;
}

/* The lines the next submit writes, for ownership, while a host with
 * nothing else in flight waits for ticket @t (gcl_tune.slot_prefetch): the
 * GPU's polls of a slot read it over PCIe, and a line that left the core's
 * caches that way costs a miss when the submit writes it again. */
static void prefetch_slot(gcl_rxloop *L, uint64_t t)
{
	uint8_t *s = (uint8_t *)loop_slot(L, t + 1);
	__builtin_prefetch(s, 1, 3);
	if (L->lp.hdr_rec) {
		for (uint32_t j = 0; j < 4; j++)
			for (uint32_t b = 0; b < 16 * L->max_burst; b += 64)
				__builtin_prefetch(s + L->lp.off_hdr + j * L->lp.rec_plane + b, 1, 3);
	} else {
		for (uint32_t b = 0; b < 8 * L->max_burst; b += 64)
			__builtin_prefetch(s + L->lp.off_offs + b, 1, 3);
	}
}

/* spin up to @spin_ns for ticket @t's burst: 0, -EAGAIN or -ESHUTDOWN */
static int loop_await(gcl_rxloop *L, uint64_t t, uint64_t spin_ns)
{
	if (L->slot_pf && t == L->next && L->slot_pf_t != t && !burst_complete(L, t)) {
		L->slot_pf_t = t;
		prefetch_slot(L, t);
	}
	const uint64_t t0 = spin_ns ? now_ns() : 0;
	uint32_t k = 0;
	while (!burst_complete(L, t)) {
		if (!spin_ns || (++k & 255) == 0) {
			if (loop_ended(L))
				return burst_complete(L, t) ? 0 : -ESHUTDOWN;
			if (!spin_ns || now_ns() - t0 >= spin_ns)
				return -EAGAIN;
		}
		__builtin_ia32_pause();
	}
	return 0;
}

/* Start the host's reads of the next ticket's verdict records while this
 * burst is delivered: they are lines the GPU writes into host memory, so
 * each costs a DRAM miss the first time (16 per 64-packet burst).  A line
 * fetched before the GPU writes it is simply fetched again. */
static void prefetch_next(gcl_rxloop *L, uint64_t t)
{
	if (t + 1 > L->next)
		return;
	const LoopSlotHdr *h = loop_slot(L, t + 1);
	const uint32_t n = (uint32_t)(h->word >> 11) & 0x1FFF;
	const uint8_t *r = (const uint8_t *)loop_recs(L, (LoopSlotHdr *)h);
	for (uint32_t b = 0; b < n * (uint32_t)sizeof(LoopRec); b += 64)
		__builtin_prefetch(r + b, 0, 3);
}

extern "C" int gcl_rxloop_peek(struct gcl_rxloop *L, int64_t ticket, uint64_t spin_ns,
                               const struct gcl_loop_rec **recs, uint32_t *n)
{
	if (!L || !recs || !n || ticket < 1 || (uint64_t)ticket > L->next)
		return -EINVAL;
	const uint64_t t = (uint64_t)ticket;
	if (t + L->lp.nslots <= L->next)
		return -ESTALE;
	const int r = loop_await(L, t, spin_ns);
	if (r)
		return r;
	LoopSlotHdr *h = loop_slot(L, t);
	*n = (uint32_t)(h->word >> 11) & 0x1FFF;
	*recs = (const struct gcl_loop_rec *)loop_recs(L, h);
	prefetch_next(L, t);
	return 0;
}

extern "C" int gcl_rxloop_release(struct gcl_rxloop *L, int64_t ticket)
{
	if (!L || ticket < 1 || (uint64_t)ticket > L->next)
		return -EINVAL;
	const uint64_t t = (uint64_t)ticket;
	if (t + L->lp.nslots <= L->next)
		return -ESTALE;
	/* the GPU may still be writing an incomplete burst's slot: it is not
	 * handed back for reuse until the burst is complete */
	if (!burst_complete(L, t))
		return -EAGAIN;
	uint64_t &r = L->retired[(t - 1) % L->lp.nslots];
	if (r < t)
		r = t;
	return 0;
}

extern "C" int gcl_rxloop_wait(struct gcl_rxloop *L, int64_t ticket, void *verdicts_out,
                               uint64_t spin_ns)
{
	if (!L || ticket < 1 || (uint64_t)ticket > L->next)
		return -EINVAL;
	const uint64_t t = (uint64_t)ticket;
	if (t + L->lp.nslots <= L->next)
		return -ESTALE;
	LoopSlotHdr *h = loop_slot(L, t);
	const int aw = loop_await(L, t, spin_ns);
	if (aw)
		return aw;
	prefetch_next(L, t);
	if (verdicts_out) {
		const uint32_t n = (uint32_t)(h->word >> 11) & 0x1FFF;
		const LoopRec *r = loop_recs(L, h);
		if (L->vbytes == 1) {
			for (uint32_t i = 0; i < n; i++)
				((uint8_t *)verdicts_out)[i] = (uint8_t)r[i].vlo;
		} else if (L->vbytes == 2) {
			for (uint32_t i = 0; i < n; i++)
				((uint16_t *)verdicts_out)[i] = (uint16_t)r[i].vlo;
		} else if (L->vbytes == 4) {
			for (uint32_t i = 0; i < n; i++)
				((uint32_t *)verdicts_out)[i] = r[i].vlo;
		} else {
			for (uint32_t i = 0; i < n; i++)
				((uint64_t *)verdicts_out)[i] = (uint64_t)r[i].vlo << 32 | r[i].hash;
		}
	}
	uint64_t &r = L->retired[(t - 1) % L->lp.nslots];
	if (r < t)
		r = t;
	return 0;
}

extern "C" int gcl_rxloop_trans(struct gcl_rxloop *L, int64_t ticket, struct gcl_trans *out)
{
	if (!L || !out || ticket < 1 || (uint64_t)ticket > L->next || !L->lp.off_trans)
		return -EINVAL;
	const uint64_t t = (uint64_t)ticket;
	if (t + L->lp.nslots <= L->next)
		return -ESTALE;
	if (!burst_complete(L, t))
		return -EAGAIN;
	const LoopSlotHdr *h = loop_slot(L, t);
	const uint32_t n = (uint32_t)(h->word >> 11) & 0x1FFF;
	const LoopRec *tr = (const LoopRec *)((const uint8_t *)h + L->lp.off_trans);
	for (uint32_t i = 0; i < n; i++) {
		out[i].h5 = tr[i].hash;
		out[i].h3 = tr[i].vlo;
	}
	return 0;
}

extern "C" int gcl_rxloop_stamps(struct gcl_rxloop *L, int64_t ticket, uint64_t out[8])
{
	if (!L || !out || !L->lp.stamps || ticket < 1 || (uint64_t)ticket > L->next)
		return -EINVAL;
	const uint64_t t = (uint64_t)ticket;
	if (t + L->lp.nslots <= L->next)
		return -ESTALE;
	const uint32_t *h = (const uint32_t *)loop_slot(L, t);
	const uint32_t a0 = __atomic_load_n(&h[4], __ATOMIC_ACQUIRE);
	const uint32_t b0 = __atomic_load_n(&h[8], __ATOMIC_ACQUIRE);
	const uint32_t c0 = __atomic_load_n(&h[12], __ATOMIC_ACQUIRE);
	if (a0 != (uint32_t)t || b0 != (uint32_t)t || c0 != (uint32_t)t)
		return -EAGAIN; /* posted after the records: not landed yet */
	out[0] = 10ull * __atomic_load_n(&h[5], __ATOMIC_RELAXED); /* hitting poll's round trip */
	out[1] = 10ull * __atomic_load_n(&h[6], __ATOMIC_RELAXED); /* hit -> classified */
	out[2] = 10ull * __atomic_load_n(&h[7], __ATOMIC_RELAXED); /* hit -> last record issued */
	out[3] = __atomic_load_n(&h[9], __ATOMIC_RELAXED);         /* polls of this wait */
	for (int i = 0; i < 3; i++) /* hit -> past the first three barriers, or (loop64) stages */
		out[4 + i] = 10ull * __atomic_load_n(&h[13 + i], __ATOMIC_RELAXED);
	out[7] = L->k64;
	return 0;
}

extern "C" int gcl_rxloop_poll_stats(struct gcl_rxloop *L, uint64_t out[3])
{
	if (!L || !out)
		return -EINVAL;
	out[0] = out[1] = out[2] = 0;
	for (uint32_t w = 0; w < L->lp.workers; w++)
		for (int k = 0; k < 3; k++)
			out[k] += __atomic_load_n(&L->ctl[kLoopCtlPolls + 4 * w + k], __ATOMIC_RELAXED);
	return 0;
}

extern "C" int gcl_rxloop_lean_bursts(struct gcl_rxloop *L, uint64_t *out)
{
	if (!L || !out)
		return -EINVAL;
	*out = 0;
	for (uint32_t w = 0; w < L->lp.workers; w++)
		*out += __atomic_load_n(&L->ctl[kLoopCtlPolls + 4 * w + 3], __ATOMIC_RELAXED);
	return 0;
}

extern "C" int gcl_rxloop_stop(struct gcl_rxloop *L)
{
	if (!L)
		return -EINVAL;
	__atomic_store_n(L->ctl, 1u, __ATOMIC_RELEASE);
	const hipError_t e = hipStreamSynchronize(L->st);
	if (L->debug) {
		fprintf(stderr, "gcl_rxloop_stop: workers on XCC");
		for (int b = 0; b < 8; b++)
			if (L->ctl[8 + b])
				fprintf(stderr, " %u", L->ctl[8 + b] - 1);
		fprintf(stderr, "\n");
	}
	(void)hipStreamDestroy(L->st);
	(void)hipHostFree(L->slots);
	(void)hipHostFree(L->img[0]);
	(void)hipHostFree(L->img[1]);
	(void)hipHostFree(L->ctl);
	if (L->c->loop == L)
		L->c->loop = nullptr;
	delete L;
	return e == hipSuccess ? 0 : -EIO;
}

extern "C" int gcl_rxloop_drive(struct gcl_rxloop *L, uint32_t n, const uint64_t *offs,
                                uint32_t iters, uint32_t depth, uint64_t *lat_ns,
                                uint64_t *elapsed_ns)
{
	if (!L || !offs || !iters || !depth || depth > L->lp.nslots)
		return -EINVAL;
	std::vector<int64_t> tk(iters);
	std::vector<uint64_t> t_sub(iters);
	uint32_t head = 0, tail = 0; /* submitted, retired */
	const uint64_t t0 = now_ns();
	while (tail < iters) {
		while (head < iters && head - tail < depth) {
			t_sub[head] = now_ns();
			const int64_t r = gcl_rxloop_submit(L, n, offs, nullptr, nullptr, nullptr, nullptr);
			if (r < 0)
				return (int)r;
			tk[head++] = r;
		}
		const int r = gcl_rxloop_wait(L, tk[tail], nullptr, 1000000000ull);
		if (r)
			return r;
		if (lat_ns)
			lat_ns[tail] = now_ns() - t_sub[tail];
		tail++;
	}
	if (elapsed_ns)
		*elapsed_ns = now_ns() - t0;
	return 0;
}
