/*
 * gcl_kern.h - the device side shared by the classify kernels (gcl_batch.hip)
 * and the persistent rx loops (gcl_loop.hip): kernel parameters, the header
 * tile, the IP table lookup, Toeplitz, and rx_one_pkt itself (classify_core,
 * classify_lean; iokernel/rx.c:116-233), plus the verdict stores and the
 * counter flush.  Integer-only; gfx950.
 */
#pragma once

#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gclassify.h"
#include "gcl_device.h"

namespace gclk {


constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kToepBytes = 12 * 256 * 4;
constexpr uint32_t kCrcBytes = 8 * 256 * 4;
constexpr uint32_t kLdsTableBudget = 96 * 1024;
constexpr int kImgUsers = 8;             /* streams tracked per table image */
/* GENERAL batches (per-packet offsets or side arrays) run on
 * classify_pair_kernel.  Against the LDS-tile kernel's GENERAL path,
 * alternating in one process (profiles/r03_general_ab.jsonl,
 * r03_ws_ab.jsonl): the cache-resident working-set row 107.4-109.5 ->
 * 95.4-98.4 us, the random pool, the JENKINS offsets-only row, PCIe
 * zero-copy and the pcap replay within +-1 %; 23 % fewer VALU instructions
 * per wave (SQ counters, profiles/r03_sq_ingress_ws_*.json).  The tile
 * kernel's GENERAL path was removed in round 5. */

/* The first failure of a sequence of HIP calls whose outcome is checked
 * once, at the end (asynchronous copies, event records and waits). */
struct HipErr {
	hipError_t e = hipSuccess;
	void operator()(hipError_t r)
	{
		if (r != hipSuccess && e == hipSuccess)
			e = r;
	}
	bool bad() const { return e != hipSuccess; }
};
/* Verdict stores are write-through (global_store sc0 sc1, a system-scope
 * relaxed atomic store): against plain stores on the same buffers, one
 * process, udp64 2.3-3.8 % faster for all verdict widths, tcp1500 2-2.4 %
 * (profiles/archive/r01_verdict_store_ab.jsonl).  Measured and removed in
 * round 5 (the A/B evidence stays in profiles/ and git history): verdicts
 * staged in LDS and stored as whole lines (within noise,
 * profiles/r04_vstage_ab.jsonl), stored one tile late (1-3 % slower,
 * profiles/archive/r02_defer_ab.jsonl), a per-XCD contiguous tile walk (7 %
 * slower, profiles/archive/r01_alloc_placement.jsonl), a dynamic per-XCD tile
 * queue (83.8 against 101.1 Gpkt/s), non-temporal verdict stores and
 * streaming-hint pair loads. */

struct RtEntry {            /* 16 B per uniqid */
	uint32_t m_lo, m_hi;     /* fastmod magic for thread_count */
	uint16_t tc, active;     /* thread_count, active_thread_count */
	uint32_t flow_off;       /* byte offset of flow_tbl in the flow area */
};
static_assert(sizeof(RtEntry) == 16, "RtEntry");

struct KParams {
	const uint8_t *frames;
	uint64_t frames_len;
	uint64_t stride;
	const uint64_t *offs;
	const uint8_t *olflags;
	const uint32_t *rss;
	const uint32_t *fdir;
	const uint32_t *dst_hint;
	uint64_t n;
	uint64_t ntiles;
	uint2 *verdicts;
	unsigned long long *counts;
	unsigned long long *stats;
	const uint8_t *tables;     /* device table image */
	uint32_t ipt_mask;         /* ip buckets - 1 (2 slots per bucket) */
	uint32_t ipt_seed;         /* lookup3 initval of the bucket hash */
	uint32_t max_rt;
	uint32_t off_rt, off_flow, off_toep, tables_lds_bytes;
	uint32_t cflags;
	uint32_t default_flags;
	uint2 *trans;    /* struct gcl_trans[n] or NULL */
	uint32_t off_seed, off_crc;
	uint32_t vcap;   /* classify_kernel, 1-/2-B verdicts: tiles of verdicts its LDS buffer
	                    holds (0: every verdict stored as it is made) */
	uint32_t vregs;  /* with vcap: tiles past a full LDS buffer held in registers */
	uint32_t plean;  /* classify_pair_kernel: plain-IPv4 waves on classify_lean */
	uint32_t tlean;  /* classify_kernel: plain-IPv4 waves on classify_lean */
	uint32_t vstage; /* classify_kernel: the last register flush staged through LDS */
	uint32_t contig; /* classify_kernel: a contiguous run of tiles per block */
};

/* classify_kernel's verdict registers: kVregs dwords per lane, so 4 * kVregs
 * tiles of 1-B verdicts (2 * kVregs of 2-B ones) past a full LDS buffer.  16
 * (one write per block for the 1024-runtime contexts, not two) measured
 * slower: tcp1500 +2.5 %, header split +2 %, udp64 unchanged
 * (profiles/r06_vregs16_ab.jsonl) */
constexpr int kVregs = 10;

/* ------------------------------------------------------------------------
 * Header tile: 256 packets x 64 B, 16-B chunks XOR-swizzled so that both the
 * coalesced ds_write_b128 fill and the row-per-lane ds_read_b128 are
 * bank-conflict free (chunk q of packet p lives at p*4 + (q ^ ((p>>2)&3))).
 */
__device__ __forceinline__ int tile_slot(int p, int q)
{
	return p * 4 + (q ^ ((p >> 2) & 3));
}

__device__ __forceinline__ uint8_t frame_byte(const KParams &k, uint64_t a)
{
	return a < k.frames_len ? k.frames[a] : 0;
}

/* frame_byte with a system-scope load when SYS (the rx loop's host frames) */
template <bool SYS>
__device__ __forceinline__ uint8_t fbyte(const KParams &k, uint64_t a)
{
	return SYS ? gcl::byte_sys(k.frames, k.frames_len, a) : frame_byte(k, a);
}

/* A caller's frame offset, clamped to frames_len: every offset at or past it
 * reads as a frame of zeros either way, and the clamp keeps a live packet
 * clear of the kNoOff sentinel (~0) the kernels use for "no packet"
 * (gcl_classify_ex refuses frames_len == ~0). */
__device__ __forceinline__ uint64_t user_off(const KParams &k, uint64_t o)
{
	return o < k.frames_len ? o : k.frames_len;
}

template <bool GENERAL>
__device__ __forceinline__ uint64_t frame_off(const KParams &k, uint64_t idx)
{
	if (GENERAL && k.offs)
		return user_off(k, k.offs[idx]);
	return idx * k.stride;
}

/* How much of a lane's header row classify_one may read: staged frame bytes
 * << 8 (the low byte, a staging shift, is always 0 here).  The rx loop's
 * header records (GCL_LOOP_HDR_RECORDS) stage frame bytes 12-15 and 20-43
 * only: ports past byte 43 (IHL >= 7) are read from the frame. */
constexpr uint32_t kSpanFull = 64u << 8;
constexpr uint32_t kSpanRec = 44u << 8;

/* "no packet" offset (frames at or past frames_len are clamped to it, so a
 * live packet never carries it) */
constexpr uint64_t kNoOff = ~0ull;

/* 16 frame bytes from @a, bytewise (frame_byte: zero past frames_len) */
__device__ __forceinline__ uint4 load16_bytes(const KParams &k, uint64_t a)
{
	uint32_t w[4];
	for (int b = 0; b < 4; b++)
		w[b] = frame_byte(k, a + 4 * b) | frame_byte(k, a + 4 * b + 1) << 8 |
		       frame_byte(k, a + 4 * b + 2) << 16 | (uint32_t)frame_byte(k, a + 4 * b + 3) << 24;
	return make_uint4(w[0], w[1], w[2], w[3]);
}

/* The tile kernel's 16-B frame loads carry the streaming hint: plain loads
 * measured 11 % slower on udp64 (88.7-89.6 vs 99.8-100.7 Gpkt/s) and 13 % on
 * tcp1500, alternating fresh processes on one box
 * (profiles/r03_dense_load_hint_ab.jsonl) -- the opposite of the pair
 * kernel, whose frames are reused from L2. */
__device__ __forceinline__ uint4 tile_load(const void *p)
{
	return gcl::load16_nt(p);
}

/*
 * Issue the four 16-B chunk loads of this lane for @tile of fixed-stride
 * slots (staged by stage_tile after the loads land).  Every lane issues all
 * four loads on every path -- a chunk past the batch or of a !@live tile
 * loads 16 B of the table image instead and is never looked at -- and
 * nothing here consumes a loaded value.  Loads retire in order and the
 * compiler's wait before staging a tile counts the loads issued after that
 * tile's on every path through the loop, so with a fixed count it waits for
 * this tile alone and the next tile's loads stay in flight (DEPTH 2); one
 * conditional load path makes it wait for everything.
 */
/*
 * Chunk c of a tile is 16-B chunk c & 3 of tile packet c >> 2; the lane's
 * j-th chunk is chunk j * NT + tid, so each wave instruction reads 1 KiB of
 * 64-B slots and the tile is complete after a block barrier.  (Round 6
 * measured the other mapping -- each wave staging and classifying its own
 * 64 packets, no barrier per tile -- 3 % slower on udp64 and tcp1500,
 * profiles/r06_stage_ab.jsonl, and removed it.)
 */
template <int NT>
__device__ __forceinline__ uint32_t tile_chunk(int j)
{
	return j * NT + threadIdx.x;
}

template <int NT>
__device__ __forceinline__ void load_tile(const KParams &k, uint64_t tile, bool live, uint4 r[4])
{
	const uint8_t *dummy = k.tables; /* device table image: >= 16 B, always mapped */
	const uint64_t t0 = tile * NT;
	const uint32_t lim = (!live || t0 >= k.n) ? 0u : k.n - t0 < NT ? (uint32_t)(k.n - t0) : NT;
	const uint8_t *base = k.frames + t0 * k.stride;
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t c = tile_chunk<NT>(j), p = c >> 2;
		const uint8_t *a = p < lim ? base + (p * (uint32_t)k.stride + (c & 3) * 16) : dummy;
		r[j] = tile_load(a);
	}
}

/*
 * What a lane loads in place of an absent per-packet array (the loop keeps
 * one load count on every path): packet @i's own offs[] entry, a line the
 * kernel has already fetched, else the table image.  (One address shared by
 * every lane of the chip, the table image, would put all these loads on one
 * L2 channel.)
 */
template <typename T>
__device__ __forceinline__ const T *side_dummy(const KParams &k, uint64_t i)
{
	return (const T *)(k.offs ? (const uint8_t *)(k.offs + i) : k.tables);
}

/* dword at byte offset b (4-aligned, < 64) of this lane's staged header */
__device__ __forceinline__ uint32_t tile_dword(const uint4 *tile, int p, int b)
{
	const uint32_t *t32 = (const uint32_t *)tile;
	return t32[tile_slot(p, b >> 4) * 4 + ((b & 15) >> 2)];
}

struct Counters {
	uint32_t flowtag, hashmiss, unreg, unhandled;
};

struct Tables {
	const uint2 *ipt;
	const RtEntry *rtab;
	const uint8_t *flow;
	const uint32_t *toep;
	const uint32_t *seed;  /* per-runtime trans_seed */
	const uint32_t *crc;   /* CRC32C slice-by-8 LUT, 8 x 256 words */
};

/* crc32q semantics (no inversion) over the 8 LE bytes of v, slice-by-8 */
__device__ __forceinline__ uint32_t crc32c_u64(const uint32_t *T, uint32_t crc, uint64_t v)
{
	const uint32_t lo = crc ^ (uint32_t)v, hi = (uint32_t)(v >> 32);
	return T[7 * 256 + (lo & 0xFF)] ^ T[6 * 256 + ((lo >> 8) & 0xFF)] ^
	       T[5 * 256 + ((lo >> 16) & 0xFF)] ^ T[4 * 256 + (lo >> 24)] ^
	       T[3 * 256 + (hi & 0xFF)] ^ T[2 * 256 + ((hi >> 8) & 0xFF)] ^
	       T[1 * 256 + ((hi >> 16) & 0xFF)] ^ T[0 * 256 + (hi >> 24)];
}

/*
 * ip_to_proc: a two-choice bucketised cuckoo table like DPDK's rte_hash (the
 * reference's dp.ip_to_proc, dp_clients.c:349-363), keyed by lookup3 of the
 * IP.  Buckets hold two {ip, uniqid} entries (16 B, one ds_read_b128); a key
 * lives in bucket h or rotl(h, 16).  The host places every key (build_image),
 * so a lookup is two independent LDS reads and four selects: no probe loop,
 * no divergence.  -1 on a miss.
 */
__device__ __forceinline__ int ipt_lookup(const uint2 *ipt, uint32_t mask, uint32_t seed,
                                          uint32_t ip)
{
	const uint32_t h = gcl::jhash_u32(ip, seed);
	const uint4 *bk = (const uint4 *)ipt;
	const uint4 x = bk[h & mask], y = bk[gcl::rotl(h, 16) & mask];
	int r = -1;
	r = (x.x == ip && x.y != kEmpty) ? (int)x.y : r;
	r = (x.z == ip && x.w != kEmpty) ? (int)x.w : r;
	r = (y.x == ip && y.y != kEmpty) ? (int)y.y : r;
	r = (y.z == ip && y.w != kEmpty) ? (int)y.w : r;
	return r;
}

/* Toeplitz over the 12-byte tuple with the per-byte LUT (12 x 256 words) */
__device__ __forceinline__ uint32_t toeplitz_lut(const uint32_t *toep, uint32_t saddr,
                                                 uint32_t daddr, uint32_t sport, uint32_t dport)
{
	return toep[0 * 256 + (saddr >> 24)] ^ toep[1 * 256 + ((saddr >> 16) & 0xFF)] ^
	       toep[2 * 256 + ((saddr >> 8) & 0xFF)] ^ toep[3 * 256 + (saddr & 0xFF)] ^
	       toep[4 * 256 + (daddr >> 24)] ^ toep[5 * 256 + ((daddr >> 16) & 0xFF)] ^
	       toep[6 * 256 + ((daddr >> 8) & 0xFF)] ^ toep[7 * 256 + (daddr & 0xFF)] ^
	       toep[8 * 256 + (sport >> 8)] ^ toep[9 * 256 + (sport & 0xFF)] ^
	       toep[10 * 256 + (dport >> 8)] ^ toep[11 * 256 + (dport & 0xFF)];
}

/*
 * Dense slots (!GENERAL): wait for everything outstanding -- the tile just
 * requested and the wave's verdict stores -- before the IP lookup of every
 * tile and before staging the first tile of each loop iteration, so a wave
 * has at most about one tile of requests in flight and the latency hides
 * behind the other resident waves.  Keeping the loads in flight across the
 * parse (the GENERAL pipelining) measured udp64 91.4 against 101 Gpkt/s, the
 * lookup drain alone 99.2-99.8 (8-B verdicts 85.9-87.3 against 92.7-93.9),
 * both drains 100.8-101.0 (92.5-92.8), a drain before both stages 86.7: the
 * HBM stream runs best with few requests outstanding per wave
 * (profiles/archive/r02_dense_depth_ab.jsonl).
 */
__device__ __forceinline__ void dense_drain()
{
	__builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0), expcnt / lgkmcnt untouched */
}

/*
 * rx_one_pkt for the packet staged in row `tid` of the tile (rx.c:116-233).
 * Written as straight-line selects: every lane runs the same instruction
 * stream (hash, probe, steer), and only the rare cases -- IHL != 5 ports, a
 * probe chain longer than one slot -- take a divergent branch.
 */
/* The header dwords rx_one_pkt's decision reads: frame bytes 12-15 and 20-43
 * (Ethertype + IHL, frag/proto or ARP opcode, saddr, daddr, L4 ports, ARP
 * target IP) as little-endian dwords. */
struct HdrWords {
	uint32_t d3, d5, d6, d7, d8, d9, d10;
};

/*
 * rx_one_pkt on the header dwords @h of packet @idx (rx.c:116-233).  Frame
 * bytes [0, @avail) were staged with shift @sh (hdr_window); @tile (REG
 * false) holds them in row @tid for the IHL != 5 port reads, which REG
 * (classify_pair_kernel: headers in registers) reads from the frame instead.
 */
/* VF: the verdict format when known at compile time (2: GCL_CFG_VERDICT2,
 * which excludes the transport pre-hash), 0: read from k.cflags.  HIST false
 * (rxloop64_kernel): no histogram add; @hist[tid] gets the packet's runtime
 * (-1: none), which the loop's writer wave counts. */
template <int MODE, bool GENERAL, bool SYS, bool REG, int VF = 0, bool HIST = true>
__device__ __forceinline__ uint64_t classify_core(const KParams &k, const HdrWords &h,
                                                  const uint4 *tile, int tid, uint64_t idx,
                                                  const Tables &tb, uint32_t *hist, Counters &cnt,
                                                  uint32_t sh, uint32_t avail, const uint32_t *pre,
                                                  uint64_t foff = kNoOff)
{
	const uint32_t d3 = h.d3, d5 = h.d5, d6 = h.d6, d7 = h.d7, d8 = h.d8, d9 = h.d9, d10 = h.d10;
	const uint32_t et = gcl::bswap16(d3 & 0xFFFF);              /* rx.c:154 */
	const uint32_t ihl = (d3 >> 16) & 0xF;
	const uint32_t frag = gcl::bswap16(d5 & 0xFFFF);            /* ARP: opcode */
	const uint32_t proto = d5 >> 24;
	const uint32_t saddr = gcl::bswap32(gcl::mid32(d6, d7));
	const uint32_t daddr = gcl::bswap32(gcl::mid32(d7, d8));     /* rx.c:157-159 */
	uint32_t arp_tip = gcl::bswap32(gcl::mid32(d9, d10));        /* rx.c:165-167 */
	/* @pre: {ol_flags, hash.rss} as loaded a tile ahead by classify_kernel
	 * (raw: the table image stands in for a missing array) */
	const uint32_t flags = !(GENERAL && k.olflags) ? k.default_flags
	                       : pre ? pre[0] & 0xFF : k.olflags[idx];
	const bool is_ip = et == GCL_ETHTYPE_IP, is_arp = et == GCL_ETHTYPE_ARP;
	if (GENERAL && !SYS && is_arp && avail < 44) {
		/* bytes 40-41 are past the staged bytes: one dword load when it is
		 * aligned and inside frames_len, else byte by byte (@foff: the frame
		 * offset when the caller has it, saving the offs[] reload) */
		const uint64_t o = foff != kNoOff ? foff : frame_off<GENERAL>(k, idx);
		const uint64_t A = (uint64_t)(uintptr_t)k.frames + o + 40;
		if (o < k.frames_len && k.frames_len - o >= 44 && (A & 3) == 0) {
			arp_tip = gcl::bswap32(gcl::mid32(d9, *(const uint32_t *)(k.frames + o + 40)));
		} else {
			const uint64_t a = o + 38;
			arp_tip = (uint32_t)frame_byte(k, a) << 24 | (uint32_t)frame_byte(k, a + 1) << 16 |
			          (uint32_t)frame_byte(k, a + 2) << 8 | frame_byte(k, a + 3);
		}
	}
	const bool azure = k.cflags & GCL_CFG_AZURE_ARP;

	/* steering hash (gclassify.h: NIC / JENKINS / TOEPLITZ) */
	uint32_t hash = 0;
	if (MODE == GCL_HASH_NIC) {
		if (k.rss)
			hash = pre ? pre[1] : k.rss[idx];
	} else {
		const bool hashable = is_ip && ihl >= 5 && (frag & 0x3FFF) == 0 &&
		                      (proto == 6 || proto == 17);
		uint32_t sport = gcl::bswap16(d8 >> 16), dport = gcl::bswap16(d9 & 0xFFFF);
		if (hashable && ihl != 5) {
			if (!REG && 20 + 4 * ihl <= avail) { /* ihl <= 11 when avail == 64 */
				const int o = 14 + 4 * (int)ihl + (int)sh;
				sport = gcl::bswap16(tile_dword(tile, tid, o - 2) >> 16);
				dport = gcl::bswap16(tile_dword(tile, tid, o + 2) & 0xFFFF);
			} else { /* past the staged header bytes */
				const uint64_t a = frame_off<GENERAL>(k, idx) + 14 + 4 * ihl;
				sport = (uint32_t)fbyte<SYS>(k, a) << 8 | fbyte<SYS>(k, a + 1);
				dport = (uint32_t)fbyte<SYS>(k, a + 2) << 8 | fbyte<SYS>(k, a + 3);
			}
		}
		const uint32_t h = MODE == GCL_HASH_JENKINS
		                       ? gcl::jhash_5tuple(saddr, daddr, sport, dport, proto)
		                       : toeplitz_lut(tb.toep, saddr, daddr, sport, dport);
		hash = hashable ? h : 0;
	}
	if (k.cflags & GCL_CFG_HASH16)
		hash &= 0xFFFF;

	/* loopback: rx_loopback's dst_ip hint lookup sets the flow tag,
	 * rx.c:249-262 (a miss leaves the mbuf's own flags) */
	uint32_t flags2 = flags, hint_mark = 0;
	if (GENERAL && k.dst_hint) {
		const uint32_t hint = k.dst_hint[idx];
		const int q = hint ? ipt_lookup(tb.ipt, k.ipt_mask, k.ipt_seed, hint) : -1;
		if (q >= 0) {
			flags2 |= GCL_F_FDIR_ID;
			hint_mark = (uint32_t)q + 1;
		}
	}

	/* hardware flow tag, rx.c:131-146 */
	int p = -1;
	uint32_t action = GCL_ACT_DELIVER;
	if (GENERAL && (flags2 & GCL_F_FDIR_ID)) {
		const uint32_t mark = hint_mark ? hint_mark - 1 : (k.fdir ? k.fdir[idx] : 0);
		cnt.flowtag++;
		if (mark < k.max_rt && tb.rtab[mark].tc != 0) {
			p = (int)mark;
			action = GCL_ACT_F_FDIR;
		}
	}
	/* Ethertype dispatch, rx.c:154-194 */
	const bool parse = p < 0;
	const bool broadcast = parse && is_arp && azure && frag == GCL_ARP_OP_REPLY;
	const bool lookup = parse && (is_ip || is_arp) && !broadcast;
	cnt.hashmiss += parse && is_ip && !(flags & GCL_F_RSS_HASH); /* rx.c:160-163 */
	const uint32_t dst = is_ip ? daddr : arp_tip;

	if constexpr (!GENERAL)
		dense_drain();
	/* ip_to_proc: open addressing keyed by rte_jhash(&ip, 4, 0), rx.c:197 */
	if (lookup)
		p = ipt_lookup(tb.ipt, k.ipt_mask, k.ipt_seed, dst);
	const bool miss = lookup && p < 0;
	const bool arp_respond = miss && azure && is_arp && frag == GCL_ARP_OP_REQUEST;
	const bool unreg = miss && !arp_respond;                    /* rx.c:205 */
	const bool bad_et = parse && !is_ip && !is_arp;              /* rx.c:191-194 */
	cnt.unreg += unreg;
	cnt.unhandled += unreg || bad_et;                            /* rx.c:232 */
	action = bad_et ? GCL_ACT_DROP_ETHERTYPE
	       : broadcast ? GCL_ACT_BROADCAST
	       : arp_respond ? GCL_ACT_ARP_RESPOND
	       : unreg ? GCL_ACT_DROP_UNREG : action;

	/* rx_send_to_runtime, rx.c:55-72: the flow_tbl slot hash % thread_count.
	 * The slot, not flow_tbl[slot], is the verdict: the host post-pass reads
	 * the live flow_tbl and active count at delivery time, as rx.c does, so
	 * a scheduler side effect earlier in the same batch (a wake that takes a
	 * core from another runtime, sched.c:208-216) steers the later packets */
	uint32_t uniq = GCL_NO_RUNTIME, thr = GCL_NO_THREAD;
	if (p >= 0) {
		const RtEntry re = tb.rtab[p];
		uniq = (uint32_t)p;
		const uint64_t M = (uint64_t)re.m_hi << 32 | re.m_lo;
		thr = gcl::fastmod(hash, M, re.tc);
		if (!re.active)
			action |= GCL_ACT_WAKE;
		if (HIST)
			atomicAdd(&hist[p], 1u);
	}
	if (!HIST)
		hist[tid] = (uint32_t)p;
	if (VF == 0 && k.trans) { /* VERDICT1/2 contexts never have the pre-hash */
		/* trans_lookup's hashes with runtime p's trans_seed
		 * (transport.c:29-42, :366-375), for the packets net_rx_one passes
		 * to net_rx_trans (core.c:203-209, :281-300) */
		const bool supported = is_ip && (d3 >> 20 & 0xF) == 4 && ihl == 5 &&
		                       !(d5 & 0x2000) && (proto == 6 || proto == 17);
		uint2 tr = make_uint2(0, 0);
		if (p >= 0 && supported) {
			const uint32_t seed = tb.seed[p];
			const uint64_t l = (uint64_t)daddr | (uint64_t)gcl::bswap16(d9 & 0xFFFF) << 32;
			const uint64_t r = (uint64_t)saddr | (uint64_t)gcl::bswap16(d8 >> 16) << 32 |
			                   (uint64_t)proto << 48;
			tr.x = crc32c_u64(tb.crc, crc32c_u64(tb.crc, seed, l), r);
			tr.y = crc32c_u64(tb.crc, seed, l | (uint64_t)proto << 48);
			action |= GCL_ACT_F_TRANS;
		}
		k.trans[idx] = tr;
	}
	const uint32_t vlo = uniq | thr << 16 | action << 24;
	if (VF == 1 || (VF == 0 && (k.cflags & GCL_CFG_VERDICT1))) {
		/* q = uniqid << thread_bits | slot; no WAKE mark (gclassify.h) */
		const uint32_t a = action & GCL_ACT_MASK;
		const uint32_t q = uniq << (k.cflags >> 24) | thr;
		return a == GCL_ACT_DELIVER || a == GCL_ACT_WAKE ? q : GCL_V1_OTHER | a;
	}
	if (VF == 2 || (VF == 0 && (k.cflags & GCL_CFG_VERDICT2))) {
		/* q = uniqid << thread_bits | thread (thread_bits in cflags[31:24]) */
		const uint32_t a = action & GCL_ACT_MASK;
		const uint32_t q = uniq << (k.cflags >> 24) | thr;
		return a == GCL_ACT_DELIVER ? q : a == GCL_ACT_WAKE ? GCL_V2_WAKE | q : GCL_V2_OTHER | a;
	}
	if (k.cflags & GCL_CFG_VERDICT4)
		return vlo;
	return (uint64_t)vlo << 32 | hash;
}

/*
 * rxloop64_kernel's lean rx_one_pkt: classify_core restricted to what a burst
 * of plain IPv4 traffic needs -- Ethertype IPv4, IHL 5, no FDIR mark, no
 * dst_ip hint, no transport pre-hash -- which the caller checks for every
 * packet of the burst (a uniform ballot) before taking it.  Same verdicts and
 * counters as classify_core on those packets (rx.c:154-163, :197-207, :55-72);
 * a burst with any other packet takes classify_core.  One wave classifies a
 * lone burst on its own, so its latency is the instruction count: this path
 * skips the FDIR, hint, options-port, ARP and action-ladder selects.
 * @flags: ol_flags (or the context default), @rss: hash.rss (NIC mode).
 */
/* HIST: add the packet to the LDS histogram (classify_pair_kernel) rather
 * than hand its runtime to the loop's writer wave in @hist[tid] */
/* DRAIN (classify_kernel's dense slots): dense_drain() before the IP
 * lookup, where classify_core drains */
/* VF: the verdict format where the caller knows it (1 / 2 B), else 0 */
template <int MODE, bool HIST = false, bool DRAIN = false, int VF = 0>
__device__ __forceinline__ uint64_t classify_lean(const KParams &k, const HdrWords &h, const Tables &tb,
                                                  uint32_t flags, uint32_t rss, uint32_t *hist, int tid,
                                                  Counters &cnt)
{
	const uint32_t frag = gcl::bswap16(h.d5 & 0xFFFF);
	const uint32_t proto = h.d5 >> 24;
	const uint32_t saddr = gcl::bswap32(gcl::mid32(h.d6, h.d7));
	const uint32_t daddr = gcl::bswap32(gcl::mid32(h.d7, h.d8));     /* rx.c:157-159 */
	uint32_t hash = 0;
	if (MODE == GCL_HASH_NIC) {
		if (k.rss)
			hash = rss;
	} else {
		const bool hashable = (frag & 0x3FFF) == 0 && (proto == 6 || proto == 17);
		const uint32_t sport = gcl::bswap16(h.d8 >> 16), dport = gcl::bswap16(h.d9 & 0xFFFF);
		const uint32_t x = MODE == GCL_HASH_JENKINS ? gcl::jhash_5tuple(saddr, daddr, sport, dport, proto)
		                                            : toeplitz_lut(tb.toep, saddr, daddr, sport, dport);
		hash = hashable ? x : 0;
	}
	if (k.cflags & GCL_CFG_HASH16)
		hash &= 0xFFFF;
	cnt.hashmiss += !(flags & GCL_F_RSS_HASH); /* rx.c:160-163 */
	if (DRAIN)
		dense_drain();
	const int p = ipt_lookup(tb.ipt, k.ipt_mask, k.ipt_seed, daddr); /* rx.c:197 */
	const bool miss = p < 0;
	cnt.unreg += miss;     /* rx.c:205 */
	cnt.unhandled += miss; /* rx.c:232 */
	uint32_t action = miss ? GCL_ACT_DROP_UNREG : GCL_ACT_DELIVER;
	uint32_t uniq = GCL_NO_RUNTIME, thr = GCL_NO_THREAD;
	if (!miss) { /* rx_send_to_runtime's slot, rx.c:55-72 */
		const RtEntry re = tb.rtab[p];
		uniq = (uint32_t)p;
		thr = gcl::fastmod(hash, (uint64_t)re.m_hi << 32 | re.m_lo, re.tc);
		if (!re.active)
			action |= GCL_ACT_WAKE;
		if (HIST)
			atomicAdd(&hist[p], 1u);
	}
	if (!HIST)
		hist[tid] = (uint32_t)p;
	const uint32_t q = uniq << (k.cflags >> 24) | thr;
	if (VF == 1 || (VF == 0 && (k.cflags & GCL_CFG_VERDICT1)))
		return miss ? GCL_V1_OTHER | GCL_ACT_DROP_UNREG : q;
	if (VF == 2 || (VF == 0 && (k.cflags & GCL_CFG_VERDICT2)))
		return miss ? GCL_V2_OTHER | GCL_ACT_DROP_UNREG : action == GCL_ACT_WAKE ? GCL_V2_WAKE | q : q;
	const uint32_t vlo = uniq | thr << 16 | action << 24;
	if (k.cflags & GCL_CFG_VERDICT4)
		return vlo;
	return (uint64_t)vlo << 32 | hash;
}

/* rx_one_pkt for the packet staged in row `tid` of the LDS tile: dense
 * slots (classify_kernel), or SYS (rxloop_kernel: frames at per-packet
 * offsets in host memory, @span's staged bytes, 64 or 44 with header
 * records, kSpanRec) */
template <int MODE, bool GENERAL, bool SYS = false>
__device__ __forceinline__ uint64_t classify_one(const KParams &k, const uint4 *tile, int tid,
                                                 uint64_t idx, const Tables &tb, uint32_t *hist,
                                                 Counters &cnt, uint32_t span = kSpanFull)
{
	static_assert(!GENERAL || SYS, "GENERAL batches run on classify_pair_kernel");
	const uint32_t avail = GENERAL ? (span >> 8 & 0xFF) : 64u;
	const uint4 w0 = tile[tile_slot(tid, 0)];
	const uint4 w1 = tile[tile_slot(tid, 1)];
	const uint4 w2 = tile[tile_slot(tid, 2)];
	HdrWords h;
	h.d3 = w0.w, h.d5 = w1.y, h.d6 = w1.z, h.d7 = w1.w;
	h.d8 = w2.x, h.d9 = w2.y, h.d10 = w2.z;
	return classify_core<MODE, GENERAL, SYS, false>(k, h, tile, tid, idx, tb, hist, cnt, 0, avail, nullptr);
}

/* bytes per verdict of the context's format (KParams.cflags) */
__device__ __forceinline__ uint32_t verdict_width(uint32_t cflags)
{
	return (cflags & GCL_CFG_VERDICT1) ? 1u : (cflags & GCL_CFG_VERDICT2) ? 2u : (cflags & GCL_CFG_VERDICT4) ? 4u : 8u;
}

/* Store verdict word @w (classify_one) of packet @idx in the context's
 * verdict format and store policy. */
__device__ __forceinline__ void put_verdict(const KParams &k, uint64_t idx, uint64_t w);

/* a write-through (sc0 sc1) store of one verdict element */
template <typename T>
__device__ __forceinline__ void store_wt(T *p, T v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* put_verdict with the format known at compile time (VF 1 / 2: the 1- or
 * 2-byte queue verdict), else read from k.cflags */
template <int VF>
__device__ __forceinline__ void put_verdict_vf(const KParams &k, uint64_t idx, uint64_t w)
{
	if (VF == 2)
		store_wt((uint16_t *)k.verdicts + idx, (uint16_t)w);
	else if (VF == 1)
		store_wt((uint8_t *)k.verdicts + idx, (uint8_t)w);
	else
		put_verdict(k, idx, w);
}

__device__ __forceinline__ void put_verdict(const KParams &k, uint64_t idx, uint64_t w)
{
	if (k.cflags & GCL_CFG_VERDICT1)
		store_wt((uint8_t *)k.verdicts + idx, (uint8_t)w);
	else if (k.cflags & GCL_CFG_VERDICT2)
		store_wt((uint16_t *)k.verdicts + idx, (uint16_t)w);
	else if (k.cflags & GCL_CFG_VERDICT4)
		store_wt((uint32_t *)k.verdicts + idx, (uint32_t)w);
	else
		store_wt((uint64_t *)k.verdicts + idx, w);
}

/* The table image into LDS at a batch kernel's start: each lane issues all
 * eight 16-B loads of a round (128 B x NT per block) before its first LDS
 * store, so staging the 1024-runtime tables (37 KiB) at 512 lanes costs one
 * L2 round trip, not one per 16 B x NT (five, each waited for before its store) */
template <int NT>
__device__ __forceinline__ void stage_tables(uint8_t *lds_tab, const uint8_t *tables, uint32_t bytes)
{
	constexpr int U = 8;
	const uint4 *src = (const uint4 *)tables;
	uint4 *dst = (uint4 *)lds_tab;
	const uint32_t n16 = bytes / 16;
	for (uint32_t base = 0; base < n16; base += U * NT) {
		uint4 r[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t i = base + u * NT + threadIdx.x;
			r[u] = src[i < n16 ? i : 0]; /* every load issued, in range */
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t i = base + u * NT + threadIdx.x;
			if (i < n16)
				dst[i] = r[u];
		}
	}
}

template <int NT>
__device__ __forceinline__ void stage_tile(uint4 *tile, const uint4 r[4])
{
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t c = tile_chunk<NT>(j);
		tile[tile_slot(c >> 2, c & 3)] = r[j];
	}
}

/* classify_kernel's MODE for gcl_access_probe: the same launch -- tiles,
 * staging, drains, barriers, deferred verdict writes -- with rx_one_pkt
 * replaced by a fold of the three header rows it reads */
constexpr int kModeProbe = 3;

/* End of a classify launch: the block's histogram (all its waves' adds
 * done) and every wave's counters into the device totals. */
template <int NT>
__device__ __forceinline__ void flush_counters(const KParams &k, const uint32_t *hist,
                                               const Counters &cnt)
{
	const int tid = threadIdx.x;
	for (uint32_t i = tid; i < k.max_rt; i += NT) {
		uint32_t v = hist[i];
		if (v && k.counts)
			atomicAdd(&k.counts[i], (unsigned long long)v);
	}
	if (k.stats) {
		uint32_t n_flowtag = cnt.flowtag, n_hashmiss = cnt.hashmiss;
		uint32_t n_unreg = cnt.unreg, n_unhandled = cnt.unhandled;
		for (int off = 32; off > 0; off >>= 1) {
			n_flowtag += __shfl_xor(n_flowtag, off);
			n_hashmiss += __shfl_xor(n_hashmiss, off);
			n_unreg += __shfl_xor(n_unreg, off);
			n_unhandled += __shfl_xor(n_unhandled, off);
		}
		if ((tid & 63) == 0) {
			if (n_flowtag)
				atomicAdd(&k.stats[GCL_RX_FLOW_TAG_MATCH], (unsigned long long)n_flowtag);
			if (n_hashmiss)
				atomicAdd(&k.stats[GCL_RX_HASH_MISSING], (unsigned long long)n_hashmiss);
			if (n_unreg)
				atomicAdd(&k.stats[GCL_RX_UNREGISTERED_MAC], (unsigned long long)n_unreg);
			if (n_unhandled)
				atomicAdd(&k.stats[GCL_RX_UNHANDLED], (unsigned long long)n_unhandled);
		}
		if (blockIdx.x == 0 && tid == 0)
			atomicAdd(&k.stats[GCL_RX_PULLED], (unsigned long long)k.n);
	}
}


/* gcl_tune.pair_lean default: classify_pair_kernel's plain-IPv4 waves on
 * classify_lean -- the ingress working set 64.6-65.3 -> 62.7-63.3 us, the
 * random pool unchanged (memory-bound), profiles/r05_pair_lean_ab.jsonl */
constexpr int kDefaultPairLean = 1;
/* gcl_tune.defer default (Geometry::defer): udp64 328.2-329.1 -> 323.4-324.2
 * us, three fresh processes (profiles/r05_defer_ab.jsonl) */
constexpr int kDefaultDefer = 1;
/* gcl_tune.tile_lean default: classify_kernel's plain-IPv4 waves on classify_lean */
constexpr int kDefaultTileLean = 1;
/* gcl_tune.vstage default: udp64 326.4-328.6 -> 324.3-327.6 us, faster in each
 * of nine interleaved pairs over three fresh processes
 * (profiles/r06_vstage_ab.jsonl) */
constexpr int kDefaultVstage = 1;
constexpr int kDefaultPairI32 = 1; /* gcl_tune.pair_i32 default */
/* gcl_tune.tile_order default: round-robin.  One contiguous run per block --
 * the order tools/read_sol's fastest pure reads use (7.21 against 6.87 TB/s)
 * -- made udp64 307.0-308.7 -> 334.5-339.3 us and its probe the same way,
 * tcp1500 1 % slower (profiles/r06_tile_order_ab.jsonl) */
constexpr int kDefaultTileOrder = 0;

} // namespace gclk
