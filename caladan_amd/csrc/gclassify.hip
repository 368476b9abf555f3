/*
 * gclassify.hip - MI355X (gfx950) rx classifier: kernels + C ABI.
 *
 * Replaces the rx_one_pkt loop of rx_burst (iokernel/rx.c:116-233, :281-287):
 * one lane per packet, the first 64 bytes of every frame staged through LDS
 * with coalesced 16-byte loads, the IP->runtime table and flow tables resident
 * in LDS when they fit, per-runtime packet counts aggregated in LDS and
 * flushed with one global atomic per (block, runtime).
 *
 * Layout in HBM: frames are fixed-stride slots (or a u64
 * offset array, like mbuf data pointers into the 2 GiB ingress region);
 * verdicts are a dense gcl_verdict[n] (8 B per packet); the table image is one
 * contiguous buffer [ip slots | runtime entries | flow bytes | toeplitz LUT].
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <new>
#include <set>
#include <utility>
#include <vector>

#include "../../include/gclassify.h"
#include "gcl_device.h"

#define GCL_VERSION "gclassify 0.1 (gfx950)"

namespace {

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
};

/* classify_kernel's verdict registers: kVregs dwords per lane, so 4 * kVregs
 * tiles of 1-B verdicts (2 * kVregs of 2-B ones) past a full LDS buffer */
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
template <int NT>
__device__ __forceinline__ void load_tile(const KParams &k, uint64_t tile, bool live, uint4 r[4])
{
	const uint8_t *dummy = k.tables; /* device table image: >= 16 B, always mapped */
	const uint64_t t0 = tile * NT;
	const uint32_t lim = (!live || t0 >= k.n) ? 0u : k.n - t0 < NT ? (uint32_t)(k.n - t0) : NT;
	const uint8_t *base = k.frames + t0 * k.stride;
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint32_t c = j * NT + threadIdx.x, p = c >> 2;
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
template <int MODE, bool HIST = false>
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
	if (k.cflags & GCL_CFG_VERDICT1)
		return miss ? GCL_V1_OTHER | GCL_ACT_DROP_UNREG : q;
	if (k.cflags & GCL_CFG_VERDICT2)
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

template <int NT>
__device__ __forceinline__ void stage_tile(uint4 *tile, const uint4 r[4])
{
#pragma unroll
	for (int j = 0; j < 4; j++) {
		int c = j * NT + (int)threadIdx.x;
		tile[tile_slot(c >> 2, c & 3)] = r[j];
	}
}

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

/*
 * The batch kernel for fixed-stride slots (classify_kernel; frames at
 * per-packet offsets or with per-packet side arrays run on
 * classify_pair_kernel).  Persistent grid: block b handles tiles b, b + G,
 * b + 2G, ... (tiles dealt round-robin, so the whole chip sweeps one window
 * of the batch), with the frames of the next DEPTH tiles in flight in
 * registers while a tile is parsed.
 */
template <int MODE, bool TLDS, int DEPTH, int NT>
/* 4 waves per SIMD (<= 128 VGPRs): the 1024 resident lanes per CU the
 * geometry policy plans for, at every tile size */
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4)))
classify_kernel(KParams k)
{
	extern __shared__ uint4 smem[];
	uint4 *tile = smem;
	uint32_t *hist = (uint32_t *)(smem + NT * 4);
	uint8_t *lds_tab = (uint8_t *)(hist + ((k.max_rt + 3) & ~3u));
	const int tid = threadIdx.x;

	/* stage tables and zero the histogram */
	for (uint32_t i = tid; i < k.max_rt; i += NT)
		hist[i] = 0;
	/* @tab is LDS or global by the template argument alone: a pointer that
	 * may be either compiles to flat loads, which count against the vector
	 * memory counter too, so every table lookup would wait for the frame
	 * loads in flight */
	const uint8_t *tab = TLDS ? lds_tab : k.tables;
	if (TLDS) {
		const uint4 *src = (const uint4 *)k.tables;
		uint4 *dst = (uint4 *)lds_tab;
		for (uint32_t i = tid; i < k.tables_lds_bytes / 16; i += NT)
			dst[i] = src[i];
	}
	Tables tb;
	tb.ipt = (const uint2 *)tab;
	tb.rtab = (const RtEntry *)(tab + k.off_rt);
	tb.flow = tab + k.off_flow;
	tb.toep = (const uint32_t *)(tab + k.off_toep);
	tb.seed = (const uint32_t *)(tab + k.off_seed);
	tb.crc = (const uint32_t *)(tab + k.off_crc);
	__syncthreads();

	Counters cnt = {0, 0, 0, 0};
	uint4 ra[4], rb[4];
	uint64_t t = blockIdx.x;
	const uint64_t step = gridDim.x, t_end = k.ntiles;
	/* k.vcap (1-/2-B verdicts): each tile's verdicts kept in LDS after the
	 * tables -- and with k.vregs, once vcap tiles are in, the next ones in a
	 * shift register of kVregs dwords per lane -- and written out when both
	 * are full and after the last tile, so the verdict stream does not
	 * interleave with the frame reads (tools/wdefer.hip) */
	const uint32_t vb = (k.cflags & GCL_CFG_VERDICT1) ? 1 : 2;
	const uint32_t rcap = k.vregs ? kVregs * 4 / vb : 0; /* tiles the registers hold */
	uint8_t *vbuf = lds_tab + ((k.tables_lds_bytes + 15) & ~15u);
	/* uniform: kl tiles in the buffer, local tiles [kf, kf + kl); nreg in
	 * the registers, local tiles [kf + vcap, kf + vcap + nreg) */
	uint32_t kl = 0, kf = 0, nreg = 0;
	uint32_t vr[kVregs];
#pragma unroll
	for (int i = 0; i < kVregs; i++)
		vr[i] = 0;
	/* every lane of every tile before t_end, live or not, so each lane's
	 * register chain stays aligned with tile_done's count (the DEPTH-2
	 * loop's empty tile past t_end is neither) */
	auto verdict = [&](uint64_t i, bool real, bool live, uint64_t w) {
		if (!k.vcap) {
			if (live)
				put_verdict(k, i, w);
		} else if (kl < k.vcap) {
			uint8_t *d = vbuf + (kl * NT + tid) * vb;
			if (vb == 1)
				*d = (uint8_t)w;
			else
				*(uint16_t *)d = (uint16_t)w;
		} else if (real) {
			const uint32_t sh = 8 * vb;
#pragma unroll
			for (int r = kVregs - 1; r > 0; r--)
				vr[r] = (vr[r] << sh) | (vr[r - 1] >> (32 - sh));
			vr[0] = (vr[0] << sh) | ((uint32_t)w & ((1u << sh) - 1));
		}
	};
	const uint64_t nb = k.n * vb;
	/* the global byte offset of local tile @j's first verdict */
	auto tile_off = [&](uint32_t j) -> uint64_t {
		return ((uint64_t)blockIdx.x + (uint64_t)j * step) * NT * vb;
	};
	/* the buffer to its places, 16 B per lane, write-through like the
	 * per-packet stores; the batch's last tile up to n only */
	auto flush_lds = [&]() {
		const uint32_t cs = vb == 1 ? __builtin_ctz(NT / 16) : __builtin_ctz(NT / 8); /* log2 chunks per tile */
		const __amdgpu_buffer_rsrc_t vrs = gcl::host_rsrc(k.verdicts, nb);
		for (uint32_t i = tid; i < kl << cs; i += NT) {
			const uint32_t j = i >> cs, c = i & ((1u << cs) - 1);
			const uint64_t o = tile_off(kf + j) + 16 * c;
			const uint8_t *src = vbuf + j * NT * vb + 16 * c;
			if (o + 16 <= nb) {
				const uint4 v = *(const uint4 *)src;
				const gcl::u32x4 x = {v.x, v.y, v.z, v.w};
				__builtin_amdgcn_raw_buffer_store_b128(x, vrs, (int)o, 0, gcl::kSysAux);
			} else {
				for (uint32_t b = 0; o + b < nb && b < 16; b++)
					store_wt((uint8_t *)k.verdicts + o + b, src[b]);
			}
		}
	};
	/* the registers, newest tile first: each lane its own packet's verdict */
	auto flush_regs = [&]() {
		const uint32_t sh = 8 * vb;
		for (uint32_t q = 0; q < nreg; q++) {
			const uint64_t o = tile_off(kf + k.vcap + nreg - 1 - q) + (uint64_t)tid * vb;
			if (o < nb) {
				if (vb == 1)
					store_wt((uint8_t *)k.verdicts + o, (uint8_t)vr[0]);
				else
					store_wt((uint16_t *)((uint8_t *)k.verdicts + o), (uint16_t)vr[0]);
			}
#pragma unroll
			for (int r = 0; r < kVregs - 1; r++)
				vr[r] = (vr[r] >> sh) | (vr[r + 1] << (32 - sh));
			vr[kVregs - 1] >>= sh;
		}
	};
	/* after a classified tile and its barrier (the buffer complete): count
	 * it; both full -> write them out (the next writes to vbuf follow the
	 * next stage's barrier) */
	auto tile_done = [&](uint64_t tt) {
		if (!k.vcap || tt >= t_end)
			return;
		if (kl < k.vcap)
			kl++;
		else
			nreg++;
		if (kl == k.vcap && nreg == rcap) {
			flush_lds();
			flush_regs();
			kf += kl + nreg;
			kl = nreg = 0;
		}
	};
	if (t < t_end)
		load_tile<NT>(k, t, true, ra);
	if (DEPTH == 2)
		load_tile<NT>(k, t + step, t + step < t_end, rb);

	while (t < t_end) {
		/* t opaque to the loop optimiser: without it every per-packet
		 * address (verdicts, ...) becomes its own 64-bit induction
		 * variable, held in VGPRs and spilled */
		if constexpr (DEPTH == 2)
			asm volatile("" : "+s"(t));
		dense_drain(); /* once per loop iteration too */
		stage_tile<NT>(tile, ra);
		__syncthreads();
		const uint64_t nxt = t + DEPTH * step;
		/* in flight while parsing */
		load_tile<NT>(k, nxt, nxt < t_end, ra);
		{
			const bool live = t * NT + tid < k.n;
			const uint64_t w = live ? classify_one<MODE, false>(k, tile, tid, t * NT + tid, tb, hist, cnt) : 0;
			verdict(t * NT + tid, true, live, w);
		}
		__syncthreads();
		tile_done(t);
		t += step;
		if (DEPTH == 2) {
			/* runs past t_end too (an empty tile: dummy loads, nothing
			 * classified) rather than leaving the loop here: a path out of
			 * the middle of the body, without the rb loads below, would
			 * make the wait before staging ra wait for everything */
			stage_tile<NT>(tile, rb);
			__syncthreads();
			load_tile<NT>(k, t + 2 * step, t + 2 * step < t_end, rb);
			{
				const bool live = t < t_end && t * NT + tid < k.n;
				const uint64_t w =
				        live ? classify_one<MODE, false>(k, tile, tid, t * NT + tid, tb, hist, cnt) : 0;
				verdict(t * NT + tid, t < t_end, live, w);
			}
			__syncthreads();
			tile_done(t);
			t += step;
		}
	}
	if (kl)
		flush_lds();
	if (nreg)
		flush_regs();
	flush_counters<NT>(k, hist, cnt);
}

/* Lane-wise select of two 16-B values (classify_pair_kernel's exchange). */
__device__ __forceinline__ uint4 sel4(bool c, const uint4 &a, const uint4 &b)
{
	return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

/* ------------------------------------------------------------------------
 * classify_pair_kernel: the GENERAL path (frames at per-packet offsets, or
 * per-packet side arrays) without a staged window.  rx_one_pkt reads frame
 * bytes 12-39 of every IPv4 packet (Ethertype, IHL, fragment field, proto,
 * saddr, daddr and -- for the computed hashes -- the L4 ports, rx.c:127-167)
 * and bytes 38-41 of an ARP packet, so each packet's header is fetched as the
 * 32 bytes [8, 40): one 128-B line for every frame that starts at least 40
 * bytes before a line end, which is every frame of the reference's ingress
 * pool (element + 344 of 9408-B elements, iokernel/defs.h:503-506).  A PAIR of
 * lanes loads it with one 16-B load each -- lane 2i bytes 8-23, lane 2i+1
 * bytes 24-39, of packet 2i and then of packet 2i+1 -- and one DPP exchange
 * gives each lane both halves of its own packet: no LDS header tile, no
 * barriers and no window arithmetic, about half the VALU work per packet of
 * the tile kernel's GENERAL loop, which is issue-bound on cache-resident
 * frames (SQ counters).  The ARP target (bytes 40-41) and the
 * ports behind IPv4 options are read from the frame when needed (REG path of
 * classify_core), as are frames that are not 4-B aligned or end past
 * frames_len (bytewise, zero past it).  Offsets, ol_flags and hash.rss are
 * loaded tiles ahead with a fixed load count on every path (the tile
 * kernel's rule for the waits).
 */
constexpr uint64_t kPairBytewise = 1ull << 63;

/* DPP move with no "old" operand: a quad_perm never leaves a lane without
 * a source, so the exchange needs no register of zeros */
template <int CTRL>
__device__ __forceinline__ uint32_t mdpp(uint32_t v)
{
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

/* Where packet @off's bytes [8, 40) come from: off + 8 when one aligned
 * pair of 16-B loads inside frames_len can read them; kPairBytewise | o
 * (o = off, or frames_len when off is past it, so every byte reads 0) when
 * they must be read byte by byte; kNoOff when there is no packet. */
__device__ __forceinline__ uint64_t pair_src(const KParams &k, uint64_t off)
{
	/* straight-line selects: every lane runs the same instructions */
	const bool in = off < k.frames_len;
	const bool fits = in && k.frames_len - off >= 40 &&
	                  (((uint32_t)(uintptr_t)k.frames + (uint32_t)off) & 3) == 0;
	const uint64_t bw = kPairBytewise | (in ? off : k.frames_len);
	return off == kNoOff ? kNoOff : fits ? off + 8 : bw;
}

typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

/* load J of this lane: half (lane & 1) of the pair's packet J, whose
 * pair_src lane J of the pair holds in @my (quad_perm broadcast) */
template <int J>
__device__ __forceinline__ uint4 pair_load(const KParams &k, uint64_t my)
{
	constexpr int B = J ? 0xF5 : 0xA0; /* quad_perm [1,1,3,3] : [0,0,2,2] */
	const uint32_t lo = mdpp<B>((uint32_t)my), hi = mdpp<B>((uint32_t)(my >> 32));
	const uint64_t s = (uint64_t)hi << 32 | lo;
	const uint8_t *a = (hi >> 31) ? k.tables : k.frames + s + 16 * (threadIdx.x & 1);
	/* plain loads: the frames stay in L2 for the next use of the same mbuf */
	const u32x4a4 v = *(const u32x4a4 *)a;
	return make_uint4(v.x, v.y, v.z, v.w);
}

/* r[j] = half (lane & 1) of pair packet j  ->  r[h] = half h of this lane's packet */
__device__ __forceinline__ void pair_exchange(uint4 r[2])
{
	const bool odd = threadIdx.x & 1;
	/* quad_perm [1,0,3,2]: the odd lane sends the even packet's second
	 * half, the even lane the odd packet's first half */
	const uint4 x = sel4(odd, r[0], r[1]);
	const uint4 y = make_uint4(mdpp<0xB1>(x.x), mdpp<0xB1>(x.y), mdpp<0xB1>(x.z), mdpp<0xB1>(x.w));
	r[0] = sel4(odd, y, r[0]);
	r[1] = sel4(odd, r[1], y);
}

template <int MODE, bool TLDS, int NT, int VF>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4)))
classify_pair_kernel(KParams k)
{
	extern __shared__ uint4 smem[];
	uint32_t *hist = (uint32_t *)smem;
	uint8_t *lds_tab = (uint8_t *)(hist + ((k.max_rt + 3) & ~3u));
	const int tid = threadIdx.x;
	for (uint32_t i = tid; i < k.max_rt; i += NT)
		hist[i] = 0;
	const uint8_t *tab = TLDS ? lds_tab : k.tables;
	if (TLDS) {
		const uint4 *src = (const uint4 *)k.tables;
		uint4 *dst = (uint4 *)lds_tab;
		for (uint32_t i = tid; i < k.tables_lds_bytes / 16; i += NT)
			dst[i] = src[i];
	}
	Tables tb;
	tb.ipt = (const uint2 *)tab;
	tb.rtab = (const RtEntry *)(tab + k.off_rt);
	tb.flow = tab + k.off_flow;
	tb.toep = (const uint32_t *)(tab + k.off_toep);
	tb.seed = (const uint32_t *)(tab + k.off_seed);
	tb.crc = (const uint32_t *)(tab + k.off_crc);
	__syncthreads();

	Counters cnt = {0, 0, 0, 0};
	const uint64_t step = gridDim.x;
	const uint64_t *offs_src = k.offs ? k.offs : (const uint64_t *)k.tables;
	auto ok = [&](uint64_t tt) { return tt < k.ntiles && tt * NT + tid < k.n; };
	auto ld_off = [&](uint64_t tt) -> uint64_t {
		return user_off(k, offs_src[k.offs && ok(tt) ? tt * NT + tid : 0]);
	};
	auto src_of = [&](uint64_t tt, uint64_t raw) -> uint64_t {
		return pair_src(k, !ok(tt) ? kNoOff : k.offs ? raw : (tt * NT + tid) * k.stride);
	};
	auto pref = [&](uint64_t tt, uint32_t pr[2]) {
		const uint64_t i = ok(tt) ? tt * NT + tid : 0;
		pr[0] = *(k.olflags ? k.olflags + i : side_dummy<uint8_t>(k, i));
		if (MODE == GCL_HASH_NIC)
			pr[1] = *(k.rss ? k.rss + i : side_dummy<uint32_t>(k, i));
	};
	auto issue = [&](uint64_t my, uint4 r[2]) {
		r[0] = pair_load<0>(k, my);
		r[1] = pair_load<1>(k, my);
	};
	/* the landed halves -> this lane's header dwords (frame bytes 12-39;
	 * d10, bytes 40-43, is not fetched: avail 40 sends ARP to the frame) */
	auto unpack = [&](uint4 r[2], uint64_t my, HdrWords &h) {
		pair_exchange(r);
		if ((my >> 63) && my != kNoOff) { /* bytewise (rare) */
			const uint64_t off = my & ~kPairBytewise;
			r[0] = load16_bytes(k, off + 8);
			r[1] = load16_bytes(k, off + 24);
		}
		h.d3 = r[0].y, h.d5 = r[0].w, h.d6 = r[1].x, h.d7 = r[1].y;
		h.d8 = r[1].z, h.d9 = r[1].w, h.d10 = 0;
	};
	/* a wave whose packets are all plain IPv4 (IHL 5, no FDIR mark) in a
	 * batch without dst_ip hints or the transport pre-hash takes
	 * classify_lean (one ballot), the others classify_core (k.plean) */
	const bool lean_ok = k.plean && !k.dst_hint && !k.trans;
	auto classify = [&](uint64_t tt, const HdrWords &h, const uint32_t pr[2], uint64_t my) {
		const uint32_t fl = k.olflags ? pr[0] & 0xFF : k.default_flags;
		const bool plain = !ok(tt) || ((h.d3 & 0x000FFFFF) == 0x00050008 && !(fl & GCL_F_FDIR_ID));
		if (lean_ok && __all(plain)) {
			if (ok(tt))
				put_verdict_vf<VF>(k, tt * NT + tid, classify_lean<MODE, true>(k, h, tb, fl, pr[1], hist, tid, cnt));
		} else if (ok(tt)) {
			const uint64_t i = tt * NT + tid;
			/* this packet's frame offset, for the ARP target's extra read */
			const uint64_t foff = (my >> 63) ? (my & ~kPairBytewise) : my - 8;
			put_verdict_vf<VF>(k, i, classify_core<MODE, true, false, true, VF>(
			                                 k, h, nullptr, tid, i, tb, hist, cnt, 0, 40, pr, foff));
		}
	};

	uint64_t t = blockIdx.x;
	uint4 ra[2], rb[2];
	uint32_t pra[2] = {0, 0}, prb[2] = {0, 0};
	/* prologue: tiles t and t + step in flight, offsets of the two after */
	uint64_t oa = ld_off(t), ob = ld_off(t + step);
	uint64_t sa = src_of(t, oa);
	issue(sa, ra);
	pref(t, pra);
	oa = ld_off(t + 2 * step);
	uint64_t sb = src_of(t + step, ob);
	issue(sb, rb);
	pref(t + step, prb);
	ob = ld_off(t + 3 * step);
	while (t < k.ntiles) {
		asm volatile("" : "+s"(t));
		HdrWords h;
		unpack(ra, sa, h);
		uint64_t my = sa;
		sa = src_of(t + 2 * step, oa);
		issue(sa, ra);
		classify(t, h, pra, my);
		pref(t + 2 * step, pra);
		oa = ld_off(t + 4 * step);
		t += step;
		/* runs past ntiles too (dummy loads, nothing classified): a path
		 * out of the middle would change the wait counts (classify_kernel) */
		unpack(rb, sb, h);
		my = sb;
		sb = src_of(t + 2 * step, ob);
		issue(sb, rb);
		classify(t, h, prb, my);
		pref(t + 2 * step, prb);
		ob = ld_off(t + 4 * step);
		t += step;
	}
	__syncthreads(); /* every wave's histogram adds are in */
	flush_counters<NT>(k, hist, cnt);
}

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
/* GCL_TUNE_PAIR_LEAN default: classify_pair_kernel's plain-IPv4 waves on
 * classify_lean -- the ingress working set 64.6-65.3 -> 62.7-63.3 us, the
 * random pool unchanged (memory-bound), profiles/r05_pair_lean_ab.jsonl */
constexpr int kDefaultPairLean = 1;
/* GCL_TUNE_DEFER default (Geometry::defer): udp64 328.2-329.1 -> 323.4-324.2
 * us, three fresh processes (profiles/r05_defer_ab.jsonl) */
constexpr int kDefaultDefer = 1;
/* GCL_TUNE_LOOP_LEAN default: bursts whose every packet is plain IPv4 (IHL 5,
 * no FDIR mark, no hint) classified by classify_lean */
constexpr uint32_t kDefaultLoopLean = 1;
/* GCL_TUNE_LOOP_PHASE default ("max,up,down" in ticks; loops of up to
 * kLoopSpecIdleWorkers workers): the poll-phase delay's ceiling and steps.
 * 1 x 1 header records, NIC hash, three fresh processes per form
 * (profiles/r05_phase_ab.jsonl, r05_phase_sweep.jsonl): back to back
 * 3.94-3.98 -> 3.11-3.19 us p50, random phase 3.61-3.90 -> 3.49-3.57, sparse
 * lone bursts unchanged (3.64-4.02 / 3.76-3.79), 2 workers x 2 in flight
 * 3.99-4.01 -> 3.14-3.45; a 200-tick ceiling let the delay outgrow the host's
 * turnaround at a random phase (3.86-4.05) */
constexpr uint32_t kDefaultLoopPhaseMax = 120, kDefaultLoopPhaseUp = 16, kDefaultLoopPhaseDown = 1;
/* GCL_TUNE_LOOP_PREFETCH default (loops of more than kLoopSpecIdleWorkers
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
	uint64_t t0;               /* tickets start after t0 (0; GCL_TUNE_LOOP_T0 tests the
	                              stamps' wrap), a multiple of nslots */
	uint32_t stamps;           /* GCL_LOOP_STAMPS: per-burst stage times into the slot header */
	uint32_t rec_plane;        /* GCL_LOOP_HDR_RECORDS: bytes between the records' chunk
	                              planes (chunk j of packet i at off_hdr + j * rec_plane + 16 i) */
	uint32_t lean;             /* rxloop64_kernel: plain-IPv4 bursts on classify_lean
	                              (GCL_TUNE_LOOP_LEAN=0: always classify_core) */
	uint32_t phase_max;        /* rxloop64_kernel: the poll-phase delay's ceiling in ticks
	                              (0: off; GCL_TUNE_LOOP_PHASE), and its steps */
	uint32_t phase_up, phase_down;
	uint32_t prefetch;         /* rxloop64_kernel: the next ticket's poll issued before a
	                              burst is classified (GCL_TUNE_LOOP_PREFETCH) */
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
 * up after one found by the second.  Round 4's form (GCL_TUNE_LOOP_HYBRID)
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
			 * GCL_TUNE_LOOP_SPEC=0 -- finds every burst "late": on time
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

/* ------------------------------------------------------------------------
 * Synthetic generator kernel: one lane per packet writes its 64-B header.
 */
struct Hdr {
	uint32_t w[16];
	__device__ void b8(int o, uint32_t v) { w[o >> 2] |= (v & 0xFF) << ((o & 3) * 8); }
	__device__ void b16(int o, uint32_t v) { b8(o, v >> 8); b8(o + 1, v); }
	__device__ void b32(int o, uint32_t v) { b16(o, v >> 16); b16(o + 2, v); }
};

__device__ __forceinline__ void gen_eth(Hdr &h, uint64_t srcbits, uint32_t et)
{
	h.b8(0, 0x02); h.b8(5, 0x01); /* dst 02:00:00:00:00:01 */
	h.b8(6, 0x02);
	h.b32(8, (uint32_t)srcbits);
	h.b16(12, et);
}

__device__ __forceinline__ void gen_ipv4(Hdr &h, uint32_t totlen, uint32_t id,
                                         uint32_t proto, uint32_t saddr, uint32_t daddr)
{
	h.b8(14, 0x45);
	h.b16(16, totlen);
	h.b16(18, id);
	h.b16(20, 0x4000);
	h.b8(22, 64);
	h.b8(23, proto);
	h.b32(26, saddr);
	h.b32(30, daddr);
	uint32_t s = 0x4500 + (totlen & 0xFFFF) + (id & 0xFFFF) + 0x4000 + (64u << 8 | proto) +
	             (saddr >> 16) + (saddr & 0xFFFF) + (daddr >> 16) + (daddr & 0xFFFF);
	while (s >> 16)
		s = (s & 0xFFFF) + (s >> 16);
	h.b16(24, ~s & 0xFFFF);
}

struct GParams {
	uint32_t workload, nruntimes;
	uint64_t seed, n, stride;
	uint32_t rank, world;
	uint64_t shard_block;
	const uint64_t *zipf;
	uint32_t nflows;
	uint8_t *frames;
	uint8_t *olflags;
	uint32_t *rss;
	uint16_t *pkt_len;
};

__device__ __forceinline__ uint32_t runtime_ip(uint32_t r) { return 0x0A000000u + r + 1; }

__global__ void __launch_bounds__(256) generate_kernel(GParams p)
{
	uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= p.n)
		return;
	uint64_t g = j;
	if (p.shard_block && p.world > 1)
		g = ((j / p.shard_block) * p.world + p.rank) * p.shard_block + j % p.shard_block;
	const uint64_t r0 = gcl::rw(p.seed, g, 0), r1 = gcl::rw(p.seed, g, 1);
	uint32_t fl = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	uint32_t len = 64;
	Hdr h;
#pragma unroll
	for (int i = 0; i < 16; i++)
		h.w[i] = 0;

	if (p.workload == GCL_WL_UDP64) {
		uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p.nruntimes) >> 32);
		gen_eth(h, r1 >> 32, GCL_ETHTYPE_IP);
		gen_ipv4(h, 50, (uint32_t)(r1 >> 16) & 0xFFFF, 17, (uint32_t)r0, runtime_ip(rt));
		h.b16(34, (uint32_t)(r0 >> 32) & 0xFFFF);
		h.b16(36, (uint32_t)(r0 >> 48));
		h.b16(38, 30);
	} else if (p.workload == GCL_WL_TCP1500_ZIPF) {
		uint32_t lo = 0, hi = p.nflows - 1;
		while (lo < hi) {
			uint32_t mid = lo + (hi - lo) / 2;
			if (r0 < p.zipf[mid])
				hi = mid;
			else
				lo = mid + 1;
		}
		const uint32_t flow = lo;
		const uint64_t fr = gcl::rw(p.seed ^ 0xF10F10F10F10F10Full, flow, 0);
		const uint32_t rt = flow % p.nruntimes;
		gen_eth(h, fr >> 16, GCL_ETHTYPE_IP);
		gen_ipv4(h, 1486, (uint32_t)r1 & 0xFFFF, 6, (uint32_t)fr, runtime_ip(rt));
		h.b16(34, (uint32_t)(fr >> 32) & 0xFFFF);
		h.b16(36, (uint32_t)(fr >> 48));
		h.b32(38, (uint32_t)(r1 >> 32));
		h.b8(46, 0x50);
		h.b8(47, 0x10);
		h.b16(48, 0xFFFF);
		len = 1500;
	} else {
		const uint64_t r2 = gcl::rw(p.seed, g, 2);
		const uint32_t kind = (uint32_t)r0 % 100;
		const uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p.nruntimes) >> 32);
		bool unreg = (uint32_t)(r0 >> 40) % 20 == 0;
		uint32_t dst = unreg ? (0xC0A80000u | (uint32_t)(r1 >> 48)) : runtime_ip(rt);
		if (kind < 70) {
			len = 64 + (uint32_t)(r1 >> 32) % (9014 - 64 + 1);
			uint32_t proto = (r0 >> 32) & 1 ? 6 : 17;
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_IP);
			gen_ipv4(h, len - 14, (uint32_t)r2 & 0xFFFF, proto, (uint32_t)r2, dst);
			h.b16(34, (uint32_t)(r2 >> 32) & 0xFFFF);
			h.b16(36, (uint32_t)(r2 >> 48));
		} else if (kind < 90) {
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_IPV6);
			h.b8(14, 0x60);
			h.b16(18, (uint32_t)(r1 >> 32) & 0x1FFF);
			h.b8(20, 17);
			h.b8(21, 64);
			h.b32(22, (uint32_t)r2);
			h.b32(38, dst);
			fl = 0;
			len = 54 + ((uint32_t)(r1 >> 32) & 0x1FFF);
			len = len < 60 ? 60 : len;
		} else {
			unreg = (uint32_t)(r0 >> 40) % 10 == 0;
			dst = unreg ? (0xC0A80000u | (uint32_t)(r1 >> 48)) : runtime_ip(rt);
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_ARP);
			h.b16(14, 1);
			h.b16(16, 0x0800);
			h.b8(18, 6);
			h.b8(19, 4);
			h.b16(20, (r0 >> 33) & 1 ? GCL_ARP_OP_REPLY : GCL_ARP_OP_REQUEST);
			h.b32(24, (uint32_t)(r2 >> 16));
			h.b32(28, (uint32_t)r2);
			h.b32(38, dst);
			fl = 0;
			len = 60;
		}
	}
	uint4 *dst4 = (uint4 *)(p.frames + j * p.stride);
#pragma unroll
	for (int i = 0; i < 4; i++)
		dst4[i] = make_uint4(h.w[4 * i], h.w[4 * i + 1], h.w[4 * i + 2], h.w[4 * i + 3]);
	if (p.olflags)
		p.olflags[j] = (uint8_t)fl;
	if (p.rss)
		p.rss[j] = (uint32_t)gcl::rw(p.seed, g, 3);
	if (p.pkt_len)
		p.pkt_len[j] = (uint16_t)len;
}

} // namespace

/* --------------------------------------------------------------------------
 * gcl_access_probe: the fewest memory requests one classify launch over the
 * batch could make, without the classification -- the layout's own ceiling.
 * One lane per packet issues one 16-B load of the 128-B line holding frame
 * byte 0 and, only when frame bytes [0, 40) (Ethernet, an IHL-5 IPv4 header,
 * the L4 ports: the common case's bytes) run into the next line, one of that
 * line too; lines shared by neighbouring packets are fetched once by the L2.
 * It also loads the packet's offset, ol_flags and hash.rss when the batch
 * has them, and stores VB bytes per packet write-through like the verdict
 * stores.  Four packets per lane are in flight before any load is used.
 */
template <int VB>
__global__ void __launch_bounds__(256) access_probe_kernel(KParams k)
{
	const uint64_t G = (uint64_t)gridDim.x * 256;
	const uint64_t base = (uint64_t)(uintptr_t)k.frames, end = base + k.frames_len;
	uint32_t acc = 0;
	for (uint64_t p0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; p0 < k.n; p0 += 4 * G) {
		uint4 v[4], w[4];
		uint32_t side[4];
#pragma unroll
		for (int u = 0; u < 4; u++) {
			const uint64_t p = p0 + u * G;
			v[u] = w[u] = make_uint4(0, 0, 0, 0);
			side[u] = 0;
			if (p < k.n) {
				const uint64_t off = k.offs ? user_off(k, k.offs[p]) : p * k.stride;
				const uint64_t A = base + off, a0 = A & ~15ull, a1 = (A + 39) & ~127ull;
				if (a0 >= base && a0 + 16 <= end)
					v[u] = gcl::load16_nt((const void *)a0);
				if (a1 > a0 && a1 + 16 <= end) /* [0, 40) crosses into the next line */
					w[u] = gcl::load16_nt((const void *)a1);
				side[u] = (k.olflags ? k.olflags[p] : 0u) ^ (k.rss ? k.rss[p] : 0u);
			}
		}
#pragma unroll
		for (int u = 0; u < 4; u++) {
			const uint64_t p = p0 + u * G;
			const uint32_t x = v[u].x ^ v[u].y ^ v[u].z ^ v[u].w ^ w[u].x ^ side[u];
			acc ^= x ^ w[u].y ^ w[u].z ^ w[u].w;
			if (p < k.n) {
				if (VB == 1)
					__hip_atomic_store((uint8_t *)k.verdicts + p, (uint8_t)x, __ATOMIC_RELAXED,
					                   __HIP_MEMORY_SCOPE_SYSTEM);
				else if (VB == 2)
					__hip_atomic_store((uint16_t *)k.verdicts + p, (uint16_t)x, __ATOMIC_RELAXED,
					                   __HIP_MEMORY_SCOPE_SYSTEM);
				else if (VB == 4)
					__hip_atomic_store((uint32_t *)k.verdicts + p, x, __ATOMIC_RELAXED,
					                   __HIP_MEMORY_SCOPE_SYSTEM);
				else
					__hip_atomic_store((uint64_t *)k.verdicts + p, (uint64_t)x, __ATOMIC_RELAXED,
					                   __HIP_MEMORY_SCOPE_SYSTEM);
			}
		}
	}
	if (acc == 0x9E3779B9u && k.stats) /* keeps every load live; practically never */
		k.stats[GCL_NR_STATS - 1] = acc;
}

/* --------------------------------------------------------------------------
 * Header gather for gcl_classify_host's COPY transport over per-packet
 * offsets (the reference's mbuf pool, frame data at element + 344): frame
 * bytes [0, kGatherRow) of every packet, read out of mapped host memory into
 * dense kGatherRow-byte rows of an HBM slab, which the batch kernel then
 * classifies like fixed slots.  kGatherRow covers everything rx_one_pkt can
 * read (ports at 14 + 4 * IHL + 4 <= 78 for IHL 15).  Eight lanes per
 * packet: lanes 0-5 load the six 16-B-aligned chunks that cover the row at
 * any alignment (coalesced into the fewest 64-B requests), lanes 0-4 funnel
 * their chunk and the next lane's into one row chunk.  Bytes at or past
 * frames_len, and every byte of a frame whose offset is, read 0.
 */
constexpr uint32_t kGatherRow = GCL_GATHER_ROW;

__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t b)
{
	return b ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * b)) : lo;
}

__global__ void __launch_bounds__(256) header_gather_kernel(const uint8_t *frames, uint64_t frames_len,
                                                            const uint64_t *offs, uint64_t n,
                                                            uint8_t *slab)
{
	const uint64_t G = (uint64_t)gridDim.x * 32; /* packets per grid pass */
	const uint32_t q = threadIdx.x & 7;
	const uint64_t base = (uint64_t)(uintptr_t)frames, end = base + frames_len;
	for (uint64_t p = (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 3); p < n; p += G) {
		const uint64_t o0 = offs[p];
		const uint64_t off = o0 < frames_len ? o0 : frames_len;
		const uint64_t A = base + off;
		const uint64_t c = (A & ~15ull) + 16ull * q;
		uint4 v = make_uint4(0, 0, 0, 0);
		if (q < 6 && off < frames_len) {
			if (c >= base && c + 16 <= end) {
				v = *(const uint4 *)c;
			} else { /* the region's first or last chunk: bytewise, 0 past it */
				uint32_t w[4];
				for (int i = 0; i < 4; i++) {
					w[i] = 0;
					for (int j = 0; j < 4; j++) {
						const uint64_t a = c + 4 * i + j;
						if (a >= base && a < end)
							w[i] |= (uint32_t)*(const uint8_t *)a << (8 * j);
					}
				}
				v = make_uint4(w[0], w[1], w[2], w[3]);
			}
		}
		/* the next lane's chunk (a packet's lanes are 8 consecutive lanes) */
		const uint32_t nx = __shfl_down(v.x, 1, 8), ny = __shfl_down(v.y, 1, 8);
		const uint32_t nz = __shfl_down(v.z, 1, 8), nw = __shfl_down(v.w, 1, 8);
		if (q < kGatherRow / 16) {
			const uint32_t sh = (uint32_t)(A & 15), d = sh >> 2, b = sh & 3;
			const uint32_t w[8] = {v.x, v.y, v.z, v.w, nx, ny, nz, nw};
			uint32_t r[4];
#pragma unroll
			for (int i = 0; i < 4; i++) {
				const uint32_t lo = d == 0 ? w[i] : d == 1 ? w[i + 1] : d == 2 ? w[i + 2] : w[i + 3];
				const uint32_t hi = d == 0 ? w[i + 1] : d == 1 ? w[i + 2] : d == 2 ? w[i + 3] : w[i + 4];
				r[i] = funnel(lo, hi, b);
			}
			*(uint4 *)(slab + p * kGatherRow + 16 * q) = make_uint4(r[0], r[1], r[2], r[3]);
		}
	}
}

/* ==========================================================================
 * Host side of the C ABI.
 */
struct gcl_ctx {
	int device;
	struct gcl_cfg cfg;
	int num_cus;
	/* host mirror of the tables (dp.clients_by_id + ip_to_proc + flow_tbl) */
	struct Rt {
		bool present;
		uint32_t ip;
		uint16_t tc, active;
		uint8_t flow[GCL_NCPU];
		uint32_t trans_seed;
	};
	std::vector<Rt> rt;
	uint32_t ipt_slots;
	uint32_t ipt_seed;    /* lookup3 initval the current image's buckets use */
	uint32_t off_rt, off_flow, off_toep, off_seed, off_crc, image_cap, image_bytes;
	uint32_t flow_used;
	bool dirty;
	bool loop_dirty;              /* tables changed since the rx loop's last image */
	struct gcl_rxloop *loop;      /* running persistent loop, or NULL */
	/* Two device images + pinned staging.  No per-launch events: each image
	 * remembers the streams that launched on it; when it stops being current
	 * an event is recorded on each of them, and the upload that next
	 * overwrites it waits on those events. */
	uint8_t *dimg[2];
	struct ImgUsers {
		int n;
		bool retired; /* events recorded, image not current */
		hipStream_t st[kImgUsers];
		hipEvent_t ev[kImgUsers];
	} users[2];
	uint8_t *staging;
	hipEvent_t staging_free;
	hipEvent_t tables_ready;   /* recorded after each table upload */
	hipStream_t tables_stream; /* stream of the last upload */
	bool tables_done;          /* tables_ready known complete */
	/* end-to-end (host buffers) resources, allocated on first use */
	struct E2E {
		int nstreams;
		uint64_t chunk;
		hipStream_t st[4];
		uint8_t *slab[4];        /* header granules of one chunk */
		uint8_t *side[4];        /* per-packet olflags/rss/fdir of one chunk */
		uint8_t *verd[4];        /* verdicts of one chunk (sized for 8-B verdicts) */
		uint64_t *acc;           /* device counts | stats */
	} e2e;
	int cur;
	hipStream_t last_stream;
	/* profiling */
	std::vector<hipEvent_t> ev_pool;
	std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
	double prof_ms;
	uint64_t prof_launches;
	uint32_t prof_every;  /* time one launch in prof_every (gcl_profile_sample) */
	uint64_t prof_seq;
	/* geometry overrides, for the tests that cover every launch shape */
	int tune_tables; /* GCL_TUNE_TABLES: 0 auto, 1 global, 2 lds-if-fits */
	int tune_depth;  /* GCL_TUNE_DEPTH: tiles in flight per block (1 or 2) */
	int tune_threads; /* GCL_TUNE_THREADS: 256, 512 or 1024 lanes per block */
	int tune_grid;    /* GCL_TUNE_GRID: blocks per launch (0: the persistent grid) */
	int tune_bpc;     /* GCL_TUNE_BLOCKS_PER_CU: cap on blocks per CU (0: none) */
	int tune_defer;   /* GCL_TUNE_DEFER: Geometry::defer for eligible batches (0-2) */
	int tune_plean;   /* GCL_TUNE_PAIR_LEAN: KParams::plean (0: off, tests and A/Bs) */
};

extern "C" {
uint32_t gcl_jenkins_hash(const void *key, size_t len);
uint32_t gcl_toeplitz(const uint8_t *key, size_t keylen, const uint8_t *input, size_t len);
}

static uint32_t pow2_at_least(uint32_t x)
{
	uint32_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

extern "C" int gcl_open(int hip_device, const struct gcl_cfg *cfg, struct gcl_ctx **out)
{
	int ndev = 0;
	if (!cfg || !out || cfg->max_runtimes == 0 || cfg->max_runtimes > GCL_MAX_PROC ||
	    cfg->hash_mode > GCL_HASH_TOEPLITZ)
		return -EINVAL;
	if ((cfg->flags & GCL_CFG_VERDICT2) &&
	    ((cfg->flags & (GCL_CFG_VERDICT4 | GCL_CFG_TRANS_HASH | GCL_CFG_VERDICT1)) ||
	     cfg->thread_bits > 8 || ((uint64_t)cfg->max_runtimes << cfg->thread_bits) > GCL_V2_QUEUES))
		return -EINVAL;
	if ((cfg->flags & GCL_CFG_VERDICT1) &&
	    ((cfg->flags & (GCL_CFG_VERDICT4 | GCL_CFG_TRANS_HASH)) || cfg->thread_bits > 7 ||
	     ((uint64_t)cfg->max_runtimes << cfg->thread_bits) > GCL_V1_QUEUES))
		return -EINVAL;
	if (hipGetDeviceCount(&ndev) != hipSuccess || hip_device < 0 || hip_device >= ndev)
		return -ENODEV;
	if (hipSetDevice(hip_device) != hipSuccess)
		return -ENODEV;

	gcl_ctx *c = new (std::nothrow) gcl_ctx();
	if (!c)
		return -ENOMEM;
	c->device = hip_device;
	c->cfg = *cfg;
	HipErr he;
	he(hipDeviceGetAttribute(&c->num_cus, hipDeviceAttributeMultiprocessorCount, hip_device));
	c->rt.resize(cfg->max_runtimes);
	c->ipt_slots = pow2_at_least(cfg->max_runtimes * 2 < 16 ? 16 : cfg->max_runtimes * 2);
	c->off_rt = c->ipt_slots * 8;
	c->off_flow = c->off_rt + cfg->max_runtimes * 16;
	/* the Toeplitz LUT offset depends on flow_used; reserve worst case */
	c->image_cap = c->off_flow + cfg->max_runtimes * GCL_NCPU + 16 + kToepBytes +
	               cfg->max_runtimes * 4 + 16 + kCrcBytes;
	c->image_bytes = 0;
	c->flow_used = 0;
	c->dirty = true;
	c->loop_dirty = true;
	c->cur = 0;
	c->last_stream = nullptr;
	c->prof_ms = 0;
	c->prof_launches = 0;
	c->prof_every = 1;
	c->prof_seq = 0;
	{
		const char *e = getenv("GCL_TUNE_TABLES");
		c->tune_tables = e ? atoi(e) : 0;
		e = getenv("GCL_TUNE_DEPTH");
		c->tune_depth = e ? atoi(e) : 0;
		e = getenv("GCL_TUNE_THREADS");
		c->tune_threads = e ? atoi(e) : 0;
		if (c->tune_threads != 256 && c->tune_threads != 512 && c->tune_threads != 1024)
			c->tune_threads = 0;
		e = getenv("GCL_TUNE_GRID");
		c->tune_grid = e ? atoi(e) : 0;
		e = getenv("GCL_TUNE_BLOCKS_PER_CU");
		c->tune_bpc = e ? atoi(e) : 0;
		e = getenv("GCL_TUNE_PAIR_LEAN");
		c->tune_plean = e ? atoi(e) != 0 : kDefaultPairLean;
		e = getenv("GCL_TUNE_DEFER");
		c->tune_defer = e ? std::min(std::max(atoi(e), 0), 2) : kDefaultDefer;
	}
	c->dimg[0] = c->dimg[1] = nullptr;
	for (int i = 0; i < 2; i++) {
		if (hipMalloc(&c->dimg[i], c->image_cap) != hipSuccess)
			goto fail;
		c->users[i].n = 0;
		c->users[i].retired = false;
		for (int j = 0; j < kImgUsers; j++)
			he(hipEventCreateWithFlags(&c->users[i].ev[j], hipEventDisableTiming));
	}
	if (hipHostMalloc(&c->staging, c->image_cap, hipHostMallocDefault) != hipSuccess)
		goto fail;
	he(hipEventCreateWithFlags(&c->staging_free, hipEventDisableTiming));
	he(hipEventCreateWithFlags(&c->tables_ready, hipEventDisableTiming));
	if (he.bad()) {
		(void)hipGetLastError();
		(void)hipHostFree(c->staging);
		goto fail;
	}
	c->tables_stream = nullptr;
	c->tables_done = true;
	memset(&c->e2e, 0, sizeof(c->e2e));
	*out = c;
	return 0;
fail:
	for (int i = 0; i < 2; i++)
		if (c->dimg[i])
			(void)hipFree(c->dimg[i]);
	delete c;
	return -ENOMEM;
}

extern "C" void gcl_close(struct gcl_ctx *c)
{
	if (!c)
		return;
	(void)hipSetDevice(c->device);
	if (c->loop)
		gcl_rxloop_stop(c->loop);
	(void)hipDeviceSynchronize();
	for (int i = 0; i < 2; i++) {
		(void)hipFree(c->dimg[i]);
		for (int j = 0; j < kImgUsers; j++)
			(void)hipEventDestroy(c->users[i].ev[j]);
	}
	(void)hipHostFree(c->staging);
	(void)hipEventDestroy(c->staging_free);
	(void)hipEventDestroy(c->tables_ready);
	for (int i = 0; i < c->e2e.nstreams; i++) {
		(void)hipStreamDestroy(c->e2e.st[i]);
		(void)hipFree(c->e2e.slab[i]);
		(void)hipFree(c->e2e.side[i]);
		(void)hipFree(c->e2e.verd[i]);
	}
	(void)hipFree(c->e2e.acc);
	for (auto &pr : c->ev_pending) {
		(void)hipEventDestroy(pr.first);
		(void)hipEventDestroy(pr.second);
	}
	for (auto e : c->ev_pool)
		(void)hipEventDestroy(e);
	delete c;
}

static uint32_t ip_owner(const gcl_ctx *c, uint32_t ip)
{
	for (uint32_t i = 0; i < c->cfg.max_runtimes; i++)
		if (c->rt[i].present && c->rt[i].ip == ip)
			return i;
	return kEmpty;
}

extern "C" int gcl_runtime_set(struct gcl_ctx *c, uint16_t uniqid, uint32_t ip_host,
                               uint16_t thread_count, uint16_t active_count,
                               const uint16_t *flow_tbl)
{
	if (!c || uniqid >= c->cfg.max_runtimes || thread_count == 0 ||
	    thread_count > GCL_NCPU || active_count > thread_count)
		return -EINVAL;
	if ((c->cfg.flags & (GCL_CFG_VERDICT2 | GCL_CFG_VERDICT1)) && thread_count > (1u << c->cfg.thread_bits))
		return -EINVAL; /* its queues would not fit the 2-byte verdict */
	if (active_count) {
		if (!flow_tbl)
			return -EINVAL;
		for (int i = 0; i < thread_count; i++)
			if (flow_tbl[i] >= thread_count)
				return -EINVAL;
	}
	uint32_t owner = ip_owner(c, ip_host);
	if (owner != kEmpty && owner != uniqid)
		return -EEXIST; /* dp_clients.c:174-179 */
	gcl_ctx::Rt &r = c->rt[uniqid];
	if (!r.present)
		r.trans_seed = 0;
	r.present = true;
	r.ip = ip_host;
	r.tc = thread_count;
	r.active = active_count;
	memset(r.flow, 0, sizeof(r.flow));
	if (active_count)
		for (int i = 0; i < thread_count; i++)
			r.flow[i] = (uint8_t)flow_tbl[i];
	c->dirty = true;
	c->loop_dirty = true;
	return 0;
}

extern "C" int gcl_runtime_set_trans_seed(struct gcl_ctx *c, uint16_t uniqid, uint32_t seed)
{
	if (!c || !(c->cfg.flags & GCL_CFG_TRANS_HASH))
		return -EINVAL;
	if (uniqid >= c->cfg.max_runtimes || !c->rt[uniqid].present)
		return -ENOENT;
	c->rt[uniqid].trans_seed = seed;
	c->dirty = true;
	c->loop_dirty = true;
	return 0;
}

extern "C" int gcl_runtime_del(struct gcl_ctx *c, uint16_t uniqid)
{
	if (!c || uniqid >= c->cfg.max_runtimes || !c->rt[uniqid].present)
		return -ENOENT;
	c->rt[uniqid] = gcl_ctx::Rt();
	c->dirty = true;
	c->loop_dirty = true;
	return 0;
}

static uint32_t jhash_u32_host(uint32_t ip, uint32_t initval)
{
	auto rot = [](uint32_t x, int k) { return (x << k) | (x >> (32 - k)); };
	uint32_t a = 0xdeadbeefu + 4u + initval, b = a, c = a;
	a += ip;
	c ^= b; c -= rot(b, 14);  /* final(), base/jenkins_hash.c:114-123 */
	a ^= c; a -= rot(c, 11);
	b ^= a; b -= rot(a, 25);
	c ^= b; c -= rot(b, 16);
	a ^= c; a -= rot(c, 4);
	b ^= a; b -= rot(a, 14);
	c ^= b; c -= rot(b, 24);
	return c;
}

/* Cuckoo placement of every present runtime's IP into @nb two-slot buckets
 * (the layout ipt_lookup reads).  Random-walk eviction; false if some key
 * could not be placed with this seed. */
static bool ipt_build(const gcl_ctx *c, uint2 *ipt, uint32_t nb, uint32_t seed)
{
	const uint32_t m = nb - 1;
	for (uint32_t i = 0; i < 2 * nb; i++)
		ipt[i] = make_uint2(0, kEmpty);
	for (uint32_t u = 0; u < c->cfg.max_runtimes; u++) {
		if (!c->rt[u].present)
			continue;
		uint2 cur = make_uint2(c->rt[u].ip, u);
		bool placed = false;
		for (uint32_t kick = 0; kick < 8 * nb + 64 && !placed; kick++) {
			const uint32_t h = jhash_u32_host(cur.x, seed);
			const uint32_t bs[2] = {h & m, ((h << 16) | (h >> 16)) & m};
			for (int j = 0; j < 4 && !placed; j++) {
				uint2 &e = ipt[2 * bs[j >> 1] + (j & 1)];
				if (e.y == kEmpty) {
					e = cur;
					placed = true;
				}
			}
			if (!placed) { /* evict a pseudo-random resident of one bucket */
				uint2 &e = ipt[2 * bs[(kick >> 1) & 1] + (kick & 1)];
				std::swap(e, cur);
			}
		}
		if (!placed)
			return false;
	}
	return true;
}

/* Serialise the host mirror into the staging buffer. Returns image bytes. */
static uint32_t build_image(gcl_ctx *c)
{
	uint8_t *img = c->staging;
	const uint32_t max_rt = c->cfg.max_runtimes;
	uint2 *ipt = (uint2 *)img;
	/* load <= 1/2 per slot: seed 0 practically always places every key */
	bool placed = false;
	for (uint32_t seed = 0; seed < 256 && !placed; seed++) {
		placed = ipt_build(c, ipt, c->ipt_slots / 2, seed);
		c->ipt_seed = seed;
	}
	if (!placed)
		return 0; /* no seed placed every key: callers return -ENOSPC */
	RtEntry *re = (RtEntry *)(img + c->off_rt);
	const uint32_t fo = 0;
	for (uint32_t u = 0; u < max_rt; u++) {
		const gcl_ctx::Rt &r = c->rt[u];
		RtEntry e = {};
		if (r.present) {
			uint64_t M = r.tc == 1 ? 0 : (UINT64_MAX / r.tc + 1);
			e.m_lo = (uint32_t)M;
			e.m_hi = (uint32_t)(M >> 32);
			e.tc = r.tc;
			e.active = r.active;
			/* no flow_tbl bytes: the device steers to a slot, the host
			 * post-pass resolves it against the live flow_tbl */
			e.flow_off = 0;
		}
		re[u] = e;
	}
	c->flow_used = fo;
	c->off_toep = align16(c->off_flow + fo);
	uint32_t bytes = c->off_toep;
	if (c->cfg.hash_mode == GCL_HASH_TOEPLITZ) {
		uint32_t *lut = (uint32_t *)(img + c->off_toep);
		for (int i = 0; i < 12; i++)
			for (int v = 0; v < 256; v++) {
				uint8_t in[12] = {0};
				in[i] = (uint8_t)v;
				lut[i * 256 + v] = gcl_toeplitz(c->cfg.rss_key, 40, in, 12);
			}
		bytes += kToepBytes;
	}
	c->off_seed = c->off_crc = 0;
	if (c->cfg.flags & GCL_CFG_TRANS_HASH) {
		c->off_seed = bytes;
		uint32_t *seed = (uint32_t *)(img + bytes);
		for (uint32_t u = 0; u < max_rt; u++)
			seed[u] = c->rt[u].present ? c->rt[u].trans_seed : 0;
		bytes = align16(bytes + max_rt * 4);
		c->off_crc = bytes;
		uint32_t *T = (uint32_t *)(img + bytes);
		for (uint32_t b = 0; b < 256; b++) {
			uint32_t x = b;
			for (int i = 0; i < 8; i++)
				x = (x >> 1) ^ (0x82F63B78u & (0u - (x & 1)));
			T[b] = x;
		}
		for (int t = 1; t < 8; t++)
			for (uint32_t b = 0; b < 256; b++)
				T[t * 256 + b] = (T[(t - 1) * 256 + b] >> 8) ^ T[T[(t - 1) * 256 + b] & 0xFF];
		bytes += kCrcBytes;
	}
	c->image_bytes = align16(bytes);
	return c->image_bytes;
}

static hipEvent_t prof_event(gcl_ctx *c)
{
	if (!c->ev_pool.empty()) {
		hipEvent_t e = c->ev_pool.back();
		c->ev_pool.pop_back();
		return e;
	}
	hipEvent_t e = nullptr;
	return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

typedef void (*ClassifyFn)(KParams);

/* Persistent grid of @fn (@nt-lane blocks, @lds bytes of LDS each): as many
 * blocks per CU as fit, capped at @bpc_cap (or @grid blocks when > 0),
 * never more than tiles. */
static hipError_t launch_fn(ClassifyFn fn, int nt, KParams k, uint32_t lds, int num_cus,
                            int bpc_cap, int grid_set, hipStream_t s)
{
	static std::mutex mu;
	static std::map<std::pair<const void *, uint32_t>, int> occ_cache;
	static std::set<const void *> raised;
	int occ;
	{
		std::lock_guard<std::mutex> g(mu);
		if (lds > 64 * 1024 && !raised.count((const void *)fn)) {
			const hipError_t e = hipFuncSetAttribute(
			        (const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
			if (e != hipSuccess)
				return e;
			raised.insert((const void *)fn);
		}
		const auto key = std::make_pair((const void *)fn, lds);
		auto it = occ_cache.find(key);
		if (it == occ_cache.end()) {
			int o = 0;
			if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, nt, lds) != hipSuccess || o < 1)
				o = 1;
			it = occ_cache.emplace(key, o).first;
		}
		occ = it->second;
	}
	if (bpc_cap > 0 && bpc_cap < occ)
		occ = bpc_cap;
	k.ntiles = (k.n + nt - 1) / nt;
	uint64_t grid = (uint64_t)num_cus * (uint64_t)occ;
	if (grid_set > 0)
		grid = (uint64_t)grid_set;
	if (grid > k.ntiles)
		grid = k.ntiles;
	if (grid < 1)
		grid = 1;
	hipLaunchKernelGGL(fn, dim3((unsigned)grid), dim3(nt), lds, s, k);
	return hipGetLastError();
}

/* Launch geometry (measured on MI355X, choose_geometry) */
struct Geometry {
	int threads;  /* packets per tile = lanes per block */
	int depth;    /* tiles in flight per block */
	int bpc_cap;  /* blocks per CU */
	int grid;     /* blocks per launch when > 0 (GCL_TUNE_GRID) */
	bool pair;    /* classify_pair_kernel (GENERAL batches): [8, 40) per packet by lane pairs */
	int defer;    /* classify_kernel with 1-/2-B verdicts kept in LDS (and past a full
	                 buffer in kVregs registers per lane) and written in batches: 1 where
	                 that takes <= 2 writes per block, 2 always (tests) */
};

/* geo.defer: what the CU's LDS leaves the block at geo.bpc_cap blocks per
 * CU holds k.vcap tiles of verdicts -- at most the block's share of the
 * batch, and only where that takes at most two writes per block */
template <int MODE, int DEPTH, int NT>
static hipError_t launch_nt(KParams k, bool tlds, uint32_t lds, int num_cus, const Geometry &geo,
                            hipStream_t s)
{
	k.vcap = 0;
	k.vregs = 0;
	if (geo.defer) {
		const uint32_t vb = (k.cflags & GCL_CFG_VERDICT1) ? 1 : 2;
		const uint32_t base = align16(lds);
		const uint32_t per_cu = 160 * 1024 / (uint32_t)std::max(geo.bpc_cap, 1);
		const uint64_t blocks = geo.grid > 0 ? (uint64_t)geo.grid : (uint64_t)num_cus * std::max(geo.bpc_cap, 1);
		const uint64_t want = ((k.n + NT - 1) / NT + blocks - 1) / blocks;
		const uint64_t room = per_cu > base ? (per_cu - base) / (NT * vb) : 0;
		const uint64_t rcap = kVregs * 4 / vb; /* tiles the registers hold past a full buffer */
		if (room && (2 * (room + rcap) >= want || geo.defer == 2)) {
			k.vcap = (uint32_t)std::min(want, room);
			k.vregs = rcap && want > room;
			lds = base + k.vcap * NT * vb;
		}
	}
	const ClassifyFn fn = tlds ? classify_kernel<MODE, true, DEPTH, NT> : classify_kernel<MODE, false, DEPTH, NT>;
	return launch_fn(fn, NT, k, lds, num_cus, geo.bpc_cap, geo.grid, s);
}

template <int MODE, int NT>
static hipError_t launch_pair(const KParams &k, bool tlds, uint32_t lds, int num_cus, const Geometry &geo,
                              hipStream_t s)
{
	/* the iokernel's ingress format, 2-byte queue verdicts, compiled in;
	 * every other format reads k.cflags.  25 % fewer static VALU
	 * instructions and SGPR spills 27 -> 8, but the working-set row is
	 * unchanged (96.5-97.3 us, profiles/r03_ws_ab_vf2.jsonl): the loop is
	 * not bound by them */
	const bool v2 = (k.cflags & GCL_CFG_VERDICT2) != 0;
	ClassifyFn fn = v2 ? (tlds ? classify_pair_kernel<MODE, true, NT, 2>
	                           : classify_pair_kernel<MODE, false, NT, 2>)
	                   : (tlds ? classify_pair_kernel<MODE, true, NT, 0>
	                           : classify_pair_kernel<MODE, false, NT, 0>);
	return launch_fn(fn, NT, k, lds, num_cus, geo.bpc_cap, geo.grid, s);
}

template <int MODE>
static hipError_t launch_mode(const KParams &k, bool tlds, const Geometry &geo,
                              uint32_t tab_lds, uint32_t hist_bytes, int num_cus, hipStream_t s)
{
	if (geo.pair) {
		const uint32_t lds = hist_bytes + tab_lds;
		if (geo.threads == 1024)
			return launch_pair<MODE, 1024>(k, tlds, lds, num_cus, geo, s);
		if (geo.threads == 512)
			return launch_pair<MODE, 512>(k, tlds, lds, num_cus, geo, s);
		return launch_pair<MODE, 256>(k, tlds, lds, num_cus, geo, s);
	}
	const uint32_t lds = (uint32_t)geo.threads * 64 + hist_bytes + tab_lds;
#define GCL_LAUNCH(D, T) \
	return launch_nt<MODE, D, T>(k, tlds, lds, num_cus, geo, s)
	if (geo.depth == 2) {
		if (geo.threads == 1024) GCL_LAUNCH(2, 1024);
		if (geo.threads == 512) GCL_LAUNCH(2, 512);
		GCL_LAUNCH(2, 256);
	}
	if (geo.threads == 1024) GCL_LAUNCH(1, 1024);
	if (geo.threads == 512) GCL_LAUNCH(1, 512);
	GCL_LAUNCH(1, 256);
#undef GCL_LAUNCH
}

/*
 * Launch geometry.  Measured on MI355X with tools/cbench.cpp (removed in round 5; interleaved, in
 * one process, against a compute-free kernel of the same traffic): the
 * classifier is fastest with about 1024 resident lanes per CU -- 256-lane
 * blocks x 4 when the tables are small, and for the 1024-runtime tables
 * (37 KiB of LDS per block) 512-lane blocks x 2, so that one LDS copy of the
 * tables serves twice the packets (tcp1500: 234 -> 206 us).  More resident
 * waves than that only add contention (udp64: 446 us at 8 x 256).
 */
static Geometry choose_geometry(const gcl_ctx *c, uint32_t tab_lds, uint32_t hist_bytes,
                                bool general, bool defer_ok)
{
	const uint32_t lds_cu = 160 * 1024, lanes_cu = 1024;
	Geometry g;
	g.depth = 1;
	g.threads = 0;
	/* GENERAL batches run on the lane-pair classify_pair_kernel.  (Round 2's
	 * register-header classify_quad_kernel was removed in round 3, and the
	 * LDS-tile kernel's GENERAL path -- 64-B windows staged per packet --
	 * in round 5: the pair kernel beat both on every row, working set 96
	 * vs 109-111 us, random pool 181 vs 189, profiles/r03_ws_ab.jsonl.) */
	g.pair = general;
	g.defer = defer_ok ? c->tune_defer : 0;
	auto per_block = [&](uint32_t nt) -> uint32_t {
		if (g.pair)
			return hist_bytes + tab_lds;
		return nt * 64 + hist_bytes + tab_lds;
	};
	for (int nt = 256; nt <= 1024 && !g.threads; nt *= 2) {
		const uint32_t pb = per_block((uint32_t)nt);
		if ((lanes_cu / nt) * pb <= lds_cu) {
			g.threads = nt;
			g.bpc_cap = (int)(lanes_cu / (uint32_t)nt);
		}
	}
	if (!g.threads) { /* big tables: as many 256-lane blocks as LDS admits */
		g.threads = 256;
		g.bpc_cap = (int)(lds_cu / per_block(256));
		if (g.bpc_cap < 1)
			g.bpc_cap = 1;
	} else if (g.threads <= 512) {
		/* a second tile in flight per block: 1.1-1.7 % faster on udp64 at
		 * 4 x 256 lanes (profiles/archive/r01_cbench_depth_*); at 2 x 512 lanes (the
		 * 1024-runtime tables) 1 % on the 8 Mi header-split layout, 3.4 % at
		 * 32 Mi, and no change on tcp1500 (profiles/archive/r01_hsplit_geometry.jsonl) */
		g.depth = 2;
	}
	if (c->tune_threads)
		g.threads = c->tune_threads;
	if (c->tune_depth)
		g.depth = c->tune_depth;
	if (c->tune_bpc)
		g.bpc_cap = c->tune_bpc;
	g.grid = c->tune_grid;
	return g;
}

/* Note that a launch on @s reads the current image.  With more streams than
 * kImgUsers, the new stream takes over the oldest one's slot after waiting
 * for what that stream has queued so far, so the slot still covers it. */
static int image_used(gcl_ctx *c, hipStream_t s)
{
	gcl_ctx::ImgUsers &u = c->users[c->cur];
	for (int i = 0; i < u.n; i++)
		if (u.st[i] == s)
			return 0;
	if (u.n == kImgUsers) {
		HipErr he;
		he(hipEventRecord(u.ev[0], u.st[0]));
		he(hipStreamWaitEvent(s, u.ev[0], 0));
		u.st[0] = s;
		return he.bad() ? -EIO : 0;
	}
	u.st[u.n++] = s;
	return 0;
}

static uint32_t verdict_bytes(const gcl_ctx *c)
{
	return (c->cfg.flags & GCL_CFG_VERDICT1) ? 1 : (c->cfg.flags & GCL_CFG_VERDICT2) ? 2
	     : (c->cfg.flags & GCL_CFG_VERDICT4) ? 4 : 8;
}

/* the kernels' cflags: cfg.flags with thread_bits in [31:24] */
static uint32_t kernel_cflags(const gcl_ctx *c)
{
	return (c->cfg.flags & 0xFFFFFFu) | (uint32_t)c->cfg.thread_bits << 24;
}

/* Upload a new table snapshot on @s if anything changed; launches on other
 * streams wait for c->tables_ready before reading the image. */
static int upload_tables(gcl_ctx *c, hipStream_t s)
{
	if (!c->dirty)
		return 0;
	HipErr he;
	he(hipEventSynchronize(c->staging_free));
	if (he.bad())
		return -EIO;
	uint32_t bytes = build_image(c);
	if (!bytes)
		return -ENOSPC;
	const int nxt = c->cur ^ 1;
	/* the image about to be overwritten: wait for its last readers */
	gcl_ctx::ImgUsers &old = c->users[nxt];
	if (old.retired)
		for (int i = 0; i < old.n; i++)
			if (old.st[i] != s)
				he(hipStreamWaitEvent(s, old.ev[i], 0));
	old.n = 0;
	old.retired = false;
	/* the image going out of use: mark where each of its streams is */
	gcl_ctx::ImgUsers &cur = c->users[c->cur];
	for (int i = 0; i < cur.n; i++)
		he(hipEventRecord(cur.ev[i], cur.st[i]));
	cur.retired = true;
	he(hipMemcpyAsync(c->dimg[nxt], c->staging, bytes, hipMemcpyHostToDevice, s));
	he(hipEventRecord(c->staging_free, s));
	he(hipEventRecord(c->tables_ready, s));
	if (he.bad())
		return -EIO; /* dirty stays set: the next call uploads again */
	c->tables_stream = s;
	c->tables_done = false;
	c->cur = nxt;
	c->dirty = false;
	return 0;
}

/* Order a launch on @s after the last table upload: free on the upload's own
 * stream, and skipped once the upload is known to have completed. */
static int wait_tables(gcl_ctx *c, hipStream_t s)
{
	if (c->tables_done || s == c->tables_stream)
		return 0;
	if (hipEventQuery(c->tables_ready) == hipSuccess) {
		c->tables_done = true;
		return 0;
	}
	return hipStreamWaitEvent(s, c->tables_ready, 0) == hipSuccess ? 0 : -EIO;
}

extern "C" int gcl_classify(struct gcl_ctx *c, const struct gcl_batch *b,
                            void *verdicts, uint64_t *runtime_counts,
                            uint64_t *stats, void *hip_stream)
{
	struct gcl_out o = {verdicts, runtime_counts, stats, nullptr};
	return gcl_classify_ex(c, b, &o, hip_stream);
}

extern "C" int gcl_header_gather(const uint8_t *frames, uint64_t frames_len, const uint64_t *offs,
                                 uint64_t n, uint8_t *rows, void *hip_stream)
{
	if (!n)
		return 0;
	if (!frames || !offs || !rows || frames_len == UINT64_MAX || n > (1ull << 40))
		return -EINVAL;
	int dev = 0, cus = 256;
	if (hipGetDevice(&dev) == hipSuccess)
		(void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
	const unsigned grid = (unsigned)std::min<uint64_t>((n + 31) / 32, (uint64_t)cus * 8);
	hipLaunchKernelGGL(header_gather_kernel, dim3(grid), dim3(256), 0, (hipStream_t)hip_stream, frames,
	                   frames_len, offs, n, rows);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int gcl_access_probe(struct gcl_ctx *c, const struct gcl_batch *b, void *out,
                                uint32_t vbytes, void *hip_stream)
{
	if (!c || !b || !out || (vbytes != 1 && vbytes != 2 && vbytes != 4 && vbytes != 8))
		return -EINVAL;
	if (b->n == 0)
		return 0;
	if (!b->frames || b->frames_len == UINT64_MAX || b->n > (1ull << 40) ||
	    (!b->offs && (b->stride < 16 || (b->stride & 15) || b->stride > (1u << 20))))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	KParams k = {};
	k.frames = b->frames;
	k.frames_len = b->frames_len;
	k.stride = b->stride;
	k.offs = b->offs;
	k.olflags = b->olflags;
	k.rss = b->rss;
	k.n = b->n;
	k.verdicts = (uint2 *)out;
	const uint64_t need = (b->n + 255) / 256;
	const unsigned grid = (unsigned)std::min<uint64_t>((uint64_t)c->num_cus * 8, need);
	hipStream_t s = (hipStream_t)hip_stream;
	if (vbytes == 1)
		hipLaunchKernelGGL(access_probe_kernel<1>, dim3(grid), dim3(256), 0, s, k);
	else if (vbytes == 2)
		hipLaunchKernelGGL(access_probe_kernel<2>, dim3(grid), dim3(256), 0, s, k);
	else if (vbytes == 4)
		hipLaunchKernelGGL(access_probe_kernel<4>, dim3(grid), dim3(256), 0, s, k);
	else
		hipLaunchKernelGGL(access_probe_kernel<8>, dim3(grid), dim3(256), 0, s, k);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int gcl_classify_ex(struct gcl_ctx *c, const struct gcl_batch *b,
                               const struct gcl_out *out, void *hip_stream)
{
	if (!c || !b || !out)
		return -EINVAL;
	void *verdicts = out->verdicts;
	uint64_t *runtime_counts = out->runtime_counts, *stats = out->stats;
	if (out->trans && !(c->cfg.flags & GCL_CFG_TRANS_HASH))
		return -EINVAL;
	hipStream_t s = (hipStream_t)hip_stream;
	if (b->n == 0)
		return 0;
	if (!b->frames || (!b->offs && (b->stride < 16 || (b->stride & 15) || b->stride > (1u << 20))))
		return -EINVAL;
	/* offsets are clamped to frames_len, which must stay clear of kNoOff */
	if (b->frames_len == UINT64_MAX)
		return -EINVAL;
	/* at most 2^40 packets, so n * stride (and the fast-path range test on
	 * it below) cannot wrap */
	if (!verdicts || b->n > (1ull << 40))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;

	const int up = upload_tables(c, s);
	if (up)
		return up;
	if (wait_tables(c, s))
		return -EIO;

	KParams k = {};
	k.frames = b->frames;
	k.frames_len = b->frames_len;
	k.stride = b->stride;
	k.offs = b->offs;
	k.olflags = b->olflags;
	k.rss = b->rss;
	k.fdir = b->fdir_hi;
	k.dst_hint = b->dst_hint;
	k.n = b->n;
	k.verdicts = (uint2 *)verdicts;
	k.counts = (unsigned long long *)runtime_counts;
	k.stats = (unsigned long long *)stats;
	k.tables = c->dimg[c->cur];
	k.ipt_mask = c->ipt_slots / 2 - 1;
	k.ipt_seed = c->ipt_seed;
	k.max_rt = c->cfg.max_runtimes;
	k.off_rt = c->off_rt;
	k.off_flow = c->off_flow;
	k.off_toep = c->off_toep;
	k.off_seed = c->off_seed;
	k.off_crc = c->off_crc;
	k.trans = (uint2 *)out->trans;
	k.cflags = kernel_cflags(c);
	k.plean = (uint32_t)c->tune_plean;
	k.default_flags = c->cfg.default_olflags;

	/* the specialised fast path needs every header granule in range */
	bool general = b->offs || b->olflags || b->fdir_hi || b->dst_hint ||
	               (c->cfg.default_olflags & GCL_F_FDIR_ID) ||
	               b->frames_len < (b->n - 1) * b->stride + GCL_HDR_GRANULE;
	uint32_t tab_bytes = c->image_bytes;
	uint32_t hist_bytes = ((c->cfg.max_runtimes + 3) & ~3u) * 4;
	bool tlds = tab_bytes <= kLdsTableBudget;
	if (c->tune_tables == 1)
		tlds = false;
	else if (c->tune_tables == 2)
		tlds = tab_bytes <= kLdsTableBudget;
	k.tables_lds_bytes = tlds ? tab_bytes : 0;
	/* dense slots with 1-/2-B verdicts, 16-B-aligned (the deferred verdicts
	 * go out 16 B at a time, through a buffer descriptor: below 4 GiB) */
	const bool defer_ok = !general && (k.cflags & (GCL_CFG_VERDICT1 | GCL_CFG_VERDICT2)) &&
	                      ((uintptr_t)verdicts & 15) == 0 && b->n * 2 < (1ull << 32);
	Geometry geo = choose_geometry(c, tlds ? tab_bytes : 0, hist_bytes, general, defer_ok);

	HipErr he;

	hipEvent_t e0 = nullptr, e1 = nullptr;
	if ((c->cfg.flags & GCL_CFG_PROFILE) && c->prof_seq++ % c->prof_every == 0) {
		e0 = prof_event(c);
		e1 = prof_event(c);
		if (!e0 || !e1) { /* no timing for this launch */
			if (e0)
				c->ev_pool.push_back(e0);
			if (e1)
				c->ev_pool.push_back(e1);
			e0 = e1 = nullptr;
		} else {
			he(hipEventRecord(e0, s));
		}
	}
	hipError_t err;
	switch (c->cfg.hash_mode) {
	case GCL_HASH_NIC:
		err = launch_mode<GCL_HASH_NIC>(k, tlds, geo, tlds ? tab_bytes : 0, hist_bytes, c->num_cus, s);
		break;
	case GCL_HASH_JENKINS:
		err = launch_mode<GCL_HASH_JENKINS>(k, tlds, geo, tlds ? tab_bytes : 0, hist_bytes, c->num_cus, s);
		break;
	default:
		err = launch_mode<GCL_HASH_TOEPLITZ>(k, tlds, geo, tlds ? tab_bytes : 0, hist_bytes, c->num_cus, s);
		break;
	}
	if (e0) {
		he(hipEventRecord(e1, s));
		if (he.bad()) { /* an unusable timing pair: back to the pool */
			c->ev_pool.push_back(e0);
			c->ev_pool.push_back(e1);
		} else {
			c->ev_pending.push_back({e0, e1});
		}
	}
	const int iu = image_used(c, s);
	c->last_stream = s;
	return err == hipSuccess && !he.bad() && !iu ? 0 : -EIO;
}

extern "C" int gcl_sync(struct gcl_ctx *c)
{
	if (!c)
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	return hipStreamSynchronize(c->last_stream) == hipSuccess ? 0 : -EIO;
}

extern "C" int gcl_profile_sample(struct gcl_ctx *c, uint32_t every)
{
	if (!c || every == 0)
		return -EINVAL;
	c->prof_every = every;
	c->prof_seq = 0;
	return 0;
}

extern "C" int gcl_kernel_time(struct gcl_ctx *c, double *ms, uint64_t *launches, int reset)
{
	if (!c)
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	for (auto &pr : c->ev_pending) {
		float f = 0;
		if (hipEventSynchronize(pr.second) == hipSuccess &&
		    hipEventElapsedTime(&f, pr.first, pr.second) == hipSuccess) {
			c->prof_ms += f;
			c->prof_launches++;
		}
		c->ev_pool.push_back(pr.first);
		c->ev_pool.push_back(pr.second);
	}
	c->ev_pending.clear();
	if (ms)
		*ms = c->prof_ms;
	if (launches)
		*launches = c->prof_launches;
	if (reset) {
		c->prof_ms = 0;
		c->prof_launches = 0;
	}
	return 0;
}

extern "C" int gcl_generate(const struct gcl_gen_params *p, uint8_t *frames, uint8_t *olflags,
                            uint32_t *rss, void *hip_stream)
{
	if (!p || !frames || p->stride < 64 || (p->stride & 15) || p->nruntimes == 0 ||
	    p->workload > GCL_WL_MIXED)
		return -EINVAL;
	if (p->workload == GCL_WL_TCP1500_ZIPF && (!p->zipf_cdf || !p->nflows))
		return -EINVAL;
	if (p->n == 0)
		return 0;
	GParams g = {};
	g.workload = p->workload;
	g.nruntimes = p->nruntimes;
	g.seed = p->seed;
	g.n = p->n;
	g.stride = p->stride;
	g.rank = p->rank;
	g.world = p->world;
	g.shard_block = p->shard_block;
	g.zipf = p->zipf_cdf;
	g.nflows = p->nflows;
	g.frames = frames;
	g.olflags = olflags;
	g.rss = rss;
	g.pkt_len = p->pkt_len;
	uint64_t blocks = (p->n + 255) / 256;
	hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(256), 0,
	                   (hipStream_t)hip_stream, g);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" const char *gcl_version(void) { return GCL_VERSION; }

extern "C" int gcl_abi_version(void) { return GCL_ABI_VERSION; }

/* Device memory for frame slabs and verdict arrays: plain hipMalloc on the
 * context's device, so large batches get the allocator's large-page path. */
extern "C" int gcl_dev_alloc(int hip_device, size_t bytes, void **out)
{
	if (!out || !bytes)
		return -EINVAL;
	if (hipSetDevice(hip_device) != hipSuccess)
		return -ENODEV;
	return hipMalloc(out, bytes) == hipSuccess ? 0 : -ENOMEM;
}

extern "C" int gcl_dev_free(void *p)
{
	return hipFree(p) == hipSuccess ? 0 : -EINVAL;
}

namespace {

/* The classify kernel's memory shape without its compute: 256-packet tiles of
 * 64-B granules read with four nt 16-B loads per lane, one VB-byte
 * write-through store per packet, like the verdict stores (tile t writes slot
 * t % wtiles of the write side). */
template <int VB>
__global__ void __launch_bounds__(256) pair_probe_kernel(const uint8_t *rd, uint64_t ntiles,
                                                         uint8_t *wr, uint64_t wtiles)
{
	__shared__ uint4 tile[1024];
	uint64_t t = blockIdx.x;
	uint4 r[4];
	auto ld = [&](uint64_t tt) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const int c = j * 256 + (int)threadIdx.x;
			r[j] = gcl::load16_nt(rd + (tt * 256 + (c >> 2)) * 64 + (c & 3) * 16);
		}
	};
	if (t < ntiles)
		ld(t);
	while (t < ntiles) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const int c = j * 256 + (int)threadIdx.x;
			tile[tile_slot(c >> 2, c & 3)] = r[j];
		}
		__syncthreads();
		const uint64_t nx = t + gridDim.x;
		if (nx < ntiles)
			ld(nx);
		const int p = threadIdx.x;
		const uint4 a = tile[tile_slot(p, 0)], b = tile[tile_slot(p, 1)];
		const uint32_t v = a.x ^ a.w ^ b.y ^ b.z;
		const uint64_t i = (t % wtiles) * 256 + p;
		if (VB == 1)
			store_wt(wr + i, (uint8_t)v);
		else if (VB == 2)
			store_wt((uint16_t *)wr + i, (uint16_t)v);
		else if (VB == 8)
			store_wt((uint64_t *)wr + i, (uint64_t)((uint64_t)v * 0x100000001ull));
		else
			store_wt((uint32_t *)wr + i, v);
		__syncthreads();
		t = nx;
	}
}

/* the probe stores to at most this much of the written side */
constexpr size_t kPairProbeWriteMax = 256ull << 20;

/* min over 3 timed launches of the probe (after one untimed), microseconds;
 * negative on a HIP error */
double pair_probe(const uint8_t *rd, size_t rd_bytes, uint8_t *wr, size_t wr_bytes, int vb,
                  hipStream_t s, hipEvent_t e0, hipEvent_t e1, int cus)
{
	/* the whole of both buffers, as the kernel walks them (a 2 GiB frame
	 * pool against a 128 MiB verdict ring is 0.35-0.4 ms): a probe of the
	 * first 512 MiB against the first 32 MiB missed the class on some boxes */
	const uint64_t ntiles = std::min<size_t>(rd_bytes, 4ull << 30) / (256 * 64);
	const uint64_t wtiles = std::min<size_t>(wr_bytes, kPairProbeWriteMax) / (256 * (size_t)vb);
	if (!ntiles || !wtiles)
		return -1;
	/* the store policy decides which pairs collide: the probe stores the
	 * way the classify kernel does (write-through) */
	auto launch = [&]() {
		const dim3 g(cus * 4), b(256);
#define GCL_PROBE(V) hipLaunchKernelGGL((pair_probe_kernel<V>), g, b, 0, s, rd, ntiles, wr, wtiles)
		if (vb == 1)
			GCL_PROBE(1);
		else if (vb == 2)
			GCL_PROBE(2);
		else if (vb == 8)
			GCL_PROBE(8);
		else
			GCL_PROBE(4);
#undef GCL_PROBE
	};
	double best = 1e30;
	for (int i = 0; i < 4; i++) {
		if (hipEventRecord(e0, s) != hipSuccess)
			return -1;
		launch();
		if (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess)
			return -1;
		float ms = 0;
		if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
			return -1;
		if (i > 0)
			best = std::min(best, (double)ms * 1e3);
	}
	return best;
}

} /* namespace */

/* The class gap: same-class pairs measured 12-18% slower than cross-class
 * ones (406 vs 343 us classify; 375-382 vs 330-341 us in the probe's shape at
 * full size, profiles/archive/r02_classmap.jsonl); run-to-run noise of one probe is
 * under 1.5%. */
constexpr double kPairGap = 0.06;
/* Of the free device memory at entry, at most this share is held by
 * candidates and spacers while searching (all but the kept buffer are freed
 * before returning). */
constexpr double kPairHoldShare = 0.6;

extern "C" int gcl_dev_alloc_paired(int hip_device, size_t bytes, const void *partner,
                                    size_t partner_bytes, uint32_t flags, void **out,
                                    struct gcl_pair_info *info)
{
	const uint32_t dir = flags & 0xFF;
	const int vb = GCL_PAIR_VBYTES_OF(flags) ? (int)GCL_PAIR_VBYTES_OF(flags) : 4;
	const bool new_reads = dir == GCL_PAIR_NEW_READS;
	if (!out || !bytes || !partner || !partner_bytes ||
	    (dir != GCL_PAIR_NEW_READS && dir != GCL_PAIR_NEW_WRITES) ||
	    (vb != 1 && vb != 2 && vb != 4 && vb != 8) || (flags >> 16))
		return -EINVAL;
	const size_t rd_bytes = new_reads ? bytes : partner_bytes;
	const size_t wr_bytes = new_reads ? partner_bytes : bytes;
	if (rd_bytes < 256 * 64 || wr_bytes < 256 * (size_t)vb)
		return -EINVAL;
	if (hipSetDevice(hip_device) != hipSuccess)
		return -ENODEV;
	int cus = 0;
	if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device) != hipSuccess)
		return -ENODEV;
	size_t free_b = 0, total_b = 0;
	if (hipMemGetInfo(&free_b, &total_b) != hipSuccess)
		return -ENODEV;
	const size_t hold_cap = (size_t)((double)free_b * kPairHoldShare);
	hipStream_t s;
	hipEvent_t e0, e1;
	if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
		return -EIO;
	if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) {
		(void)hipStreamDestroy(s);
		return -EIO;
	}
	const bool dbg = getenv("GCL_PAIR_DEBUG") != nullptr;
	std::vector<std::pair<void *, double>> cand;
	std::vector<void *> spacers;
	size_t held = 0, spacer_held = 0;
	int ret = 0, nspacers = 0, classes = 1;
	for (int i = 0; i < GCL_PAIR_TRIES; i++) {
		void *p = nullptr;
		if (i && i % GCL_PAIR_RUN == 0) {
			/* one class so far: step past the run.  Runs of one class span
			 * 4-34 GiB of consecutive allocations (profiles/archive/r02_classmap.jsonl),
			 * so the spacer grows: 2, 4, 8, then 16 x @bytes */
			size_t sp_bytes = bytes * (2ull << std::min(nspacers, 3));
			if (held + sp_bytes + bytes > hold_cap)
				sp_bytes = hold_cap > held + 2 * bytes ? hold_cap - held - bytes : 0;
			void *sp = nullptr;
			if (sp_bytes && hipMalloc(&sp, sp_bytes) == hipSuccess) {
				spacers.push_back(sp);
				held += sp_bytes;
				spacer_held += sp_bytes;
				nspacers++;
			} else {
				(void)hipGetLastError();
			}
			if (dbg)
				fprintf(stderr, "gcl_dev_alloc_paired: spacer %p (%zu MiB)\n", sp, sp_bytes >> 20);
		}
		if (held + bytes > hold_cap && !cand.empty())
			break;
		if (hipMalloc(&p, bytes) != hipSuccess) {
			(void)hipGetLastError();
			break;
		}
		held += bytes;
		const double us = new_reads
		        ? pair_probe((const uint8_t *)p, rd_bytes, (uint8_t *)partner, wr_bytes, vb, s, e0, e1, cus)
		        : pair_probe((const uint8_t *)partner, rd_bytes, (uint8_t *)p, wr_bytes, vb, s, e0, e1, cus);
		if (dbg)
			fprintf(stderr, "gcl_dev_alloc_paired: candidate %d %p probe %.2f us\n", i, p, us);
		if (us < 0) {
			(void)hipFree(p);
			ret = -EIO;
			break;
		}
		cand.emplace_back(p, us);
		double lo = 1e30, hi = 0;
		for (auto &c : cand) {
			lo = std::min(lo, c.second);
			hi = std::max(hi, c.second);
		}
		if (hi > lo * (1 + kPairGap)) {
			classes = 2;
			break; /* both classes seen */
		}
	}
	size_t best = 0;
	double worst = 0;
	for (size_t i = 0; i < cand.size(); i++) {
		if (cand[i].second < cand[best].second)
			best = i;
		worst = std::max(worst, cand[i].second);
	}
	for (size_t i = 0; i < cand.size(); i++)
		if (ret || i != best)
			(void)hipFree(cand[i].first);
	for (void *sp : spacers)
		(void)hipFree(sp);
	(void)hipEventDestroy(e0);
	(void)hipEventDestroy(e1);
	(void)hipStreamDestroy(s);
	if (ret)
		return ret;
	if (cand.empty())
		return -ENOMEM;
	*out = cand[best].first;
	if (classes == 1 && !getenv("GCL_PAIR_QUIET"))
		fprintf(stderr, "gcl_dev_alloc_paired: warning: one placement class in %zu candidates "
		        "(%.1f-%.1f us, %zu MiB of spacers); the pair may be the slow one\n",
		        cand.size(), cand[best].second, worst, spacer_held >> 20);
	if (info) {
		memset(info, 0, sizeof(*info));
		info->chosen_us = cand[best].second;
		info->worst_us = worst;
		info->candidates = (uint32_t)cand.size();
		info->classes = (uint32_t)classes;
		info->spacer_bytes = spacer_held;
		info->probe_write_bytes = std::min<size_t>(wr_bytes, kPairProbeWriteMax) / (256 * vb) * (256 * vb);
	}
	return 0;
}

/* ==========================================================================
 * End-to-end: frames in host memory (the NIC's mbufs), verdicts back to host.
 */
extern "C" int gcl_host_register(void *p, size_t len)
{
	if (!p || !len)
		return -EINVAL;
	return hipHostRegister(p, len, hipHostRegisterMapped | hipHostRegisterPortable) == hipSuccess
	               ? 0 : -ENOMEM;
}

extern "C" int gcl_host_unregister(void *p)
{
	return hipHostUnregister(p) == hipSuccess ? 0 : -EINVAL;
}

/* Per-packet sub-arrays of a COPY chunk's side buffer, at multiples of this
 * many bytes: ol_flags [0, C), hash.rss [C, 5C), hash.fdir.hi [5C, 9C),
 * dst_hint [9C, 13C), offsets [13C, 21C).  A multiple of 16, so every
 * sub-array is 16-B aligned whatever chunk the caller asks for. */
static uint64_t side_stride(uint64_t chunk)
{
	return (chunk + 15) & ~15ull;
}

static int e2e_setup(gcl_ctx *c, int nstreams, uint64_t chunk)
{
	gcl_ctx::E2E &e = c->e2e;
	if (e.nstreams == nstreams && e.chunk == chunk)
		return 0;
	for (int i = 0; i < e.nstreams; i++) {
		(void)hipStreamDestroy(e.st[i]);
		(void)hipFree(e.slab[i]);
		(void)hipFree(e.side[i]);
		(void)hipFree(e.verd[i]);
	}
	if (!e.acc && hipMalloc(&e.acc, (GCL_MAX_PROC + GCL_NR_STATS) * 8) != hipSuccess)
		return -ENOMEM;
	e.nstreams = 0;
	for (int i = 0; i < nstreams; i++) {
		if (hipStreamCreateWithFlags(&e.st[i], hipStreamNonBlocking) != hipSuccess ||
		    hipMalloc(&e.slab[i], chunk * kGatherRow) != hipSuccess ||
		    hipMalloc(&e.side[i], side_stride(chunk) * 21) != hipSuccess ||
		    hipMalloc(&e.verd[i], chunk * sizeof(struct gcl_verdict)) != hipSuccess)
			return -ENOMEM;
		e.nstreams = i + 1;
	}
	e.chunk = chunk;
	return 0;
}

/* device address of pinned / registered host memory, or NULL */
static void *mapped(const void *h)
{
	void *d = nullptr;
	if (!h)
		return nullptr;
	if (hipHostGetDevicePointer(&d, (void *)h, 0) != hipSuccess) {
		(void)hipGetLastError(); /* not registered: do not leave a sticky error */
		return nullptr;
	}
	return d;
}

extern "C" int gcl_classify_host(struct gcl_ctx *c, const struct gcl_batch *hb,
                                 void *host_verdicts, uint64_t *host_counts,
                                 uint64_t *host_stats, const struct gcl_e2e_opts *o)
{
	if (!c || !hb || !host_verdicts || !o || o->mode > GCL_E2E_ZEROCOPY)
		return -EINVAL;
	if (hb->n == 0)
		return 0;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	const uint32_t max_rt = c->cfg.max_runtimes;
	const uint64_t vsize = verdict_bytes(c);
	int nst = o->nstreams ? (int)o->nstreams : 2;
	if (nst > 4)
		nst = 4;
	uint64_t chunk = o->chunk ? o->chunk : (1ull << 20);
	int ret = e2e_setup(c, nst, chunk);
	if (ret)
		return ret;
	gcl_ctx::E2E &e = c->e2e;
	hipStream_t s0 = e.st[0];
	HipErr he; /* every asynchronous step below; checked after the final sync */
	he(hipMemsetAsync(e.acc, 0, (max_rt + GCL_NR_STATS) * 8, s0));
	if (upload_tables(c, s0))
		return -EIO;
	hipEvent_t ready;
	if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess)
		return -EIO;
	he(hipEventRecord(ready, s0));
	for (int i = 1; i < nst; i++)
		he(hipStreamWaitEvent(e.st[i], ready, 0));

	uint64_t *dcounts = e.acc, *dstats = e.acc + max_rt;
	if (o->mode == GCL_E2E_ZEROCOPY) {
		/* the kernel reads the headers straight out of host memory over
		 * PCIe and writes verdicts straight into host memory */
		struct gcl_batch db = *hb;
		db.frames = (const uint8_t *)mapped(hb->frames);
		db.offs = (const uint64_t *)mapped(hb->offs);
		db.olflags = (const uint8_t *)mapped(hb->olflags);
		db.rss = (const uint32_t *)mapped(hb->rss);
		db.fdir_hi = (const uint32_t *)mapped(hb->fdir_hi);
		db.dst_hint = (const uint32_t *)mapped(hb->dst_hint);
		void *dv = mapped(host_verdicts);
		if (!db.frames || !dv || (hb->offs && !db.offs) || (hb->olflags && !db.olflags) ||
		    (hb->rss && !db.rss) || (hb->fdir_hi && !db.fdir_hi) ||
		    (hb->dst_hint && !db.dst_hint)) {
			(void)hipEventDestroy(ready);
			return -EFAULT; /* not pinned/registered: see gcl_host_register */
		}
		ret = gcl_classify(c, &db, dv, dcounts, dstats, s0);
	} else {
		/* frames at per-packet offsets are gathered by a kernel reading the
		 * mapped region; fixed slots by the DMA engine */
		const uint8_t *dframes = hb->offs ? (const uint8_t *)mapped(hb->frames) : nullptr;
		const uint64_t *doffs = hb->offs ? (const uint64_t *)mapped(hb->offs) : nullptr;
		if (!hb->offs && ((hb->stride & 15) || hb->stride < GCL_HDR_GRANULE)) {
			(void)hipEventDestroy(ready);
			return -EINVAL;
		}
		if (hb->offs && (!dframes || hb->frames_len == UINT64_MAX)) {
			(void)hipEventDestroy(ready);
			return dframes ? -EINVAL : -EFAULT; /* the gather reads the registered region */
		}
		/* a row holds frame bytes [0, 80) (IHL 15's ports end at 78); a
		 * 64-B slot stride is its own row (the next frame follows, as in
		 * the host buffer) */
		const uint64_t row = hb->offs || hb->stride >= kGatherRow ? kGatherRow : GCL_HDR_GRANULE;
		const uint64_t C = side_stride(chunk);
		for (uint64_t s = 0, ci = 0; s < hb->n && !ret; s += chunk, ci++) {
			const int i = (int)(ci % nst);
			const uint64_t m = hb->n - s < chunk ? hb->n - s : chunk;
			hipStream_t st = e.st[i];
			if (hb->offs) {
				const uint64_t *so = doffs ? doffs + s : (const uint64_t *)(e.side[i] + 13 * C);
				if (!doffs)
					he(hipMemcpyAsync((void *)so, hb->offs + s, m * 8, hipMemcpyHostToDevice, st));
				if (gcl_header_gather(dframes, hb->frames_len, so, m, e.slab[i], st))
					he(hipErrorLaunchFailure);
			} else {
				/* H2D of each slot's header row (2D DMA) */
				const uint8_t *src = hb->frames + s * hb->stride;
				uint64_t avail = hb->frames_len > s * hb->stride ? hb->frames_len - s * hb->stride : 0;
				if (avail < (m - 1) * hb->stride + row) {
					ret = -EINVAL;
					break;
				}
				if (hb->stride == row)
					he(hipMemcpyAsync(e.slab[i], src, m * row, hipMemcpyHostToDevice, st));
				else
					he(hipMemcpy2DAsync(e.slab[i], row, src, hb->stride, row, m, hipMemcpyHostToDevice, st));
			}
			struct gcl_batch db = {};
			db.frames = e.slab[i];
			db.frames_len = m * row;
			db.stride = row;
			db.n = m;
			uint8_t *side = e.side[i];
			if (hb->olflags) {
				he(hipMemcpyAsync(side, hb->olflags + s, m, hipMemcpyHostToDevice, st));
				db.olflags = side;
			}
			if (hb->rss) {
				he(hipMemcpyAsync(side + C, hb->rss + s, m * 4, hipMemcpyHostToDevice, st));
				db.rss = (const uint32_t *)(side + C);
			}
			if (hb->fdir_hi) {
				he(hipMemcpyAsync(side + 5 * C, hb->fdir_hi + s, m * 4, hipMemcpyHostToDevice, st));
				db.fdir_hi = (const uint32_t *)(side + 5 * C);
			}
			if (hb->dst_hint) {
				he(hipMemcpyAsync(side + 9 * C, hb->dst_hint + s, m * 4, hipMemcpyHostToDevice, st));
				db.dst_hint = (const uint32_t *)(side + 9 * C);
			}
			ret = gcl_classify(c, &db, e.verd[i], dcounts, dstats, st);
			he(hipMemcpyAsync((uint8_t *)host_verdicts + s * vsize, e.verd[i], m * vsize,
			                  hipMemcpyDeviceToHost, st));
		}
		for (int i = 1; i < nst; i++) {
			he(hipEventRecord(ready, e.st[i]));
			he(hipStreamWaitEvent(s0, ready, 0));
		}
	}
	uint64_t tmp[GCL_MAX_PROC + GCL_NR_STATS];
	he(hipMemcpyAsync(tmp, e.acc, (max_rt + GCL_NR_STATS) * 8, hipMemcpyDeviceToHost, s0));
	hipError_t err = hipStreamSynchronize(s0);
	(void)hipEventDestroy(ready);
	if (ret)
		return ret;
	if (he.bad())
		return -EIO;
	if (err != hipSuccess)
		return -EIO;
	if (host_counts)
		for (uint32_t i = 0; i < max_rt; i++)
			host_counts[i] += tmp[i];
	if (host_stats)
		for (int i = 0; i < GCL_NR_STATS; i++)
			host_stats[i] += tmp[max_rt + i];
	c->last_stream = s0;
	return 0;
}

/* ==========================================================================
 * Persistent rx loop (host side).  Ring slots and table images live in
 * coherent, mapped host memory; the CPU publishes a slot with a release store
 * of its ticket, the kernel answers with a release store of `done`.
 */
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

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
 * GCL_TUNE_LOOP64=0: the tests' way to run short bursts through it) */
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
	{
		uint64_t t0 = 0;
		if (const char *e = getenv("GCL_TUNE_LOOP_T0")) /* tests: start near a stamp wrap */
			t0 = strtoull(e, nullptr, 0) / cfg->slots * cfg->slots;
		L->lp.t0 = t0;
		L->next = t0;
		L->retired.assign(cfg->slots, t0);
	}
	L->max_burst = cfg->max_burst;
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
	lp.lean = kDefaultLoopLean;
	if (const char *e = getenv("GCL_TUNE_LOOP_LEAN"))
		lp.lean = atoi(e) != 0;
	lp.off_hdr = (cfg->flags & (GCL_LOOP_INLINE_HDRS | GCL_LOOP_HDR_RECORDS))
	                     ? lp.off_verd + sizeof(LoopRec) * mb : 0;
	lp.rec_plane = (uint32_t)(16 * mb);
	lp.spec = (!lp.off_hdr || lp.hdr_rec) && cfg->max_burst <= 64;
	lp.spec_ticks = cfg->workers <= kLoopSpecIdleWorkers ? kLoopSpecIdle : kLoopSpecTicks;
	L->k64 = cfg->max_burst <= 64;
	if (const char *e = getenv("GCL_TUNE_LOOP64")) /* 0: tests, the general loop */
		L->k64 = L->k64 && atoi(e) != 0;
	if (const char *e = getenv("GCL_TUNE_LOOP_SPEC")) /* experiments: ticks of 10 ns */
		lp.spec_ticks = (uint32_t)atoi(e);
	/* the poll-phase delay: closed-loop submitters are the few-worker case;
	 * a deep pipeline finds its bursts queued */
	lp.phase_max = cfg->workers <= kLoopSpecIdleWorkers ? kDefaultLoopPhaseMax : 0;
	lp.phase_up = kDefaultLoopPhaseUp;
	lp.phase_down = kDefaultLoopPhaseDown;
	if (const char *e = getenv("GCL_TUNE_LOOP_PHASE")) { /* "max[,up[,down]]", ticks */
		unsigned m = 0, u = lp.phase_up, d = lp.phase_down;
		if (sscanf(e, "%u,%u,%u", &m, &u, &d) >= 1 && m <= 1000 && u && d <= u) {
			lp.phase_max = m;
			lp.phase_up = u;
			lp.phase_down = d;
		}
	}
	/* the next ticket's poll during classification: for workers that find
	 * their bursts queued (more than the closed-loop few) */
	lp.prefetch = cfg->workers > kLoopSpecIdleWorkers && !lp.hdr_rec ? kDefaultLoopPrefetch : 0;
	if (const char *e = getenv("GCL_TUNE_LOOP_PREFETCH"))
		lp.prefetch = atoi(e) != 0;
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
	if (getenv("GCL_LOOP_DEBUG"))
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
	/* (prefetching 6 ahead, or the record lines for ownership, measured
	 * the same: profiles/r03_hdr_records_prefetch_ab.jsonl) */
	for (uint32_t i = 0; i < n; i++, q++) {
		if (i + 2 < n && offs[i + 2] < L->region_len)
			__builtin_prefetch(L->region + offs[i + 2] + 12, 0, 3);
		const uint64_t o = offs[i];
		/* frame dwords 3-6 and 7-10 (bytes 12-43) in two registers, shuffled
		 * into the chunks without a trip through memory */
		u32x4_h v0, v1;
		if (o < L->region_len && L->region_len - o >= 44) {
			memcpy(&v0, L->region + o + 12, 16);
			memcpy(&v1, L->region + o + 28, 16);
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

/* spin up to @spin_ns for ticket @t's burst: 0, -EAGAIN or -ESHUTDOWN */
static int loop_await(gcl_rxloop *L, uint64_t t, uint64_t spin_ns)
{
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
	if (getenv("GCL_LOOP_DEBUG")) {
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
