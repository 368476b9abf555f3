/*
 * gcl_batch.hip - the batch classify kernels and their launch: the rx_one_pkt
 * loop of rx_burst (iokernel/rx.c:116-233, :281-287) over a whole batch of
 * device-resident (or mapped host) frames.
 *
 *   classify_kernel       fixed-stride slots: 64-B header granules staged
 *                         through an XOR-swizzled LDS tile, one lane per packet
 *   classify_pair_kernel  per-packet offsets or side arrays: bytes [8, 40) of
 *                         each frame by lane pairs with a DPP exchange
 *   access_probe_kernel   the fewest requests the frame layout allows
 *                         (GCL_PROBE_MIN; the kernels' own shapes run in
 *                         kModeProbe for gcl_access_probe)
 *
 * Layout in HBM: frames are fixed-stride slots (or a u64 offset
 * array, like mbuf data pointers into the 2 GiB ingress region); verdicts are
 * dense u8 / u16 / gcl_verdict4 / gcl_verdict arrays.
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "../../include/gclassify.h"
#include "gcl_ctx.h"

namespace gclk {

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
	if (TLDS)
		stage_tables<NT>(lds_tab, k.tables, k.tables_lds_bytes);
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
	/* tiles first, first + step, ... before t_end: dealt round-robin (the
	 * whole chip sweeps one window of the batch), or with k.contig one run
	 * of ceil(ntiles / G) tiles per block (each block streams its own part) */
	uint64_t first = blockIdx.x, step = gridDim.x, t_end = k.ntiles;
	if (k.contig) {
		const uint64_t per = (k.ntiles + gridDim.x - 1) / gridDim.x;
		first = (uint64_t)blockIdx.x * per;
		step = 1;
		t_end = std::min(first + per, k.ntiles);
	}
	uint64_t t = first;
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
		return (first + (uint64_t)j * step) * NT * vb;
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
	/* rx_one_pkt on this lane's row, or (gcl_access_probe) the rows it
	 * reads folded, after the same drain */
	/* a wave whose packets are all plain IPv4 (IHL 5; a dense batch has no
	 * FDIR marks or hints) takes classify_lean (k.tlean, one ballot over the
	 * live lanes), the others classify_core; no transport pre-hash in lean */
	const bool lean_ok = k.tlean && !k.trans;
	auto classify = [&](uint64_t tt) -> uint64_t {
		if constexpr (MODE == kModeProbe) {
			dense_drain();
			const uint4 a = tile[tile_slot(tid, 0)], b = tile[tile_slot(tid, 1)], c = tile[tile_slot(tid, 2)];
			return a.w ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z;
		} else {
			const uint64_t idx = tt * NT + tid;
			const uint4 w0 = tile[tile_slot(tid, 0)], w1 = tile[tile_slot(tid, 1)], w2 = tile[tile_slot(tid, 2)];
			HdrWords h;
			h.d3 = w0.w, h.d5 = w1.y, h.d6 = w1.z, h.d7 = w1.w;
			h.d8 = w2.x, h.d9 = w2.y, h.d10 = w2.z;
			if (lean_ok && __all((h.d3 & 0x000FFFFFu) == 0x00050008u)) {
				const uint32_t rss = MODE == GCL_HASH_NIC && k.rss ? k.rss[idx] : 0u;
				return classify_lean<MODE, true, true>(k, h, tb, k.default_flags, rss, hist, tid, cnt);
			}
			return classify_core<MODE, false, false, false>(k, h, tile, tid, idx, tb, hist, cnt, 0, 64, nullptr);
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
			const uint64_t w = live ? classify(t) : 0;
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
				const uint64_t w = live ? classify(t) : 0;
				verdict(t * NT + tid, t < t_end, live, w);
			}
			__syncthreads();
			tile_done(t);
			t += step;
		}
	}
	if (kl)
		flush_lds();
	if (nreg && k.vstage && nreg <= k.vcap) {
		/* the registers through the buffer (its stores above have their
		 * data: a barrier and it is free), then out 16 B per lane like the
		 * buffer, not one verdict per lane per tile */
		__syncthreads();
		for (uint32_t q = 0; q < nreg; q++) {
			uint8_t *d = vbuf + ((nreg - 1 - q) * NT + tid) * vb;
			if (vb == 1)
				*d = (uint8_t)vr[0];
			else
				*(uint16_t *)d = (uint16_t)vr[0];
			const uint32_t sh = 8 * vb;
#pragma unroll
			for (int r = 0; r < kVregs - 1; r++)
				vr[r] = (vr[r] >> sh) | (vr[r + 1] << (32 - sh));
			vr[kVregs - 1] >>= sh;
		}
		__syncthreads();
		kf += k.vcap;
		kl = nreg;
		flush_lds();
	} else if (nreg) {
		flush_regs();
	}
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

/* I32: a batch whose frames, offsets, side arrays and verdicts all lie within
 * 2 GiB (pair_i32_ok) runs its per-packet arithmetic in 32 bits: packet
 * indices and frame offsets as u32, every load and store through a buffer
 * descriptor with a 32-bit offset (no 64-bit address per lane), one DPP move
 * per broadcast instead of two */
constexpr uint32_t kBw32 = 0x80000000u;   /* I32 pair_src: read bytewise */
constexpr uint32_t kNoOff32 = 0xFFFFFFFFu; /* I32 pair_src: no packet */

template <int MODE, bool TLDS, int NT, int VF, bool I32>
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
	if (TLDS)
		stage_tables<NT>(lds_tab, k.tables, k.tables_lds_bytes);
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
	using Src = std::conditional_t<I32, uint32_t, uint64_t>; /* pair_src's encoding */
	const uint64_t *offs_src = k.offs ? k.offs : (const uint64_t *)k.tables;
	/* I32: buffer descriptors (a missing array reads 16 B of the tables) */
	const __amdgpu_buffer_rsrc_t rs_fr = gcl::host_rsrc(k.frames, I32 ? k.frames_len : 16);
	const __amdgpu_buffer_rsrc_t rs_off = gcl::host_rsrc(k.offs ? (const void *)k.offs : k.tables,
	                                                     I32 && k.offs ? 8 * k.n : 16);
	const __amdgpu_buffer_rsrc_t rs_olf = gcl::host_rsrc(k.olflags ? (const void *)k.olflags : k.tables,
	                                                     I32 && k.olflags ? k.n : 16);
	const __amdgpu_buffer_rsrc_t rs_rss = gcl::host_rsrc(k.rss ? (const void *)k.rss : k.tables,
	                                                     I32 && k.rss ? 4 * k.n : 16);
	const uint32_t vbytes = VF ? VF : verdict_width(k.cflags);
	const __amdgpu_buffer_rsrc_t rs_v = gcl::host_rsrc(k.verdicts, I32 ? vbytes * k.n : 16);
	const uint32_t flen32 = (uint32_t)k.frames_len, n32 = (uint32_t)k.n;
	const uint32_t nt32 = (uint32_t)k.ntiles; /* I32: n < 2^28, so every tile index fits */
	const uint32_t fbase3 = (uint32_t)(uintptr_t)k.frames & 3;
	/* I32 pair_src: [off + 8, off + 40) fits below frames_len iff off <= fit_lim */
	const bool fit_any = flen32 >= 40;
	const uint32_t fit_lim = fit_any ? flen32 - 40 : 0u;
	const uint32_t half16 = 16u * (uint32_t)(tid & 1);
	auto idx = [&](uint64_t tt) -> uint64_t {
		if constexpr (I32)
			return (uint32_t)tt * (uint32_t)NT + (uint32_t)tid;
		else
			return tt * NT + tid;
	};
	auto ok = [&](uint64_t tt) {
		if constexpr (I32) /* 32-bit compares: the tile test stays scalar */
			return (uint32_t)tt < nt32 && (uint32_t)idx(tt) < n32;
		else
			return tt < k.ntiles && tt * NT + tid < k.n;
	};
	/* the raw offset: clamped (user_off) where it is used, two half-steps
	 * later -- clamped here, the compare right after the load made every
	 * half-step wait for it, and so for every load issued before it */
	auto ld_off = [&](uint64_t tt) -> uint64_t {
		if constexpr (I32) {
			const uint32_t o = k.offs && ok(tt) ? 8u * (uint32_t)idx(tt) : 0u;
			const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs_off, (int)o, 0, 0);
			return (uint64_t)v[1] << 32 | v[0];
		} else {
			return offs_src[k.offs && ok(tt) ? tt * NT + tid : 0];
		}
	};
	auto src_of = [&](uint64_t tt, uint64_t raw) -> Src {
		if constexpr (I32) {
			/* pair_src in 32 bits: frames_len < 2^31 - 64, so off + 8 and
			 * kBw32 | off never meet each other or kNoOff32 */
			const uint32_t off = k.offs ? (raw < k.frames_len ? (uint32_t)raw : flen32)
			                            : (uint32_t)idx(tt) * (uint32_t)k.stride;
			/* bitwise, not short-circuit: straight-line selects, no exec-mask
			 * branches; off <= fit_lim implies off < frames_len */
			const bool fits = fit_any & (off <= fit_lim) & (((fbase3 + off) & 3) == 0);
			const uint32_t my = fits ? off + 8 : kBw32 | __builtin_elementwise_min(off, flen32);
			return ok(tt) ? my : kNoOff32;
		} else {
			return pair_src(k, !ok(tt) ? kNoOff : k.offs ? user_off(k, raw) : (tt * NT + tid) * k.stride);
		}
	};
	auto pref = [&](uint64_t tt, uint32_t pr[2]) {
		if constexpr (I32) {
			const uint32_t i = ok(tt) ? (uint32_t)idx(tt) : 0u;
			pr[0] = __builtin_amdgcn_raw_buffer_load_b8(rs_olf, (int)(k.olflags ? i : 0u), 0, 0);
			if (MODE == GCL_HASH_NIC || (MODE == kModeProbe && k.rss))
				pr[1] = __builtin_amdgcn_raw_buffer_load_b32(rs_rss, (int)(k.rss ? 4u * i : 0u), 0, 0);
		} else {
			const uint64_t i = ok(tt) ? tt * NT + tid : 0;
			pr[0] = *(k.olflags ? k.olflags + i : side_dummy<uint8_t>(k, i));
			if (MODE == GCL_HASH_NIC || (MODE == kModeProbe && k.rss)) /* the probe: a NIC-mode context's */
				pr[1] = *(k.rss ? k.rss + i : side_dummy<uint32_t>(k, i));
		}
	};
	/* load J of this lane: half (lane & 1) of the pair's packet J */
	auto load32 = [&](uint32_t s) -> uint4 {
		/* s with its top bit set (bytewise, or no packet) needs no select:
		 * kBw32 | o + 16 lies past frames_len (< 2^31 - 64), where the
		 * descriptor's range check returns zeros, and kNoOff32 + 16 wraps to
		 * 15, an in-range read nothing uses */
		const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_fr, (int)(s + half16), 0, 0);
		return make_uint4(v[0], v[1], v[2], v[3]);
	};
	auto issue = [&](Src my, uint4 r[2]) {
		if constexpr (I32) {
			r[0] = load32(mdpp<0xA0>(my)); /* quad_perm [0,0,2,2] */
			r[1] = load32(mdpp<0xF5>(my)); /* quad_perm [1,1,3,3] */
		} else {
			r[0] = pair_load<0>(k, my);
			r[1] = pair_load<1>(k, my);
		}
	};
	auto bytewise = [&](Src my) {
		if constexpr (I32)
			return (my >> 31) && my != kNoOff32;
		else
			return (my >> 63) && my != kNoOff;
	};
	/* this packet's frame offset from its pair_src encoding */
	auto frame_off_of = [&](Src my) -> uint64_t {
		if constexpr (I32)
			return (my >> 31) ? (uint64_t)(my & ~kBw32) : (uint64_t)my - 8;
		else
			return (my >> 63) ? (my & ~kPairBytewise) : my - 8;
	};
	auto put = [&](uint64_t i, uint64_t v) {
		if constexpr (I32) {
			const int o = (int)((uint32_t)i * vbytes);
			if (vbytes == 1)
				__builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, rs_v, o, 0, gcl::kSysAux);
			else if (vbytes == 2)
				__builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, rs_v, o, 0, gcl::kSysAux);
			else if (vbytes == 4)
				__builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, rs_v, o, 0, gcl::kSysAux);
			else
				__builtin_amdgcn_raw_buffer_store_b64(
				        (gcl::u32x2){(uint32_t)v, (uint32_t)(v >> 32)}, rs_v, o, 0, gcl::kSysAux);
		} else {
			put_verdict_vf<VF>(k, i, v);
		}
	};
	/* the landed halves -> this lane's header dwords (frame bytes 12-39;
	 * d10, bytes 40-43, is not fetched: avail 40 sends ARP to the frame) */
	auto unpack = [&](uint4 r[2], Src my, HdrWords &h) {
		/* every loaded dword live until here: a dword nothing reads (bytes
		 * 8-11) let the compiler reuse its register right after the load
		 * was issued, and wait for that load there, a latency per
		 * half-step */
		asm volatile("" : "+v"(r[0].x), "+v"(r[0].y), "+v"(r[0].z), "+v"(r[0].w), "+v"(r[1].x), "+v"(r[1].y),
		             "+v"(r[1].z), "+v"(r[1].w));
		pair_exchange(r);
		if (bytewise(my)) { /* bytewise (rare) */
			const uint64_t off = frame_off_of(my);
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
	auto classify = [&](uint64_t tt, const HdrWords &h, const uint32_t pr[2], Src my) {
		if constexpr (MODE == kModeProbe) {
			/* gcl_access_probe: the words rx_one_pkt would read, folded, and
			 * stored as the verdict is (no tables, hashes or histogram) */
			if (ok(tt))
				put(idx(tt), h.d3 ^ h.d5 ^ h.d6 ^ h.d7 ^ h.d8 ^ h.d9 ^ (k.olflags ? pr[0] & 0xFF : 0u) ^
				                     (k.rss ? pr[1] : 0u));
			return;
		}
		const uint32_t fl = k.olflags ? pr[0] & 0xFF : k.default_flags;
		const bool plain = !ok(tt) || ((h.d3 & 0x000FFFFF) == 0x00050008 && !(fl & GCL_F_FDIR_ID));
		if constexpr (MODE != kModeProbe) {
			if (lean_ok && __all(plain)) {
				if (ok(tt))
					put(idx(tt), classify_lean<MODE, true, false, VF>(k, h, tb, fl, pr[1], hist, tid, cnt));
			} else if (ok(tt)) {
				const uint64_t i = tt * NT + tid;
				/* this packet's frame offset, for the ARP target's extra read */
				put(i, classify_core<MODE, true, false, true, VF>(k, h, nullptr, tid, i, tb, hist, cnt, 0, 40, pr,
				                                                   frame_off_of(my)));
			}
		}
	};

	uint64_t t = blockIdx.x;
	uint4 ra[2], rb[2];
	uint32_t pra[2] = {0, 0}, prb[2] = {0, 0};
	/* prologue: tiles t and t + step in flight, offsets of the two after */
	uint64_t oa = ld_off(t), ob = ld_off(t + step);
	Src sa = src_of(t, oa);
	issue(sa, ra);
	pref(t, pra);
	oa = ld_off(t + 2 * step);
	Src sb = src_of(t + step, ob);
	issue(sb, rb);
	pref(t + step, prb);
	ob = ld_off(t + 3 * step);
	while (I32 ? (uint32_t)t < nt32 : t < k.ntiles) {
		asm volatile("" : "+s"(t));
		HdrWords h;
		unpack(ra, sa, h);
		Src my = sa;
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

} // namespace gclk

using namespace gclk;

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
	int grid;     /* blocks per launch when > 0 (gcl_tune.grid) */
	bool pair;    /* classify_pair_kernel (GENERAL batches): [8, 40) per packet by lane pairs */
	bool i32;     /* ... with 32-bit indices and offsets (pair_i32_ok) */
	int defer;    /* classify_kernel with 1-/2-B verdicts kept in LDS (and past a full
	                 buffer in kVregs registers per lane) and written in batches: 1 where
	                 that takes <= 2 writes per block, 2 always (tests) */
};

/* geo.defer: what the CU's LDS leaves the block at geo.bpc_cap blocks per
 * CU holds k.vcap tiles of verdicts -- at most the block's share of the
 * batch, and only where that takes at most two writes per block */
static bool plan_defer(const KParams &k, uint32_t &lds, int num_cus, const Geometry &geo, uint32_t nt,
                       uint32_t &vcap, uint32_t &vregs)
{
	vcap = vregs = 0;
	if (!geo.defer)
		return false;
	const uint32_t vb = (k.cflags & GCL_CFG_VERDICT1) ? 1 : 2;
	const uint32_t base = align16(lds);
	const uint32_t per_cu = 160 * 1024 / (uint32_t)std::max(geo.bpc_cap, 1);
	const uint64_t blocks = geo.grid > 0 ? (uint64_t)geo.grid : (uint64_t)num_cus * std::max(geo.bpc_cap, 1);
	const uint64_t want = ((k.n + nt - 1) / nt + blocks - 1) / blocks;
	const uint64_t room = per_cu > base ? (per_cu - base) / (nt * vb) : 0;
	const uint64_t rcap = kVregs * 4 / vb; /* tiles the registers hold past a full buffer */
	if (!room || (2 * (room + rcap) < want && geo.defer != 2))
		return false;
	vcap = (uint32_t)std::min(want, room);
	vregs = rcap && want > room;
	lds = base + vcap * nt * vb;
	return true;
}

template <int MODE, int DEPTH, int NT>
static hipError_t launch_nt(KParams k, bool tlds, uint32_t lds, int num_cus, const Geometry &geo,
                            hipStream_t s)
{
	plan_defer(k, lds, num_cus, geo, NT, k.vcap, k.vregs);
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
#define GCL_PAIR(I) (v2 ? (tlds ? classify_pair_kernel<MODE, true, NT, 2, I> \
	                        : classify_pair_kernel<MODE, false, NT, 2, I>) \
	                : (tlds ? classify_pair_kernel<MODE, true, NT, 0, I> \
	                        : classify_pair_kernel<MODE, false, NT, 0, I>))
	ClassifyFn fn = geo.i32 ? GCL_PAIR(true) : GCL_PAIR(false);
#undef GCL_PAIR
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
	g.i32 = false; /* batch_launch decides */
	g.defer = defer_ok ? tuned(c->tune.defer, kDefaultDefer) : 0;
	auto per_block = [&](uint32_t nt) -> uint32_t {
		if (g.pair)
			return hist_bytes + tab_lds;
		return nt * 64 + hist_bytes + tab_lds;
	};
	/* dense slots: 512-lane tiles, two blocks per CU (one generation of
	 * blocks over the chip), then 1024 x 1; GENERAL batches (the pair kernel,
	 * no tile): 2 x 256, below.  Round 6 re-measured the dense shape with the
	 * lean waves and the deferred verdicts: 2 x 512 at depth 1 307-318 us on
	 * udp64 against 317-328 for round 5's 4 x 256 at depth 2, fastest in six
	 * of six rounds (profiles/r06_geometry_ab.jsonl); the pair kernel at
	 * 2 x 512: random pool 151.8-152.5 -> 150.0-151.0 us, working set
	 * 52.6-53.3 -> 52.0-52.6 (profiles/r06_pair_geometry_ab.jsonl) */
	/* The pair kernel keeps two tiles of frame loads in flight, so half the
	 * lanes -- 2 x 256 per CU -- halves the lines in flight (as wide slots
	 * do on the tile kernel, batch_launch): working set 50.2-50.3 ->
	 * 48.3-48.7 us, random pool 1 % faster; 4 x 256 slower
	 * (profiles/r06_pair_lanes_ab.jsonl) */
	static const int order_dense[] = {512, 1024, 256}, order_pair[] = {256, 512, 1024};
	const uint32_t lanes = g.pair ? 512 : lanes_cu;
	for (int nt : g.pair ? order_pair : order_dense) {
		const uint32_t pb = per_block((uint32_t)nt);
		const uint32_t bpc = std::max(lanes / (uint32_t)nt, 1u);
		if (!g.threads && bpc * pb <= lds_cu) {
			g.threads = nt;
			g.bpc_cap = (int)bpc;
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
		 * 32 Mi, and no change on tcp1500 (profiles/archive/r01_hsplit_geometry.jsonl).
		 * A block that defers its verdicts runs at depth 1 (batch_launch) */
		g.depth = 2;
	}
	g.threads = tuned(c->tune.threads, g.threads);
	g.depth = tuned(c->tune.depth, g.depth);
	g.bpc_cap = tuned(c->tune.blocks_per_cu, g.bpc_cap);
	g.grid = tuned(c->tune.grid, 0);
	return g;
}

extern "C" int gcl_classify(struct gcl_ctx *c, const struct gcl_batch *b,
                            void *verdicts, uint64_t *runtime_counts,
                            uint64_t *stats, void *hip_stream)
{
	struct gcl_out o = {verdicts, runtime_counts, stats, nullptr};
	return gcl_classify_ex(c, b, &o, hip_stream);
}

static int batch_launch(gcl_ctx *c, const gcl_batch *b, const gcl_out *out, hipStream_t s, bool probe);

/* a dense batch: fixed slots, no side arrays, every header granule in range
 * (classify_kernel's batches; the others run on classify_pair_kernel) --
 * whether gcl_access_probe's kernel shape is the tile or the pair kernel's */
static bool dense_batch(const gcl_ctx *c, const gcl_batch *b)
{
	return !(b->offs || b->olflags || b->fdir_hi || b->dst_hint || (c->cfg.default_olflags & GCL_F_FDIR_ID) ||
	         b->frames_len < (b->n - 1) * b->stride + GCL_HDR_GRANULE);
}

extern "C" int gcl_access_probe(struct gcl_ctx *c, const struct gcl_batch *b, void *out,
                                uint32_t vbytes, void *hip_stream)
{
	const bool minimal = vbytes & GCL_PROBE_MIN;
	vbytes &= ~(uint32_t)GCL_PROBE_MIN;
	if (!c || !b || !out || (vbytes != 1 && vbytes != 2 && vbytes != 4 && vbytes != 8))
		return -EINVAL;
	if (b->n == 0)
		return 0;
	if (!b->frames || b->frames_len == UINT64_MAX || b->n > (1ull << 40) ||
	    (!b->offs && (b->stride < 16 || (b->stride & 15) || b->stride > (1u << 20))))
		return -EINVAL;
	if (hipSetDevice(c->device) != hipSuccess)
		return -ENODEV;
	if (!minimal && vbytes == verdict_bytes(c)) {
		/* the classify launch itself (tile or pair kernel), rx_one_pkt folded away */
		const struct gcl_out o = {out, nullptr, nullptr, nullptr};
		return batch_launch(c, b, &o, (hipStream_t)hip_stream, true);
	}
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
	return batch_launch(c, b, out, (hipStream_t)hip_stream, false);
}

/* gcl_classify_ex, or with @probe (gcl_access_probe) the same launch in
 * kModeProbe: no counts, stats or timing */
static int batch_launch(gcl_ctx *c, const gcl_batch *b, const gcl_out *out, hipStream_t s, bool probe)
{
	void *verdicts = out->verdicts;
	uint64_t *runtime_counts = out->runtime_counts, *stats = out->stats;
	if (out->trans && !(c->cfg.flags & GCL_CFG_TRANS_HASH))
		return -EINVAL;
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
	/* a probe loads hash.rss where the context's own launch would */
	k.rss = probe && c->cfg.hash_mode != GCL_HASH_NIC ? nullptr : b->rss;
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
	k.plean = (uint32_t)tuned(c->tune.pair_lean, kDefaultPairLean);
	k.tlean = (uint32_t)tuned(c->tune.tile_lean, kDefaultTileLean);
	k.vstage = (uint32_t)tuned(c->tune.vstage, kDefaultVstage);
	k.contig = (uint32_t)tuned(c->tune.tile_order, kDefaultTileOrder);
	k.default_flags = c->cfg.default_olflags;

	/* the specialised fast path needs every header granule in range */
	const bool general = !dense_batch(c, b);
	uint32_t tab_bytes = c->image_bytes;
	uint32_t hist_bytes = ((c->cfg.max_runtimes + 3) & ~3u) * 4;
	const bool tlds = tab_bytes <= kLdsTableBudget && c->tune.tables != 1;
	k.tables_lds_bytes = tlds ? tab_bytes : 0;
	/* dense slots with 1-/2-B verdicts, 16-B-aligned (the deferred verdicts
	 * go out 16 B at a time, through a buffer descriptor: below 4 GiB) */
	const bool defer_ok = !general && (k.cflags & (GCL_CFG_VERDICT1 | GCL_CFG_VERDICT2)) &&
	                      ((uintptr_t)verdicts & 15) == 0 && b->n * 2 < (1ull << 32);
	Geometry geo = choose_geometry(c, tlds ? tab_bytes : 0, hist_bytes, general, defer_ok);
	if (!general && geo.depth == 2 && c->tune.depth == GCL_TUNE_AUTO && b->stride <= GCL_HDR_GRANULE) {
		/* a block that keeps its verdicts until after its reads streams a
		 * dense slab best with one tile in flight (udp64 1-B at 2 x 512:
		 * 307-318 against 308-319 us at depth 2, profiles/r06_geometry_ab.jsonl);
		 * per-packet stores, and headers one per line of a wide slot
		 * (tcp1500: depth 1 3 % slower), keep two */
		uint32_t l = (uint32_t)geo.threads * 64 + hist_bytes + (tlds ? tab_bytes : 0), vc, vr;
		if (plan_defer(k, l, c->num_cus, geo, (uint32_t)geo.threads, vc, vr))
			geo.depth = 1;
	}
	if (!general && b->stride > GCL_HDR_GRANULE && geo.threads == 512 && c->tune.threads == GCL_TUNE_AUTO &&
	    c->tune.depth == GCL_TUNE_AUTO) {
		/* wide slots (one header per 128-B line or more): 256-lane tiles at
		 * depth 1, still two blocks per CU -- 512 lines (64 KiB) in flight
		 * per CU, what the dense 2 x 512 shape keeps at 64 B per header,
		 * instead of 2048: tcp1500 172.3-173.2 -> 164.8-165.7 us, and
		 * 166.5 at depth 2 (profiles/r06_wide_geometry_ab.jsonl) */
		geo.threads = 256;
		geo.depth = 1;
	}
	/* the pair kernel's 32-bit form: frames (and the largest slot offset),
	 * offsets, side arrays and verdicts each within 2 GiB */
	geo.i32 = general && tuned(c->tune.pair_i32, kDefaultPairI32) && b->frames_len < (1ull << 31) - 64 &&
	          b->n < (1ull << 28) && (b->offs || b->n * (uint64_t)b->stride <= (1ull << 31));

	HipErr he;

	hipEvent_t e0 = nullptr, e1 = nullptr;
	if (!probe && (c->cfg.flags & GCL_CFG_PROFILE) && c->prof_seq++ % c->prof_every == 0) {
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
	switch (probe ? kModeProbe : (int)c->cfg.hash_mode) {
	case kModeProbe:
		err = launch_mode<kModeProbe>(k, tlds, geo, tlds ? tab_bytes : 0, hist_bytes, c->num_cus, s);
		break;
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

