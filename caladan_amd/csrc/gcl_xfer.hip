/*
 * gcl_xfer.hip - where the frames come from and the buffers live: the header
 * gather over the reference's mbuf pool (frame data at element + 344,
 * iokernel/defs.h:503-506), the placed device allocation of the frame pool /
 * verdict ring pair (gcl_dev_alloc_paired), host registration, and the
 * end-to-end batch from host memory (gcl_classify_host: zero-copy, or a DMA /
 * gather into HBM on 2-4 streams).
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "../../include/gclassify.h"
#include "gcl_ctx.h"

using namespace gclk;


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

namespace gclk {

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
	    (vb != 1 && vb != 2 && vb != 4 && vb != 8) || (flags & ~(uint32_t)(0xFFFF | GCL_PAIR_QUIET | GCL_PAIR_VERBOSE)))
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
	const bool dbg = (flags & GCL_PAIR_VERBOSE) != 0;
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
	if (classes == 1 && !(flags & GCL_PAIR_QUIET))
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
void *gclk::mapped(const void *h)
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

