/*
 * gcl_group.hip - the multi-GPU step behind the C ABI (include/gcl_group.h).
 *
 * One process, one dataplane thread (iokernel/dpdk.c:276-280,
 * iokernel/main.c:144-150), every GPU of the node: one gcl_ctx per GPU with
 * replicated tables, batches split round-robin in blocks, and the
 * per-runtime counts + rx counters (iokernel/defs.h:417-460) all-gathered
 * with RCCL over xGMI.
 *
 * Counters.  Every GPU accumulates u64[R + 8] ([counts | stats]) in its own
 * `acc` with the classify kernels' atomics.  An exchange first snapshots
 * `acc` on the GPU's compute stream (a 1-8 KiB D2D copy, in order with the
 * launches before it), so launches enqueued after the exchange never race
 * the gather; the gather and the sum then run on a side stream per GPU and
 * overlap the next batches.  Snapshots rotate over kSlots buffers, each
 * guarded by the event that ends its exchange.
 */
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <new>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "../../include/gcl_group.h"
#include "../../include/gclassify.h"

namespace {

constexpr int kSlots = 4; /* exchanges in flight */

struct HipErr {
	hipError_t e = hipSuccess;
	void operator()(hipError_t r)
	{
		if (r != hipSuccess && e == hipSuccess)
			e = r;
	}
	bool bad() const { return e != hipSuccess; }
};

/* out[i] = sum over the @rows gathered vectors of element i */
__global__ void __launch_bounds__(256) sum_rows_kernel(const unsigned long long *rows, int nrows,
                                                       int len, unsigned long long *out)
{
	const int i = blockIdx.x * 256 + threadIdx.x;
	if (i >= len)
		return;
	unsigned long long s = 0;
	for (int r = 0; r < nrows; r++)
		s += rows[(size_t)r * len + i];
	out[i] = s;
}

uint32_t verdict_size(uint32_t flags)
{
	return (flags & GCL_CFG_VERDICT1) ? 1 : (flags & GCL_CFG_VERDICT2) ? 2 : (flags & GCL_CFG_VERDICT4) ? 4 : 8;
}

} // namespace

struct gcl_group {
	int n;
	uint32_t R, L;      /* runtimes; vector length R + GCL_NR_STATS */
	uint64_t block;
	uint32_t xchg;
	uint32_t vsize;
	int nst;            /* work streams per GPU (host batches) */
	struct Dev {
		int dev;
		gcl_ctx *ctx;
		hipStream_t st[GCL_GROUP_MAX_STREAMS]; /* st[0]: device-resident launches */
		hipEvent_t st_ev[GCL_GROUP_MAX_STREAMS];
		hipStream_t xs;                        /* exchange stream */
		uint64_t *acc;                         /* u64[L] */
		uint64_t *snap;                        /* u64[kSlots][L] */
		uint64_t *gath;                        /* u64[kSlots][n * L] */
		uint64_t *node;                        /* u64[kSlots][L] */
		hipEvent_t snap_ev[kSlots];
		hipEvent_t done_ev[kSlots];
		bool pending[kSlots];
		/* COPY staging per work stream, sized for one block */
		uint8_t *slab[GCL_GROUP_MAX_STREAMS];
		uint8_t *side[GCL_GROUP_MAX_STREAMS];
		uint8_t *verd[GCL_GROUP_MAX_STREAMS];
		ncclComm_t comm;
	} d[GCL_GROUP_MAX_DEV];
	uint64_t *host_node; /* pinned u64[kSlots][L]: GPU 0's node vector */
	uint64_t *host_gath; /* pinned u64[kSlots][n * L]: GPU 0's gathered vectors */
	uint64_t seq;        /* exchanges enqueued */
	int last;            /* slot of the last exchange, -1 = none */
	uint32_t timeout_ms; /* bound on RCCL init and on a non-blocking call's completion */
	bool diverged;       /* a table change reached some replicas only: every
	                        later call fails with -EIO (the GPUs would steer
	                        with different tables) */
	bool failed;         /* an exchange's RCCL enqueue failed or timed out: the
	                        communicators were aborted, and every later call
	                        fails with -EIO (a collective may still hold the
	                        snapshot slots; the communicators' state is unknown) */
	uint32_t fault;      /* gcl_group_test_fault: GCL_GROUP_FAULT_* injected (tests) */
};

/* a group that must refuse all work */
static bool broken(const gcl_group *g)
{
	return g->diverged || g->failed;
}

/* Abort every communicator (RCCL's bounded teardown, for communicators in
 * an unknown state) and mark the group failed. */
static void fail_group(gcl_group *g)
{
	for (int i = 0; i < g->n; i++)
		if (g->d[i].comm) {
			(void)hipSetDevice(g->d[i].dev);
			(void)ncclCommAbort(g->d[i].comm);
			g->d[i].comm = nullptr;
		}
	g->failed = true;
}

static uint64_t mono_ms()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000ull + (uint64_t)ts.tv_nsec / 1000000ull;
}

/* Non-blocking communicators: every RCCL call returns at once, possibly with
 * ncclInProgress, and the state is polled here until each communicator is
 * ready, has failed, or @deadline (CLOCK_MONOTONIC ms) passes.  0, -EIO
 * (an RCCL error) or -ETIMEDOUT. */
static int comms_wait(gcl_group *g, uint64_t deadline)
{
	for (;;) {
		bool busy = false;
		for (int i = 0; i < g->n; i++) {
			ncclResult_t st = ncclSuccess;
			if (ncclCommGetAsyncError(g->d[i].comm, &st) != ncclSuccess)
				return -EIO;
			if (st == ncclInProgress)
				busy = true;
			else if (st != ncclSuccess)
				return -EIO;
		}
		if (!busy)
			return 0;
		if (mono_ms() >= deadline)
			return -ETIMEDOUT;
		usleep(100);
	}
}

/* One communicator rank per GPU, initialised together from this thread as
 * ncclCommInitAll does, but non-blocking so that a C caller gets -ETIMEDOUT
 * after g->timeout_ms instead of blocking in RCCL's bootstrap; the partial
 * communicators are aborted then. */
static int comms_init(gcl_group *g, const int *devs)
{
	ncclUniqueId id;
	if (ncclGetUniqueId(&id) != ncclSuccess)
		return -EIO;
	ncclConfig_t conf = NCCL_CONFIG_INITIALIZER;
	conf.blocking = 0;
	const uint64_t deadline = mono_ms() + g->timeout_ms;
	bool ok = ncclGroupStart() == ncclSuccess;
	for (int i = 0; i < g->n && ok; i++) {
		ok = hipSetDevice(devs[i]) == hipSuccess;
		const ncclResult_t r = ok ? ncclCommInitRankConfig(&g->d[i].comm, g->n, id, i, &conf)
		                          : ncclInternalError;
		ok = r == ncclSuccess || r == ncclInProgress;
	}
	const ncclResult_t e = ncclGroupEnd();
	ok = ok && (e == ncclSuccess || e == ncclInProgress);
	int ret = ok ? comms_wait(g, deadline) : -EIO;
	if (ret) {
		for (int i = 0; i < g->n; i++)
			if (g->d[i].comm) {
				(void)hipSetDevice(g->d[i].dev);
				(void)ncclCommAbort(g->d[i].comm);
				g->d[i].comm = nullptr;
			}
	}
	return ret;
}

extern "C" uint64_t gcl_shard_count(uint64_t n, uint32_t world, uint32_t rank, uint64_t block)
{
	if (world <= 1 || block == 0)
		return rank == 0 ? n : 0;
	if (rank >= world)
		return 0;
	const uint64_t full = n / block, tail = n % block;
	/* blocks rank, rank + world, ... below full, plus the ragged last block */
	uint64_t c = (full > rank ? (full - rank + world - 1) / world : 0) * block;
	if (tail && full % world == rank)
		c += tail;
	return c;
}

extern "C" uint64_t gcl_shard_global(uint64_t j, uint32_t world, uint32_t rank, uint64_t block)
{
	if (world <= 1 || block == 0)
		return j;
	return ((j / block) * world + rank) * block + j % block;
}

/* zero a GPU's accumulators, complete before returning: the group's streams
 * are non-blocking, so a null-stream hipMemset (which may return before it
 * lands) is not ordered before the next exchange's snapshot on st[0] */
static hipError_t zero_acc(gcl_group::Dev &D, size_t bytes)
{
	hipError_t e = hipMemsetAsync(D.acc, 0, bytes, D.st[0]);
	return e != hipSuccess ? e : hipStreamSynchronize(D.st[0]);
}

static void free_dev(gcl_group::Dev &D, bool rccl)
{
	if (D.dev < 0)
		return;
	(void)hipSetDevice(D.dev);
	if (rccl && D.comm)
		(void)ncclCommDestroy(D.comm);
	for (int i = 0; i < GCL_GROUP_MAX_STREAMS; i++) {
		if (D.st[i])
			(void)hipStreamDestroy(D.st[i]);
		if (D.st_ev[i])
			(void)hipEventDestroy(D.st_ev[i]);
		if (D.slab[i])
			(void)hipFree(D.slab[i]);
		if (D.side[i])
			(void)hipFree(D.side[i]);
		if (D.verd[i])
			(void)hipFree(D.verd[i]);
	}
	if (D.xs)
		(void)hipStreamDestroy(D.xs);
	for (int s = 0; s < kSlots; s++) {
		if (D.snap_ev[s])
			(void)hipEventDestroy(D.snap_ev[s]);
		if (D.done_ev[s])
			(void)hipEventDestroy(D.done_ev[s]);
	}
	for (uint64_t *p : {D.acc, D.snap, D.gath, D.node})
		if (p)
			(void)hipFree(p);
	if (D.ctx)
		gcl_close(D.ctx);
}

extern "C" void gcl_group_close(struct gcl_group *g)
{
	if (!g)
		return;
	(void)gcl_group_sync(g);
	for (int i = 0; i < g->n; i++)
		free_dev(g->d[i], g->xchg == GCL_XCHG_RCCL);
	if (g->host_node)
		(void)hipHostFree(g->host_node);
	if (g->host_gath)
		(void)hipHostFree(g->host_gath);
	delete g;
}

extern "C" int gcl_group_open_v2(int ndev, const int *devs, const struct gcl_cfg *cfg,
                                 const struct gcl_group_cfg *gcfg, struct gcl_group **out)
{
	if (!out || !devs || !cfg || ndev < 1 || ndev > GCL_GROUP_MAX_DEV)
		return -EINVAL;
	if (gcfg && gcfg->size != sizeof(struct gcl_group_cfg))
		return -EINVAL; /* a struct of another layout */
	*out = nullptr;
	const uint64_t block = gcfg && gcfg->block ? gcfg->block : GCL_GROUP_BLOCK;
	const uint32_t xchg = gcfg ? gcfg->exchange : GCL_XCHG_RCCL;
	const uint32_t nst = gcfg && gcfg->nstreams ? gcfg->nstreams : 2;
	if ((block & 255) || block > (1ull << 32) || xchg > GCL_XCHG_HOST ||
	    nst > GCL_GROUP_MAX_STREAMS)
		return -EINVAL;
	int visible = 0;
	if (hipGetDeviceCount(&visible) != hipSuccess)
		return -ENODEV;
	for (int i = 0; i < ndev; i++) {
		if (devs[i] < 0 || devs[i] >= visible)
			return -ENODEV;
		for (int j = 0; j < i && xchg == GCL_XCHG_RCCL; j++)
			if (devs[j] == devs[i])
				return -EINVAL; /* one communicator rank per GPU */
	}

	gcl_group *g = new (std::nothrow) gcl_group();
	if (!g)
		return -ENOMEM;
	g->n = ndev;
	g->R = cfg->max_runtimes;
	g->L = cfg->max_runtimes + GCL_NR_STATS;
	g->block = block;
	g->xchg = xchg;
	g->vsize = verdict_size(cfg->flags);
	g->nst = (int)nst;
	g->seq = 0;
	g->last = -1;
	for (int i = 0; i < GCL_GROUP_MAX_DEV; i++)
		g->d[i].dev = -1;
	const size_t L8 = (size_t)g->L * 8;
	int ret = 0;
	for (int i = 0; i < ndev && !ret; i++) {
		gcl_group::Dev &D = g->d[i];
		D.dev = devs[i];
		ret = gcl_open(devs[i], cfg, &D.ctx);
		if (ret)
			break;
		HipErr he;
		he(hipSetDevice(D.dev));
		for (int s = 0; s < g->nst; s++) {
			he(hipStreamCreateWithFlags(&D.st[s], hipStreamNonBlocking));
			he(hipEventCreateWithFlags(&D.st_ev[s], hipEventDisableTiming));
		}
		he(hipStreamCreateWithFlags(&D.xs, hipStreamNonBlocking));
		for (int s = 0; s < kSlots; s++) {
			he(hipEventCreateWithFlags(&D.snap_ev[s], hipEventDisableTiming));
			he(hipEventCreateWithFlags(&D.done_ev[s], hipEventDisableTiming));
		}
		he(hipMalloc(&D.acc, L8));
		he(hipMalloc(&D.snap, L8 * kSlots));
		he(hipMalloc(&D.gath, L8 * kSlots * ndev));
		he(hipMalloc(&D.node, L8 * kSlots));
		if (!he.bad())
			he(zero_acc(D, L8));
		if (he.bad())
			ret = he.e == hipErrorOutOfMemory ? -ENOMEM : -EIO;
	}
	if (!ret) {
		HipErr he;
		he(hipHostMalloc(&g->host_node, L8 * kSlots, hipHostMallocDefault));
		he(hipHostMalloc(&g->host_gath, L8 * kSlots * ndev, hipHostMallocDefault));
		if (he.bad())
			ret = -ENOMEM;
	}
	if (!ret && xchg == GCL_XCHG_RCCL) {
		g->timeout_ms = gcfg && gcfg->init_timeout_ms ? gcfg->init_timeout_ms
		                                               : GCL_GROUP_INIT_TIMEOUT_MS;
		ret = comms_init(g, devs);
	}
	if (ret) {
		gcl_group_close(g);
		return ret;
	}
	*out = g;
	return 0;
}

/* The exported gcl_group_open symbol reads the 16-B struct gcl_group_cfg of
 * rounds 1-3 (block, exchange, nstreams), with the default RCCL init bound;
 * the current header maps gcl_group_open to gcl_group_open_v2.  A binary
 * built against the round-4 header (a 24-B struct with init_timeout_ms and a
 * pad word, passed to this same symbol) loses its init_timeout_ms here until
 * it is rebuilt against the current header: the two layouts cannot be told
 * apart at run time. */
struct gcl_group_cfg_v1 {
	uint64_t block;
	uint32_t exchange;
	uint32_t nstreams;
};

#undef gcl_group_open
extern "C" int gcl_group_open(int ndev, const int *devs, const struct gcl_cfg *cfg,
                              const struct gcl_group_cfg_v1 *gcfg, struct gcl_group **out)
{
	struct gcl_group_cfg c = {};
	c.size = sizeof(c);
	if (gcfg) {
		c.block = gcfg->block;
		c.exchange = gcfg->exchange;
		c.nstreams = gcfg->nstreams;
	}
	return gcl_group_open_v2(ndev, devs, cfg, &c, out);
}

extern "C" int gcl_group_size(const struct gcl_group *g) { return g ? g->n : -EINVAL; }

extern "C" struct gcl_ctx *gcl_group_ctx(struct gcl_group *g, int i)
{
	return g && i >= 0 && i < g->n ? g->d[i].ctx : nullptr;
}

extern "C" void *gcl_group_stream(struct gcl_group *g, int i)
{
	return g && i >= 0 && i < g->n ? (void *)g->d[i].st[0] : nullptr;
}

/* A table change is checked by context 0 first: every context has the same
 * cfg and the same tables, so a refusal there (-EINVAL, -EEXIST, -ENOENT)
 * leaves all replicas untouched.  The replicas' setters only edit a host
 * mirror and cannot fail differently; if one ever did, the group is marked
 * diverged and refuses all further work rather than classify with tables
 * that differ between GPUs. */
template <typename F>
static int fan_out(struct gcl_group *g, F f)
{
	if (!g)
		return -EINVAL;
	if (broken(g))
		return -EIO;
	const int r0 = f(g->d[0].ctx);
	if (r0)
		return r0;
	for (int i = 1; i < g->n; i++)
		if (f(g->d[i].ctx)) {
			g->diverged = true;
			return -EIO;
		}
	return 0;
}

extern "C" int gcl_group_runtime_set(struct gcl_group *g, uint16_t uniqid, uint32_t ip_host,
                                     uint16_t thread_count, uint16_t active_count,
                                     const uint16_t *flow_tbl)
{
	return fan_out(g, [&](gcl_ctx *c) {
		return gcl_runtime_set(c, uniqid, ip_host, thread_count, active_count, flow_tbl);
	});
}

extern "C" int gcl_group_runtime_del(struct gcl_group *g, uint16_t uniqid)
{
	return fan_out(g, [&](gcl_ctx *c) { return gcl_runtime_del(c, uniqid); });
}

extern "C" int gcl_group_runtime_set_trans_seed(struct gcl_group *g, uint16_t uniqid, uint32_t seed)
{
	return fan_out(g, [&](gcl_ctx *c) { return gcl_runtime_set_trans_seed(c, uniqid, seed); });
}

extern "C" int gcl_group_classify(struct gcl_group *g, const struct gcl_batch *shards,
                                  void *const *verdicts)
{
	if (!g || !shards || !verdicts)
		return -EINVAL;
	if (broken(g))
		return -EIO;
	for (int i = 0; i < g->n; i++) {
		gcl_group::Dev &D = g->d[i];
		const int r = gcl_classify(D.ctx, &shards[i], verdicts[i], D.acc, D.acc + g->R, D.st[0]);
		if (r)
			return r;
	}
	return 0;
}

/* device address of registered host memory on the current device, or NULL */
static void *mapped(const void *h)
{
	void *d = nullptr;
	if (!h)
		return nullptr;
	if (hipHostGetDevicePointer(&d, (void *)h, 0) != hipSuccess) {
		(void)hipGetLastError();
		return nullptr;
	}
	return d;
}

/* Work streams 0 .. @nst - 1 on every GPU (a host batch may ask for more
 * than the group opened with); exchanges and syncs cover all of them. */
static int grow_streams(gcl_group *g, int nst)
{
	for (int i = 0; i < g->n && nst > g->nst; i++) {
		gcl_group::Dev &D = g->d[i];
		if (hipSetDevice(D.dev) != hipSuccess)
			return -ENODEV;
		for (int s = g->nst; s < nst; s++)
			if (!D.st[s] && (hipStreamCreateWithFlags(&D.st[s], hipStreamNonBlocking) != hipSuccess ||
			                 hipEventCreateWithFlags(&D.st_ev[s], hipEventDisableTiming) != hipSuccess))
				return -ENOMEM;
	}
	if (nst > g->nst)
		g->nst = nst;
	return 0;
}

static int ensure_staging(gcl_group *g, gcl_group::Dev &D, int nst)
{
	if (hipSetDevice(D.dev) != hipSuccess)
		return -ENODEV;
	for (int s = 0; s < nst; s++) {
		if (D.slab[s])
			continue;
		if (hipMalloc(&D.slab[s], g->block * GCL_GATHER_ROW) != hipSuccess ||
		    hipMalloc(&D.side[s], g->block * 21) != hipSuccess ||
		    hipMalloc(&D.verd[s], g->block * 8) != hipSuccess)
			return -ENOMEM;
	}
	return 0;
}

/* Sub-batch of block @b: packets [b * block, min(n, (b + 1) * block)). */
static gcl_batch block_batch(const gcl_batch &hb, uint64_t b, uint64_t block)
{
	gcl_batch s = hb;
	const uint64_t i0 = b * block;
	s.n = hb.n - i0 < block ? hb.n - i0 : block;
	if (hb.offs) {
		s.offs = hb.offs + i0;
	} else {
		const uint64_t o = i0 * hb.stride;
		s.frames = hb.frames + o;
		s.frames_len = hb.frames_len > o ? hb.frames_len - o : 0;
	}
	if (hb.olflags)
		s.olflags = hb.olflags + i0;
	if (hb.rss)
		s.rss = hb.rss + i0;
	if (hb.fdir_hi)
		s.fdir_hi = hb.fdir_hi + i0;
	if (hb.dst_hint)
		s.dst_hint = hb.dst_hint + i0;
	if (hb.pkt_len)
		s.pkt_len = hb.pkt_len + i0;
	return s;
}

extern "C" int gcl_group_classify_host(struct gcl_group *g, const struct gcl_batch *hb,
                                       void *host_verdicts, const struct gcl_e2e_opts *o)
{
	if (!g || !hb || !host_verdicts || !o || o->mode > GCL_E2E_ZEROCOPY ||
	    o->nstreams > GCL_GROUP_MAX_STREAMS)
		return -EINVAL;
	if (broken(g))
		return -EIO;
	if (hb->n == 0)
		return 0;
	if (!hb->frames || (!hb->offs && (hb->stride < 16 || (hb->stride & 15))))
		return -EINVAL;
	const int nst = o->nstreams ? (int)o->nstreams : g->nst;
	const int G = g->n;
	const uint64_t nb = (hb->n + g->block - 1) / g->block;
	int ret = grow_streams(g, nst);
	if (ret)
		return ret;
	HipErr he;
	if (o->mode == GCL_E2E_ZEROCOPY) {
		/* every GPU reads its blocks straight out of registered host
		 * memory and writes their verdicts back in place */
		gcl_batch db[GCL_GROUP_MAX_DEV];
		uint8_t *dv[GCL_GROUP_MAX_DEV];
		for (int i = 0; i < G; i++) {
			if (hipSetDevice(g->d[i].dev) != hipSuccess)
				return -ENODEV;
			db[i] = *hb;
			db[i].frames = (const uint8_t *)mapped(hb->frames);
			db[i].offs = (const uint64_t *)mapped(hb->offs);
			db[i].olflags = (const uint8_t *)mapped(hb->olflags);
			db[i].rss = (const uint32_t *)mapped(hb->rss);
			db[i].fdir_hi = (const uint32_t *)mapped(hb->fdir_hi);
			db[i].dst_hint = (const uint32_t *)mapped(hb->dst_hint);
			db[i].pkt_len = nullptr;
			dv[i] = (uint8_t *)mapped(host_verdicts);
			if (!db[i].frames || !dv[i] || (hb->offs && !db[i].offs) ||
			    (hb->olflags && !db[i].olflags) || (hb->rss && !db[i].rss) ||
			    (hb->fdir_hi && !db[i].fdir_hi) || (hb->dst_hint && !db[i].dst_hint))
				return -EFAULT; /* not registered: gcl_host_register */
		}
		/* blocks in batch order, so every GPU has work from the start */
		for (uint64_t b = 0; b < nb && !ret; b++) {
			const int i = (int)(b % G);
			gcl_group::Dev &D = g->d[i];
			const gcl_batch s = block_batch(db[i], b, g->block);
			ret = gcl_classify(D.ctx, &s, dv[i] + b * g->block * g->vsize, D.acc, D.acc + g->R,
			                   D.st[(b / G) % nst]);
		}
	} else {
		/* a row holds frame bytes [0, 80) (IHL 15's ports end at 78): 80-B
		 * rows by 2D DMA from slots of >= 80 B, the 64-B slots themselves,
		 * or gathered by gcl_header_gather from per-packet offsets */
		const uint64_t row = hb->offs || hb->stride >= GCL_GATHER_ROW ? GCL_GATHER_ROW : GCL_HDR_GRANULE;
		if (!hb->offs && (hb->stride < GCL_HDR_GRANULE ||
		                  hb->frames_len < (hb->n - 1) * hb->stride + row))
			return -EINVAL;
		if (hb->offs && hb->frames_len == UINT64_MAX)
			return -EINVAL;
		const uint8_t *dfr[GCL_GROUP_MAX_DEV];
		const uint64_t *dof[GCL_GROUP_MAX_DEV];
		for (int i = 0; i < G && hb->offs; i++) {
			if (hipSetDevice(g->d[i].dev) != hipSuccess)
				return -ENODEV;
			dfr[i] = (const uint8_t *)mapped(hb->frames);
			dof[i] = (const uint64_t *)mapped(hb->offs);
			if (!dfr[i])
				return -EFAULT; /* the gather reads the registered region */
		}
		for (int i = 0; i < G; i++)
			if ((ret = ensure_staging(g, g->d[i], nst)))
				return ret;
		for (uint64_t b = 0; b < nb && !ret; b++) {
			const int i = (int)(b % G);
			gcl_group::Dev &D = g->d[i];
			const int si = (int)((b / G) % nst);
			hipStream_t st = D.st[si];
			const gcl_batch s = block_batch(*hb, b, g->block);
			const uint64_t m = s.n, B = g->block;
			if (hipSetDevice(D.dev) != hipSuccess)
				return -ENODEV;
			if (hb->offs) {
				/* the block's offsets: mapped, or copied beside the side arrays */
				const uint64_t *so = dof[i] ? dof[i] + b * B : (const uint64_t *)(D.side[si] + 13 * B);
				if (!dof[i])
					he(hipMemcpyAsync((void *)so, s.offs, m * 8, hipMemcpyHostToDevice, st));
				if (gcl_header_gather(dfr[i], hb->frames_len, so, m, D.slab[si], st))
					he(hipErrorLaunchFailure);
			} else if (hb->stride == row) {
				he(hipMemcpyAsync(D.slab[si], s.frames, m * row, hipMemcpyHostToDevice, st));
			} else { /* H2D of each slot's header row (2D DMA) */
				he(hipMemcpy2DAsync(D.slab[si], row, s.frames, hb->stride, row, m,
				                    hipMemcpyHostToDevice, st));
			}
			gcl_batch db = {};
			db.frames = D.slab[si];
			db.frames_len = m * row;
			db.stride = row;
			db.n = m;
			uint8_t *side = D.side[si];
			if (s.olflags) {
				he(hipMemcpyAsync(side, s.olflags, m, hipMemcpyHostToDevice, st));
				db.olflags = side;
			}
			if (s.rss) {
				he(hipMemcpyAsync(side + B, s.rss, m * 4, hipMemcpyHostToDevice, st));
				db.rss = (const uint32_t *)(side + B);
			}
			if (s.fdir_hi) {
				he(hipMemcpyAsync(side + 5 * B, s.fdir_hi, m * 4, hipMemcpyHostToDevice, st));
				db.fdir_hi = (const uint32_t *)(side + 5 * B);
			}
			if (s.dst_hint) {
				he(hipMemcpyAsync(side + 9 * B, s.dst_hint, m * 4, hipMemcpyHostToDevice, st));
				db.dst_hint = (const uint32_t *)(side + 9 * B);
			}
			ret = gcl_classify(D.ctx, &db, D.verd[si], D.acc, D.acc + g->R, st);
			he(hipMemcpyAsync((uint8_t *)host_verdicts + b * B * g->vsize, D.verd[si],
			                  m * g->vsize, hipMemcpyDeviceToHost, st));
		}
	}
	const int sr = gcl_group_sync(g);
	if (ret)
		return ret;
	return he.bad() ? -EIO : sr;
}

extern "C" int gcl_group_rccl_ranks(const struct gcl_group *g, int *ranks)
{
	if (!g || !ranks)
		return -EINVAL;
	*ranks = 0;
	if (g->xchg != GCL_XCHG_RCCL)
		return 0;
	if (broken(g))
		return -EIO;
	for (int i = 0; i < g->n; i++) {
		int c = 0;
		if (!g->d[i].comm || ncclCommCount(g->d[i].comm, &c) != ncclSuccess || (i && c != *ranks))
			return -EIO;
		*ranks = c;
	}
	return 0;
}

extern "C" int gcl_group_test_fault(struct gcl_group *g, uint32_t what)
{
	if (!g || (what & ~(uint32_t)GCL_GROUP_FAULT_EXCHANGE))
		return -EINVAL;
	g->fault = what;
	return 0;
}

extern "C" int gcl_group_exchange(struct gcl_group *g)
{
	if (!g)
		return -EINVAL;
	if (broken(g))
		return -EIO;
	const int b = (int)(g->seq % kSlots);
	const size_t L = g->L, L8 = L * 8;
	HipErr he;
	for (int i = 0; i < g->n; i++) {
		gcl_group::Dev &D = g->d[i];
		he(hipSetDevice(D.dev));
		hipStream_t c = D.st[0];
		/* the snapshot follows every launch enqueued so far, on every
		 * work stream of this GPU */
		for (int s = 1; s < g->nst; s++) {
			he(hipEventRecord(D.st_ev[s], D.st[s]));
			he(hipStreamWaitEvent(c, D.st_ev[s], 0));
		}
		if (D.pending[b]) /* slot b's previous exchange must be done with it */
			he(hipStreamWaitEvent(c, D.done_ev[b], 0));
		he(hipMemcpyAsync(D.snap + b * L, D.acc, L8, hipMemcpyDeviceToDevice, c));
		he(hipEventRecord(D.snap_ev[b], c));
		he(hipStreamWaitEvent(D.xs, D.snap_ev[b], 0));
	}
	if (he.bad())
		return -EIO;
	if (g->xchg == GCL_XCHG_RCCL) {
		bool ok = ncclGroupStart() == ncclSuccess;
		for (int i = 0; i < g->n && ok; i++) {
			gcl_group::Dev &D = g->d[i];
			const ncclResult_t r = ncclAllGather(D.snap + b * L, D.gath + b * L * g->n, L,
			                                     ncclUint64, D.comm, D.xs);
			ok = r == ncclSuccess || r == ncclInProgress;
		}
		const ncclResult_t e = ncclGroupEnd();
		ok = ok && (e == ncclSuccess || e == ncclInProgress);
		/* non-blocking communicators: the enqueue itself may still be in
		 * progress (the first all-gather connects the ring) */
		int w = !ok ? -EIO : e == ncclInProgress ? comms_wait(g, mono_ms() + g->timeout_ms) : 0;
		if (!w && (g->fault & GCL_GROUP_FAULT_EXCHANGE))
			w = -ETIMEDOUT; /* injected: as a timed-out enqueue */
		if (w) {
			/* the all-gather may still be enqueued on D.xs, reading and
			 * writing slot b: abort the communicators and refuse all
			 * further work rather than reuse the slot or the communicators */
			fail_group(g);
			return w;
		}
		for (int i = 0; i < g->n; i++) {
			gcl_group::Dev &D = g->d[i];
			he(hipSetDevice(D.dev));
			hipLaunchKernelGGL(sum_rows_kernel, dim3((unsigned)((L + 255) / 256)), dim3(256), 0, D.xs,
			                   (const unsigned long long *)(D.gath + b * L * g->n), g->n, (int)L,
			                   (unsigned long long *)(D.node + b * L));
			he(hipGetLastError());
			if (i == 0) {
				he(hipMemcpyAsync(g->host_node + b * L, D.node + b * L, L8, hipMemcpyDeviceToHost, D.xs));
				he(hipMemcpyAsync(g->host_gath + b * L * g->n, D.gath + b * L * g->n, L8 * g->n,
				                  hipMemcpyDeviceToHost, D.xs));
			}
		}
	} else {
		for (int i = 0; i < g->n; i++) {
			gcl_group::Dev &D = g->d[i];
			he(hipSetDevice(D.dev));
			he(hipMemcpyAsync(g->host_gath + (b * g->n + i) * L, D.snap + b * L, L8,
			                  hipMemcpyDeviceToHost, D.xs));
		}
	}
	for (int i = 0; i < g->n; i++) {
		gcl_group::Dev &D = g->d[i];
		he(hipSetDevice(D.dev));
		he(hipEventRecord(D.done_ev[b], D.xs));
		D.pending[b] = true;
	}
	g->last = b;
	g->seq++;
	return he.bad() ? -EIO : 0;
}

extern "C" int gcl_group_read(struct gcl_group *g, uint64_t *node_counts, uint64_t *node_stats,
                              uint64_t *per_gpu)
{
	if (!g)
		return -EINVAL;
	if (broken(g))
		return -EIO;
	if (g->last < 0)
		return -ENODATA;
	const int b = g->last;
	const size_t L = g->L;
	for (int i = 0; i < g->n; i++) {
		gcl_group::Dev &D = g->d[i];
		if (hipSetDevice(D.dev) != hipSuccess || hipEventSynchronize(D.done_ev[b]) != hipSuccess)
			return -EIO;
	}
	const uint64_t *rows = g->host_gath + b * L * g->n;
	for (size_t k = 0; k < L; k++) {
		uint64_t v;
		if (g->xchg == GCL_XCHG_RCCL) {
			v = g->host_node[b * L + k];
		} else {
			v = 0;
			for (int i = 0; i < g->n; i++)
				v += rows[i * L + k];
		}
		if (k < g->R) {
			if (node_counts)
				node_counts[k] = v;
		} else if (node_stats) {
			node_stats[k - g->R] = v;
		}
	}
	if (per_gpu)
		memcpy(per_gpu, rows, L * 8 * g->n);
	return 0;
}

extern "C" int gcl_group_sync(struct gcl_group *g)
{
	if (!g)
		return -EINVAL;
	/* a failed group's streams are still drained (close relies on it), but
	 * the call reports the failure like every other one */
	int ret = broken(g) ? -EIO : 0;
	for (int i = 0; i < g->n; i++) {
		gcl_group::Dev &D = g->d[i];
		if (D.dev < 0 || hipSetDevice(D.dev) != hipSuccess)
			continue;
		for (int s = 0; s < g->nst; s++)
			if (D.st[s] && hipStreamSynchronize(D.st[s]) != hipSuccess)
				ret = -EIO;
		if (D.xs && hipStreamSynchronize(D.xs) != hipSuccess)
			ret = -EIO;
	}
	return ret;
}

extern "C" int gcl_group_reset(struct gcl_group *g)
{
	if (!g)
		return -EINVAL;
	if (broken(g))
		return -EIO; /* the accumulators may still feed an aborted all-gather */
	int ret = gcl_group_sync(g);
	for (int i = 0; i < g->n && !ret; i++) {
		gcl_group::Dev &D = g->d[i];
		if (hipSetDevice(D.dev) != hipSuccess || zero_acc(D, (size_t)g->L * 8) != hipSuccess)
			ret = -EIO;
	}
	return ret;
}
