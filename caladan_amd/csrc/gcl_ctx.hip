/*
 * gcl_ctx.hip - the classifier context: gcl_open / gcl_close, the host mirror
 * of the reference's tables (dp.clients_by_id, dp.ip_to_proc, flow_tbl;
 * dp_clients.c:156-250, :349-363, sched.c:122-147), the table image and its
 * snapshot upload, the test/A-B overrides (gcl_ctx_tune), kernel timing and
 * the version calls.  No kernels live here.
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <utility>
#include <vector>

#include "../../include/gclassify.h"
#include "gcl_ctx.h"

#define GCL_VERSION "gclassify 0.1 (gfx950)"

using namespace gclk;

static uint32_t pow2_at_least(uint32_t x)
{
	uint32_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

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
	gcl_tune_init(&c->tune);
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
uint32_t gclk::build_image(gcl_ctx *c)
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

hipEvent_t gclk::prof_event(gcl_ctx *c)
{
	if (!c->ev_pool.empty()) {
		hipEvent_t e = c->ev_pool.back();
		c->ev_pool.pop_back();
		return e;
	}
	hipEvent_t e = nullptr;
	return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

/* Note that a launch on @s reads the current image.  With more streams than
 * kImgUsers, the new stream takes over the oldest one's slot after waiting
 * for what that stream has queued so far, so the slot still covers it. */
int gclk::image_used(gcl_ctx *c, hipStream_t s)
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

uint32_t gclk::verdict_bytes(const gcl_ctx *c)
{
	return (c->cfg.flags & GCL_CFG_VERDICT1) ? 1 : (c->cfg.flags & GCL_CFG_VERDICT2) ? 2
	     : (c->cfg.flags & GCL_CFG_VERDICT4) ? 4 : 8;
}

/* the kernels' cflags: cfg.flags with thread_bits in [31:24] */
uint32_t gclk::kernel_cflags(const gcl_ctx *c)
{
	return (c->cfg.flags & 0xFFFFFFu) | (uint32_t)c->cfg.thread_bits << 24;
}

/* Upload a new table snapshot on @s if anything changed; launches on other
 * streams wait for c->tables_ready before reading the image. */
int gclk::upload_tables(gcl_ctx *c, hipStream_t s)
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
int gclk::wait_tables(gcl_ctx *c, hipStream_t s)
{
	if (c->tables_done || s == c->tables_stream)
		return 0;
	if (hipEventQuery(c->tables_ready) == hipSuccess) {
		c->tables_done = true;
		return 0;
	}
	return hipStreamWaitEvent(s, c->tables_ready, 0) == hipSuccess ? 0 : -EIO;
}

extern "C" void gcl_tune_init(struct gcl_tune *t)
{
	if (!t)
		return;
	memset(t, 0, sizeof(*t));
	t->size = sizeof(*t);
	t->tables = t->depth = t->threads = t->grid = t->blocks_per_cu = GCL_TUNE_AUTO;
	t->defer = t->pair_lean = t->tile_lean = GCL_TUNE_AUTO;
	t->loop64 = t->loop_lean = t->loop_spec = t->loop_prefetch = GCL_TUNE_AUTO;
	t->loop_phase_max = t->loop_phase_up = t->loop_phase_down = GCL_TUNE_AUTO;
	t->rec_prefetch = t->slot_prefetch = t->vstage = t->pair_i32 = t->tile_order = GCL_TUNE_AUTO;
	t->loop_t0 = 0;
	t->debug = 0;
}

/* every field GCL_TUNE_AUTO or in its range; the loop's three phase fields
 * all AUTO or all set (max <= 1000 ticks, up > 0, down <= up) */
static bool tune_valid(const struct gcl_tune *t)
{
	auto in = [](int32_t v, int32_t lo, int32_t hi) { return v == GCL_TUNE_AUTO || (v >= lo && v <= hi); };
	auto flag = [&](int32_t v) { return in(v, 0, 1); };
	const bool ph_auto = t->loop_phase_max == GCL_TUNE_AUTO && t->loop_phase_up == GCL_TUNE_AUTO &&
	                     t->loop_phase_down == GCL_TUNE_AUTO;
	const bool ph_set = t->loop_phase_max >= 0 && t->loop_phase_max <= 1000 && t->loop_phase_up > 0 &&
	                    t->loop_phase_down >= 0 && t->loop_phase_down <= t->loop_phase_up;
	return t->size == sizeof(*t) && flag(t->tables) && in(t->depth, 1, 2) &&
	       (t->threads == GCL_TUNE_AUTO || t->threads == 256 || t->threads == 512 || t->threads == 1024) &&
	       in(t->grid, 1, 1 << 20) && in(t->blocks_per_cu, 1, 64) && in(t->defer, 0, 2) &&
	       flag(t->pair_lean) && flag(t->tile_lean) && flag(t->loop64) && flag(t->loop_lean) && in(t->loop_spec, 0, 100000000) &&
	       flag(t->loop_prefetch) && (ph_auto || ph_set) && t->debug <= 1 && in(t->rec_prefetch, 0, 64) &&
	       flag(t->slot_prefetch) && flag(t->vstage) && flag(t->pair_i32) &&
	       flag(t->tile_order);
}

extern "C" int gcl_ctx_tune(struct gcl_ctx *c, const struct gcl_tune *t)
{
	if (!c)
		return -EINVAL;
	if (!t) {
		gcl_tune_init(&c->tune);
		return 0;
	}
	if (!tune_valid(t))
		return -EINVAL;
	c->tune = *t;
	return 0;
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

extern "C" const char *gcl_version(void) { return GCL_VERSION; }

extern "C" int gcl_abi_version(void) { return GCL_ABI_VERSION; }

