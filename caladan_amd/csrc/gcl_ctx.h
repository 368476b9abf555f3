/*
 * gcl_ctx.h - the classifier context (struct gcl_ctx, opaque in the C ABI)
 * and the host-side helpers the library's translation units share: the table
 * image and its snapshot upload (gcl_ctx.hip), the mapped views of host
 * memory (gcl_xfer.hip).  Not installed; include/gclassify.h is the ABI.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <vector>

#include "../../include/gclassify.h"
#include "gcl_kern.h"

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
		hipStream_t st[gclk::kImgUsers];
		hipEvent_t ev[gclk::kImgUsers];
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
	/* overrides of the measured defaults for tests and A/Bs (gcl_ctx_tune;
	 * GCL_TUNE_AUTO everywhere in production) */
	struct gcl_tune tune;
};

namespace gclk {

constexpr uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

/* gcl_ctx.hip */
uint32_t build_image(gcl_ctx *c);           /* host mirror -> c->staging; image bytes, 0: -ENOSPC */
hipEvent_t prof_event(gcl_ctx *c);          /* a timing event from the context's pool */
int image_used(gcl_ctx *c, hipStream_t s);  /* a launch on @s reads the current image */
uint32_t verdict_bytes(const gcl_ctx *c);
uint32_t kernel_cflags(const gcl_ctx *c);   /* cfg.flags with thread_bits in [31:24] */
int upload_tables(gcl_ctx *c, hipStream_t s);
int wait_tables(gcl_ctx *c, hipStream_t s);
/* a tune field, or @dflt where it is GCL_TUNE_AUTO */
inline int32_t tuned(int32_t v, int32_t dflt) { return v == GCL_TUNE_AUTO ? dflt : v; }

/* gcl_xfer.hip: device address of pinned / registered host memory, or NULL */
void *mapped(const void *h);

} // namespace gclk
