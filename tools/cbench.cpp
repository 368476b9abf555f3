// cbench.cpp - drive libgclassify.so through its C ABI alone (no Python, no
// torch) and A/B kernel configurations inside one process.
//
//   cbench <workload> <steps> [cfg ...]
// (env CBENCH_N, CBENCH_STRIDE, CBENCH_R override the workload's shape)
//
// Each cfg is "ABLATE:GRID:DEPTH:THREADS:BPC:SCHED:V4[:NT]" (NT = GCL_TUNE_NT_STORE;
// a ninth field, the removed GCL_TUNE_DEFER knob, is refused) (GCL_TUNE_* knobs, 0 = default;
// V4=1 classifies into 4-byte verdicts, GCL_CFG_VERDICT4; V4=2 into 2-byte queue
// verdicts, GCL_CFG_VERDICT2).
// CBENCH_NOISE_US=X co-runs, on a second stream, 32 one-wave blocks that each
// spin for X us at the start of every classify launch (stand-in for an RCCL
// kernel sharing the chip).  Rounds
// interleave the configs (plus "ref", a compute-free kernel with the same
// tile/LDS/traffic shape) so box-to-box and drift effects cancel; the median
// kernel time per config is printed as JSON.
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/cbench tools/cbench.cpp \
//          -Lcaladan_amd -lgclassify -Wl,-rpath,'$ORIGIN/../caladan_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "gclassify.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// same traffic and tile structure as classify_kernel, no classification
__global__ void __launch_bounds__(256) ref_kernel(const unsigned char *buf, unsigned long long npkt,
                                                  unsigned long long stride, unsigned long long *out)
{
	__shared__ u32x4 tile[1024];
	const unsigned long long ntiles = npkt / 256;
	unsigned long long t = blockIdx.x;
	u32x4 r[4];
	auto ld = [&](unsigned long long tt) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			int c = j * 256 + threadIdx.x;
			r[j] = __builtin_nontemporal_load(
			    (const u32x4 *)(buf + (tt * 256 + (c >> 2)) * stride + (c & 3) * 16));
		}
	};
	if (t < ntiles)
		ld(t);
	while (t < ntiles) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			int c = j * 256 + threadIdx.x;
			int p = c >> 2, q = c & 3;
			tile[p * 4 + (q ^ ((p >> 2) & 3))] = r[j];
		}
		__syncthreads();
		if (t + gridDim.x < ntiles)
			ld(t + gridDim.x);
		int p = threadIdx.x;
		u32x4 a = tile[p * 4 + ((p >> 2) & 3)], b = tile[p * 4 + (1 ^ ((p >> 2) & 3))];
		out[t * 256 + p] = ((unsigned long long)(a.w ^ b.y) << 32) | (b.z ^ a.x);
		__syncthreads();
		t += gridDim.x;
	}
}

// bounded spinner: every wave leaves after @us microseconds (100 MHz clock)
__global__ void noise_kernel(unsigned us, unsigned long long *sink)
{
	const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
	unsigned long long x = threadIdx.x;
	while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us)
		x = x * 6364136223846793005ull + 1;
	if (x == 42)
		sink[0] = x;
}

struct Cfg {
	std::string name;
	int ablate, grid, depth, threads, bpc, sched, v4, nt, defer; /* defer: must stay -1 */
	bool ref;
	std::vector<double> us, wall;
};

int main(int argc, char **argv)
{
	const int wl = argc > 1 ? atoi(argv[1]) : GCL_WL_UDP64;
	const int steps = argc > 2 ? atoi(argv[2]) : 20;
	/* CBENCH_N / CBENCH_STRIDE / CBENCH_R override the workload's packets per
	 * launch, slot stride (64 with the tcp1500 stream = the header-split
	 * layout) and runtime count */
	auto env_u64 = [](const char *k, uint64_t d) { const char *e = getenv(k); return e ? strtoull(e, nullptr, 0) : d; };
	const uint64_t n = env_u64("CBENCH_N", wl == GCL_WL_UDP64 ? (32ull << 20) : (8ull << 20));
	const uint64_t stride = env_u64("CBENCH_STRIDE", wl == GCL_WL_UDP64 ? 64 : 1536);
	const uint32_t R = (uint32_t)env_u64("CBENCH_R", wl == GCL_WL_UDP64 ? 16 : 1024);
	const uint32_t T = wl == GCL_WL_UDP64 ? 8 : 4;
	if (!n || n > (64ull << 20) || stride < 64 || stride % 16 || n * stride > (48ull << 30) || !R || R > 4096) {
		fprintf(stderr, "bad CBENCH_N/STRIDE/R\n");
		return 1;
	}
	std::vector<Cfg> cfgs;
	cfgs.push_back({"ref", 0, 0, 0, 0, 0, 0, 0, 0, -1, true, {}, {}});
	for (int i = 3; i < argc; i++) {
		Cfg c = {argv[i], 0, 0, 0, 0, 0, 0, 0, 0, -1, false, {}, {}};
		sscanf(argv[i], "%d:%d:%d:%d:%d:%d:%d:%d:%d", &c.ablate, &c.grid, &c.depth, &c.threads, &c.bpc,
		       &c.sched, &c.v4, &c.nt, &c.defer);
		if (c.defer != -1) {
			fprintf(stderr, "cfg %s: GCL_TUNE_DEFER was removed from the library\n", argv[i]);
			return 1;
		}
		cfgs.push_back(c);
	}
	if (cfgs.size() == 1)
		cfgs.push_back({"default", 0, 0, 0, 0, 0, 0, 0, 0, -1, false, {}, {}});
	const char *pe = getenv("CBENCH_PROFILE");
	const bool profile = !pe || atoi(pe) != 0; /* 0: no per-launch events, wall time only */
	const char *ne = getenv("CBENCH_NOISE_US");
	const unsigned noise_us = ne ? (unsigned)atoi(ne) : 0;
	if (noise_us > 1000) {
		fprintf(stderr, "CBENCH_NOISE_US too large\n");
		return 1;
	}
	hipStream_t s1, s2;
	CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
	CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
	hipEvent_t start_ev;
	CHECK(hipEventCreateWithFlags(&start_ev, hipEventDisableTiming));

	uint8_t *frames;
	struct gcl_verdict *v;
	uint64_t *acc, *zipf = nullptr;
	CHECK(hipMalloc(&v, n * sizeof(*v)));
	if (getenv("CBENCH_PAIRED")) { /* frame pool placed against the verdict ring */
		struct gcl_pair_info pi;
		if (gcl_dev_alloc_paired(0, n * stride, v, n * 4, GCL_PAIR_NEW_READS, (void **)&frames, &pi)) {
			fprintf(stderr, "gcl_dev_alloc_paired failed\n");
			return 1;
		}
		fprintf(stderr, "paired: probe %.2f us (worst %.2f, %u candidates, %u classes)\n",
		        pi.chosen_us, pi.worst_us, pi.candidates, pi.classes);
	} else {
		CHECK(hipMalloc(&frames, n * stride));
	}
	CHECK(hipMalloc(&acc, (R + GCL_NR_STATS) * 8));
	CHECK(hipMemset(frames, 0, n * stride));
	CHECK(hipMemset(acc, 0, (R + GCL_NR_STATS) * 8));
	struct gcl_gen_params gp = {};
	gp.workload = wl;
	gp.nruntimes = R;
	gp.seed = 0xCA1ADA4;
	gp.n = n;
	gp.stride = stride;
	gp.world = 1;
	if (wl == GCL_WL_TCP1500_ZIPF) {
		const uint32_t nf = 1 << 20;
		uint64_t *h = (uint64_t *)malloc(nf * 8);
		gcl_zipf_cdf(nf, 0.99, h);
		CHECK(hipMalloc(&zipf, nf * 8));
		CHECK(hipMemcpy(zipf, h, nf * 8, hipMemcpyHostToDevice));
		free(h);
		gp.zipf_cdf = zipf;
		gp.nflows = nf;
	}
	if (gcl_generate(&gp, frames, nullptr, nullptr, nullptr)) {
		fprintf(stderr, "gcl_generate failed\n");
		return 1;
	}
	struct gcl_batch b = {};
	b.frames = frames;
	b.frames_len = n * stride;
	b.stride = stride;
	b.n = n;
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

	for (int round = 0; round < 7; round++) {
		for (Cfg &c : cfgs) {
			if (c.ref) {
				hipLaunchKernelGGL(ref_kernel, dim3(cus * 8), dim3(256), 0, 0, frames, n, stride,
				                   (unsigned long long *)v);
				CHECK(hipEventRecord(e0, nullptr));
				for (int i = 0; i < steps; i++)
					hipLaunchKernelGGL(ref_kernel, dim3(cus * 8), dim3(256), 0, 0, frames, n,
					                   stride, (unsigned long long *)v);
				CHECK(hipEventRecord(e1, nullptr));
				CHECK(hipEventSynchronize(e1));
				float ms = 0;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				c.us.push_back(ms * 1e3 / steps);
				c.wall.push_back(ms * 1e3 / steps);
				continue;
			}
			char buf[32];
			snprintf(buf, sizeof(buf), "%d", c.ablate);
			setenv("GCL_TUNE_ABLATE", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.grid);
			setenv("GCL_TUNE_GRID", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.depth);
			setenv("GCL_TUNE_DEPTH", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.threads);
			setenv("GCL_TUNE_THREADS", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.bpc);
			setenv("GCL_TUNE_BLOCKS_PER_CU", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.sched);
			setenv("GCL_TUNE_SCHED", buf, 1);
			snprintf(buf, sizeof(buf), "%d", c.nt);
			setenv("GCL_TUNE_NT_STORE", buf, 1);
			struct gcl_cfg cfg = {};
			cfg.max_runtimes = R;
			cfg.hash_mode = GCL_HASH_JENKINS;
			cfg.flags = (profile ? GCL_CFG_PROFILE : 0) |
			            (c.v4 == 2 ? GCL_CFG_VERDICT2 : c.v4 ? GCL_CFG_VERDICT4 : 0);
			cfg.thread_bits = (uint8_t)(T <= 4 ? 2 : 3);
			cfg.default_olflags = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
			struct gcl_ctx *ctx;
			if (gcl_open(0, &cfg, &ctx)) {
				fprintf(stderr, "gcl_open failed\n");
				return 1;
			}
			uint16_t act[GCL_NCPU], flow[GCL_NCPU];
			for (uint32_t r = 0; r < R; r++) {
				uint16_t na = (uint16_t)(r % T + 1);
				for (uint16_t i = 0; i < na; i++)
					act[i] = i;
				gcl_steer_flows((uint16_t)T, act, na, flow);
				gcl_runtime_set(ctx, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow);
			}
			gcl_classify(ctx, &b, v, acc, acc + R, s1);
			CHECK(hipDeviceSynchronize());
			double ms;
			uint64_t launches;
			gcl_kernel_time(ctx, &ms, &launches, 1);
			CHECK(hipEventRecord(e0, s1));
			for (int i = 0; i < steps; i++) {
				if (noise_us) {
					CHECK(hipEventRecord(start_ev, s1));
					CHECK(hipStreamWaitEvent(s2, start_ev, 0));
					hipLaunchKernelGGL(noise_kernel, dim3(32), dim3(64), 0, s2, noise_us,
					                   (unsigned long long *)acc);
				}
				gcl_classify(ctx, &b, v, acc, acc + R, s1);
			}
			CHECK(hipEventRecord(e1, s1));
			CHECK(hipDeviceSynchronize());
			float wms = 0;
			CHECK(hipEventElapsedTime(&wms, e0, e1));
			c.wall.push_back(wms * 1e3 / steps);
			gcl_kernel_time(ctx, &ms, &launches, 1);
			c.us.push_back(launches ? ms / launches * 1e3 : wms * 1e3 / steps);
			gcl_close(ctx);
		}
	}
	double ref = 0;
	for (Cfg &c : cfgs) {
		std::sort(c.us.begin(), c.us.end());
		std::sort(c.wall.begin(), c.wall.end());
		double med = c.us[c.us.size() / 2], wmed = c.wall[c.wall.size() / 2];
		if (c.ref)
			ref = med;
		printf("{\"workload\": %d, \"n\": %llu, \"stride\": %llu, \"R\": %u, \"cfg\": \"%s\", "
		       "\"profile\": %d, \"median_us\": %.2f, "
		       "\"min_us\": %.2f, \"max_us\": %.2f, \"wall_us_per_step\": %.2f, \"Mpkts\": %.1f, "
		       "\"ref_over_this\": %.4f}\n",
		       wl, (unsigned long long)n, (unsigned long long)stride, R, c.name.c_str(), (int)profile,
		       med, c.us.front(), c.us.back(), wmed, n / (med * 1e-6) / 1e6, ref / med);
	}
	return 0;
}
