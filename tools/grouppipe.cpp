// grouppipe.cpp - the multi-GPU rx step as the single dataplane thread of the
// iokernel would drive it (iokernel/dpdk.c:276-280, main.c:144-150), from C:
// one gcl_group over <ndev> GPUs (include/gcl_group.h), batches of frames in
// pinned host memory -- the ingress region -- split round-robin in 64 Ki-packet
// blocks over the GPUs (gcl_group_classify_host: PCIe zero-copy, then the
// header DMA-gather), the per-runtime counts and rx counters all-gathered
// through RCCL (gcl_group_exchange / gcl_group_read), every verdict of the last
// batch checked against a one-context classification of the same batch.
//
//   grouppipe <ndev> [pkts] [iters]   -> one JSON line
//
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/grouppipe tools/grouppipe.cpp
//         -Lcaladan_amd -lgclgroup -lgclassify -Wl,-rpath,'$ORIGIN/../caladan_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <vector>

#include "gcl_group.h"
#include "gclassify.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
#define GCHECK(x) do { int r_ = (x); if (r_) { \
	fprintf(stderr, "%s:%d %s = %d\n", __FILE__, __LINE__, #x, r_); exit(1); } } while (0)

static double now_s()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
	int visible = 0;
	CHECK(hipGetDeviceCount(&visible));
	const int ndev = argc > 1 ? atoi(argv[1]) : visible;
	const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 0) : (8ull << 20);
	const int iters = argc > 3 ? atoi(argv[3]) : 5;
	const uint32_t R = 16, T = 8, stride = 64;
	if (ndev < 1 || ndev > visible || ndev > GCL_GROUP_MAX_DEV || !n || n > (256ull << 20) || iters < 1) {
		fprintf(stderr, "bad arguments (%d GPUs visible)\n", visible);
		return 1;
	}

	/* the ingress region: udp64 frames generated on GPU 0, copied to pinned host memory */
	uint8_t *dfr, *region;
	CHECK(hipSetDevice(0));
	CHECK(hipMalloc(&dfr, n * stride));
	CHECK(hipMemset(dfr, 0, n * stride));
	struct gcl_gen_params gp = {};
	gp.workload = GCL_WL_UDP64;
	gp.nruntimes = R;
	gp.seed = 0xCA1ADA4;
	gp.n = n;
	gp.stride = stride;
	gp.world = 1;
	GCHECK(gcl_generate(&gp, dfr, nullptr, nullptr, nullptr));
	CHECK(hipHostMalloc((void **)&region, n * stride, hipHostMallocMapped | hipHostMallocPortable));
	CHECK(hipMemcpy(region, dfr, n * stride, hipMemcpyDeviceToHost));
	CHECK(hipFree(dfr));
	uint16_t *v, *v1;
	CHECK(hipHostMalloc((void **)&v, n * 2, hipHostMallocMapped | hipHostMallocPortable));
	CHECK(hipHostMalloc((void **)&v1, n * 2, hipHostMallocMapped | hipHostMallocPortable));

	struct gcl_cfg cfg = {};
	cfg.max_runtimes = R;
	cfg.hash_mode = GCL_HASH_JENKINS;
	cfg.flags = GCL_CFG_VERDICT2;
	cfg.thread_bits = 3;
	cfg.default_olflags = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	std::vector<int> devs(ndev);
	for (int i = 0; i < ndev; i++)
		devs[i] = i;
	struct gcl_group_cfg gc = GCL_GROUP_CFG_INIT;
	gc.block = GCL_GROUP_BLOCK;
	gc.exchange = GCL_XCHG_RCCL;
	gc.nstreams = 2;
	struct gcl_group *grp;
	GCHECK(gcl_group_open(ndev, devs.data(), &cfg, &gc, &grp));
	struct gcl_ctx *one; /* the check: the same batch through one context */
	GCHECK(gcl_open(0, &cfg, &one));
	for (uint32_t r = 0; r < R; r++) {
		uint16_t act[GCL_NCPU], flow[GCL_NCPU];
		const uint16_t na = (uint16_t)(r % T + 1);
		for (uint16_t i = 0; i < na; i++)
			act[i] = (uint16_t)((i * 3) % T);
		GCHECK(gcl_steer_flows((uint16_t)T, act, na, flow));
		GCHECK(gcl_group_runtime_set(grp, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow));
		GCHECK(gcl_runtime_set(one, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow));
	}

	struct gcl_batch hb = {};
	hb.frames = region;
	hb.frames_len = n * stride;
	hb.stride = stride;
	hb.n = n;
	double rate[2] = {0, 0};
	uint64_t calls = 0;
	const uint32_t modes[2] = {GCL_E2E_ZEROCOPY, GCL_E2E_COPY};
	for (int m = 0; m < 2; m++) {
		struct gcl_e2e_opts o = {};
		o.mode = modes[m];
		GCHECK(gcl_group_classify_host(grp, &hb, v, &o)); /* warm */
		calls++;
		const double t0 = now_s();
		for (int i = 0; i < iters; i++)
			GCHECK(gcl_group_classify_host(grp, &hb, v, &o));
		rate[m] = (double)n * iters / (now_s() - t0) / 1e6;
		calls += iters;
	}
	GCHECK(gcl_group_exchange(grp));
	std::vector<uint64_t> counts(R), stats(GCL_NR_STATS), per((size_t)ndev * (R + GCL_NR_STATS));
	GCHECK(gcl_group_read(grp, counts.data(), stats.data(), per.data()));

	/* the last batch's verdicts against one context over the whole batch */
	struct gcl_e2e_opts o1 = {};
	o1.mode = GCL_E2E_ZEROCOPY;
	GCHECK(gcl_classify_host(one, &hb, v1, nullptr, nullptr, &o1));
	const bool verdicts_ok = memcmp(v, v1, n * 2) == 0;
	uint64_t total = 0;
	for (uint32_t r = 0; r < R; r++)
		total += counts[r];
	bool per_ok = true;
	for (int i = 0; i < ndev; i++)
		per_ok = per_ok && per[(size_t)i * (R + GCL_NR_STATS) + R + GCL_RX_PULLED] ==
		                           gcl_shard_count(n, (uint32_t)ndev, (uint32_t)i, GCL_GROUP_BLOCK) * calls;
	const bool counts_ok = total == n * calls && stats[GCL_RX_PULLED] == n * calls && per_ok;
	printf("{\"n_gpus\": %d, \"pkts\": %llu, \"iters\": %d, \"zerocopy_mpps\": %.1f, \"copy_hdr_mpps\": %.1f, "
	       "\"exchange\": \"rccl\", \"counts_check\": \"%s\", \"verdicts_check\": \"%s\"}\n",
	       ndev, (unsigned long long)n, iters, rate[0], rate[1], counts_ok ? "ok" : "MISMATCH",
	       verdicts_ok ? "ok" : "MISMATCH");
	gcl_close(one);
	gcl_group_close(grp);
	CHECK(hipHostFree(v));
	CHECK(hipHostFree(v1));
	CHECK(hipHostFree(region));
	return counts_ok && verdicts_ok ? 0 : 2;
}
