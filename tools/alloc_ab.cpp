// alloc_ab.cpp - does the classify rate depend on how the frame buffer was
// allocated?  One process, identical bytes in each buffer, rounds interleaved:
//   A  first hipMalloc of the process
//   B  hipMalloc after a 3 GiB buffer was allocated (and stays allocated)
//   C  hipMalloc into the hole a freed 3 GiB buffer left, after many small
//      allocations were made and half of them freed (fragmented free space)
//   D  hipExtMallocWithFlags(hipDeviceMallocContiguous)
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/alloc_ab tools/alloc_ab.cpp \
//          -Lcaladan_amd -lgclassify -Wl,-rpath,'$ORIGIN/../caladan_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gclassify.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

/* read-only stream over the buffer: 16 B per lane per step, 4 in flight */
__global__ void __launch_bounds__(256) read_kernel(const u32x4 *p, unsigned long long n16,
                                                   unsigned long long *sink)
{
	unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
	const unsigned long long G = (unsigned long long)gridDim.x * 256;
	unsigned x = 0;
	for (; i + 3 * G < n16; i += 4 * G) {
		u32x4 a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + G);
		u32x4 c = __builtin_nontemporal_load(p + i + 2 * G), d = __builtin_nontemporal_load(p + i + 3 * G);
		x ^= a.x ^ b.y ^ c.z ^ d.w;
	}
	for (; i < n16; i += G)
		x ^= p[i].x;
	if (x == 0x12345678u)
		sink[0] = x;
}

int main(int argc, char **argv)
{
	const int steps = argc > 1 ? atoi(argv[1]) : 20;
	const uint64_t n = 32ull << 20, stride = 64, bytes = n * stride;
	const uint32_t R = 16, T = 8;
	std::vector<uint8_t *> bufs;
	std::vector<const char *> names;
	uint8_t *a, *b, *c, *d, *big, *big2;
	const int sweep = argc > 2 && !strcmp(argv[2], "sweep") ? (argc > 3 ? atoi(argv[3]) : 24) : 0;
	if (sweep) {
		/* @sweep plain 2 GiB buffers in allocation order */
		static char nm[64][16];
		for (int i = 0; i < sweep && i < 64; i++) {
			uint8_t *p;
			CHECK(hipMalloc(&p, bytes));
			snprintf(nm[i], sizeof(nm[i]), "seq%02d", i);
			bufs.push_back(p); names.push_back(nm[i]);
		}
	} else if (argc > 2 && !strcmp(argv[2], "cfirst")) {
		/* contiguous first, then plain, then contiguous again */
		uint8_t *p;
		CHECK(hipExtMallocWithFlags((void **)&p, bytes, hipDeviceMallocContiguous));
		bufs.push_back(p); names.push_back("contig_first");
		CHECK(hipMalloc(&p, bytes));
		bufs.push_back(p); names.push_back("plain_second");
		CHECK(hipExtMallocWithFlags((void **)&p, bytes, hipDeviceMallocContiguous));
		bufs.push_back(p); names.push_back("contig_third");
		CHECK(hipMalloc(&p, bytes));
		bufs.push_back(p); names.push_back("plain_fourth");
	} else {
	CHECK(hipMalloc(&a, bytes));
	bufs.push_back(a); names.push_back("A_first");
	CHECK(hipMalloc(&big, 3ull << 30));
	CHECK(hipMalloc(&b, bytes));
	bufs.push_back(b); names.push_back("B_after_3GiB");
	/* fragment: many 6 MiB allocations, free every other one, then free a 3 GiB */
	std::vector<uint8_t *> small;
	for (int i = 0; i < 512; i++) {
		uint8_t *p;
		CHECK(hipMalloc(&p, 6ull << 20));
		small.push_back(p);
	}
	for (size_t i = 0; i < small.size(); i += 2)
		CHECK(hipFree(small[i]));
	CHECK(hipMalloc(&big2, 1ull << 30));
	CHECK(hipFree(big));
	CHECK(hipMalloc(&c, bytes));
	bufs.push_back(c); names.push_back("C_fragmented");
	if (hipExtMallocWithFlags((void **)&d, bytes, hipDeviceMallocContiguous) == hipSuccess) {
		bufs.push_back(d); names.push_back("D_contiguous");
	} else {
		fprintf(stderr, "contiguous alloc failed\n");
		(void)hipGetLastError();
	}
	}
	struct gcl_gen_params gp = {};
	gp.workload = GCL_WL_UDP64;
	gp.nruntimes = R;
	gp.seed = 0xCA1ADA4;
	gp.n = n;
	gp.stride = stride;
	gp.world = 1;
	for (uint8_t *p : bufs)
		if (gcl_generate(&gp, p, nullptr, nullptr, nullptr))
			return 1;
	uint32_t *v, *v2;
	uint64_t *acc;
	CHECK(hipMalloc(&v, n * 4));
	{
		uint8_t *gap;
		CHECK(hipMalloc(&gap, 1ull << 30)); /* place v2 1 GiB away from v */
		CHECK(hipMalloc(&v2, n * 4));
	}
	CHECK(hipMalloc(&acc, (R + GCL_NR_STATS) * 8));
	struct gcl_cfg cfg = {};
	cfg.max_runtimes = R;
	cfg.hash_mode = GCL_HASH_JENKINS;
	cfg.flags = GCL_CFG_VERDICT4;
	cfg.default_olflags = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	/* ctx: round-robin tiles over XCDs; ctx2: a contiguous eighth per XCD */
	struct gcl_ctx *ctx, *ctx2;
	setenv("GCL_TUNE_XCD_MAP", "0", 1);
	if (gcl_open(0, &cfg, &ctx))
		return 1;
	setenv("GCL_TUNE_XCD_MAP", "1", 1);
	if (gcl_open(0, &cfg, &ctx2))
		return 1;
	uint16_t act[GCL_NCPU], flow[GCL_NCPU];
	for (uint32_t r = 0; r < R; r++) {
		uint16_t na = (uint16_t)(r % T + 1);
		for (uint16_t i = 0; i < na; i++)
			act[i] = i;
		gcl_steer_flows((uint16_t)T, act, na, flow);
		gcl_runtime_set(ctx, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow);
		gcl_runtime_set(ctx2, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow);
	}
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	std::vector<std::vector<double>> us(bufs.size()), us2(bufs.size()), rd(bufs.size());
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	const int rounds = sweep ? 3 : 7;
	for (int round = 0; round < rounds; round++) {
		for (size_t i = 0; i < bufs.size(); i++) {
			struct gcl_batch bt = {};
			bt.frames = bufs[i];
			bt.frames_len = bytes;
			bt.stride = stride;
			bt.n = n;
			gcl_classify(ctx, &bt, v, acc, acc + R, nullptr);
			CHECK(hipEventRecord(e0, nullptr));
			for (int s = 0; s < steps; s++)
				gcl_classify(ctx, &bt, v, acc, acc + R, nullptr);
			CHECK(hipEventRecord(e1, nullptr));
			CHECK(hipEventSynchronize(e1));
			float ms;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			us[i].push_back(ms * 1e3 / steps);
			/* same frames, per-XCD contiguous tile walk */
			gcl_classify(ctx2, &bt, v2, acc, acc + R, nullptr);
			CHECK(hipEventRecord(e0, nullptr));
			for (int s2 = 0; s2 < steps; s2++)
				gcl_classify(ctx2, &bt, v2, acc, acc + R, nullptr);
			CHECK(hipEventRecord(e1, nullptr));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			us2[i].push_back(ms * 1e3 / steps);
			/* read-only stream */
			CHECK(hipEventRecord(e0, nullptr));
			for (int s2 = 0; s2 < steps; s2++)
				hipLaunchKernelGGL(read_kernel, dim3(cus * 8), dim3(256), 0, nullptr,
				                   (const u32x4 *)bufs[i], (unsigned long long)(bytes / 16),
				                   (unsigned long long *)acc);
			CHECK(hipEventRecord(e1, nullptr));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			rd[i].push_back(ms * 1e3 / steps);
		}
	}
	for (size_t i = 0; i < bufs.size(); i++) {
		std::sort(us[i].begin(), us[i].end());
		std::sort(us2[i].begin(), us2[i].end());
		std::sort(rd[i].begin(), rd[i].end());
		printf("{\"buffer\": \"%s\", \"va\": \"%p\", \"median_us\": %.2f, \"min_us\": %.2f, \"max_us\": %.2f, "
		       "\"median_us_xcdmap\": %.2f, \"read_only_us\": %.2f, \"read_TBs\": %.2f}\n",
		       names[i], (void *)bufs[i], us[i][us[i].size() / 2], us[i].front(), us[i].back(),
		       us2[i][us2[i].size() / 2], rd[i][rd[i].size() / 2], bytes / (rd[i][rd[i].size() / 2] * 1e-6) / 1e12);
	}
	gcl_close(ctx);
	gcl_close(ctx2);
	return 0;
}
