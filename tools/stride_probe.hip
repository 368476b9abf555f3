// stride_probe.hip - what does one 64-B header per 1536-B slot cost, by
// allocation kind and load cache policy?
//
// tcp1500 (config 3) reads the first 64 B of every 1536-B slot.  On ordinary
// (coarse-grained, cached) device memory every such read fetches a whole
// 128-B L2 line and the line rate, not the byte rate, bounds the kernel
// (profiles/archive/r01_halfline.jsonl, r01_membench.jsonl).  An uncached or
// fine-grained allocation changes the memory type the L2 applies, and a
// system-scope load changes how the L2 treats the request; if either lets the
// fabric move 64 B instead of 128 B per slot, the layout's ceiling moves.
// This times a pure read of 64 B per slot over 8 Mi slots (12 GiB) for every
// combination, plus the dense 2 GiB stream as a yardstick.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/stride_probe tools/stride_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

enum { LD_PLAIN, LD_NT, LD_SYS, LD_SYS_NT };

template <int LD>
__device__ __forceinline__ u32x4 ld16(const unsigned char *p)
{
	if constexpr (LD == LD_NT)
		return __builtin_nontemporal_load((const u32x4 *)p);
	else
		return *(const u32x4 *)p;
}

// four independent loads; the system-scope forms go through inline asm, which
// the compiler's wait-count pass cannot see, so they end in their own vmcnt(0)
template <int LD>
__device__ __forceinline__ void ld16x4(const unsigned char *p0, const unsigned char *p1,
                                       const unsigned char *p2, const unsigned char *p3, u32x4 v[4])
{
	if constexpr (LD == LD_SYS)
		asm volatile("global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
		             "global_load_dwordx4 %1, %5, off sc0 sc1\n\t"
		             "global_load_dwordx4 %2, %6, off sc0 sc1\n\t"
		             "global_load_dwordx4 %3, %7, off sc0 sc1\n\t"
		             "s_waitcnt vmcnt(0)"
		             : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
		             : "v"(p0), "v"(p1), "v"(p2), "v"(p3) : "memory");
	else if constexpr (LD == LD_SYS_NT)
		asm volatile("global_load_dwordx4 %0, %4, off sc0 sc1 nt\n\t"
		             "global_load_dwordx4 %1, %5, off sc0 sc1 nt\n\t"
		             "global_load_dwordx4 %2, %6, off sc0 sc1 nt\n\t"
		             "global_load_dwordx4 %3, %7, off sc0 sc1 nt\n\t"
		             "s_waitcnt vmcnt(0)"
		             : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
		             : "v"(p0), "v"(p1), "v"(p2), "v"(p3) : "memory");
	else {
		v[0] = ld16<LD>(p0);
		v[1] = ld16<LD>(p1);
		v[2] = ld16<LD>(p2);
		v[3] = ld16<LD>(p3);
	}
}

// 4 lanes per slot, each one 16-B chunk of the slot's first BYTES bytes
// (BYTES/16 lanes per slot); UNROLL independent slots per lane in flight.
template <int LD, int BYTES>
__global__ void __launch_bounds__(256) slot_kernel(const unsigned char *buf, unsigned long long slots,
                                                   unsigned stride, unsigned *out)
{
	constexpr int L = BYTES / 16;
	const unsigned long long n = slots * L;
	const unsigned long long G = (unsigned long long)gridDim.x * 256;
	unsigned acc = 0;
	unsigned long long c = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
	for (; c + 3 * G < n; c += 4 * G) {
		u32x4 v[4];
		const unsigned long long c1 = c + G, c2 = c + 2 * G, c3 = c + 3 * G;
		ld16x4<LD>(buf + (c / L) * stride + (c % L) * 16, buf + (c1 / L) * stride + (c1 % L) * 16,
		           buf + (c2 / L) * stride + (c2 % L) * 16, buf + (c3 / L) * stride + (c3 % L) * 16, v);
#pragma unroll
		for (int d = 0; d < 4; d++)
			acc ^= v[d].x ^ v[d].w;
	}
	for (; c < n; c += G)
		acc ^= ld16<LD_PLAIN>(buf + (c / L) * stride + (c % L) * 16).y;
	if (acc == 0x9E3779B9u)
		out[0] = acc;
}

template <int LD, int BYTES>
static void run(const char *kind, const char *ld, const unsigned char *buf, unsigned long long slots,
                unsigned stride, unsigned *out, int blocks, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	for (int w = 0; w < 3; w++)
		hipLaunchKernelGGL((slot_kernel<LD, BYTES>), dim3(blocks), dim3(256), 0, 0, buf, slots, stride, out);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		hipLaunchKernelGGL((slot_kernel<LD, BYTES>), dim3(blocks), dim3(256), 0, 0, buf, slots, stride, out);
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	const double us = ms * 1e3 / reps;
	printf("{\"alloc\": \"%s\", \"load\": \"%s\", \"stride\": %u, \"bytes_per_slot\": %d, \"slots\": %llu, "
	       "\"blocks\": %d, \"us\": %.2f, \"Gslots_per_s\": %.2f, \"useful_GBs\": %.1f}\n",
	       kind, ld, stride, BYTES, slots, blocks, us, slots / us / 1e3, slots * (double)BYTES / us / 1e3);
	fflush(stdout);
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
}

template <int BYTES>
static void all_loads(const char *kind, const unsigned char *buf, unsigned long long slots, unsigned stride,
                      unsigned *out, int blocks, int reps)
{
	run<LD_PLAIN, BYTES>(kind, "plain", buf, slots, stride, out, blocks, reps);
	run<LD_NT, BYTES>(kind, "nt", buf, slots, stride, out, blocks, reps);
	run<LD_SYS, BYTES>(kind, "sc0sc1", buf, slots, stride, out, blocks, reps);
	run<LD_SYS_NT, BYTES>(kind, "sc0sc1nt", buf, slots, stride, out, blocks, reps);
}

int main(int argc, char **argv)
{
	const int reps = argc > 1 ? atoi(argv[1]) : 20;
	const unsigned long long slots = 8ull << 20;
	const unsigned stride = 1536;
	const unsigned long long bytes = slots * stride;
	unsigned *out;
	CHECK(hipMalloc(&out, 64));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	struct { const char *name; unsigned flags; int ext; } kinds[] = {
		{"hipMalloc", 0, 0},
		{"uncached", hipDeviceMallocUncached, 1},
		{"finegrained", hipDeviceMallocFinegrained, 1},
	};
	for (auto &k : kinds) {
		unsigned char *buf = nullptr;
		if (k.ext)
			CHECK(hipExtMallocWithFlags((void **)&buf, bytes, k.flags));
		else
			CHECK(hipMalloc(&buf, bytes));
		CHECK(hipMemset(buf, 1, bytes));
		CHECK(hipDeviceSynchronize());
		for (int g : {cus * 4, cus * 8}) {
			all_loads<64>(k.name, buf, slots, stride, out, g, reps);
			// the same bytes as a dense stream: 2 GiB read as 128-B "slots"
			if (g == cus * 8)
				all_loads<128>(k.name, buf, (2ull << 30) / 128, 128, out, g, reps);
		}
		CHECK(hipFree(buf));
	}
	CHECK(hipFree(out));
	return 0;
}
