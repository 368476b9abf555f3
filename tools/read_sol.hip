// read_sol.hip - the HBM read speed of light on this box, for the udp64
// slab's size (32 Mi x 64 B = 2 GiB): pure streaming reads in
// the common shapes (grid-stride or one contiguous chunk per block; 2-8
// 16-B loads per lane in flight; plain or non-temporal; 1-8 blocks of 256-1024
// lanes per CU), each timed with HIP events over REPS launches after a
// warm-up.  Every loaded dword feeds an xor whose result is stored only if it
// equals a value no slab of zeros produces, so nothing is written and the
// loads cannot be dropped.  One JSON line per shape, then the best.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/read_sol tools/read_sol.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p)
{
	if constexpr (NT)
		return __builtin_nontemporal_load(p);
	else
		return *p;
}

/* grid-stride: iteration i of lane g reads chunks (i * U + u) * G + g */
template <int U, bool NT>
__global__ void stride_kernel(const u32x4 *src, unsigned long long nchunks, unsigned *sink)
{
	const unsigned long long G = (unsigned long long)gridDim.x * blockDim.x;
	const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
	unsigned acc = 0;
	for (unsigned long long base = 0; base + (unsigned long long)U * G <= nchunks; base += (unsigned long long)U * G) {
		u32x4 r[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			r[u] = ld16<NT>(src + base + u * G + g);
#pragma unroll
		for (int u = 0; u < U; u++)
			acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[g] = acc;
}

/* one contiguous chunk per block, the block's lanes side by side */
template <int U, bool NT>
__global__ void block_kernel(const u32x4 *src, unsigned long long nchunks, unsigned *sink)
{
	const unsigned long long per = nchunks / gridDim.x;
	const u32x4 *p = src + per * blockIdx.x;
	const unsigned T = blockDim.x;
	unsigned acc = 0;
	for (unsigned long long base = 0; base + (unsigned long long)U * T <= per; base += (unsigned long long)U * T) {
		u32x4 r[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			r[u] = ld16<NT>(p + base + u * T + threadIdx.x);
#pragma unroll
		for (int u = 0; u < U; u++)
			acc ^= r[u].x ^ r[u].y ^ r[u].z ^ r[u].w;
	}
	if (acc == 0x9E3779B9u)
		sink[(unsigned long long)blockIdx.x * T + threadIdx.x] = acc;
}

typedef void (*kfn)(const u32x4 *, unsigned long long, unsigned *);

struct Shape {
	const char *name;
	int unroll;
	bool nt;
	kfn fn;
};

int main(int argc, char **argv)
{
	const unsigned long long bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (2ull << 30);
	const int reps = argc > 2 ? atoi(argv[2]) : 20;
	const unsigned long long nchunks = bytes / 16;
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	u32x4 *src;
	unsigned *sink;
	CHECK(hipMalloc(&src, bytes));
	CHECK(hipMemset(src, 0, bytes));
	CHECK(hipMalloc(&sink, 64ull << 20));
	const Shape shapes[] = {
		{"stride", 2, false, stride_kernel<2, false>}, {"stride", 4, false, stride_kernel<4, false>},
		{"stride", 8, false, stride_kernel<8, false>}, {"stride", 4, true, stride_kernel<4, true>},
		{"stride", 8, true, stride_kernel<8, true>},   {"block", 4, false, block_kernel<4, false>},
		{"block", 8, false, block_kernel<8, false>},   {"block", 4, true, block_kernel<4, true>},
		{"block", 8, true, block_kernel<8, true>},
	};
	const int threads[] = {256, 512, 1024};
	const int per_cu[] = {1, 2, 4, 8};
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	double best = 0;
	char best_desc[160] = "";
	for (const Shape &s : shapes)
		for (int nt : threads)
			for (int k : per_cu) {
				if ((long)nt * k > 2048) /* at most 32 waves per CU */
					continue;
				const unsigned grid = (unsigned)(cus * k);
				/* the bytes a launch reads: whole iterations only */
				const unsigned long long step = (unsigned long long)s.unroll * grid * nt;
				const unsigned long long per_blk = nchunks / grid;
				const unsigned long long read =
				        (s.name[0] == 's' ? nchunks / step * step
				                          : per_blk / ((unsigned long long)s.unroll * nt) * s.unroll * nt * grid) * 16;
				for (int w = 0; w < 3; w++)
					hipLaunchKernelGGL(s.fn, dim3(grid), dim3(nt), 0, 0, src, nchunks, sink);
				CHECK(hipGetLastError());
				CHECK(hipEventRecord(e0, 0));
				for (int r = 0; r < reps; r++)
					hipLaunchKernelGGL(s.fn, dim3(grid), dim3(nt), 0, 0, src, nchunks, sink);
				CHECK(hipEventRecord(e1, 0));
				CHECK(hipEventSynchronize(e1));
				float ms = 0;
				CHECK(hipEventElapsedTime(&ms, e0, e1));
				const double us = ms * 1e3 / reps, gbs = read / (us * 1e3);
				printf("{\"shape\": \"%s\", \"unroll\": %d, \"nt\": %d, \"threads\": %d, \"blocks_per_cu\": %d, "
				       "\"bytes\": %llu, \"us\": %.1f, \"GBs\": %.1f}\n",
				       s.name, s.unroll, (int)s.nt, nt, k, read, us, gbs);
				fflush(stdout);
				if (gbs > best) {
					best = gbs;
					snprintf(best_desc, sizeof best_desc, "%s unroll %d nt %d, %d x %d per CU", s.name,
					         s.unroll, (int)s.nt, k, nt);
				}
			}
	printf("{\"best_GBs\": %.1f, \"best\": \"%s\", \"cus\": %d}\n", best, best_desc, cus);
	CHECK(hipFree(src));
	CHECK(hipFree(sink));
	return 0;
}
