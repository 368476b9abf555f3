// wmix.hip - what the verdict stores cost beside the header read stream (gfx950).
//
// The classify kernel reads one 64-B header granule per packet and writes one
// 4-B verdict.  membench's rw_* patterns showed that the small write stream
// costs far more than its bytes (udp64: +~70 us for 128 MiB; tcp1500: +~40 us
// for 32 MiB).  This tool times the same tile loop (256 packets per block
// iteration, 4 x 16-B nt loads per lane, persistent grid) with the write
// stream in different shapes, to find the one the memory system absorbs:
//   none      : no verdict stores (one word per block at the end)
//   st4       : global_store_dword per packet, default policy
//   st4_nt    : the same, non-temporal
//   st4_sc    : the same, sc0 sc1 (write-through to memory)
//   batch<B>  : verdicts of B tiles kept in LDS, then written 16 B per lane
//   copy      : 1 GiB -> 1 GiB copy, for the mixed read/write ceiling
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/wmix tools/wmix.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

enum { W_NONE, W_ST4, W_ST4_NT, W_ST4_SC, W_BATCH, W_WRAP, W_FRAC };

__device__ __forceinline__ void st4_sc(unsigned *p, unsigned v)
{
	asm volatile("global_store_dword %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

template <int W, int B>
__global__ void __launch_bounds__(256) tile_kernel(const unsigned char *buf, unsigned long long ntiles,
                                                   unsigned long long stride, unsigned *out)
{
	__shared__ u32x4 tile[1024];
	__shared__ unsigned vst[W == W_BATCH ? B * 256 : 1];
	unsigned long long t = blockIdx.x;
	unsigned acc = 0;
	u32x4 r[4];
	int nb = 0;
	unsigned long long tb0 = t;
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
		unsigned long long nx = t + gridDim.x;
		if (nx < ntiles)
			ld(nx);
		int p = threadIdx.x;
		u32x4 a = tile[p * 4 + (0 ^ ((p >> 2) & 3))], b = tile[p * 4 + (1 ^ ((p >> 2) & 3))];
		unsigned v = a.x ^ a.w ^ b.y ^ b.z;
		unsigned long long idx = t * 256 + p;
		if (W == W_NONE) {
			acc ^= v;
		} else if (W == W_ST4) {
			out[idx] = v;
		} else if (W == W_ST4_NT) {
			__builtin_nontemporal_store(v, &out[idx]);
		} else if (W == W_ST4_SC) {
			st4_sc(&out[idx], v);
		} else if (W == W_WRAP) {
			/* B = log2 of the words of a wrapped window: stays in L2 / MALL */
			out[idx & ((1ull << B) - 1)] = v;
		} else if (W == W_FRAC) {
			/* only one tile in B writes: 1/B of the write volume */
			if (t % B == 0)
				out[idx] = v;
		} else {
			/* B tiles of one block are t, t+G, ... : not contiguous, so the
			 * batch is B separate 1-KiB runs written 16 B per lane by 64 lanes */
			vst[nb * 256 + p] = v;
			nb++;
			if (nb == B || nx >= ntiles) {
				__syncthreads();
				for (int i = threadIdx.x; i < nb * 64; i += 256) {
					int bt = i >> 6, o = i & 63;
					unsigned long long tt = tb0 + (unsigned long long)bt * gridDim.x;
					*(u32x4 *)&out[tt * 256 + o * 4] = *(u32x4 *)&vst[bt * 256 + o * 4];
				}
				nb = 0;
				tb0 = nx;
			}
		}
		__syncthreads();
		t = nx;
	}
	if (W == W_NONE && acc == 0x9E3779B9u)
		out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) copy_kernel(const u32x4 *in, u32x4 *out, unsigned long long n16)
{
	unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
	for (unsigned long long c = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; c < n16;
	     c += nthreads)
		out[c] = __builtin_nontemporal_load(&in[c]);
}

template <typename F>
static float timeit(F launch, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	launch();
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		launch();
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms * 1e3f / reps;
}

template <int W, int B>
static void run(const char *name, const char *shape, const unsigned char *buf, unsigned long long npkt,
                unsigned long long stride, unsigned *out, int blocks, int reps)
{
	const unsigned long long nt = npkt / 256;
	float us = timeit([&] { hipLaunchKernelGGL((tile_kernel<W, B>), dim3(blocks), dim3(256), 0, 0,
	                                          buf, nt, stride, out); }, reps);
	printf("{\"shape\": \"%s\", \"writes\": \"%s\", \"blocks\": %d, \"us\": %.2f, \"Mpkts\": %.1f, "
	       "\"alg_GBs\": %.1f}\n", shape, name, blocks, us, npkt / us, npkt * 68.0 / us / 1e3);
	fflush(stdout);
}

int main(int argc, char **argv)
{
	int reps = argc > 1 ? atoi(argv[1]) : 20;
	const unsigned long long bytes = 12ull << 30;
	unsigned char *buf;
	unsigned *out;
	CHECK(hipMalloc(&buf, bytes));
	CHECK(hipMalloc(&out, (32ull << 20) * 4));
	CHECK(hipMemset(buf, 1, bytes));
	CHECK(hipMemset(out, 0, (32ull << 20) * 4));
	CHECK(hipDeviceSynchronize());
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	struct { const char *name; unsigned long long n, stride; } shapes[] = {
		{"udp64", 32ull << 20, 64}, {"tcp1500", 8ull << 20, 1536}};
	for (auto &s : shapes) {
		for (int g : {cus * 4}) {
			run<W_NONE, 1>("none", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_ST4, 1>("st4", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_ST4_NT, 1>("st4_nt", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_ST4_SC, 1>("st4_sc", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_BATCH, 4>("batch4", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_BATCH, 16>("batch16", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_WRAP, 18>("wrap_1MiB", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_WRAP, 22>("wrap_16MiB", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_WRAP, 24>("wrap_64MiB", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_FRAC, 2>("frac_1of2", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_FRAC, 8>("frac_1of8", s.name, buf, s.n, s.stride, out, g, reps);
			run<W_FRAC, 64>("frac_1of64", s.name, buf, s.n, s.stride, out, g, reps);
		}
	}
	for (int g : {cus * 4, cus * 8}) {
		unsigned long long n16 = (1ull << 30) / 16;
		float us = timeit([&] { hipLaunchKernelGGL(copy_kernel, dim3(g), dim3(256), 0, 0,
		                                          (const u32x4 *)buf, (u32x4 *)(buf + (4ull << 30)), n16); }, reps);
		printf("{\"shape\": \"copy_1GiB\", \"blocks\": %d, \"us\": %.2f, \"GBs_rw\": %.1f}\n", g, us,
		       2.0 * (1ull << 30) / us / 1e3);
	}
	CHECK(hipFree(buf));
	CHECK(hipFree(out));
	return 0;
}
