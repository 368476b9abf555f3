// place.hip - does the udp64 read+write shape depend on where the verdict
// array sits relative to the frame array?  tools/alloc_ab.cpp found the
// classify kernel bimodal (343 vs 406 us) across buffers of the same process
// and across processes.  Here the frames stay put and the verdict array
// slides through a 1 GiB pool by power-of-two offsets (and the frames slide
// through a 4 GiB allocation), timing the same tile loop as tools/wmix.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/place tools/place.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void __launch_bounds__(256) tile_kernel(const unsigned char *buf, unsigned long long ntiles,
                                                   unsigned long long stride, unsigned *out)
{
	__shared__ u32x4 tile[1024];
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
		unsigned long long nx = t + gridDim.x;
		if (nx < ntiles)
			ld(nx);
		int p = threadIdx.x;
		u32x4 a = tile[p * 4 + (0 ^ ((p >> 2) & 3))], b = tile[p * 4 + (1 ^ ((p >> 2) & 3))];
		out[t * 256 + p] = a.x ^ a.w ^ b.y ^ b.z;
		__syncthreads();
		t = nx;
	}
}

static float timeit(const unsigned char *f, unsigned *v, unsigned long long n, unsigned long long stride,
                    int blocks, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL(tile_kernel, dim3(blocks), dim3(256), 0, 0, f, n / 256, stride, v);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		hipLaunchKernelGGL(tile_kernel, dim3(blocks), dim3(256), 0, 0, f, n / 256, stride, v);
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms * 1e3f / reps;
}

int main(int argc, char **argv)
{
	const int reps = argc > 1 ? atoi(argv[1]) : 10;
	const unsigned long long n = 32ull << 20, stride = 64;
	unsigned char *fpool, *vpool;
	CHECK(hipMalloc(&fpool, 4ull << 30));
	CHECK(hipMalloc(&vpool, 1ull << 30));
	CHECK(hipMemset(fpool, 1, 4ull << 30));
	CHECK(hipMemset(vpool, 0, 1ull << 30));
	CHECK(hipDeviceSynchronize());
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	const int G = cus * 4;
	printf("{\"fpool\": \"%p\", \"vpool\": \"%p\"}\n", (void *)fpool, (void *)vpool);
	/* verdict array offsets: 0, then powers of two 4 KiB .. 512 MiB, then
	 * a few odd multiples of 2 MiB */
	std::initializer_list<unsigned long long> offs = {
		0, 4096, 8192, 16384, 32768, 65536, 1 << 17, 1 << 18, 1 << 19, 1 << 20, 2 << 20, 4 << 20,
		8 << 20, 16 << 20, 32 << 20, 64 << 20, 128 << 20, 256 << 20, 512 << 20,
		3 << 20, 5 << 20, 6 << 20, 7 << 20, 3 << 21, 3 << 22, 3 << 23, 3 << 24, 3 << 25, 3 << 26};
	for (unsigned long long o : offs) {
		float us = timeit(fpool, (unsigned *)(vpool + o), n, stride, G, reps);
		printf("{\"vary\": \"verdict\", \"off\": %llu, \"us\": %.2f}\n", o, us);
		fflush(stdout);
	}
	for (unsigned long long o : offs) {
		if (o > (1ull << 31))
			continue;
		float us = timeit(fpool + o, (unsigned *)vpool, n, stride, G, reps);
		printf("{\"vary\": \"frames\", \"off\": %llu, \"us\": %.2f}\n", o, us);
		fflush(stdout);
	}
	for (unsigned long long o : {0ull, 1ull << 30, 1ull << 31, 3ull << 30}) {
		if (o + (2ull << 30) > (4ull << 30))
			continue;
		float us = timeit(fpool + o, (unsigned *)vpool, n, stride, G, reps);
		printf("{\"vary\": \"frames_big\", \"off\": %llu, \"us\": %.2f}\n", o, us);
	}
	CHECK(hipFree(fpool));
	CHECK(hipFree(vpool));
	return 0;
}
