// halfline.hip - does a read of part of a 128-B line cost the whole line?
//
// FETCH_SIZE counts TCC_EA0_RDREQ x 64 B whatever the request size, and on
// gfx950 a full-line streaming read is one 128-B request per line (guide:
// "FETCH_SIZE reports half").  tcp1500 reads 64 B of every 1536-B slot; the
// request count cannot tell whether those are 64-B or 128-B requests.  Time
// can, when the lines are dense: read 128, 64 and 32 B of every 128-B line of
// a 2 GiB buffer (the same 16 Mi lines each time).  If a partial read fetched
// only what it asks for, the 64-B pass would move half the bytes.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/halfline tools/halfline.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

// PER = 16-B chunks read per line (8 = whole line, 4 = 64 B, 2 = 32 B)
template <int PER>
__global__ void __launch_bounds__(256) part_kernel(const unsigned char *buf, unsigned long long lines,
                                                   unsigned *out)
{
	const unsigned long long n = lines * PER;
	const unsigned long long G = (unsigned long long)gridDim.x * 256;
	unsigned acc = 0;
	unsigned long long c = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
	for (; c + 3 * G < n; c += 4 * G) {
		u32x4 v[4];
#pragma unroll
		for (int d = 0; d < 4; d++) {
			const unsigned long long cc = c + d * G;
			v[d] = __builtin_nontemporal_load((const u32x4 *)(buf + (cc / PER) * 128 + (cc % PER) * 16));
		}
#pragma unroll
		for (int d = 0; d < 4; d++)
			acc ^= v[d].x ^ v[d].w;
	}
	for (; c < n; c += G)
		acc ^= ((const u32x4 *)(buf + (c / PER) * 128 + (c % PER) * 16))->y;
	if (acc == 0x9E3779B9u)
		out[0] = acc;
}

template <int PER>
static void run(const unsigned char *buf, unsigned long long lines, unsigned *out, int blocks, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL(part_kernel<PER>, dim3(blocks), dim3(256), 0, 0, buf, lines, out);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		hipLaunchKernelGGL(part_kernel<PER>, dim3(blocks), dim3(256), 0, 0, buf, lines, out);
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	const double us = ms * 1e3 / reps;
	printf("{\"bytes_per_line\": %d, \"lines\": %llu, \"blocks\": %d, \"us\": %.2f, \"Glines_per_s\": %.2f, "
	       "\"requested_GBs\": %.1f}\n", PER * 16, lines, blocks, us, lines / us / 1e3,
	       lines * PER * 16.0 / us / 1e3);
	fflush(stdout);
}

int main(int argc, char **argv)
{
	const int reps = argc > 1 ? atoi(argv[1]) : 20;
	const unsigned long long bytes = 2ull << 30, lines = bytes / 128;
	unsigned char *buf;
	unsigned *out;
	CHECK(hipMalloc(&buf, bytes));
	CHECK(hipMalloc(&out, 64));
	CHECK(hipMemset(buf, 1, bytes));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	for (int g : {cus * 4, cus * 8}) {
		run<8>(buf, lines, out, g, reps);
		run<4>(buf, lines, out, g, reps);
		run<2>(buf, lines, out, g, reps);
	}
	CHECK(hipFree(buf));
	CHECK(hipFree(out));
	return 0;
}
