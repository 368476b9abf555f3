// clock_probe.hip - what the two GPU clocks cost a wave that reads them.
//
// The rx loop's poll reads s_memrealtime (the 100 MHz real-time counter) for
// its speculative window and its lifetime bound.  This times, on one wave,
// K back-to-back dependent reads of s_memrealtime and of s_memtime (the
// shader clock), each read's value used before the next is issued, and the
// shader clock's rate against the real-time counter over ~10 ms.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/clock_probe tools/clock_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void probe(unsigned long long *o, int K)
{
	if (threadIdx.x)
		return;
	unsigned long long acc = 0;
	unsigned long long t0 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < K; i++)
		acc += __builtin_amdgcn_s_memrealtime() & 1; /* used: waits for each */
	unsigned long long t1 = __builtin_amdgcn_s_memtime();
	for (int i = 0; i < K; i++)
		acc += __builtin_amdgcn_s_memtime() & 1;
	unsigned long long t2 = __builtin_amdgcn_s_memtime();
	/* shader clock rate: spin ~10 ms of real time */
	const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
	unsigned long long r1;
	do {
		r1 = __builtin_amdgcn_s_memrealtime();
	} while (r1 - r0 < 1000000);
	const unsigned long long c1 = __builtin_amdgcn_s_memtime();
	o[0] = t1 - t0;
	o[1] = t2 - t1;
	o[2] = c1 - c0;
	o[3] = r1 - r0;
	o[4] = acc;
}

int main()
{
	unsigned long long *d, h[5];
	const int K = 1000;
	CHECK(hipMalloc(&d, sizeof(h)));
	for (int rep = 0; rep < 3; rep++) {
		hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, K);
		CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
		const double mhz = h[2] / (h[3] * 10e-3); /* shader ticks per us */
		printf("{\"memrealtime_ns\": %.1f, \"memtime_ns\": %.1f, \"memtime_mhz\": %.1f}\n",
		       h[0] / (double)K / mhz * 1e3, h[1] / (double)K / mhz * 1e3, mhz);
	}
	return 0;
}
