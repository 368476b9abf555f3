// membench.hip - HBM ceilings for the rx classify access patterns (gfx950).
//
// Measures, with hipEvents, the bandwidth a trivial kernel reaches for:
//   stream   : every byte of a buffer, 16 B per lane, fully coalesced
//   hdr<S>   : the first 64 B of every S-byte slot (4 lanes x 16 B per slot)
//   hdr32<S> : the first 32 B of every S-byte slot
// so the classify kernel's roofline fraction can be read against what the
// memory system delivers for the same pattern.  Each kernel xor-reduces what
// it reads into one word per block so nothing is optimised away.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

// chunks: number of 16-B pieces; piece c lives at (c / per) * stride + (c % per) * 16
template <int DEPTH>
__global__ void __launch_bounds__(256) read_kernel(const unsigned char *buf, unsigned long long chunks,
                                                   unsigned per, unsigned long long stride,
                                                   unsigned *out)
{
	unsigned acc = 0;
	unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
	unsigned long long c = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
	for (; c + (DEPTH - 1) * nthreads < chunks; c += DEPTH * nthreads) {
		u32x4 v[DEPTH];
#pragma unroll
		for (int d = 0; d < DEPTH; d++) {
			unsigned long long cc = c + d * nthreads;
			const unsigned char *p = buf + (cc / per) * stride + (cc % per) * 16;
			v[d] = __builtin_nontemporal_load((const u32x4 *)p);
		}
#pragma unroll
		for (int d = 0; d < DEPTH; d++)
			acc ^= v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
	}
	for (; c < chunks; c += nthreads) {
		const unsigned char *p = buf + (c / per) * stride + (c % per) * 16;
		u32x4 v = *(const u32x4 *)p;
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x9E3779B9u)
		out[blockIdx.x] = acc;
}

// the classify kernel's traffic without its compute: 64 B read per packet
// (4 lanes x 16 B at the slot stride, staged like the real tile) + 8 B written
__global__ void __launch_bounds__(256) rw_kernel(const unsigned char *buf, unsigned long long npkt,
                                                 unsigned long long stride, unsigned long long *out)
{
	unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
	for (unsigned long long base = (unsigned long long)blockIdx.x * blockDim.x; base < npkt * 4;
	     base += nthreads) {
		unsigned long long c = base + threadIdx.x;
		unsigned x = 0;
		if (c < npkt * 4) {
			const unsigned char *p = buf + (c >> 2) * stride + (c & 3) * 16;
			u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
			x = v.x ^ v.y ^ v.z ^ v.w;
		}
		// combine the 4 lanes of a packet, one 8-B store per packet
		x ^= __shfl_xor(x, 1);
		x ^= __shfl_xor(x, 2);
		if (c < npkt * 4 && (c & 3) == 0)
			out[c >> 2] = x;
	}
}

// variants of the classify traffic shape (udp64: 64-B slots), one tile of 256
// packets per block iteration, staged through LDS like the real kernel:
//  V=0: 8-B verdict store per lane; V=1: verdicts staged in LDS and written
//  16 B per lane by half the lanes; V=2: as 0 with non-temporal stores;
//  V=3: as 0 with two tiles in flight.
template <int V>
__global__ void __launch_bounds__(256) tile_kernel(const unsigned char *buf, unsigned long long npkt,
                                                   unsigned long long stride, unsigned long long *out)
{
	__shared__ u32x4 tile[1024];
	__shared__ unsigned long long vst[256];
	const unsigned long long ntiles = npkt / 256;
	unsigned long long t = blockIdx.x;
	u32x4 r[4], r2[4];
	auto ld = [&](unsigned long long tt, u32x4 *rr) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			int c = j * 256 + threadIdx.x;
			rr[j] = __builtin_nontemporal_load((const u32x4 *)(buf + (tt * 256 + (c >> 2)) * stride + (c & 3) * 16));
		}
	};
	if (t < ntiles) ld(t, r);
	if (V == 3 && t + gridDim.x < ntiles) ld(t + gridDim.x, r2);
	while (t < ntiles) {
#pragma unroll
		for (int j = 0; j < 4; j++) {
			int c = j * 256 + threadIdx.x;
			int p = c >> 2, q = c & 3;
			tile[p * 4 + (q ^ ((p >> 2) & 3))] = r[j];
		}
		__syncthreads();
		unsigned long long nx = t + (V == 3 ? 2 : 1) * gridDim.x;
		if (V == 3) {
#pragma unroll
			for (int j = 0; j < 4; j++) r[j] = r2[j];
			if (nx < ntiles) ld(nx, r2);
		} else if (nx < ntiles) {
			ld(nx, r);
		}
		int p = threadIdx.x;
		u32x4 a = tile[p * 4 + (0 ^ ((p >> 2) & 3))], b = tile[p * 4 + (1 ^ ((p >> 2) & 3))];
		unsigned long long v = ((unsigned long long)(a.w ^ b.y) << 32) | (b.z ^ a.x);
		unsigned long long idx = t * 256 + p;
		if (V == 1) {
			vst[p] = v;
			__syncthreads();
			if (p < 128) {
				u32x4 w = *(u32x4 *)&vst[2 * p];
				*(u32x4 *)&out[t * 256 + 2 * p] = w;
			}
		} else if (V == 2) {
			__builtin_nontemporal_store(v, &out[idx]);
		} else {
			out[idx] = v;
		}
		__syncthreads();
		t += gridDim.x;
	}
}

template <int V>
static void run_tile(const char *name, const unsigned char *buf, unsigned long long npkt,
                     unsigned long long stride, unsigned long long *out, int blocks, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL(tile_kernel<V>, dim3(blocks), dim3(256), 0, 0, buf, npkt, stride, out);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		hipLaunchKernelGGL(tile_kernel<V>, dim3(blocks), dim3(256), 0, 0, buf, npkt, stride, out);
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	double bytes = (double)npkt * 72;
	printf("{\"pattern\": \"%s\", \"blocks\": %d, \"depth\": %d, \"useful_bytes\": %.0f, \"us\": %.2f, \"GBs\": %.1f, \"Mpkts\": %.1f}\n",
	       name, blocks, V, bytes, ms * 1e3 / reps, bytes * reps / (ms * 1e-3) / 1e9,
	       (double)npkt * reps / (ms * 1e-3) / 1e6);
	fflush(stdout);
}

// pure streaming write of B bytes, 16 B per lane
__global__ void __launch_bounds__(256) write_kernel(u32x4 *out, unsigned long long n16)
{
	unsigned long long nthreads = (unsigned long long)gridDim.x * blockDim.x;
	for (unsigned long long c = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += nthreads)
		out[c] = u32x4{(unsigned)c, 1, 2, 3};
}

static double run_rw(const char *name, const unsigned char *buf, unsigned long long npkt,
                     unsigned long long stride, unsigned long long *out, int blocks, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	hipLaunchKernelGGL(rw_kernel, dim3(blocks), dim3(256), 0, 0, buf, npkt, stride, out);
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		hipLaunchKernelGGL(rw_kernel, dim3(blocks), dim3(256), 0, 0, buf, npkt, stride, out);
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	double bytes = (double)npkt * 72;
	printf("{\"pattern\": \"%s\", \"blocks\": %d, \"depth\": 1, \"useful_bytes\": %.0f, \"us\": %.2f, \"GBs\": %.1f, \"Mpkts\": %.1f}\n",
	       name, blocks, bytes, ms * 1e3 / reps, bytes * reps / (ms * 1e-3) / 1e9,
	       (double)npkt * reps / (ms * 1e-3) / 1e6);
	fflush(stdout);
	return 0;
}

static double run(const char *name, const unsigned char *buf, unsigned long long chunks, unsigned per,
                  unsigned long long stride, unsigned *out, int blocks, int depth, int reps)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	auto launch = [&]() {
		switch (depth) {
		case 1: hipLaunchKernelGGL(read_kernel<1>, dim3(blocks), dim3(256), 0, 0, buf, chunks, per, stride, out); break;
		case 2: hipLaunchKernelGGL(read_kernel<2>, dim3(blocks), dim3(256), 0, 0, buf, chunks, per, stride, out); break;
		case 4: hipLaunchKernelGGL(read_kernel<4>, dim3(blocks), dim3(256), 0, 0, buf, chunks, per, stride, out); break;
		default: hipLaunchKernelGGL(read_kernel<8>, dim3(blocks), dim3(256), 0, 0, buf, chunks, per, stride, out); break;
		}
	};
	launch();
	CHECK(hipDeviceSynchronize());
	CHECK(hipEventRecord(a, 0));
	for (int i = 0; i < reps; i++)
		launch();
	CHECK(hipEventRecord(b, 0));
	CHECK(hipEventSynchronize(b));
	float ms = 0;
	CHECK(hipEventElapsedTime(&ms, a, b));
	double bytes = (double)chunks * 16;
	double gbs = bytes * reps / (ms * 1e-3) / 1e9;
	printf("{\"pattern\": \"%s\", \"blocks\": %d, \"depth\": %d, \"useful_bytes\": %.0f, \"us\": %.2f, \"GBs\": %.1f}\n",
	       name, blocks, depth, bytes, ms * 1e3 / reps, gbs);
	fflush(stdout);
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return gbs;
}

int main(int argc, char **argv)
{
	int calib = argc > 1 && !strcmp(argv[1], "calib");
	int reps = calib ? 1 : (argc > 1 ? atoi(argv[1]) : 20);
	const unsigned long long bytes = 12ull << 30; // 12 GiB: the tcp1500 slot array
	unsigned char *buf;
	unsigned *out;
	CHECK(hipMalloc(&buf, bytes));
	CHECK(hipMalloc(&out, 1 << 20));
	CHECK(hipMemset(buf, 1, bytes));
	CHECK(hipDeviceSynchronize());
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	unsigned long long *vout;
	CHECK(hipMalloc(&vout, (32ull << 20) * 8));
	if (calib) {
		// one dispatch per pattern, for FETCH_SIZE / WRITE_SIZE calibration
		run("stream_2GiB", buf, (2ull << 30) / 16, 1, 16, out, cus * 8, 2, 1);
		run("hdr64_stride1536", buf, (8ull << 20) * 4, 4, 1536, out, cus * 8, 2, 1);
		run("hdr128_stride1536", buf, (8ull << 20) * 8, 8, 1536, out, cus * 8, 2, 1);
		run("hdr32_stride1536", buf, (8ull << 20) * 2, 2, 1536, out, cus * 8, 2, 1);
		run_rw("rw_udp64", buf, 32ull << 20, 64, vout, cus * 8, 1);
		run_rw("rw_tcp1500", buf, 8ull << 20, 1536, vout, cus * 8, 1);
		return 0;
	}
	if (argc > 2 && !strcmp(argv[2], "tile")) {
		for (int gi : {cus * 4, cus * 8, cus * 16}) {
			run_tile<0>("tile_v0_store8", buf, 32ull << 20, 64, vout, gi, reps);
			run_tile<1>("tile_v1_store16", buf, 32ull << 20, 64, vout, gi, reps);
			run_tile<2>("tile_v2_store8_nt", buf, 32ull << 20, 64, vout, gi, reps);
			run_tile<3>("tile_v3_depth2", buf, 32ull << 20, 64, vout, gi, reps);
			run_tile<0>("tile_v0_tcp1500", buf, 8ull << 20, 1536, vout, gi, reps);
		}
		for (int gi : {cus * 4, cus * 8}) {
			hipEvent_t a, b;
			CHECK(hipEventCreate(&a));
			CHECK(hipEventCreate(&b));
			unsigned long long n16 = (2ull << 30) / 16;
			hipLaunchKernelGGL(write_kernel, dim3(gi), dim3(256), 0, 0, (u32x4 *)buf, n16);
			CHECK(hipEventRecord(a, 0));
			for (int i = 0; i < reps; i++)
				hipLaunchKernelGGL(write_kernel, dim3(gi), dim3(256), 0, 0, (u32x4 *)buf, n16);
			CHECK(hipEventRecord(b, 0));
			CHECK(hipEventSynchronize(b));
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, a, b));
			printf("{\"pattern\": \"write_2GiB\", \"blocks\": %d, \"GBs\": %.1f}\n", gi,
			       (2ull << 30) * (double)reps / (ms * 1e-3) / 1e9);
		}
		return 0;
	}
	for (int gi : {cus * 4, cus * 8, cus * 16}) {
		run_rw("rw_udp64", buf, 32ull << 20, 64, vout, gi, reps);
		run_rw("rw_tcp1500", buf, 8ull << 20, 1536, vout, gi, reps);
	}
	const int grids[] = {cus * 4, cus * 8, cus * 16};
	const int depths[] = {1, 2, 4, 8};
	// stream 2 GiB (the udp64 frame array)
	for (int gi = 0; gi < 3; gi++)
		for (int d : depths)
			run("stream_2GiB", buf, (2ull << 30) / 16, 1, 16, out, grids[gi], d, reps);
	// header granules of 1536-B slots (8 Mi slots = 12 GiB)
	const unsigned long long slots = bytes / 1536;
	for (int gi = 0; gi < 3; gi++)
		for (int d : depths) {
			run("hdr64_stride1536", buf, slots * 4, 4, 1536, out, grids[gi], d, reps);
			run("hdr32_stride1536", buf, slots * 2, 2, 1536, out, grids[gi], d, reps);
			run("hdr128_stride1536", buf, slots * 8, 8, 1536, out, grids[gi], d, reps);
		}
	// header granules of 9216-B slots (the jumbo layout)
	const unsigned long long jslots = bytes / 9216;
	for (int d : depths)
		run("hdr64_stride9216", buf, jslots * 4, 4, 9216, out, grids[1], d, reps);
	CHECK(hipFree(buf));
	CHECK(hipFree(out));
	return 0;
}
