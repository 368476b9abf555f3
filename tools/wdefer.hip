// wdefer.hip - is the udp64 verdict stream's cost a
// floor of interleaving reads and writes, or of when the writes are issued?
//
// The headline kernel reads 32 Mi 64-B header granules (2 GiB) and writes one
// 1-B verdict per packet (32 MiB) write-through at the end of each 256-packet
// tile.  This probe runs the same persistent grid (1024 blocks x 256 lanes,
// 4 x 16-B streaming loads per lane per tile, round-robin tiles) with no
// classification and the 1-B write stream in different shapes:
//   none         no verdict stores (one word per block at the end)
//   tile         1 B per lane per tile, write-through (the classify kernel)
//   defer        every verdict of the block kept in LDS (32 KB per block),
//                all written after the block's last tile, 16 B per lane
//   defer_half   the same, flushed twice (after half of the block's tiles)
//   contig_tile  block b walks tiles [b*C, (b+1)*C) (C = tiles per block),
//                per-tile stores
//   contig_defer the same walk, its 32 KB of verdicts written as one run at
//                the end
// Each shape is timed with HIP events over 20 launches after 3 warm-ups,
// shapes interleaved over 3 rounds; one JSON line per (round, shape).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/wdefer tools/wdefer.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

enum { S_NONE, S_TILE, S_DEFER, S_DEFER_HALF, S_CONTIG_TILE, S_CONTIG_DEFER, S_N };
static const char *kNames[S_N] = {"none", "tile", "defer", "defer_half", "contig_tile", "contig_defer"};

constexpr int NT = 256;
constexpr int kMaxTilesPerBlock = 128; /* 32 KB of 1-B verdicts */

__device__ __forceinline__ uint4 ld_nt(const void *p)
{
	typedef unsigned int v4 __attribute__((ext_vector_type(4)));
	const v4 v = __builtin_nontemporal_load((const v4 *)p);
	return make_uint4(v.x, v.y, v.z, v.w);
}

template <int S>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4)))
probe_kernel(const unsigned char *frames, unsigned long long ntiles, unsigned char *verd, unsigned *sink)
{
	extern __shared__ unsigned char vbuf[];
	const int tid = threadIdx.x;
	const unsigned long long G = gridDim.x;
	const bool contig = S == S_CONTIG_TILE || S == S_CONTIG_DEFER;
	const unsigned long long per = (ntiles + G - 1) / G;
	unsigned long long t = contig ? blockIdx.x * per : blockIdx.x;
	const unsigned long long t_end = contig ? (blockIdx.x + 1) * per < ntiles ? (blockIdx.x + 1) * per : ntiles
	                                        : ntiles;
	const unsigned long long step = contig ? 1 : G;
	unsigned acc = 0;
	int k = 0;
	auto flush = [&](int k0, int k1) { /* tiles k0..k1-1 of this block, 16 B per lane */
		for (int i = tid; i < (k1 - k0) * (NT / 16); i += NT) {
			const int kk = k0 + i / (NT / 16), c = i % (NT / 16);
			const unsigned long long tt = contig ? blockIdx.x * per + kk : blockIdx.x + kk * G;
			const uint4 v = *(const uint4 *)(vbuf + kk * NT + 16 * c);
			__hip_atomic_store((unsigned long long *)(verd + tt * NT + 16 * c),
			                   (unsigned long long)v.x | (unsigned long long)v.y << 32,
			                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
			__hip_atomic_store((unsigned long long *)(verd + tt * NT + 16 * c + 8),
			                   (unsigned long long)v.z | (unsigned long long)v.w << 32,
			                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		}
	};
	for (; t < t_end; t += step, k++) {
		uint4 r[4];
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const int c = j * NT + tid, p = c >> 2;
			r[j] = ld_nt(frames + (t * NT + p) * 64 + (c & 3) * 16);
		}
		unsigned x = 0;
#pragma unroll
		for (int j = 0; j < 4; j++)
			x ^= r[j].x ^ r[j].y ^ r[j].z ^ r[j].w;
		acc ^= x;
		if (S == S_TILE || S == S_CONTIG_TILE)
			__hip_atomic_store(verd + t * NT + tid, (unsigned char)x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
		else if (S != S_NONE)
			vbuf[k * NT + tid] = (unsigned char)x;
		if (S == S_DEFER_HALF && k + 1 == kMaxTilesPerBlock / 2) {
			__syncthreads();
			flush(0, k + 1);
		}
	}
	if (S == S_DEFER || S == S_CONTIG_DEFER || S == S_DEFER_HALF) {
		__syncthreads();
		flush(S == S_DEFER_HALF && k > kMaxTilesPerBlock / 2 ? kMaxTilesPerBlock / 2 : 0, k);
	}
	if (acc == 0x9E3779B9u)
		sink[0] = acc;
}

int main(int argc, char **argv)
{
	const unsigned long long n = argc > 1 ? strtoull(argv[1], 0, 0) : (32ull << 20);
	const int grid = argc > 2 ? atoi(argv[2]) : 1024;
	const unsigned long long ntiles = n / NT;
	if (ntiles > (unsigned long long)grid * kMaxTilesPerBlock) {
		fprintf(stderr, "too many tiles per block for the LDS buffer\n");
		return 1;
	}
	unsigned char *frames, *verd;
	unsigned *sink;
	CHECK(hipMalloc(&frames, n * 64));
	CHECK(hipMalloc(&verd, n));
	CHECK(hipMalloc(&sink, 64));
	CHECK(hipMemset(frames, 0x5A, n * 64));
	CHECK(hipMemset(verd, 0, n));
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	const unsigned lds = kMaxTilesPerBlock * NT;
	auto launch = [&](int s) {
#define L(S) hipLaunchKernelGGL(probe_kernel<S>, dim3(grid), dim3(NT), S == S_NONE || S == S_TILE || S == S_CONTIG_TILE ? 0 : lds, 0, frames, ntiles, verd, sink)
		switch (s) {
		case S_NONE: L(S_NONE); break;
		case S_TILE: L(S_TILE); break;
		case S_DEFER: L(S_DEFER); break;
		case S_DEFER_HALF: L(S_DEFER_HALF); break;
		case S_CONTIG_TILE: L(S_CONTIG_TILE); break;
		default: L(S_CONTIG_DEFER); break;
		}
#undef L
	};
	for (int round = 0; round < 3; round++) {
		for (int s = 0; s < S_N; s++) {
			for (int i = 0; i < 3; i++)
				launch(s);
			CHECK(hipEventRecord(e0, 0));
			for (int i = 0; i < 20; i++)
				launch(s);
			CHECK(hipEventRecord(e1, 0));
			CHECK(hipEventSynchronize(e1));
			CHECK(hipGetLastError());
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, e0, e1));
			const double us = ms * 1e3 / 20;
			const double bytes = (double)n * (s == S_NONE ? 64 : 65);
			printf("{\"round\": %d, \"shape\": \"%s\", \"pkts\": %llu, \"blocks\": %d, \"us\": %.2f, "
			       "\"alg_GBs\": %.1f, \"frac\": %.4f}\n",
			       round, kNames[s], n, grid, us, (double)n * 65 / (us * 1e-6) / 1e9,
			       (double)n * 65 / (us * 1e-6) / 8e12);
			(void)bytes;
			fflush(stdout);
		}
	}
	return 0;
}
