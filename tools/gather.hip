// gather.hip - the read ceiling of the integrated ingress shape (bench.py
// e2e.ingress_pool): 64-B header windows gathered through a u64 descriptor
// array from the reference's mbuf pool geometry (131072 elements of 9408 B,
// 222 per 2 MiB page, frame data at element + 344; iokernel/defs.h:503-523),
// 64 passes per batch.  No classification, no verdicts: the descriptor read
// and one 16-B-aligned 64-B window per packet (four 16-B loads, as the
// classify kernel's windowed staging issues), in three descriptor orders:
//   random    64 random permutations of the pool (the bench's order)
//   address   the pool in address order, 64 times
//   dense     a dense 64-B slot array of the same packet count (udp64 shape)
//   working_set_4096  a random 4096-mbuf subset of the pool in random order
// Two kernels: `gather` (one 16-B chunk per lane, its descriptor loaded
// right before it) and `gather_lds` (the classify kernel's form: descriptors
// shared through LDS, one tile ahead).  Prints the kernel time and packets/s.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather tools/gather.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one packet per 4 lanes: lane q of the packet reads 16 B at (off & ~15) + 16 q
__global__ void __launch_bounds__(256) gather_kernel(const unsigned char *pool, const unsigned long long *offs,
                                                     unsigned long long n, unsigned *out)
{
	unsigned acc = 0;
	const unsigned long long nthr = (unsigned long long)gridDim.x * blockDim.x;
	for (unsigned long long c = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; c < n * 4;
	     c += nthr) {
		const unsigned long long o = (__builtin_nontemporal_load(offs + (c >> 2)) & ~15ull) + (c & 3) * 16;
		const u32x4 v = __builtin_nontemporal_load((const u32x4 *)(pool + o));
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x9E3779B9u)
		out[blockIdx.x] = acc;
}

// the classify kernel's decoupled form: a 256-lane block takes 256
// descriptors per tile, each lane loading its own packet's descriptor one
// tile ahead; after a barrier the descriptors come from LDS and the four
// lanes of each 64-B window issue their 16-B loads (coalesced), two tiles of
// loads in flight
__global__ void __launch_bounds__(256) gather_lds_kernel(const unsigned char *pool,
                                                         const unsigned long long *offs,
                                                         unsigned long long n, unsigned *out)
{
	__shared__ unsigned long long s_off[2][256];
	unsigned acc = 0;
	const unsigned long long ntiles = n / 256, G = gridDim.x;
	unsigned long long t = blockIdx.x;
	unsigned long long mine = t < ntiles ? __builtin_nontemporal_load(offs + t * 256 + threadIdx.x) : 0;
	int par = 0;
	for (; t < ntiles; t += G, par ^= 1) {
		s_off[par][threadIdx.x] = mine;
		__syncthreads();
		if (t + G < ntiles)
			mine = __builtin_nontemporal_load(offs + (t + G) * 256 + threadIdx.x);
		u32x4 v[4];
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const int c = j * 256 + (int)threadIdx.x;
			v[j] = __builtin_nontemporal_load(
			        (const u32x4 *)(pool + (s_off[par][c >> 2] & ~15ull) + (c & 3) * 16));
		}
#pragma unroll
		for (int j = 0; j < 4; j++)
			acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
	}
	if (acc == 0x9E3779B9u)
		out[blockIdx.x] = acc;
}

int main(int argc, char **argv)
{
	const int reps = argc > 1 ? atoi(argv[1]) : 10;
	const unsigned long long P = 131072, per_page = 222, elt = 9408, data = 344, cycles = 64;
	const unsigned long long region = (P + per_page - 1) / per_page * (2ull << 20);
	const unsigned long long n = P * cycles;
	std::vector<unsigned long long> pool(P), rnd(n), adr(n), dense(n), wset(n);
	for (unsigned long long i = 0; i < P; i++)
		pool[i] = (i / per_page) * (2ull << 20) + (i % per_page) * elt + data;
	std::mt19937_64 rng(0xCA1ADA4);
	std::vector<unsigned long long> perm(P);
	for (unsigned long long c = 0; c < cycles; c++) {
		for (unsigned long long i = 0; i < P; i++)
			perm[i] = i;
		std::shuffle(perm.begin(), perm.end(), rng);
		for (unsigned long long i = 0; i < P; i++) {
			rnd[c * P + i] = pool[perm[i]];
			adr[c * P + i] = pool[i];
		}
	}
	for (unsigned long long i = 0; i < n; i++)
		dense[i] = i * 64;
	{ /* a 4096-mbuf working set in random order (RX ring + mempool cache) */
		const unsigned long long W = 4096;
		for (unsigned long long i = 0; i < P; i++)
			perm[i] = i;
		std::shuffle(perm.begin(), perm.end(), rng);
		std::vector<unsigned long long> sub(perm.begin(), perm.begin() + W);
		for (unsigned long long c = 0; c < n / W; c++) {
			std::shuffle(sub.begin(), sub.end(), rng);
			for (unsigned long long i = 0; i < W; i++)
				wset[c * W + i] = pool[sub[i]];
		}
	}
	const unsigned long long bytes = std::max(region, n * 64);
	unsigned char *buf;
	unsigned long long *d_offs;
	unsigned *out;
	CHECK(hipMalloc(&buf, bytes));
	CHECK(hipMemset(buf, 1, bytes));
	CHECK(hipMalloc(&d_offs, n * 8));
	CHECK(hipMalloc(&out, 1 << 20));
	int cus = 0;
	CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	const struct { const char *name; std::vector<unsigned long long> *o; } orders[] = {
		{"random", &rnd}, {"address", &adr}, {"dense", &dense}, {"working_set_4096", &wset}};
	for (auto &ord : orders) {
		CHECK(hipMemcpy(d_offs, ord.o->data(), n * 8, hipMemcpyHostToDevice));
		for (int g : {cus * 4, cus * 8, cus * 16}) {
			hipLaunchKernelGGL(gather_kernel, dim3(g), dim3(256), 0, 0, buf, d_offs, n, out);
			CHECK(hipEventRecord(a, 0));
			for (int r = 0; r < reps; r++)
				hipLaunchKernelGGL(gather_kernel, dim3(g), dim3(256), 0, 0, buf, d_offs, n, out);
			CHECK(hipEventRecord(b, 0));
			CHECK(hipEventSynchronize(b));
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, a, b));
			const double us = ms * 1e3 / reps;
			printf("{\"order\": \"%s\", \"kernel\": \"gather\", \"blocks\": %d, \"pkts\": %llu, \"us\": %.2f, "
			       "\"Mpkts\": %.1f, \"desc_plus_window_GBs\": %.1f}\n", ord.name, g, n, us, n / us,
			       n * 72.0 / (us * 1e-6) / 1e9);
			fflush(stdout);
		}
		for (int g : {cus * 4, cus * 8, cus * 16}) {
			hipLaunchKernelGGL(gather_lds_kernel, dim3(g), dim3(256), 0, 0, buf, d_offs, n, out);
			CHECK(hipEventRecord(a, 0));
			for (int r = 0; r < reps; r++)
				hipLaunchKernelGGL(gather_lds_kernel, dim3(g), dim3(256), 0, 0, buf, d_offs, n, out);
			CHECK(hipEventRecord(b, 0));
			CHECK(hipEventSynchronize(b));
			float ms = 0;
			CHECK(hipEventElapsedTime(&ms, a, b));
			const double us = ms * 1e3 / reps;
			printf("{\"order\": \"%s\", \"kernel\": \"gather_lds\", \"blocks\": %d, \"pkts\": %llu, "
			       "\"us\": %.2f, \"Mpkts\": %.1f, \"desc_plus_window_GBs\": %.1f}\n", ord.name, g, n, us,
			       n / us, n * 72.0 / (us * 1e-6) / 1e9);
			fflush(stdout);
		}
	}
	return 0;
}
