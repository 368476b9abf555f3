// xcd_lat.hip - host-memory load latency seen from each XCD.
//
// The persistent rx loop (one workgroup per worker) lands on whatever XCD
// the dispatcher's round-robin has reached, and a 64-packet burst is ~4
// dependent round trips to host memory.  This measures one such round trip
// from every XCD: 64 one-wave blocks, lane 0 of each walks a chain of
// dependent system-scope loads through coherent host memory (and, as a
// control, through device memory), timed with s_memrealtime (100 MHz), and
// reports its XCC_ID.
//
//   xcd_lat [chain]    -> one JSON line per XCD
//
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/xcd_lat tools/xcd_lat.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void __launch_bounds__(64) lat_kernel(const uint32_t *host, const uint32_t *dev, uint32_t chain,
                                                 uint32_t mask, uint64_t *out)
{
	if (threadIdx.x != 0)
		return;
	const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20); /* XCC_ID[3:0] */
	uint32_t i = blockIdx.x * 97u & mask;
	const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
	for (uint32_t k = 0; k < chain; k++)
		i = __hip_atomic_load(&host[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & mask;
	const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
	for (uint32_t k = 0; k < chain; k++)
		i = __hip_atomic_load(&dev[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & mask;
	const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
	out[3 * blockIdx.x] = xcc;
	out[3 * blockIdx.x + 1] = t1 - t0;
	out[3 * blockIdx.x + 2] = (t2 - t1) | (uint64_t)(i == 0xFFFFFFFFu) << 63;
}

int main(int argc, char **argv)
{
	const uint32_t chain = argc > 1 ? (uint32_t)atoi(argv[1]) : 256;
	const uint32_t n = 1 << 16, mask = n - 1, nb = 64;
	std::vector<uint32_t> perm(n);
	for (uint32_t i = 0; i < n; i++)
		perm[i] = (i * 40503u + 12345u) & mask; /* odd multiplier: a permutation */
	uint32_t *host, *hostd, *dev;
	uint64_t *out;
	CHECK(hipHostMalloc((void **)&host, n * 4, hipHostMallocCoherent | hipHostMallocMapped));
	CHECK(hipHostGetDevicePointer((void **)&hostd, host, 0));
	for (uint32_t i = 0; i < n; i++)
		host[i] = perm[i];
	CHECK(hipMalloc(&dev, n * 4));
	CHECK(hipMemcpy(dev, perm.data(), n * 4, hipMemcpyHostToDevice));
	CHECK(hipMalloc(&out, nb * 3 * 8));
	std::vector<std::vector<double>> hl(16), dl(16);
	for (int rep = 0; rep < 5; rep++) {
		hipLaunchKernelGGL(lat_kernel, dim3(nb), dim3(64), 0, 0, hostd, dev, chain, mask, out);
		CHECK(hipDeviceSynchronize());
		std::vector<uint64_t> o(nb * 3);
		CHECK(hipMemcpy(o.data(), out, nb * 3 * 8, hipMemcpyDeviceToHost));
		if (rep == 0)
			continue;
		for (uint32_t b = 0; b < nb; b++) {
			const uint32_t x = (uint32_t)o[3 * b] & 15;
			hl[x].push_back(o[3 * b + 1] * 10.0 / chain);
			dl[x].push_back((o[3 * b + 2] & ~(1ull << 63)) * 10.0 / chain);
		}
	}
	for (int x = 0; x < 16; x++) {
		if (hl[x].empty())
			continue;
		std::sort(hl[x].begin(), hl[x].end());
		std::sort(dl[x].begin(), dl[x].end());
		printf("{\"xcc\": %d, \"blocks\": %zu, \"host_load_ns_p50\": %.0f, \"host_load_ns_min\": %.0f, "
		       "\"dev_load_ns_p50\": %.0f}\n", x, hl[x].size(), hl[x][hl[x].size() / 2], hl[x][0],
		       dl[x][dl[x].size() / 2]);
	}
	CHECK(hipHostFree(host));
	CHECK(hipFree(dev));
	CHECK(hipFree(out));
	return 0;
}
