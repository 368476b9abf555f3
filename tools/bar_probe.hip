// bar_probe.hip - can the host write device memory through the PCIe BAR, and
// does a doorbell there beat one in host memory for the persistent loop?
//
// 1. For hipMalloc, fine-grained and uncached device allocations: can the CPU
//    read and write the device pointer (guarded by a SIGSEGV handler)?
// 2. Ping-pong, one wave: the host rings doorbell i (optionally after writing
//    a 4 KiB burst next to it), the GPU polls the doorbell with system-scope
//    loads, reads the burst, and answers with a system-scope store into
//    coherent host memory; the host spins on the answer.  Doorbell + burst in
//    host memory (the loop's current design) vs in device memory (BAR).
//
//   bar_probe [iters]    -> JSON lines
//
// The kernel leaves after @iters rounds or 2 s (s_memrealtime, 100 MHz),
// whichever comes first, and the host gives up after 2 s too.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/bar_probe tools/bar_probe.hip
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }

static uint64_t now_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

/* host access to @p: 0 ok, 1 fault on write, 2 fault on read, 3 wrong value */
static int host_access(volatile uint32_t *p)
{
	struct sigaction sa = {}, old;
	sa.sa_handler = on_segv;
	sigaction(SIGSEGV, &sa, &old);
	sigaction(SIGBUS, &sa, nullptr);
	int r = 0;
	if (sigsetjmp(jb, 1)) {
		r = r ? r : 9;
	} else {
		r = 1;
		p[0] = 0x12345678u;
		r = 2;
		const uint32_t v = p[0];
		r = v == 0x12345678u ? 0 : 3;
	}
	sigaction(SIGSEGV, &old, nullptr);
	sigaction(SIGBUS, &old, nullptr);
	return r;
}

__device__ __forceinline__ uint32_t ld_sys(const uint32_t *p)
{
	return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys(uint32_t *p, uint32_t v)
{
	__hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* @bell: doorbell (u32) followed by a @burst-byte payload; @reply: host memory */
__global__ void __launch_bounds__(64) pong_kernel(const uint32_t *bell, uint32_t burst, uint32_t *reply,
                                                  uint32_t iters)
{
	const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 200000000ull; /* 2 s */
	__shared__ uint32_t s_go;
	for (uint32_t i = 1; i <= iters; i++) {
		if (threadIdx.x == 0) {
			uint32_t go = 0;
			for (;;) {
				if (ld_sys(bell) == i) {
					go = 1;
					break;
				}
				if (__builtin_amdgcn_s_memrealtime() > t_end)
					break;
				__builtin_amdgcn_s_sleep(1);
			}
			s_go = go;
		}
		__syncthreads();
		if (!s_go)
			return;
		uint32_t acc = 0;
		for (uint32_t o = 4 * threadIdx.x; o < burst; o += 4 * 64)
			acc ^= ld_sys((const uint32_t *)((const uint8_t *)bell + 64 + o));
		for (int off = 32; off > 0; off >>= 1)
			acc ^= __shfl_xor(acc, off);
		if (threadIdx.x == 0)
			st_sys(&reply[0], i ^ (acc & 0)); /* acc keeps the loads alive */
		if (threadIdx.x == 0 && acc == 0xDEADBEEFu)
			st_sys(&reply[1], acc);
		__syncthreads();
	}
}

static void pingpong(const char *where, uint32_t *bell_host_view, const uint32_t *bell_dev, uint32_t burst,
                     uint32_t *reply, uint32_t iters)
{
	volatile uint32_t *hb = bell_host_view;
	volatile uint32_t *rp = reply;
	hb[0] = 0;
	rp[0] = 0;
	__atomic_thread_fence(__ATOMIC_SEQ_CST);
	hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, 0, bell_dev, burst, reply, iters);
	std::vector<double> lat;
	std::vector<uint32_t> payload(burst / 4 + 1, 0x5A5A5A5Au);
	bool ok = true;
	for (uint32_t i = 1; i <= iters && ok; i++) {
		const uint64_t t0 = now_ns();
		if (burst)
			memcpy((void *)(hb + 16), payload.data(), burst);
		__atomic_thread_fence(__ATOMIC_SEQ_CST);
		hb[0] = i;
		__atomic_thread_fence(__ATOMIC_SEQ_CST);
		while (rp[0] != i) {
			if (now_ns() - t0 > 2000000000ull) {
				ok = false;
				break;
			}
			__builtin_ia32_pause();
		}
		lat.push_back((now_ns() - t0) * 1e-3);
	}
	CHECK(hipDeviceSynchronize());
	std::sort(lat.begin(), lat.end());
	printf("{\"pingpong\": \"%s\", \"burst_bytes\": %u, \"iters\": %u, \"ok\": %s, \"p50_us\": %.2f, "
	       "\"p99_us\": %.2f, \"min_us\": %.2f}\n", where, burst, (unsigned)lat.size(), ok ? "true" : "false",
	       lat[lat.size() / 2], lat[lat.size() * 99 / 100], lat[0]);
	fflush(stdout);
}

int main(int argc, char **argv)
{
	const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
	int lb = 0;
	CHECK(hipDeviceGetAttribute(&lb, hipDeviceAttributeIsLargeBar, 0));
	printf("{\"large_bar\": %d}\n", lb);

	struct Kind { const char *name; unsigned flags; bool ext; } kinds[] = {
		{"hipMalloc", 0, false},
		{"fine_grained", hipDeviceMallocFinegrained, true},
		{"uncached", hipDeviceMallocUncached, true},
	};
	void *dev[3] = {};
	int acc[3] = {};
	for (int k = 0; k < 3; k++) {
		if (kinds[k].ext)
			CHECK(hipExtMallocWithFlags(&dev[k], 1 << 20, kinds[k].flags));
		else
			CHECK(hipMalloc(&dev[k], 1 << 20));
		acc[k] = host_access((volatile uint32_t *)dev[k]);
		printf("{\"alloc\": \"%s\", \"ptr\": \"%p\", \"host_access\": %d}\n", kinds[k].name, dev[k], acc[k]);
		fflush(stdout);
	}

	uint32_t *hbell, *reply;
	CHECK(hipHostMalloc((void **)&hbell, 1 << 20, hipHostMallocCoherent | hipHostMallocMapped));
	CHECK(hipHostMalloc((void **)&reply, 4096, hipHostMallocCoherent | hipHostMallocMapped));
	uint32_t *hbell_dev, *reply_dev;
	CHECK(hipHostGetDevicePointer((void **)&hbell_dev, hbell, 0));
	CHECK(hipHostGetDevicePointer((void **)&reply_dev, reply, 0));
	for (uint32_t burst : {0u, 4096u}) {
		pingpong("host_memory", hbell, hbell_dev, burst, reply_dev, iters);
		for (int k = 1; k < 3; k++)
			if (acc[k] == 0) {
				char name[64];
				snprintf(name, sizeof(name), "device_%s", kinds[k].name);
				pingpong(name, (uint32_t *)dev[k], (const uint32_t *)dev[k], burst, reply_dev, iters);
			}
	}
	for (int k = 0; k < 3; k++)
		CHECK(hipFree(dev[k]));
	CHECK(hipHostFree(hbell));
	CHECK(hipHostFree(reply));
	return 0;
}
