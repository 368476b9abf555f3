/*
 * gcl_device.h - device-side building blocks shared by the classify and
 * generator kernels (gfx950).  Integer-only: lookup3, Toeplitz, header field
 * extraction from little-endian dwords, Lemire fastmod.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gcl {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

/* 16-byte streaming load that does not keep the line (read-once frames) */
__device__ __forceinline__ uint4 load16_nt(const void *p)
{
	u32x4 v = __builtin_nontemporal_load((const u32x4 *)p);
	return make_uint4(v.x, v.y, v.z, v.w);
}

/* System-scope (sc0 sc1) accesses for host memory the CPU rewrites while a
 * persistent kernel runs (the rx loop's burst slots, table images and the
 * frames of a recycled mbuf pool): they miss in every GPU cache, so a line
 * cached by an earlier burst can never be returned stale. */
__device__ __forceinline__ uint32_t ld_sys32(const void *p)
{
	return __hip_atomic_load((const uint32_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint64_t ld_sys64(const void *p)
{
	return __hip_atomic_load((const uint64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_sys32(void *p, uint32_t v)
{
	__hip_atomic_store((uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/* byte @a of a host region of @len bytes, system scope; 0 past the end */
__device__ __forceinline__ uint8_t byte_sys(const uint8_t *base, uint64_t len, uint64_t a)
{
	return a < len ? (uint8_t)(ld_sys32(base + (a & ~3ull)) >> (8 * (a & 3))) : 0;
}

/* 16 bytes at byte offset @a (any alignment) of a host region of @len bytes,
 * system scope, bytes past the end read as 0: the dwords covering the range,
 * funnel-shifted.  A dword that straddles @len lies inside the page that
 * holds byte len-1, so loading it whole is safe. */
__device__ __forceinline__ uint4 load16_sys(const uint8_t *base, uint64_t len, uint64_t a)
{
	const uint64_t a0 = a & ~3ull;
	const uint32_t sh = (uint32_t)(a & 3);
	uint32_t w[5];
#pragma unroll
	for (int i = 0; i < 5; i++) {
		const uint64_t q = a0 + 4 * (uint64_t)i;
		w[i] = (q < len && (i < 4 || sh)) ? ld_sys32(base + q) : 0;
	}
	uint32_t o[4];
#pragma unroll
	for (int i = 0; i < 4; i++)
		o[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
	if (a + 16 > len) {
#pragma unroll
		for (int b = 0; b < 16; b++)
			if (a + b >= len)
				o[b >> 2] &= ~(0xFFu << (8 * (b & 3)));
	}
	return make_uint4(o[0], o[1], o[2], o[3]);
}

/* Buffer-op cache policy sc0 | sc1: system scope, misses every GPU cache. */
constexpr int kSysAux = 17;

/* Buffer descriptor over host memory (< 4 GiB) the persistent loop reads or
 * writes; build it from wave-uniform values only.  The base and size go
 * through readfirstlane, so the descriptor sits in scalar registers even where
 * the compiler cannot prove them uniform (a loop variable, a value read from
 * LDS): otherwise every buffer access gets a readfirstlane waterfall loop. */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t host_rsrc(const void *p, uint64_t bytes)
{
	const uint64_t a = (uint64_t)(uintptr_t)p;
	const uint64_t u = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32 |
	                   (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
	const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0xFFFFFFFFull ? bytes : 0xFFFFFFFFull));
	return __builtin_amdgcn_make_buffer_rsrc((void *)(uintptr_t)u, 0, n, 0x00020000);
}

/* load16_sys as one 16-B (or two 8-B) system-scope buffer loads when the
 * range is aligned and inside a region below 4 GiB: one PCIe read per lane
 * instead of five dword reads */
__device__ __forceinline__ uint4 load16_host(__amdgpu_buffer_rsrc_t rs, const uint8_t *base,
                                             uint64_t len, uint64_t a)
{
	if (a + 16 <= len && len <= 0xFFFFFFFFull) {
		if (!(a & 15)) {
			const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)a, 0, kSysAux);
			return make_uint4(v[0], v[1], v[2], v[3]);
		}
		if (!(a & 7)) {
			const auto x = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)a, 0, kSysAux);
			const auto y = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)a + 8, 0, kSysAux);
			return make_uint4(x[0], x[1], y[0], y[1]);
		}
	}
	return load16_sys(base, len, a);
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int k)
{
	return (x << k) | (x >> (32 - k));
}

/* lookup3 mix / final (base/jenkins_hash.c:79-87, :114-123) */
__device__ __forceinline__ void jmix(uint32_t &a, uint32_t &b, uint32_t &c)
{
	a -= c; a ^= rotl(c, 4);  c += b;
	b -= a; b ^= rotl(a, 6);  a += c;
	c -= b; c ^= rotl(b, 8);  b += a;
	a -= c; a ^= rotl(c, 16); c += b;
	b -= a; b ^= rotl(a, 19); a += c;
	c -= b; c ^= rotl(b, 4);  b += a;
}

__device__ __forceinline__ void jfinal(uint32_t &a, uint32_t &b, uint32_t &c)
{
	c ^= b; c -= rotl(b, 14);
	a ^= c; a -= rotl(c, 11);
	b ^= a; b -= rotl(a, 25);
	c ^= b; c -= rotl(b, 16);
	a ^= c; a -= rotl(c, 4);
	b ^= a; b -= rotl(a, 14);
	c ^= b; c -= rotl(b, 24);
}

/* jenkins_hash(&ip, 4): the rte_jhash key of dp.ip_to_proc (dp_clients.c:360) */
__device__ __forceinline__ uint32_t jhash_u32(uint32_t ip, uint32_t initval = 0)
{
	uint32_t a = 0xdeadbeefu + 4u + initval, b = a, c = a;
	a += ip;
	jfinal(a, b, c);
	return c;
}

/* jenkins_hash over the 13-byte flow key {saddr, daddr, dport, sport, proto}
 * (host-order fields, little-endian bytes): one 12-byte block + 1 tail byte. */
__device__ __forceinline__ uint32_t jhash_5tuple(uint32_t saddr, uint32_t daddr,
                                                 uint32_t sport, uint32_t dport,
                                                 uint32_t proto)
{
	uint32_t a = 0xdeadbeefu + 13u, b = a, c = a;
	a += saddr;
	b += daddr;
	c += dport | (sport << 16);
	jmix(a, b, c);
	a += proto;
	jfinal(a, b, c);
	return c;
}

__device__ __forceinline__ uint32_t bswap16(uint32_t x)
{
	return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
	return __builtin_bswap32(x);
}

/* bytes [2..5] of the 8-byte little-endian pair (lo, hi) */
__device__ __forceinline__ uint32_t mid32(uint32_t lo, uint32_t hi)
{
	return __builtin_amdgcn_alignbit(hi, lo, 16);
}

/* n % d for d in [1, 2^16) with M = ceil(2^64 / d) (0 for d == 1). */
__device__ __forceinline__ uint32_t fastmod(uint32_t n, uint64_t M, uint32_t d)
{
	uint64_t low = M * (uint64_t)n;
	uint32_t lo = (uint32_t)low, hi = (uint32_t)(low >> 32);
	uint64_t t = (uint64_t)hi * d + __umulhi(lo, d);
	return (uint32_t)(t >> 32);
}

/* splitmix64 output function at stream position x (generator) */
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t rw(uint64_t seed, uint64_t g, uint64_t k)
{
	return mix64(seed + (g * 8 + k + 1) * 0x9E3779B97F4A7C15ull);
}

} // namespace gcl
