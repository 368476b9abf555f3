/*
 * gcl_gen.hip - the synthetic traffic generator (gcl_generate): packet g of
 * the global stream is a pure function of (seed, g) through splitmix64, so
 * every rank and the CPU oracle (oracle/orc.c) produce identical bytes.  Test
 * and bench infrastructure beside the rx path, not part of it.
 */
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gclassify.h"
#include "gcl_device.h"

namespace gclk {

/* ------------------------------------------------------------------------
 * Synthetic generator kernel: one lane per packet writes its 64-B header.
 */
struct Hdr {
	uint32_t w[16];
	__device__ void b8(int o, uint32_t v) { w[o >> 2] |= (v & 0xFF) << ((o & 3) * 8); }
	__device__ void b16(int o, uint32_t v) { b8(o, v >> 8); b8(o + 1, v); }
	__device__ void b32(int o, uint32_t v) { b16(o, v >> 16); b16(o + 2, v); }
};

__device__ __forceinline__ void gen_eth(Hdr &h, uint64_t srcbits, uint32_t et)
{
	h.b8(0, 0x02); h.b8(5, 0x01); /* dst 02:00:00:00:00:01 */
	h.b8(6, 0x02);
	h.b32(8, (uint32_t)srcbits);
	h.b16(12, et);
}

__device__ __forceinline__ void gen_ipv4(Hdr &h, uint32_t totlen, uint32_t id,
                                         uint32_t proto, uint32_t saddr, uint32_t daddr)
{
	h.b8(14, 0x45);
	h.b16(16, totlen);
	h.b16(18, id);
	h.b16(20, 0x4000);
	h.b8(22, 64);
	h.b8(23, proto);
	h.b32(26, saddr);
	h.b32(30, daddr);
	uint32_t s = 0x4500 + (totlen & 0xFFFF) + (id & 0xFFFF) + 0x4000 + (64u << 8 | proto) +
	             (saddr >> 16) + (saddr & 0xFFFF) + (daddr >> 16) + (daddr & 0xFFFF);
	while (s >> 16)
		s = (s & 0xFFFF) + (s >> 16);
	h.b16(24, ~s & 0xFFFF);
}

struct GParams {
	uint32_t workload, nruntimes;
	uint64_t seed, n, stride;
	uint32_t rank, world;
	uint64_t shard_block;
	const uint64_t *zipf;
	uint32_t nflows;
	uint8_t *frames;
	uint8_t *olflags;
	uint32_t *rss;
	uint16_t *pkt_len;
};

__device__ __forceinline__ uint32_t runtime_ip(uint32_t r) { return 0x0A000000u + r + 1; }

__global__ void __launch_bounds__(256) generate_kernel(GParams p)
{
	uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (j >= p.n)
		return;
	uint64_t g = j;
	if (p.shard_block && p.world > 1)
		g = ((j / p.shard_block) * p.world + p.rank) * p.shard_block + j % p.shard_block;
	const uint64_t r0 = gcl::rw(p.seed, g, 0), r1 = gcl::rw(p.seed, g, 1);
	uint32_t fl = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	uint32_t len = 64;
	Hdr h;
#pragma unroll
	for (int i = 0; i < 16; i++)
		h.w[i] = 0;

	if (p.workload == GCL_WL_UDP64) {
		uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p.nruntimes) >> 32);
		gen_eth(h, r1 >> 32, GCL_ETHTYPE_IP);
		gen_ipv4(h, 50, (uint32_t)(r1 >> 16) & 0xFFFF, 17, (uint32_t)r0, runtime_ip(rt));
		h.b16(34, (uint32_t)(r0 >> 32) & 0xFFFF);
		h.b16(36, (uint32_t)(r0 >> 48));
		h.b16(38, 30);
	} else if (p.workload == GCL_WL_TCP1500_ZIPF) {
		uint32_t lo = 0, hi = p.nflows - 1;
		while (lo < hi) {
			uint32_t mid = lo + (hi - lo) / 2;
			if (r0 < p.zipf[mid])
				hi = mid;
			else
				lo = mid + 1;
		}
		const uint32_t flow = lo;
		const uint64_t fr = gcl::rw(p.seed ^ 0xF10F10F10F10F10Full, flow, 0);
		const uint32_t rt = flow % p.nruntimes;
		gen_eth(h, fr >> 16, GCL_ETHTYPE_IP);
		gen_ipv4(h, 1486, (uint32_t)r1 & 0xFFFF, 6, (uint32_t)fr, runtime_ip(rt));
		h.b16(34, (uint32_t)(fr >> 32) & 0xFFFF);
		h.b16(36, (uint32_t)(fr >> 48));
		h.b32(38, (uint32_t)(r1 >> 32));
		h.b8(46, 0x50);
		h.b8(47, 0x10);
		h.b16(48, 0xFFFF);
		len = 1500;
	} else {
		const uint64_t r2 = gcl::rw(p.seed, g, 2);
		const uint32_t kind = (uint32_t)r0 % 100;
		const uint32_t rt = (uint32_t)(((uint64_t)(uint32_t)r1 * p.nruntimes) >> 32);
		bool unreg = (uint32_t)(r0 >> 40) % 20 == 0;
		uint32_t dst = unreg ? (0xC0A80000u | (uint32_t)(r1 >> 48)) : runtime_ip(rt);
		if (kind < 70) {
			len = 64 + (uint32_t)(r1 >> 32) % (9014 - 64 + 1);
			uint32_t proto = (r0 >> 32) & 1 ? 6 : 17;
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_IP);
			gen_ipv4(h, len - 14, (uint32_t)r2 & 0xFFFF, proto, (uint32_t)r2, dst);
			h.b16(34, (uint32_t)(r2 >> 32) & 0xFFFF);
			h.b16(36, (uint32_t)(r2 >> 48));
		} else if (kind < 90) {
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_IPV6);
			h.b8(14, 0x60);
			h.b16(18, (uint32_t)(r1 >> 32) & 0x1FFF);
			h.b8(20, 17);
			h.b8(21, 64);
			h.b32(22, (uint32_t)r2);
			h.b32(38, dst);
			fl = 0;
			len = 54 + ((uint32_t)(r1 >> 32) & 0x1FFF);
			len = len < 60 ? 60 : len;
		} else {
			unreg = (uint32_t)(r0 >> 40) % 10 == 0;
			dst = unreg ? (0xC0A80000u | (uint32_t)(r1 >> 48)) : runtime_ip(rt);
			gen_eth(h, r2 >> 8, GCL_ETHTYPE_ARP);
			h.b16(14, 1);
			h.b16(16, 0x0800);
			h.b8(18, 6);
			h.b8(19, 4);
			h.b16(20, (r0 >> 33) & 1 ? GCL_ARP_OP_REPLY : GCL_ARP_OP_REQUEST);
			h.b32(24, (uint32_t)(r2 >> 16));
			h.b32(28, (uint32_t)r2);
			h.b32(38, dst);
			fl = 0;
			len = 60;
		}
	}
	uint4 *dst4 = (uint4 *)(p.frames + j * p.stride);
#pragma unroll
	for (int i = 0; i < 4; i++)
		dst4[i] = make_uint4(h.w[4 * i], h.w[4 * i + 1], h.w[4 * i + 2], h.w[4 * i + 3]);
	if (p.olflags)
		p.olflags[j] = (uint8_t)fl;
	if (p.rss)
		p.rss[j] = (uint32_t)gcl::rw(p.seed, g, 3);
	if (p.pkt_len)
		p.pkt_len[j] = (uint16_t)len;
}

} // namespace gclk

using namespace gclk;

extern "C" int gcl_generate(const struct gcl_gen_params *p, uint8_t *frames, uint8_t *olflags,
                            uint32_t *rss, void *hip_stream)
{
	if (!p || !frames || p->stride < 64 || (p->stride & 15) || p->nruntimes == 0 ||
	    p->workload > GCL_WL_MIXED)
		return -EINVAL;
	if (p->workload == GCL_WL_TCP1500_ZIPF && (!p->zipf_cdf || !p->nflows))
		return -EINVAL;
	if (p->n == 0)
		return 0;
	GParams g = {};
	g.workload = p->workload;
	g.nruntimes = p->nruntimes;
	g.seed = p->seed;
	g.n = p->n;
	g.stride = p->stride;
	g.rank = p->rank;
	g.world = p->world;
	g.shard_block = p->shard_block;
	g.zipf = p->zipf_cdf;
	g.nflows = p->nflows;
	g.frames = frames;
	g.olflags = olflags;
	g.rss = rss;
	g.pkt_len = p->pkt_len;
	uint64_t blocks = (p->n + 255) / 256;
	hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(256), 0,
	                   (hipStream_t)hip_stream, g);
	return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

