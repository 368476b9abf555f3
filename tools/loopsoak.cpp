// loopsoak.cpp - soak of the persistent rx loop's stamped offsets (DESIGN.md
// §4 rxloop_kernel: a burst's offsets arrive with the poll that finds it when
// every entry carries the slot's current use stamp).  Random bursts of 1..64
// packets at random offsets into a mixed-traffic region (IPv4 TCP/UDP, IPv6,
// ARP), pushed through few slots by a tight host loop with several bursts in
// flight and random pauses, so the host's slot writes race the workers'
// polls; every verdict is compared with the batch kernel's verdict for the
// same packet (the batch path is the one the parity tests pin to the oracle).
// A torn or stale offset that passed the stamp check would show as a
// mismatch.  With a fifth argument `records` the bursts go in as stamped
// header records (GCL_LOOP_HDR_RECORDS), whose 16-B chunks the workers read
// with their polls: a torn or stale chunk that passed would show the same way.
//
//   loopsoak <bursts> <workers> <slots> <depth> [records]   -> one JSON line, exit 2 on a mismatch
//
// Build: hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/loopsoak tools/loopsoak.cpp
//         -Lcaladan_amd -lgclassify -Wl,-rpath,'$ORIGIN/../caladan_amd'
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <deque>
#include <random>
#include <utility>
#include <vector>

#include "gclassify.h"
#include "tune_env.h"

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)
#define GCHECK(x) do { int r_ = (int)(x); if (r_ < 0) { \
	fprintf(stderr, "%s:%d %s = %d\n", __FILE__, __LINE__, #x, r_); exit(1); } } while (0)

static uint64_t now_ns()
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int main(int argc, char **argv)
{
	const uint64_t nbursts = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1000000;
	const uint32_t workers = argc > 2 ? (uint32_t)atoi(argv[2]) : 4;
	const uint32_t slots = argc > 3 ? (uint32_t)atoi(argv[3]) : 4;
	const uint32_t depth = argc > 4 ? (uint32_t)atoi(argv[4]) : 4;
	const bool records = argc > 5 && !strcmp(argv[5], "records");
	const uint32_t R = 16, T = 8, stride = 128;
	const uint64_t n = 1 << 16;
	if (!nbursts || !workers || workers > 64 || slots < 2 || slots > 1024 || (slots & (slots - 1)) ||
	    !depth || depth > slots) {
		fprintf(stderr, "bad arguments\n");
		return 1;
	}

	/* the region: mixed headers generated on the GPU, copied to pinned host memory */
	uint8_t *dfr, *region;
	CHECK(hipMalloc(&dfr, n * stride));
	CHECK(hipMemset(dfr, 0, n * stride));
	struct gcl_gen_params gp = {};
	gp.workload = GCL_WL_MIXED;
	gp.nruntimes = R;
	gp.seed = 0x50A4;
	gp.n = n;
	gp.stride = stride;
	gp.world = 1;
	GCHECK(gcl_generate(&gp, dfr, nullptr, nullptr, nullptr));
	CHECK(hipHostMalloc((void **)&region, n * stride, hipHostMallocMapped));
	CHECK(hipMemcpy(region, dfr, n * stride, hipMemcpyDeviceToHost));
	CHECK(hipFree(dfr));

	struct gcl_cfg cfg = {};
	cfg.max_runtimes = R;
	cfg.hash_mode = GCL_HASH_JENKINS;
	cfg.default_olflags = GCL_F_RSS_HASH | GCL_F_IP_CKSUM_GOOD;
	struct gcl_ctx *ctx;
	GCHECK(gcl_open(0, &cfg, &ctx));
	GCHECK(tune_from_env(ctx));
	for (uint32_t r = 0; r < R; r++) {
		uint16_t act[GCL_NCPU], flow[GCL_NCPU];
		const uint16_t na = (uint16_t)(r % T + 1);
		for (uint16_t i = 0; i < na; i++)
			act[i] = (uint16_t)((i * 5) % T);
		GCHECK(gcl_steer_flows((uint16_t)T, act, na, flow));
		GCHECK(gcl_runtime_set(ctx, (uint16_t)r, gcl_runtime_ip(r), (uint16_t)T, na, flow));
	}

	/* reference verdicts: the batch kernel over every packet of the region */
	std::vector<uint64_t> offs(n);
	for (uint64_t i = 0; i < n; i++)
		offs[i] = i * stride;
	struct gcl_verdict *vref;
	CHECK(hipHostMalloc((void **)&vref, n * sizeof(*vref), hipHostMallocMapped));
	struct gcl_batch hb = {};
	hb.frames = region;
	hb.frames_len = n * stride;
	hb.stride = stride;
	hb.n = n;
	struct gcl_e2e_opts o = {};
	o.mode = GCL_E2E_ZEROCOPY;
	GCHECK(gcl_classify_host(ctx, &hb, vref, nullptr, nullptr, &o));

	struct gcl_rxloop_cfg lc = {};
	lc.slots = slots;
	lc.max_burst = 64;
	lc.workers = workers;
	lc.lifetime_ms = 600000;
	lc.region = region;
	lc.region_len = n * stride;
	lc.flags = records ? GCL_LOOP_HDR_RECORDS : 0;
	struct gcl_rxloop *loop;
	GCHECK(gcl_rxloop_start(ctx, &lc, &loop));

	std::mt19937_64 rng(12345);
	std::vector<std::vector<uint32_t>> idx(depth);
	std::vector<uint64_t> so(64);
	std::vector<gcl_verdict> got(64);
	std::deque<std::pair<int64_t, uint32_t>> inflight; /* ticket, idx slot */
	uint64_t sub = 0, done = 0, checked = 0, bad = 0, first_bad = ~0ull, slot_rr = 0;
	const uint64_t t0 = now_ns();
	while (done < nbursts) {
		while (sub < nbursts && inflight.size() < depth) {
			const uint32_t m = (rng() & 1) ? 64 : (uint32_t)(rng() % 64) + 1;
			const uint32_t k = (uint32_t)(slot_rr++ % depth);
			idx[k].resize(m);
			for (uint32_t i = 0; i < m; i++) {
				idx[k][i] = (uint32_t)(rng() % n);
				so[i] = offs[idx[k][i]];
			}
			/* now and then a pause, so some bursts land while a worker polls */
			if ((rng() & 7) == 0) {
				const uint64_t until = now_ns() + rng() % 6000;
				while (now_ns() < until)
					;
			}
			const int64_t tk = gcl_rxloop_submit(loop, m, so.data(), nullptr, nullptr, nullptr, nullptr);
			GCHECK(tk);
			inflight.emplace_back(tk, k);
			sub++;
		}
		const auto [tk, k] = inflight.front();
		inflight.pop_front();
		const uint32_t m = (uint32_t)idx[k].size();
		GCHECK(gcl_rxloop_wait(loop, tk, got.data(), 2000000000ull));
		for (uint32_t i = 0; i < m; i++) {
			if (memcmp(&got[i], &vref[idx[k][i]], sizeof(gcl_verdict))) {
				if (!bad)
					first_bad = done;
				bad++;
			}
		}
		checked += m;
		done++;
	}
	const double sec = (now_ns() - t0) * 1e-9;
	uint64_t ps[3] = {0, 0, 0};
	gcl_rxloop_poll_stats(loop, ps);
	gcl_rxloop_stop(loop);
	printf("{\"bursts\": %llu, \"workers\": %u, \"slots\": %u, \"depth\": %u, \"records\": %s, "
	       "\"packets_checked\": %llu, "
	       "\"mismatches\": %llu, \"first_mismatch_burst\": %lld, \"seconds\": %.1f, \"mpps\": %.1f, "
	       "\"bursts_early\": %llu, \"bursts_stale\": %llu, \"bursts_late\": %llu}\n",
	       (unsigned long long)nbursts, workers, slots, depth, records ? "true" : "false",
	       (unsigned long long)checked,
	       (unsigned long long)bad, bad ? (long long)first_bad : -1LL, sec, checked / sec / 1e6,
	       (unsigned long long)ps[0], (unsigned long long)ps[1], (unsigned long long)ps[2]);
	gcl_close(ctx);
	CHECK(hipHostFree(vref));
	CHECK(hipHostFree(region));
	return bad ? 2 : 0;
}
