/*
 * pinning.h - tools only: CPU choice for the host threads of the pipeline
 * tools (tools/rxpipe, tools/cpupipe): the dataplane core is pinned as the
 * iokernel pins its lcore (iokernel/dpdk.c:276-280), to the idlest physical
 * core near the GPU; helper threads (the NIC emulation) to other idle cores.
 */
#pragma once

#include <hip/hip_runtime.h>
#include <ctype.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <unistd.h>

#include <algorithm>
#include <utility>
#include <vector>

/* the process's affinity mask before pin_near_gpu narrowed this thread's
 * (threads created later inherit the narrowed one) */
static cpu_set_t g_allowed;
static bool g_allowed_set = false;

/* Idle jiffies of every CPU from /proc/stat (index = CPU), empty on error. */
static inline std::vector<uint64_t> cpu_idle()
{
	std::vector<uint64_t> idle;
	FILE *f = fopen("/proc/stat", "r");
	if (!f)
		return idle;
	char line[512];
	while (fgets(line, sizeof(line), f)) {
		int cpu;
		unsigned long long v[8] = {0};
		if (strncmp(line, "cpu", 3) || !isdigit((unsigned char)line[3]))
			continue;
		if (sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, &v[0], &v[1], &v[2],
		           &v[3], &v[4], &v[5], &v[6], &v[7]) < 5 || cpu < 0 || cpu >= CPU_SETSIZE)
			continue;
		if ((size_t)cpu >= idle.size())
			idle.resize(cpu + 1, 0);
		idle[cpu] = v[3] + v[4]; /* idle + iowait */
	}
	fclose(f);
	return idle;
}

/* The SMT siblings of @cpu (sysfs thread_siblings_list), @cpu included. */
static inline std::vector<int> siblings(int cpu)
{
	std::vector<int> out;
	char path[128];
	snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/topology/thread_siblings_list", cpu);
	FILE *f = fopen(path, "r");
	if (f) {
		int lo, hi;
		char sep;
		while (fscanf(f, "%d", &lo) == 1) {
			hi = lo;
			if (fscanf(f, "%c", &sep) == 1 && sep == '-' && fscanf(f, "%d", &hi) == 1)
				(void)fscanf(f, "%c", &sep);
			for (int c = lo; c <= hi; c++)
				out.push_back(c);
		}
		fclose(f);
	}
	if (out.empty())
		out.push_back(cpu);
	return out;
}

/* Pin this thread to one CPU, as the iokernel pins its dataplane lcore
 * (iokernel/dpdk.c:276-280): among the CPUs of our affinity mask local to
 * GPU @dev's PCIe node (sysfs local_cpulist; else the whole mask), the one
 * whose physical core was idlest over 100 ms -- the CPU and its SMT
 * siblings, from /proc/stat -- highest number first on a tie, away from
 * CPU 0's housekeeping.  On a host shared with other jobs a fixed pick (the
 * last local CPU, before) could land on a busy core and swing the rate 3x
 * from run to run.  RXPIPE_PIN=0 in the environment leaves the thread
 * unpinned.  Returns the CPU, or -1. */
static inline int pin_near_gpu(int dev)
{
	const char *env = getenv("RXPIPE_PIN");
	if (env && !strcmp(env, "0"))
		return -1;
	cpu_set_t allowed;
	if (sched_getaffinity(0, sizeof(allowed), &allowed))
		return -1;
	if (!g_allowed_set) {
		g_allowed = allowed;
		g_allowed_set = true;
	}
	std::vector<int> cand;
	char bus[64] = {0}, path[160];
	if (hipDeviceGetPCIBusId(bus, sizeof(bus), dev) == hipSuccess) {
		for (char *c = bus; *c; c++)
			*c = (char)tolower(*c);
		snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/local_cpulist", bus);
		FILE *f = fopen(path, "r");
		if (f) {
			int lo, hi;
			char sep;
			while (fscanf(f, "%d", &lo) == 1) {
				hi = lo;
				if (fscanf(f, "%c", &sep) == 1 && sep == '-' && fscanf(f, "%d", &hi) == 1)
					(void)fscanf(f, "%c", &sep);
				for (int cpu = lo; cpu <= hi; cpu++)
					if (cpu < CPU_SETSIZE && CPU_ISSET(cpu, &allowed))
						cand.push_back(cpu);
			}
			fclose(f);
		}
	}
	if (cand.empty())
		for (int cpu = 0; cpu < CPU_SETSIZE; cpu++)
			if (CPU_ISSET(cpu, &allowed))
				cand.push_back(cpu);
	if (cand.empty())
		return -1;
	int pick = cand.back();
	const std::vector<uint64_t> a = cpu_idle();
	struct timespec ts = {0, 100 * 1000 * 1000};
	nanosleep(&ts, nullptr);
	const std::vector<uint64_t> b = cpu_idle();
	if (!a.empty() && a.size() == b.size()) {
		int64_t best = -1;
		for (int cpu : cand) {
			int64_t score = 0;
			for (int sib : siblings(cpu))
				if ((size_t)sib < a.size())
					score += (int64_t)(b[sib] - a[sib]);
			if (score >= best) {
				best = score;
				pick = cpu;
			}
		}
	}
	cpu_set_t one;
	CPU_ZERO(&one);
	CPU_SET(pick, &one);
	return sched_setaffinity(0, sizeof(one), &one) ? -1 : pick;
}


/* @k CPUs of our affinity mask for helper threads (the NIC emulation): the
 * idlest physical cores over 100 ms, one CPU per core, none sharing a core
 * with @busy (the dataplane's CPU, or -1); fewer when the mask has fewer. */
static inline std::vector<int> pick_other_cpus(uint32_t k, int busy)
{
	std::vector<int> out;
	cpu_set_t allowed;
	if (g_allowed_set) /* the mask before the dataplane thread was pinned */
		allowed = g_allowed;
	else if (sched_getaffinity(0, sizeof(allowed), &allowed))
		return out;
	std::vector<int> skip = busy >= 0 ? siblings(busy) : std::vector<int>();
	const std::vector<uint64_t> a = cpu_idle();
	struct timespec ts = {0, 100 * 1000 * 1000};
	nanosleep(&ts, nullptr);
	const std::vector<uint64_t> b = cpu_idle();
	std::vector<std::pair<int64_t, int>> cand;
	std::vector<char> seen(CPU_SETSIZE, 0);
	for (int cpu = 0; cpu < CPU_SETSIZE; cpu++) {
		if (!CPU_ISSET(cpu, &allowed) || seen[cpu] || std::find(skip.begin(), skip.end(), cpu) != skip.end())
			continue;
		int64_t score = 0;
		for (int sib : siblings(cpu)) {
			if (sib < CPU_SETSIZE)
				seen[sib] = 1;
			if ((size_t)sib < a.size() && a.size() == b.size())
				score += (int64_t)(b[sib] - a[sib]);
		}
		cand.push_back({-score, cpu});
	}
	std::sort(cand.begin(), cand.end());
	for (size_t i = 0; i < cand.size() && out.size() < k; i++)
		out.push_back(cand[i].second);
	return out;
}
