/*
 * tune_env.h - tools only: a struct gcl_tune filled from GCL_TUNE_* variables
 * in the tool's own environment, so that A/B recipes (tools/runs/) can set
 * the library's overrides per run.  The library itself reads no environment
 * (gcl_ctx_tune, include/gclassify.h).
 *
 *   GCL_TUNE_TABLES, _DEPTH, _THREADS, _GRID, _BLOCKS_PER_CU, _DEFER,
 *   _PAIR_LEAN, _TILE_LEAN, _LOOP64, _LOOP_LEAN, _LOOP_SPEC, _LOOP_PREFETCH,
 *   _REC_PREFETCH, _SLOT_PREFETCH, _VSTAGE, _PAIR_I32  integers
 *   GCL_TUNE_LOOP_PHASE  "max[,up[,down]]" (ticks; up 16, down 1 by default)
 *   GCL_TUNE_LOOP_T0, GCL_TUNE_DEBUG
 */
#pragma once

#include <stdio.h>
#include <stdlib.h>

#include "gclassify.h"

static inline void tune_env_int(const char *name, int32_t *f)
{
	const char *e = getenv(name);
	if (e && *e)
		*f = (int32_t)atoi(e);
}

/* gcl_ctx_tune(@ctx) with the environment's overrides; 0 or -errno */
static inline int tune_from_env(struct gcl_ctx *ctx)
{
	struct gcl_tune t;
	gcl_tune_init(&t);
	tune_env_int("GCL_TUNE_TABLES", &t.tables);
	tune_env_int("GCL_TUNE_DEPTH", &t.depth);
	tune_env_int("GCL_TUNE_THREADS", &t.threads);
	tune_env_int("GCL_TUNE_GRID", &t.grid);
	tune_env_int("GCL_TUNE_BLOCKS_PER_CU", &t.blocks_per_cu);
	tune_env_int("GCL_TUNE_DEFER", &t.defer);
	tune_env_int("GCL_TUNE_PAIR_LEAN", &t.pair_lean);
	tune_env_int("GCL_TUNE_LOOP64", &t.loop64);
	tune_env_int("GCL_TUNE_LOOP_LEAN", &t.loop_lean);
	tune_env_int("GCL_TUNE_LOOP_SPEC", &t.loop_spec);
	tune_env_int("GCL_TUNE_LOOP_PREFETCH", &t.loop_prefetch);
	tune_env_int("GCL_TUNE_TILE_LEAN", &t.tile_lean);
	tune_env_int("GCL_TUNE_REC_PREFETCH", &t.rec_prefetch);
	tune_env_int("GCL_TUNE_SLOT_PREFETCH", &t.slot_prefetch);
	tune_env_int("GCL_TUNE_VSTAGE", &t.vstage);
	tune_env_int("GCL_TUNE_PAIR_I32", &t.pair_i32);
	if (const char *e = getenv("GCL_TUNE_LOOP_PHASE")) {
		unsigned m = 0, u = 16, d = 1;
		if (sscanf(e, "%u,%u,%u", &m, &u, &d) >= 1) {
			t.loop_phase_max = (int32_t)m;
			t.loop_phase_up = (int32_t)u;
			t.loop_phase_down = (int32_t)d;
		}
	}
	if (const char *e = getenv("GCL_TUNE_LOOP_T0"))
		t.loop_t0 = strtoull(e, nullptr, 0);
	if (const char *e = getenv("GCL_TUNE_DEBUG"))
		t.debug = atoi(e) != 0;
	const int r = gcl_ctx_tune(ctx, &t);
	if (r)
		fprintf(stderr, "tune_from_env: gcl_ctx_tune refused the GCL_TUNE_* settings (%d)\n", r);
	return r;
}
