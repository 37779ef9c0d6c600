/*
 * sg_ctx.hpp - host-side context shared by the C-ABI translation units (sg_api.cpp,
 * sg_register.hip): one entry per device with its HIP stream, events and HBM workspaces.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string>
#include <vector>
#include "../../include/sirilgpu.h"

#define SG_LIT_THREADS 65536

struct SgBuf {
	void *p = nullptr;
	size_t size = 0;
};

struct SgDevice {
	int id = 0;
	hipStream_t stream = nullptr;
	hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
	SgBuf flag_list, flag_map, flag_count, rej, sum_buf, maxim, shifts, norm, tables, scratch, frames, out, stats_buf;
	/* registration workspaces (sg_register.hip) */
	SgBuf reg_sel, reg_spec, reg_work, reg_tw, reg_best, reg_qbuf, reg_qacc;
	SgBuf redo;	/* redo list of the histogram stacking path */
	SgBuf zeros;	/* zero page for out-of-frame sample loads */
	uint16_t *pinned[2] = {nullptr, nullptr};
	size_t pinned_size = 0;
	/* file decode path (sg_io.hip): pinned staging of raw frames, device raw buffers */
	void *io_stage[2] = {nullptr, nullptr};
	size_t io_stage_size = 0;
	SgBuf io_raw, io_bad;
	SgBuf warp_tab;		/* sg_warp.hip interpolation table */
	int warp_tab_interp = -1;
	hipEvent_t io_ev[2] = {nullptr, nullptr};
	int io_ev_used[2] = {0, 0};
};

struct sg_ctx {
	std::vector<SgDevice> dev;
	std::string err;
	sg_stack_stats stats;
};

static inline int set_err(sg_ctx *ctx, int code, const char *fmt, const char *a = "", long b = 0) {
	char buf[512];
	snprintf(buf, sizeof buf, fmt, a, b);
	if (ctx)
		ctx->err = buf;
	return code;
}

#define HIPCHK(call)                                                                       \
	do {                                                                               \
		hipError_t _e = (call);                                                    \
		if (_e != hipSuccess)                                                      \
			return set_err(ctx, SG_ERR_DEVICE, "HIP error %s at line %ld",     \
					hipGetErrorString(_e), (long)__LINE__);            \
	} while (0)

static inline hipError_t ensure(SgBuf &b, size_t bytes) {
	if (b.size >= bytes && b.p)
		return hipSuccess;
	if (b.p)
		(void)hipFree(b.p);
	b.p = nullptr;
	b.size = 0;
	size_t sz = bytes ? bytes : 16;
	hipError_t e = hipMalloc(&b.p, sz);
	if (e == hipSuccess)
		b.size = sz;
	return e;
}

