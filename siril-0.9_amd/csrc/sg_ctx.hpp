/*
 * sg_ctx.hpp - host-side context shared by the C-ABI translation units (sg_api.cpp,
 * sg_register.hip): one entry per device with its HIP stream, events and HBM workspaces.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <mutex>
#include <string>
#include <vector>
#include "../../include/sirilgpu.h"

#define SG_LIT_THREADS 65536

struct SgBuf {
	void *p = nullptr;
	size_t size = 0;
};

/* one host reader of the host-pull path (sg_stack_u16): it pulls top-down row chunks through the
 * region callback into its pinned buffers, copies them on its own stream to a device staging
 * buffer and flips them into the frame planes; ev[k] marks buffer k (host and device) free */
struct SgReader {
	hipStream_t stream = nullptr;
	uint16_t *pin[2] = {nullptr, nullptr};
	uint16_t *dstage[2] = {nullptr, nullptr};
	hipEvent_t ev[2] = {nullptr, nullptr};
	bool used[2] = {false, false};
	size_t cap = 0;		/* elements per buffer */
};

/* per-call device buffers of one stacking counter slot.  An async call flagged
 * SG_STACK_RESULT_AT_COLLECT runs everything after its main kernel on the device's tail stream,
 * beside the next call's main kernel, which uses the other slot's buffers (a slot is reused only
 * once the call two back has been folded).  Synchronous calls use slot 0. */
struct SgSlot {
	SgBuf inb;		/* the call's inputs (shift table, normalisation pairs, chain tables) */
	SgBuf flag_list, flag_map, redo, cmp_cols, cmp_list, scratch, lin_tab, wx;
	/* pinned, host-mapped staging of the inputs (k_stage_copy reads it); stage_ev marks the copy
	 * done before the host block is rewritten */
	void *stage_h = nullptr, *stage_d = nullptr;
	size_t stage_h_size = 0;
	bool stage_pending = false;
	hipEvent_t stage_ev = nullptr;
	int flag_epoch = 0;	/* flag_map epoch of the slot's last call (0: clear the map first) */
};

struct SgDevice {
	int id = 0;
	int shared = 1;		/* context slots on this physical device (sg_init(devs = {0, 0}) shares one card) */
	sg_stack_stats stats;	/* last stack call on this device (published to sg_ctx::stats) */
	std::vector<SgReader> readers;
	hipStream_t stream = nullptr;
	hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
	SgBuf sum_buf, frames, out, stats_buf;
	SgSlot sl[2];
	hipStream_t tail = nullptr;	/* SG_STACK_RESULT_AT_COLLECT calls: their post-processing */
	hipEvent_t tail_ev = nullptr;	/* the main kernel of such a call has finished */
	hipEvent_t tail_done_ev = nullptr;	/* sg_stack_wait_tail: the tail work queued so far has finished */
	/* registration workspaces (sg_register.hip) */
	SgBuf reg_sel, reg_spec, reg_work, reg_tw, reg_tw32, reg_best, reg_qbuf, reg_qacc;
	/* registration: the quality estimate runs on its own stream beside the FFT passes; its
	 * sums come back into a pinned block, aux_ev marks them landed */
	hipStream_t aux = nullptr;
	hipEvent_t aux_ev[2] = {nullptr, nullptr};
	unsigned long long *qacc_h = nullptr;
	size_t qacc_h_n = 0;
	/* registration tables cached per side (reg_tw for reg_tab_S / reg_tab_generic, reg_tw32 for
	 * reg_tw32_S), the pinned pair-table / result block, and aux2: the reference spectrum's
	 * stream beside the pairs' forward rows */
	int reg_tab_S = 0, reg_tab_generic = -1, reg_tw32_S = 0;
	void *reg_pin = nullptr;
	size_t reg_pin_n = 0;
	hipStream_t aux2 = nullptr;
	hipEvent_t aux2_ev[2] = {nullptr, nullptr};
	SgBuf zeros;	/* zero page for out-of-frame sample loads */
	/* stacking counters (rejection shards, flag / redo counts, sum maximum) in one device block,
	 * cleared by one memset and read back by one D2H copy into ctr_h (pinned) */
	SgBuf ctr;
	void *ctr_h = nullptr;
	/* two counter slots (device block + pinned host copy each): sg_stack_u16_device_async queues a
	 * call's read-back into its slot and returns; the slot is folded (event wait, fault checks,
	 * counters added to acc_*) by the next call that needs it or by sg_stack_collect.
	 * cev[slot] = {start, main kernel end, read-back done} */
	hipEvent_t cev[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
	unsigned long long *ctr_hd = nullptr;	/* ctr_h as the device sees it (k_ctr_finalize writes it) */
	bool ctr_clean[2] = {false, false};	/* the slot's device counters are zero (k_ctr_finalize left them so) */

	bool pend[2] = {false, false};
	unsigned long long pend_seq[2] = {0, 0}, seq = 0;
	sg_stack_stats pstats[2];	/* a pending call's statistics (timings filled in when folded) */
	int pend_sum_read[2] = {0, 0};	/* the call reports the SUM maximum */
	uint64_t acc_rej[3][2] = {{0, 0}, {0, 0}, {0, 0}};
	uint64_t acc_max = 0;
	int acc_rc = 0;
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

/* A/B and test knobs from the environment, read once when the context is created
 * (sg_init): the product path never consults the environment per call.  An unset or
 * invalid value gives the measured default. */
static inline int sg_env_int(const char *name, int lo, int hi, int def) {
	const char *e = getenv(name);
	if (!e || !*e)
		return def;
	char *end = nullptr;
	const long v = strtol(e, &end, 10);
	return (*end == 0 && v >= lo && v <= hi) ? (int)v : def;
}

struct SgKnobs {
	int hist_dbg = 0;		/* SG_HIST_DBG: k_stack_hist phase / timing A/B (0 = production) */
	int hist_prio = 1;		/* SG_HIST_PRIO: build-phase wave priority (1 measured best, scripts/gpu_prio.sh) */
	int hist_ldspad = 0;		/* SG_HIST_LDSPAD: extra LDS bytes per histogram workgroup (occupancy A/B) */
	int hist_ni = 1;		/* SG_HIST_NI: pixel pairs per lane of the histogram tiles (2: 256-px tiles) */
	int wins_cap = 64;		/* SG_WINS_CAP: histogram Winsorize inner iterations per pass before the redo list */
	int redo_replay = 1;		/* SG_REDO_REPLAY: 0 = redo list always through the sorted kernel */
	int hist_compact = 1;		/* SG_HIST_COMPACT: 0 = normalised redo pixels gather their columns again,
					 * >= 2: the compact list's capacity in pixels (tests of the overflow) */
	int reduce1 = 0;		/* SG_REDUCE1: 1 = one pixel per lane, 2 = the per-lane pixel-pair kernel, in the SUM/MAX/MIN/MEAN reduce (A/B) */
	long long host_budget = 0;	/* SG_HOST_BUDGET_BYTES: host-pull HBM budget (0 = 85 % of free HBM) */
	int reduce_seg = 1;		/* SG_REDUCE_SEG: 256-byte segments per wave in k_stack_reduce3 (1, 2, 4; 1 measured best: 512 x 4096^2 mean 3.52 / 3.59 / 4.33 ms, profiles/r05g) */
	int hist_sigmedian = 1;		/* SG_HIST_SIGMEDIAN: 0 = SIGMEDIAN on the sorted kernel only (A/B) */
	int pull_overlap = 1;		/* SG_PULL_OVERLAP: 0 = host-pull bands read and stacked one after the other (A/B) */
	int qsub_threads = 64;		/* SG_QSUB_THREADS: 64 measured best (scripts/gpu_qsub.sh) */
	int qgrad_threads = 128;	/* SG_QGRAD_THREADS: 128 measured best (scripts/gpu_qgrad.sh) */
	int reg_batch = 0;		/* SG_REG_BATCH: pairs per launch (0 = up to 2 GB of pair planes) */
	int reg_cw = 0;			/* SG_REG_CW: columns per column-pass workgroup (0 = 8192 / S) */
	int reg_path = 2;		/* SG_REG_PATH: 2 = half-spectrum passes (power-of-two sides), 3 = the generic passes */
	int reg_xcd = 1;		/* SG_REG_XCD: 0 = column strips in dispatch order */
	int reg_pb = 1;			/* SG_REG_PB: pairs per strip block of the fused column pass (1 = pair-major) */
	int reg_fp = 32;		/* SG_REG_FP: 32 = fp32 half-spectrum passes, near ties re-run in fp64; 64 = fp64 only */
	int reg_cw32 = 4;		/* SG_REG_CW32: columns per strip of the fp32 column pass (4: 32-B row segments, no spill; 8: 64-B segments, 16 elements per thread) */
	int reg_colocc = 1;		/* SG_REG_COLOCC: 1 = fp32 column pass held to 64 VGPRs (two 1024-thread workgroups per CU: registration 6.86 -> 6.21 ms on configs[1], profiles/r03t_ab_reg_cols.log), 0 = 76 VGPRs, one workgroup */
	int reg_wcol = 1;		/* SG_REG_WCOL: 1 = wave-level fp32 column pass at S = 2048 (k_reg_cols_xpower_w), 0 = block-level */
	int reg_genfuse = 1;		/* SG_REG_GENFUSE: 1 = generic sides' fused column pass (k_gen_cols_xpower), 0 = rows + k_gen_xpower + rows */
	int reg_rpw = 8;		/* SG_REG_RPW: rows per wave of the wave-level forward row pass (the next row fetched during this one's transform) */
	int reg_qafter = 0;		/* SG_REG_QAFTER: 1 = the quality estimate queued after the first batch's forward rows (beside the column pass) */
	int reg_qfold = 12;		/* SG_REG_QFOLD = r (3, 6, 9 ...): QualityEstimate's 3x3 subsample folded into the wave-level forward row pass, r consecutive rows per wave (S = 2048, fp32; configs[1] registration 3.10 -> 2.95 ms, r = 6-12 equal, 24 / 48 slower, profiles/r06s_*, r06t_*); 0 = k_quality_sub */
	int linfit_waves = 8;		/* SG_LINFIT_WAVES: waves per 64-pixel k_stack_linfit tile (4, 8 or 16 (KM = 8)) */
	int wins_export = 0;		/* SG_WINS_EXPORT = k > 0: histogram WINSORIZED (no normalisation) exports its columns holding 1 .. k zero / 65535 samples to k_hist_slow */
	int linfit_pair = 0;		/* SG_LINFIT_PAIR: 1 = both pixels of a sorted pair through one lockstep pass loop (lfx_pixel2_m) */
	int linfit_fast = 1;		/* SG_LINFIT_FAST: 1 = LINEARFIT through the decision-exact k_stack_linfit (16 <= N <= 1024), redo pixels to the sorted kernel; 0 = every pixel through the sorted kernel */
	int qgrad_stream = 1;		/* SG_QGRAD_STREAM: 1 = the quality gradient streamed down 60-column bands (k_quality_grad_s), 0 = tiled */
	int reg_wcolw = 8;		/* SG_REG_WCOLW: columns per strip of the wave-level column pass (8: 64-B row segments, one workgroup per CU: configs[1] registration 3.33 -> 3.20 ms and the pass's HBM writes 1.57x -> 1.0x the plane, profiles/r05w_*; 4: 32-B segments, two workgroups per CU) */
	int reg_specp = 1;		/* SG_REG_SPECP: 1 = the wave-level column pass reads the reference spectrum in lane order (k_spec_perm), 0 = through LDS */
	int reg_refconc = 1;		/* SG_REG_REFCONC: 1 = fp32 reference spectrum on its own stream beside the first batch's forward rows */
	int norm_fma = 2;		/* SG_NORM_FMA: normalised histogram stacks load with one fma per sample (1, 2) or, additive with
					 * scale 1, an integer offset (2) when a device check (k_norm_fma_check) finds that equal to the
					 * reference's roundings for every u16 value of every frame; 0 = the reference's operations */
	int reg_rpb = 4;		/* SG_REG_RPB: rows per forward-row workgroup of the half-spectrum path (1 -> 4: 6.46 -> 5.92 ms registration on configs[1], profiles/r03u_ab_reg_rows.log) */
	void read() {
		hist_dbg = sg_env_int("SG_HIST_DBG", 0, 1000, 0);
		hist_prio = sg_env_int("SG_HIST_PRIO", 0, 3, 1);
		hist_ldspad = sg_env_int("SG_HIST_LDSPAD", 0, 160 * 1024, 0);
		hist_ni = sg_env_int("SG_HIST_NI", 1, 2, 1);
		wins_cap = sg_env_int("SG_WINS_CAP", 4, 100000, 64);
		redo_replay = sg_env_int("SG_REDO_REPLAY", 0, 1, 1);
		hist_compact = sg_env_int("SG_HIST_COMPACT", 0, 1 << 30, 1);
		reduce1 = sg_env_int("SG_REDUCE1", 0, 2, 0);
		pull_overlap = sg_env_int("SG_PULL_OVERLAP", 0, 1, 1);
		hist_sigmedian = sg_env_int("SG_HIST_SIGMEDIAN", 0, 1, 1);
		reduce_seg = sg_env_int("SG_REDUCE_SEG", 1, 4, 1);
		if (reduce_seg == 3)
			reduce_seg = 2;
		if (const char *e = getenv("SG_HOST_BUDGET_BYTES"))
			host_budget = atoll(e) > 0 ? atoll(e) : 0;
		const int qs = sg_env_int("SG_QSUB_THREADS", 64, 1024, 64);
		qsub_threads = qs % 64 == 0 ? qs : 64;
		const int qg = sg_env_int("SG_QGRAD_THREADS", 64, 256, 128);
		qgrad_threads = (qg == 64 || qg == 128 || qg == 256) ? qg : 128;
		reg_batch = sg_env_int("SG_REG_BATCH", 1, 1024, 0);
		reg_cw = sg_env_int("SG_REG_CW", 1, 64, 0);
		while (reg_cw & (reg_cw - 1))	/* strips of a power of two columns (the FFT helpers split indices by shifts) */
			reg_cw &= reg_cw - 1;
		reg_path = sg_env_int("SG_REG_PATH", 2, 3, 2);
		reg_xcd = sg_env_int("SG_REG_XCD", 0, 1, 1);
		reg_pb = sg_env_int("SG_REG_PB", 1, 64, 1);
		reg_fp = sg_env_int("SG_REG_FP", 32, 64, 32) == 64 ? 64 : 32;
		reg_genfuse = sg_env_int("SG_REG_GENFUSE", 0, 1, 1);
		reg_wcol = sg_env_int("SG_REG_WCOL", 0, 1, 1);
		reg_cw32 = sg_env_int("SG_REG_CW32", 1, 16, 4);
		while (reg_cw32 & (reg_cw32 - 1))
			reg_cw32 &= reg_cw32 - 1;
		reg_colocc = sg_env_int("SG_REG_COLOCC", 0, 1, 1);
		reg_rpb = sg_env_int("SG_REG_RPB", 1, 64, 4);
		reg_refconc = sg_env_int("SG_REG_REFCONC", 0, 1, 1);
		reg_specp = sg_env_int("SG_REG_SPECP", 0, 1, 1);
		reg_wcolw = sg_env_int("SG_REG_WCOLW", 4, 8, 8) == 8 ? 8 : 4;
		qgrad_stream = sg_env_int("SG_QGRAD_STREAM", 0, 1, 1);
		linfit_fast = sg_env_int("SG_LINFIT_FAST", 0, 1, 1);
		linfit_waves = sg_env_int("SG_LINFIT_WAVES", 4, 16, 8);
		linfit_pair = sg_env_int("SG_LINFIT_PAIR", 0, 1, 0);
		wins_export = sg_env_int("SG_WINS_EXPORT", 0, 65535, 0);
		reg_qafter = sg_env_int("SG_REG_QAFTER", 0, 1, 0);
		reg_rpw = sg_env_int("SG_REG_RPW", 1, 64, 8);
		reg_qfold = sg_env_int("SG_REG_QFOLD", 0, 63, 12) / 3 * 3;
		norm_fma = sg_env_int("SG_NORM_FMA", 0, 2, 2);
	}
};

struct sg_ctx {
	std::vector<SgDevice> dev;
	std::mutex mu;		/* err / stats: the host-pull path drives every device from its own thread */
	std::string err;
	sg_stack_stats stats;
	SgKnobs knobs;
};

/* internal: a stale-state chain left the resident rows (mapped to SG_ERR_GENERIC at the ABI;
 * the host-pull path retries the band with more rows resident) */
#define SG_ERR_WALK -20

static inline int set_err(sg_ctx *ctx, int code, const char *fmt, const char *a = "", long b = 0) {
	char buf[512];
	snprintf(buf, sizeof buf, fmt, a, b);
	if (ctx) {
		std::lock_guard<std::mutex> lk(ctx->mu);
		ctx->err = buf;
	}
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

