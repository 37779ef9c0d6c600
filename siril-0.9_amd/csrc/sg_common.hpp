/*
 * sg_common.hpp - shared device-side definitions for the stacking kernels (gfx950).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SG_TILE_W 64		/* pixels per stacking tile (one 128-B row segment) */
#define SG_STAGE_STRIDE 66	/* u16 per staged frame row: 64 px + 2 pad -> 33 dwords, bank-conflict free */
#define SG_SORT_THREADS 256
#define SG_REJ_SHARDS 1024
/* A/B probe modes of the stacking kernels (SG_HIST_DBG: phase timings, loads only, timelines,
 * occupancy reports): compiled in only by a probe build (make EXTRA=-DSG_DBG_MODES=1 BUILD=...);
 * the product kernels carry no branch on them */
#ifndef SG_DBG_MODES
#define SG_DBG_MODES 0
#endif
#define SG_DBG(p) (SG_DBG_MODES ? (p).dbg : 0)

enum { SG_CLS_OK = 0, SG_CLS_LITERAL = 1, SG_CLS_CHAIN = 2, SG_CLS_DONE = 3,
	SG_CLS_NOTERM = 4 /* SIGMEDIAN whose reference loop never ends (p.loop_fault; the call fails) */,
	SG_CLS_CHAIN_DONE = 5 /* a CHAIN pixel k_stack_literal's phase 2 finished (still a chain link for walks) */ };
/* k_stack_replay: waves per block (one pixel per wave, ~18 KB of LDS each), max frames */
#define SG_REPLAY_WAVES 2
#define SG_REPLAY_MAXN 2048
#define SG_REDO_REPLAY_MAX 32768	/* histogram redo pixels sent straight to k_stack_replay (measured: 22 k faster there, 113 k slower) */

/* dwords per pixel column of the histogram kernels' LDS histogram: 64 band dwords (256 u8 bins)
 * and the out-of-band count (sg_stack_hist.hip SGH_HROWS) */
#define SG_HIST_HROWS 65

/* everything the stacking kernels need, passed by value */
struct SgStackParams {
	const uint16_t *frames;
	int64_t frame_stride, plane_stride;	/* elements */
	uint16_t *out;
	int N, W, H, C;
	int method, rejection, normalize;
	int use_shift;
	double sig0, sig1;
	const int *shiftx, *shifty;		/* device [N] */
	int dbg;				/* A/B timing knob (SG_HIST_DBG), 0 in production */
	int prio;				/* histogram path: wave priority of the build phase (SG_HIST_PRIO) */
	int wins_cap;				/* histogram WINSORIZED: inner iterations of a pass before the pixel goes to the
						 * redo list (SG_WINS_CAP): the rare pixels that need hundreds hold a whole
						 * wave in lockstep, the wave-per-pixel replay runs them alone */
	const int *hist_tab;			/* device: c1[hist_npad] = shifty*W*2 + 2*shiftx, then int16 sx2[hist_npad] = 2*shiftx */
	int hist_npad;				/* N rounded up to a multiple of 16 */
	int hist_norm_fold;			/* additive pairs carry offset - 0.5 (NORM 3 kernels) */
	int hist_maxsx;				/* max |shiftx| (interior-tile test of the histogram path) */
	const double *hist_norm;		/* device: {scale, offset | mul} per frame (hist_npad pairs), normalised stacks */
	/* additive normalisation with shifts: per border row (rows 0 .. ztab_k1 - 1, then
	 * H - ztab_k2 .. H - 1) the normalised zeros round_to_WORD(-offset_f) of the frames whose
	 * shifted row leaves the frame, those that are neither 0 nor 65535: int[8] {count, sum,
	 * sum of squares lo, hi, min, max, 0, 0} (null: none) */
	const int *ztab;
	int ztab_k1, ztab_k2;
	const double *offset, *mul, *scale;	/* device [N] or null */
	int row_begin, row_end;			/* memory rows to compute */
	int res_begin, res_end;			/* memory rows present at `frames` (desc->resident_rows) */
	int sy_min, sy_max;			/* range of shifty (0, 0 without shifts) */
	unsigned int *walk_fault;		/* set when a stale-state chain needs rows that are not resident */
	unsigned int *loop_fault;		/* set when a SIGMEDIAN pixel's reference loop never ends */
	unsigned long long *rej;		/* [SG_REJ_SHARDS][3][2] */
	unsigned int *flag_count;
	unsigned int *flag_list;		/* encoded (c*H + R)*W + x */
	unsigned int flag_cap;
	uint8_t *flag_map;			/* [C][H][W] class per pixel (chain walk): (epoch << 3) | class, an entry of
						 * another epoch reads as SG_CLS_OK (the host clears the map when epochs wrap) */
	unsigned int flag_epoch;		/* 1 .. 31, this call's */
	/* histogram path, normalised SIGMA / WINSORIZED: a redo pixel whose only out-of-band
	 * samples besides 0 / 65535 are the few the build captured (SGH_OVK) leaves its whole sorted
	 * column at cmp_cols[slot][N] and its pixel at cmp_list[slot] (slot < cmp_cap), so the
	 * sorted kernel reads N contiguous values instead of gathering N scattered lines */
	uint16_t *cmp_cols;
	unsigned int *cmp_list, *cmp_count;
	unsigned int cmp_cap;
	const uint16_t *cmp_src;		/* k_stack_sorted<., true>: stage the listed columns from here (sorted) */
	unsigned int list_minn;			/* k_stack_sorted<., true> on the redo list: do nothing unless the device count
						 * exceeds this (0: take any list); the replay takes the shorter lists */
	/* k_stack_replay: the histogram path's redo list taken directly when its count is at most
	 * rp_maxn (null: only the flag list) */
	const unsigned int *rp_list, *rp_count;
	unsigned int rp_maxn;
	const double *linfit_tab;		/* LINEARFIT: gsl_fit_linear's m_x, m_dx2 per N (k_linfit_tables) */
	/* histogram WINSORIZED without normalisation (SG_WINS_EXPORT): the tile exports the columns that
	 * hold a zero or a 65535 sample (the slow Winsorize pixels) instead of finishing them, and
	 * k_hist_slow finishes them in waves of their own: wx[j * wx_cap + slot], rows j < SGH_HROWS the
	 * column's histogram dwords, then lo, nz | ns << 16, the pixel index; wx_count (device) the slots
	 * taken (null wx: every column finished in its tile) */
	uint32_t *wx;				/* [SG_HIST_HROWS + 3][wx_cap] */
	unsigned int wx_cap;
	unsigned int *wx_count;
	int wx_kmax;				/* export a column with 1 .. wx_kmax zero / 65535 samples (more: the rows a
						 * registration shift empties, whose tiles are slow throughout: finished there) */
	uint32_t *sum_buf;			/* SUM: raw sums [C][H][W] */
	unsigned int *maxim;			/* SUM: global max of sums */
};

/* pixel classes of this call (entries written by earlier calls read as SG_CLS_OK) */
__device__ __forceinline__ int sg_flag_get(const SgStackParams &p, int64_t pix) {
	const unsigned int v = p.flag_map[pix];
	return (v >> 3) == p.flag_epoch ? (int)(v & 7u) : (int)SG_CLS_OK;
}
__device__ __forceinline__ void sg_flag_set(const SgStackParams &p, int64_t pix, int cls) {
	p.flag_map[pix] = (uint8_t)((p.flag_epoch << 3) | (unsigned int)cls);
}

/* round_to_WORD, src/core/utils.c:68-74 */
__device__ __forceinline__ uint16_t sg_round_to_WORD(double x) {
	if (x <= 0.0)
		return 0;
	if (x > 65535.0)
		return 65535;
	return (uint16_t)(x + 0.5);
}

/* normalisation of one gathered sample, src/stacking/stacking.c:1635-1652 (and :750-764) */
__device__ __forceinline__ uint16_t sg_normalize(const SgStackParams &p, int f, uint16_t v) {
	switch (p.normalize) {
	default:
	case 0:
		return v;
	case 1:	/* ADDITIVE */
	case 3: {	/* ADDITIVE_SCALING */
		double tmp = (double)v * (p.scale ? p.scale[f] : 1.0);
		return sg_round_to_WORD(tmp - (p.offset ? p.offset[f] : 0.0));
	}
	case 2:	/* MULTIPLICATIVE */
	case 4: {
		double tmp = (double)v * (p.scale ? p.scale[f] : 1.0);
		return sg_round_to_WORD(tmp * (p.mul ? p.mul[f] : 1.0));
	}
	}
}

/* sample of frame f at output pixel (c, R, x) (memory coords): the rejection stacker's
 * y-shifted band read (:1550-1577) leaves zero rows in the block buffer, and those zeros
 * ARE normalised like read samples (:1644-1650); the x shift writes 0 directly into the
 * stack, bypassing normalisation (:1628-1632).  The median stacker ignores shifts (:703-722). */
__device__ __forceinline__ uint16_t sg_gather(const SgStackParams &p, int f, int c, int R, int x) {
	int sx = 0, sy = 0;
	if (p.use_shift) {
		sx = p.shiftx[f];
		sy = p.shifty[f];
	}
	int sr = R - sy, sc = x - sx;
	if ((unsigned)sc >= (unsigned)p.W)
		return 0;
	uint16_t v = 0;
	if ((unsigned)sr < (unsigned)p.H)
		v = p.frames[(int64_t)f * p.frame_stride + (int64_t)c * p.plane_stride +
			(int64_t)sr * p.W + sc];
	return sg_normalize(p, f, v);
}
