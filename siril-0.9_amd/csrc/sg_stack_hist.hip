/*
 * sg_stack_hist.hip - gfx950 fast path of stack_mean_with_rejection, SIGMA rejection
 * (src/stacking/stacking.c:1674-1695 + sigma_clipping :1148-1161) and WINSORIZED
 * (:1710-1749), any normalisation (:1635-1652, applied at load), without sorting.
 *
 * Why: the reference sorts every pixel column (quicksort_s) on every clipping pass.  A
 * sort of N = 512 u16 per pixel costs ~O(N log^2 N) compare-exchanges on a GPU, far more
 * VALU than the N*2 bytes the pixel reads from HBM can hide.  But every quantity a
 * sigma-clip pass needs is a function of the column's value HISTOGRAM:
 *   - the kept set after any number of passes is {v : A <= v <= B} (low clips remove the
 *     lowest values, high clips the highest; the set stays a value interval);
 *   - median of the kept set = value at a rank, counts below/above a threshold = ranks;
 *   - sigma comes from exact integer moments n, S, SS of the kept set.
 * So each 128-pixel tile builds, per pixel, an exact histogram of 256 unit-wide bins
 * [lo, lo+255] around the median of the first 16 frames (u8 counts packed 4 per dword),
 * plus a counter of the samples above the band and of the zeros / 65535s (the number
 * below the band follows from N) (out-of-frame zero fill, dead pixels, saturation, cosmics).  4 waves stream the
 * N frames into it, one lane per PAIR of adjacent pixels: each frame row is one 256-byte
 * coalesced dword load per wave (2-byte aligned dword loads are legal on gfx950), the
 * per-frame buffer descriptor makes out-of-frame rows read 0 through the hardware bounds
 * check (the zero fill of :1550-1577 for free), and the pixel pair is binned with packed
 * u16 arithmetic and branch-free LDS atomics.  Tiles whose shifted columns can leave the
 * image (the two image-edge tile columns) load pixel by pixel with the column check of
 * :1628-1632 (one latency per 16-frame block; they are 2 of every W/128 tiles).  The
 * finish then prefix-sums the bins once and runs the reference's pass loop as O(log)
 * histogram queries: SIGMA with a lane pair per pixel on all 4 waves, WINSORIZED with one
 * lane per pixel on waves 0 / 1.
 *
 * Exactness: decisions use exact moments; a pixel whose decision falls within a rounding
 * band of a threshold (GSL's long-double sd vs exact), whose loop would hit the
 * reference's early `break` (N - r <= 4, :1684, stale rejected[]), whose median falls
 * outside the band, which has out-of-band samples other than 0 / 65535, or whose u8
 * counters overflow (detected: the counts must add up to N) is appended to a redo list
 * and recomputed by the
 * sorted kernel (k_stack_sorted<.., true>), which in turn hands knife-edge pixels to the
 * literal (fp80) path.  Output is therefore bit-identical to the sorted path.
 */
#include "sg_common.hpp"

#define SGH_BINS 256
#define SGH_DW (SGH_BINS / 4)	/* band dwords per pixel */
/* A tile is NI * 128 pixels of one row, streamed by NI * 4 waves: every lane loads NI dwords
 * (pixel pairs) per frame, instruction i covering the tile's 256-byte segment i.  Pixel pair i
 * of lane l = pixels 128 i + 2 l (column 64 (2 i) + l) and 128 i + 2 l + 1 (column
 * 64 (2 i + 1) + l).  NI = 2 reads each frame row as one contiguous 512-byte segment (a
 * shifted row straddles 5 128-B lines per 512 B instead of 3 per 256 B: tools/bw_probe4.hip
 * streams the 512 x 4096^2 sequence in 2.94 ms against 3.20 ms), but two 8-wave workgroups per
 * CU overlap one tile's finish with the other's loads worse than four 4-wave ones: 4.62 ms
 * against 4.22 ms for the whole kernel, so NI = 1 is the default (SG_HIST_NI=2 selects 2). */
#define SGH_WAVES_PER_NI 4
/* waves per 256-pixel tile (NI = 2, the A/B SG_HIST_NI=2): 8, or 4 (-DSGH_WAVES_NI2=4: each
 * lane loads both dwords of a 512-byte row segment, two 4-wave workgroups per CU with up to
 * 256 VGPRs).  Measured (scripts/gpu_r4h.sh, profiles/r02x_ab_ni2_waves.log): 4 waves 5.02-5.08
 * ms (loads only 3.36), 8 waves 4.37 ms, the 128-pixel default 3.50 ms (loads only 3.23) */
#ifndef SGH_WAVES_NI2
#define SGH_WAVES_NI2 8
#endif
#ifndef SGH_NB2
#define SGH_NB2 1	/* blocks in flight for NI = 2 (4 waves: NB2 = 2 5.08 ms, 1 5.02 ms) */
#endif
template <int NI>
struct SghCfg {
	static constexpr int WAVES = NI == 1 ? SGH_WAVES_PER_NI : SGH_WAVES_NI2;
	static constexpr int WPE = NI == 1 ? 4 : (SGH_WAVES_NI2 == 4 ? 2 : 4);	/* waves per SIMD (launch bound) */
};
#ifndef SGH_WINS_WAVES
#define SGH_WINS_WAVES 2	/* waves per 128-pixel WINSORIZED tile: 2, each building twice the frames, so 4 tiles fit a CU at 2 waves per SIMD (26.5 -> 25.7 ms on configs[4], profiles/r03_wins_ab.log); 4: the SIGMA shape */
#endif
/* waves of a tile of kernel k_stack_hist<REJ, ., NI> */
template <int REJ, int NI>
struct SghW {
	static constexpr int WAVES = (REJ == 4 && NI == 1) ? SGH_WINS_WAVES : SghCfg<NI>::WAVES;
};
#ifndef SGH_CENTER
#define SGH_CENTER 16		/* frames used for the centre estimate */
#endif
#ifndef SGH_NBUF
#define SGH_NBUF 2		/* register buffers of 16 frames per wave (NBUF-1 blocks in flight while binning) */
#endif
#define SGH_BAND 1e-13		/* same rounding band as the sorted path (SG_BAND) */
/* largest frame count whose Winsorized moments n SS and S^2 (values relative to lo, |v - lo| <=
 * 65535) stay integers below 2^53: 1448^2 65535^2 < 2^53 */
#define SGH_WIN_DBL_MAXN 1448

typedef unsigned short sgh_u16x2 __attribute__((ext_vector_type(2)));

/* Histogram layout: pixel column c = 64 half + l (half 0 = the low u16 of a lane's pixel
 * pair, half 1 the high one, l = lane) keeps its band in h[half][j][l]: a wave's 64 lanes
 * always address 64 different banks, whatever bins they hit.
 *   h[half][j][l] byte b (j < 64): count of value lo + 4 j + b   (u8 counters)
 *   h[half][64][l]               : samples outside the band (u32: zeros, 65535s; anything
 *                                  else sends the pixel to the redo list) */
#define SGH_HROWS (SGH_DW + 1)
static_assert(SGH_HROWS == SG_HIST_HROWS, "sg_common.hpp's column size");
#define SGH_OVK 4	/* out-of-band sample values captured per column (normalised stacks) */
template <int NI>
struct alignas(16) SghLds {
	uint32_t h[2 * NI][SGH_HROWS][64];
	uint32_t nz[128 * NI], ns[128 * NI];	/* zeros / 65535s (all of them lie outside the band) */
	uint32_t na[128 * NI];			/* samples above the band (stack_median / PERCENTILE kernels only) */
	uint32_t lo2[NI][64];			/* band starts of the lane pixel pairs (u16 halves) */
	uint32_t cs[NI][8][64];			/* wave 1's first 8 frames for the band centre (SGH_CENTER2W) */
	uint8_t perm[128];			/* WINSORIZED finish order of the columns (SGH_WINS_ORDER) */
	/* normalised SIGMA / WINSORIZED builds: the first SGH_OVK out-of-band samples of a column
	 * that are neither 0 nor 65535, and how many there were (sgh_capture, sgh_compact) */
	uint16_t ov[SGH_OVK][128 * NI];
	uint32_t ovn[128 * NI];
#ifdef SGH_WPROF
	uint64_t wp[SghCfg<NI>::WAVES][16];	/* probe build: per-wave region cycles and events (sgh_wp) */
#endif
};

/* Finish-phase queries.  The band is cut into SGH_NGRP groups of SGH_GRP dwords (32 bins);
 * the exclusive prefix count / moments at each group start are kept in registers, so a
 * rank or prefix query is one lane-local table select plus SGH_GRP independent LDS reads
 * (one LDS round trip) instead of a dependent walk. */
#define SGH_GRP 8
#define SGH_NGRP (SGH_DW / SGH_GRP)

/* count / sum / sum of squares of (v - lo) over a set of samples */
struct SghM {
	int c;
	long long s;
	unsigned long long ss;
};

struct SghPix {
	int lo;			/* value of bin 0, 1 <= lo <= 65279 */
	int nz, ns, nb;		/* zeros, 65535s, band samples (nz + nb + ns == N) */
	int col;
	const uint32_t *hb;	/* the tile's histogram h[0][0][0] */
	/* band prefix (count, sum, sum of squares of t) before group g, kept at index g ^ hx: a lane
	 * of a pair holds its own 4 groups first (hx = 4 for the high half), so the exchange of
	 * the halves' prefixes needs no reordering */
	uint32_t pc[SGH_NGRP], ps[SGH_NGRP], pss[SGH_NGRP];
	int hx;
#ifdef SGH_WPROF
	uint64_t *wp;		/* probe build: this wave's region accumulators in LDS */
#endif
	SghM Z;			/* moments of the zeros (and of the border row's normalised zeros, ztab) */
	int zmax;		/* > 0: the below-band samples include normalised zeros (or captured samples) up to this
				 * value; a count query at v in [0, zmax) or a rank among them is not decided here */
	int omin;		/* < 65535: captured samples above the band from this value on (CAP SIGMA); a count
				 * query at v in [omin, 65535) or a rank among the above-band samples is not decided here */
	SghM T;			/* moments of all samples */
	double zs, zss;		/* Z.s, Z.ss as doubles (exact: below 2^53) for the Winsorized queries */
};

/* t[k] for a lane-varying k in [0, 8): a 3-level select tree on the bits of k */
__device__ __forceinline__ uint32_t sgh_sel(const uint32_t (&t)[SGH_NGRP], int k) {
	static_assert(SGH_NGRP == 8, "3-level tree");
	const bool b0 = (k & 1) != 0, b1 = (k & 2) != 0, b2 = (k & 4) != 0;
	const uint32_t a0 = b0 ? t[1] : t[0], a1 = b0 ? t[3] : t[2], a2 = b0 ? t[5] : t[4], a3 = b0 ? t[7] : t[6];
	const uint32_t c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
	return b2 ? c1 : c0;
}
/* prefix entry of group g */
__device__ __forceinline__ uint32_t sgh_pre(const SghPix &P, const uint32_t (&t)[SGH_NGRP], int g) {
	return sgh_sel(t, g ^ P.hx);
}
/* the band group holding band rank r (0 for r < 0): the number of groups g >= 1 whose
 * prefix count is <= r, counted over the 8 entries in any order (group 0's prefix is 0) */
__device__ __forceinline__ int sgh_grp_of(const SghPix &P, int r) {
	int grp = r >= 0 ? -1 : 0;
#pragma unroll
	for (int k = 0; k < SGH_NGRP; k++)
		grp += (int)P.pc[k] <= r ? 1 : 0;
	return grp;
}

__device__ __forceinline__ void sgh_grp(const SghPix &P, int g, uint32_t (&d)[SGH_GRP]) {
	const uint32_t *b = P.hb + ((P.col >> 6) * SGH_HROWS + g * SGH_GRP) * 64 + (P.col & 63);
#pragma unroll
	for (int k = 0; k < SGH_GRP; k++)
		d[k] = b[k * 64];
}


/* moments of the bins of one group, relative to the group's first bin: the dword K of the
 * group holds bins j = 4 K + b; sum j c_j is a u8 dot product on constant weights, and with
 * j < 32, j^2 < 1024, sum j^2 c_j = sum lo8(j^2) c_j + 256 sum hi8(j^2) c_j: two more u8 dot
 * products per dword (the high one only for K >= 4, where j^2 >= 256) - 29 VALU per 8-dword
 * group against 48 with the bytes unpacked to u16 for v_dot2_u32_u16 (round 1) */
template <int K>
__device__ __forceinline__ void sgh_dw_moments_b(uint32_t dd, uint32_t &c, uint32_t &s, uint32_t &sl, uint32_t &sh) {
	constexpr uint32_t j0 = 4 * K, j1 = j0 + 1, j2 = j0 + 2, j3 = j0 + 3;
	constexpr uint32_t w1 = j0 | (j1 << 8) | (j2 << 16) | (j3 << 24);
	constexpr uint32_t wl = ((j0 * j0) & 0xFFu) | (((j1 * j1) & 0xFFu) << 8) | (((j2 * j2) & 0xFFu) << 16) |
		(((j3 * j3) & 0xFFu) << 24);
	constexpr uint32_t wh = ((j0 * j0) >> 8) | (((j1 * j1) >> 8) << 8) | (((j2 * j2) >> 8) << 16) | (((j3 * j3) >> 8) << 24);
	c = __builtin_amdgcn_sad_u8(dd, 0u, c);
	s = __builtin_amdgcn_udot4(dd, w1, s, false);
	sl = __builtin_amdgcn_udot4(dd, wl, sl, false);
	if (wh != 0u)
		sh = __builtin_amdgcn_udot4(dd, wh, sh, false);
}

template <bool COUNT = true>
__device__ __forceinline__ void sgh_grp_moments(const uint32_t (&d)[SGH_GRP], uint32_t &c, uint32_t &s, uint32_t &ss) {
	static_assert(SGH_GRP == 8, "unrolled for 8 dwords");
	uint32_t sl = 0, sh = 0, cx = 0;
	uint32_t &cc = COUNT ? c : cx;	/* !COUNT: the caller has the count already */
	sgh_dw_moments_b<0>(d[0], cc, s, sl, sh);
	sgh_dw_moments_b<1>(d[1], cc, s, sl, sh);
	sgh_dw_moments_b<2>(d[2], cc, s, sl, sh);
	sgh_dw_moments_b<3>(d[3], cc, s, sl, sh);
	sgh_dw_moments_b<4>(d[4], cc, s, sl, sh);
	sgh_dw_moments_b<5>(d[5], cc, s, sl, sh);
	sgh_dw_moments_b<6>(d[6], cc, s, sl, sh);
	sgh_dw_moments_b<7>(d[7], cc, s, sl, sh);
	ss += sl + (sh << 8);
}

/* a prefix query "samples with value <= v" (v in [-1, 65535]): the group of the band bin is
 * read once; the count is cheap and the moments are only formed for the passes that
 * actually remove samples */
struct SghQ {
	int v, t, g, kb;
	uint32_t d[SGH_GRP];	/* the group's dwords below the boundary dword kb, others 0 */
	uint32_t bd;		/* the boundary dword (group dword kb, the one holding bin t), masked to bins <= t */
	uint32_t cp;		/* band samples <= t inside the group (d and bd) */
};

/* the group is read as 8 dwords plus the boundary dword once more (one more LDS read, no
 * select tree): dwords k < kb are kept whole with one compare + select each, the boundary
 * dword is masked to its bins <= t and enters the sums separately */
__device__ __forceinline__ void sgh_q_load(const SghPix &P, int v, SghQ &q) {
	int t = v - P.lo;
	t = t < -1 ? -1 : (t > SGH_BINS - 1 ? SGH_BINS - 1 : t);
	q.v = v;
	q.t = t;
	const int tc = t < 0 ? 0 : t;
	q.g = tc >> 5;
	sgh_grp(P, q.g, q.d);
	q.bd = P.hb[((P.col >> 6) * SGH_HROWS + (tc >> 2)) * 64 + (P.col & 63)];
	const int kb = (t >> 2) - q.g * SGH_GRP;	/* -1 for t = -1: nothing counted */
	q.kb = kb;
#pragma unroll
	for (int k = 0; k < SGH_GRP; k++)
		q.d[k] = k < kb ? q.d[k] : 0u;
	const uint32_t mt = 0xFFFFFFFFu >> (24 - 8 * (t & 3));
	q.bd = t >= 0 ? (q.bd & mt) : 0u;
	uint32_t c = __builtin_amdgcn_sad_u8(q.bd, 0u, 0u);
#pragma unroll
	for (int k = 0; k < SGH_GRP; k++)
		c = __builtin_amdgcn_sad_u8(q.d[k], 0u, c);
	q.cp = c;
}

__device__ __forceinline__ int sgh_q_count(const SghPix &P, const SghQ &q) {
	const uint32_t c = sgh_pre(P, P.pc, q.g) + q.cp;
	if (q.v < 0)
		return 0;
	if (q.v >= 65535)
		return P.T.c;
	return P.nz + (int)c;
}

__device__ __forceinline__ SghM sgh_q_moments(const SghPix &P, const SghQ &q) {
	uint32_t c = q.cp, s = 0, ss = 0;
	sgh_grp_moments<false>(q.d, c, s, ss);
	/* the boundary dword: bins j = 4 kb + b, j^2 = (4 kb)^2 + 2 (4 kb) b + b^2 */
	const uint32_t cb = __builtin_amdgcn_sad_u8(q.bd, 0u, 0u);
	const uint32_t sb = __builtin_amdgcn_udot4(q.bd, 0x03020100u, 0u, false);
	const uint32_t qb = __builtin_amdgcn_udot4(q.bd, 0x09040100u, 0u, false);
	/* 24-bit multiplies throughout (all factors < 2^24: k4 <= 28, b0 <= 224, c <= 32 * 255) */
	const uint32_t k4 = 4u * (uint32_t)(q.kb < 0 ? 0 : q.kb);
	ss += qb + __umul24(2u * k4, sb) + __umul24(__umul24(k4, k4), cb);
	s += sb + __umul24(k4, cb);
	const uint32_t b0 = (uint32_t)q.g * (4u * SGH_GRP);	/* first bin of the group */
	SghM m;
	m.c = P.nz + (int)(sgh_pre(P, P.pc, q.g) + c);
	m.s = P.Z.s + (long long)(sgh_pre(P, P.ps, q.g) + s + __umul24(b0, c));
	m.ss = P.Z.ss + (unsigned long long)(sgh_pre(P, P.pss, q.g) + ss + __umul24(2u * b0, s) + __umul24(__umul24(b0, b0), c));
	if (q.v < 0) {
		m.c = 0;
		m.s = 0;
		m.ss = 0;
	}
	if (q.v >= 65535)
		m = P.T;
	return m;
}

/* moments of the samples with value <= v (rare paths) */
__device__ __forceinline__ int sgh_cnt_le(const SghPix &P, int v) {
	SghQ q;
	sgh_q_load(P, v, q);
	return sgh_q_count(P, q);
}

/* value of band rank r inside group g (d = the group's dwords, base = samples before it) */
__device__ __forceinline__ int sgh_locate(const SghPix &P, int g, const uint32_t (&d)[SGH_GRP], uint32_t base, uint32_t r) {
	uint32_t cum = base, before = base, kk = 0, dsel = d[0];
#pragma unroll
	for (int k = 0; k < SGH_GRP - 1; k++) {
		cum += __builtin_amdgcn_sad_u8(d[k], 0u, 0u);
		const bool past = cum <= r;	/* rank r lies after dword k */
		kk += past ? 1u : 0u;
		before = past ? cum : before;
		dsel = past ? d[k + 1] : dsel;
	}
	const uint32_t b0 = before + (dsel & 0xFFu), b1 = b0 + ((dsel >> 8) & 0xFFu), b2 = b1 + ((dsel >> 16) & 0xFFu);
	const int i = (b0 <= r ? 1 : 0) + (b1 <= r ? 1 : 0) + (b2 <= r ? 1 : 0);
	return P.lo + 4 * (g * SGH_GRP + (int)kk) + i;
}

/* values at global ranks g1 and g2 (g2 == g1 or g1 + 1), one group read when both lie
 * in the same band group */
__device__ __forceinline__ void sgh_value_at2(const SghPix &P, int g1, int g2, int &m1, int &m2) {
	const int r1 = g1 - P.nz, r2 = g2 - P.nz;
	const bool in1 = r1 >= 0 && r1 < P.nb, in2 = r2 >= 0 && r2 < P.nb;
	const int grp1 = sgh_grp_of(P, r1), grp2 = sgh_grp_of(P, r2);
	uint32_t d[SGH_GRP];
	sgh_grp(P, grp1, d);
	const uint32_t base1 = sgh_pre(P, P.pc, grp1);
	m1 = in1 ? sgh_locate(P, grp1, d, base1, (uint32_t)r1) : (r1 < 0 ? 0 : 65535);
	if (in2 && grp2 == grp1) {
		m2 = sgh_locate(P, grp1, d, base1, (uint32_t)r2);
	} else if (in2) {
		sgh_grp(P, grp2, d);
		m2 = sgh_locate(P, grp2, d, sgh_pre(P, P.pc, grp2), (uint32_t)r2);
	} else {
		m2 = r2 < 0 ? 0 : 65535;
	}
}

/* sgh_value_at2 with nbl samples below the band (a rank below them reads 0, one past the band
 * 65535: the caller has checked those samples are zeros / 65535s) */
__device__ __forceinline__ void sgh_value_at2n(const SghPix &P, int nbl, int g1, int g2, int &m1, int &m2) {
	const int r1 = g1 - nbl, r2 = g2 - nbl;
	const bool in1 = r1 >= 0 && r1 < P.nb, in2 = r2 >= 0 && r2 < P.nb;
	const int grp1 = sgh_grp_of(P, r1), grp2 = sgh_grp_of(P, r2);
	uint32_t d[SGH_GRP];
	sgh_grp(P, grp1, d);
	const uint32_t base1 = sgh_pre(P, P.pc, grp1);
	m1 = in1 ? sgh_locate(P, grp1, d, base1, (uint32_t)r1) : (r1 < 0 ? 0 : 65535);
	if (in2 && grp2 == grp1) {
		m2 = sgh_locate(P, grp1, d, base1, (uint32_t)r2);
	} else if (in2) {
		sgh_grp(P, grp2, d);
		m2 = sgh_locate(P, grp2, d, sgh_pre(P, P.pc, grp2), (uint32_t)r2);
	} else {
		m2 = r2 < 0 ? 0 : 65535;
	}
}

/* ceil(x) clamped to [0, 65536] (NaN -> 0), floor(x) clamped to [-1, 65535] (NaN -> 65535);
 * written as selects so the pass loop stays one basic block */
__device__ __forceinline__ int sgh_ceil_clamp(double x) {
	double y = x > 0.0 ? x : 0.0;
	y = y > 65536.0 ? 65536.0 : y;
	return (int)ceil(y);
}
__device__ __forceinline__ int sgh_floor_clamp(double x) {
	double y = x < 65535.0 ? x : 65535.0;
	y = y < -1.0 ? -1.0 : y;
	return (int)floor(y);
}

/* centre estimate of the two pixels of a lane from 16 samples each (16-bit halves of
 * p[]): median of the samples that are neither 0 nor 65535 (the out-of-frame zero fill of
 * edge pixels must not drag the band away); packed bitonic network */
__device__ __forceinline__ void sgh_centre2(const uint32_t (&p)[SGH_CENTER], int &lo_a, int &lo_b) {
	sgh_u16x2 v[SGH_CENTER];
	sgh_u16x2 nzc = {0, 0}, sc = {0, 0};
#pragma unroll
	for (int i = 0; i < SGH_CENTER; i++) {
		v[i] = __builtin_bit_cast(sgh_u16x2, p[i]);
		nzc += __builtin_elementwise_min(v[i], (sgh_u16x2){1, 1});
		sc += __builtin_elementwise_sub_sat(v[i], (sgh_u16x2){65534, 65534});
	}
#pragma unroll
	for (int k = 2; k <= SGH_CENTER; k <<= 1) {
#pragma unroll
		for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
			for (int i = 0; i < SGH_CENTER; i++) {
				const int l = i ^ j;
				if (l > i) {
					const bool up = (i & k) == 0;
					const sgh_u16x2 a = v[i], b = v[l];
					const sgh_u16x2 mn = __builtin_elementwise_min(a, b), mx = __builtin_elementwise_max(a, b);
					v[i] = up ? mn : mx;
					v[l] = up ? mx : mn;
				}
			}
		}
	}
	int lo2[2];
#pragma unroll
	for (int h = 0; h < 2; h++) {
		const int z = SGH_CENTER - (int)nzc[h], s = (int)sc[h];
		int idx = z + (SGH_CENTER - z - s) / 2;
		if (idx > SGH_CENTER - 1)
			idx = SGH_CENTER - 1;
		int r = v[0][h];
#pragma unroll
		for (int i = 1; i < SGH_CENTER; i++)
			r = (i == idx) ? (int)v[i][h] : r;
		r -= SGH_BINS / 2;
		if (r < 1)
			r = 1;
		if (r > 65535 - SGH_BINS)
			r = 65535 - SGH_BINS;
		lo2[h] = r;
	}
	lo_a = lo2[0];
	lo_b = lo2[1];
}

/* per-tile load context */
struct SghFrame {
	const char *plane0;		/* channel plane of frame 0 */
	int64_t fstride2;		/* bytes between frames */
	uint32_t plane_bytes;
	int rw2;			/* R * W * 2 */
	int w2;				/* W * 2 */
	uint32_t xa2;			/* 2 * x of the lane's first pixel */
	uint32_t x02;			/* 2 * x0, the tile's first column */
};

/* shift table of the 16 frames f0..f0+15 (f0 % 16 == 0): c1 = shifty*W*2 + 2*shiftx (one
 * s_load_dwordx16) and int16 sx2 = 2*shiftx (one s_load_dwordx8); zero padded to a
 * multiple of 16 frames */
struct SghTab16 {
	int c1[16];
	uint32_t sx2p[8];
};
/* the shift table and the normalisation pairs reach the kernel as __restrict__ kernel
 * arguments (SghRo): nothing the kernel stores can alias them, so their uniform loads compile
 * to scalar loads (s_load_dwordx16 / x8 / x4) instead of vector loads that would queue
 * behind the frame loads in vmcnt order */
struct SghRo {
	const int *tab;		/* SgStackParams::hist_tab */
	const int4 *norm;	/* SgStackParams::hist_norm as int4 pairs */
	int npad;
};
__device__ __forceinline__ void sgh_tab16(const SghRo &ro, int f0, SghTab16 &T) {
	const int4 *q = (const int4 *)(ro.tab + f0);
	const int4 *r = (const int4 *)(ro.tab + ro.npad + f0 / 2);
#pragma unroll
	for (int i = 0; i < 4; i++) {
		const int4 v = q[i];
		T.c1[4 * i] = __builtin_amdgcn_readfirstlane(v.x);
		T.c1[4 * i + 1] = __builtin_amdgcn_readfirstlane(v.y);
		T.c1[4 * i + 2] = __builtin_amdgcn_readfirstlane(v.z);
		T.c1[4 * i + 3] = __builtin_amdgcn_readfirstlane(v.w);
	}
#pragma unroll
	for (int i = 0; i < 2; i++) {
		const int4 v = r[i];
		T.sx2p[4 * i] = (uint32_t)__builtin_amdgcn_readfirstlane(v.x);
		T.sx2p[4 * i + 1] = (uint32_t)__builtin_amdgcn_readfirstlane(v.y);
		T.sx2p[4 * i + 2] = (uint32_t)__builtin_amdgcn_readfirstlane(v.z);
		T.sx2p[4 * i + 3] = (uint32_t)__builtin_amdgcn_readfirstlane(v.w);
	}
}

/* cache policy bits of the frame loads (A/B builds: -DSGH_LOAD_AUX=...; 0 = default policy) */
#ifndef SGH_LOAD_AUX
#define SGH_LOAD_AUX 0
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sgh_rsrc(const char *base, uint32_t nrec) {
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nrec, 0x00020000);
}

/* 16 frames f0..f0+15, one 2-byte aligned dword load per frame and lane at
 * (R - sy) W 2 + 2 (x - sx) (the lane's pixel pair); a row outside the frame reads 0
 * through the bounds check, frames >= N get num_records = 0 (read 0; never binned).
 * EDGE (image-edge tiles, where a shifted column can leave the image; the x shift writes 0
 * there, :1628-1632): a pair with both columns outside loads out of bounds (0); a pair
 * straddling the left edge loads one pixel to the right and the binning moves the valid
 * pixel to the high half (<< 16), one straddling the right edge loads one pixel to the
 * left (>> 16); two fix bits per frame in `fix` */
template <bool FULL, bool EDGE, int NI, int MB = 16, int MO = 0>
__device__ __forceinline__ void sgh_loadblk(const SghFrame &F, const SghTab16 &T, int N, int f0,
		uint32_t (&dst)[MB][NI], uint32_t (&fix)[NI]) {
	const char *b = F.plane0 + (int64_t)f0 * F.fstride2;
	if (EDGE) {
#pragma unroll
		for (int i = 0; i < NI; i++)
			fix[i] = 0;
	}
#pragma unroll
	for (int m = 0; m < MB; m++) {
		const uint32_t nrec = (FULL || f0 + m < N) ? F.plane_bytes : 0u;
		const uint32_t k = (uint32_t)(F.rw2 - T.c1[MO + m]);
#pragma unroll
		for (int i = 0; i < NI; i++) {
			const uint32_t xa2 = F.xa2 + 256u * i;	/* the lane's pair in segment i */
			uint32_t off = k + xa2;
			if (EDGE) {
				const int mt = MO + m;
				const int sx2 = (mt & 1) ? ((int)T.sx2p[mt >> 1] >> 16) : (int)(int16_t)(T.sx2p[mt >> 1] & 0xFFFFu);
				const uint32_t sca = xa2 - (uint32_t)sx2;
				const bool bada = sca >= (uint32_t)F.w2, badb = sca + 2u >= (uint32_t)F.w2;
				off = bada ? (badb ? 0x80000000u : off + 2u) : (badb ? off - 2u : off);
				fix[i] |= ((bada && !badb) ? 1u : ((!bada && badb) ? 2u : ((bada && badb) ? 3u : 0u))) << (2 * m);
			}
			/* interior tiles: the frame's term (R - sy) W 2 + 2 (x0 - sx), the shifted start of
			 * the tile's row segment, goes in the SGPR offset and the lane's voffset 4 l + 256 i
			 * stays fixed (no VALU per load).  The segment start is >= 0 for a row inside the
			 * frame (x0 >= max |sx| in an interior tile) and < 0 for a row above it; gfx950
			 * bounds-checks the unsigned sum voffset + soffset without wrapping
			 * (tools/soffset_probe.hip), so the latter (2^32 + start as unsigned) reads 0 */
			if (EDGE)
				dst[m][i] = __builtin_amdgcn_raw_buffer_load_b32(sgh_rsrc(b, nrec), (int)off, 0, SGH_LOAD_AUX);
			else
				dst[m][i] = __builtin_amdgcn_raw_buffer_load_b32(sgh_rsrc(b, nrec), (int)(xa2 - F.x02),
						(int)(k + F.x02), SGH_LOAD_AUX);
		}
		b += F.fstride2;
	}
}

template <bool EDGE>
__device__ __forceinline__ uint32_t sgh_fixup(uint32_t v, uint32_t fix, int m) {
	if (!EDGE)
		return v;
	const uint32_t f = (fix >> (2 * m)) & 3u;
	return f == 1u ? v << 16 : (f == 2u ? v >> 16 : v);
}

/* normalisation of a loaded pixel pair (:1635-1652): NORM 1 = round_to_WORD(v scale - offset),
 * 2 = round_to_WORD(v scale mul), 3 = NORM 1 with the + 0.5 folded into the offset, in the
 * reference's double operations; 4 (additive) / 5 (multiplicative) = trunc(fma(v, a, b)), one
 * rounding, with {a, b} from k_norm_fma_check, which ran only because that equals the reference's
 * operations for every u16 v of every frame; 6 (additive, scale 1) = clamp(v - K, 0, 65535) with an
 * integer K per frame, admitted the same way; rows outside the
 * frame (read as 0) are normalised like read samples, but columns outside the image (EDGE
 * fix codes 1..3) stay 0, as the x shift writes 0 straight into the stack (:1628-1632) */
template <int NORM, bool EDGE>
__device__ __forceinline__ uint32_t sgh_norm_pair(uint32_t v, double a, double b, uint32_t fix, int m) {
	if (NORM == 0)
		return v;
	if (NORM == 6) {
		/* additive with scale 1: sat(sat(v + kneg) - kpos) per half, K = kpos - kneg the frame's
		 * integer offset (the pair's bits: a = {kpos, kneg} replicated in both halves) */
		const sgh_u16x2 kp = __builtin_bit_cast(sgh_u16x2, (uint32_t)__double2loint(a));
		const sgh_u16x2 kn = __builtin_bit_cast(sgh_u16x2, (uint32_t)__double2hiint(a));
		uint32_t r = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_elementwise_add_sat(
				__builtin_bit_cast(sgh_u16x2, v), kn), kp));
		(void)b;
		if (EDGE) {
			const uint32_t f = (fix >> (2 * m)) & 3u;
			r &= f == 0u ? 0xFFFFFFFFu : (f == 1u ? 0xFFFF0000u : (f == 2u ? 0x0000FFFFu : 0u));
		}
		return r;
	}
	/* round_to_WORD(y) = min(trunc(y + 0.5), 65535) with the conversion's clamp of
	 * negative values to 0 (y <= 0 gives y + 0.5 <= 0.5, truncated to 0 either way) */
	auto g = [&](uint32_t x) -> uint32_t {
		const double t = (double)x * a;
		/* NORM 3: b = offset - 0.5 (exact, checked on the host), so trunc(t - b) is
		 * trunc(round(t - offset) + 0.5) of the reference with one add less */
		const double y = NORM >= 4 ? __builtin_fma((double)x, a, b) :
			NORM == 3 ? t - b : (NORM == 1 ? t - b : t * b) + 0.5;
		uint32_t r;
		asm("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(y));
		return r;
	};
	/* the two u32 results clamped to 65535 and packed by one v_cvt_pk_u16_u32 (saturating) */
	uint32_t r = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_u16((int)g(v & 0xFFFFu), (int)g(v >> 16)));
	if (EDGE) {
		const uint32_t f = (fix >> (2 * m)) & 3u;
		r &= f == 0u ? 0xFFFFFFFFu : (f == 1u ? 0xFFFF0000u : (f == 2u ? 0x0000FFFFu : 0u));
	}
	return r;
}

/* per-frame normalisation pair {scale, offset | mul} (one scalar load) */
__device__ __forceinline__ void sgh_coef(const SghRo &ro, int f, double &a, double &b) {
	const int4 v = ro.norm[f];
	const int x = __builtin_amdgcn_readfirstlane(v.x), y = __builtin_amdgcn_readfirstlane(v.y);
	const int z = __builtin_amdgcn_readfirstlane(v.z), w = __builtin_amdgcn_readfirstlane(v.w);
	a = __hiloint2double(y, x);
	b = __hiloint2double(w, z);
}

/* packed u16 min / saturating sub kept as single instructions (LLVM otherwise rewrites
 * min(v, 1) and sat(v - 65534) into per-half compares and selects) */
__device__ __forceinline__ uint32_t sgh_pk_min(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "s"(b));
	return r;
}
__device__ __forceinline__ uint32_t sgh_pk_sub_sat(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "s"(b));
	return r;
}
__device__ __forceinline__ uint32_t sgh_pk_add(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
}

__device__ __forceinline__ uint32_t sgh_pk_sub_wrap(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
}
__device__ __forceinline__ uint32_t sgh_pk_shl(uint32_t a, int n) {
	uint32_t r;
	asm("v_pk_lshlrev_b16 %0, %2, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "i"(n));
	return r;
}

/* bin the pixel pair of one frame (low half -> h[0], high half -> h[1], lane l4 = 4 l):
 * t = min(v - lo (mod 2^16), 256) is the band bin, or 256 = the out-of-band counter (row
 * 64) for anything below or above the band; row t >> 2 is at byte 256 (t >> 2), i.e. byte 1
 * of t << 6 (one byte permute each), the counter byte is t & 3, so the increment is
 * 1 << 8 (t & 3) = 1 << (8 t mod 32).  Zeros and 65535s are counted per half. */
/* The packed ops are written as vector builtins: the hazard recognizer cannot see into inline
 * asm and pads every asm result with an s_nop before its first use (31 per 8-frame half block
 * in the round-2 build).  The two counter constants (1, 65534 per half) come in as opaque SGPRs
 * (sgh_opaque, set once per tile), because LLVM rewrites a packed min(v, 1) / sat(v - 65534)
 * with literal operands into per-half compares and selects. */
#ifndef SGH_BIN_ASM
#define SGH_BIN_ASM 0
#endif
#ifndef SGH_BIN2
#define SGH_BIN2 1	/* interior whole half blocks bin two frames at a time (sgh_bin_pair2) */
#endif
__device__ __forceinline__ uint32_t sgh_opaque(uint32_t k) {
	uint32_t r;
	asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "i"(k));
	return r;
}
/* AB (stack_median / PERCENTILE kernels): also count the samples above the band, min(sat(v - hi), 1)
 * per half with hi = lo + 255, so the finish can place ranks and counts beside out-of-band samples
 * other than 0 / 65535 (unregistered stars in a median stack) */
template <bool AB = false>
__device__ __forceinline__ void sgh_bin_pair(uint32_t *h, uint32_t l4, uint32_t lo2, uint32_t vv,
		uint32_t &nonzero, uint32_t &nsat, uint32_t k1 = 0x00010001u, uint32_t ksat = 0xFFFEFFFEu,
		uint32_t *nab = nullptr, uint32_t hi2 = 0u) {
#if !SGH_BIN_ASM
	const sgh_u16x2 v16 = __builtin_bit_cast(sgh_u16x2, vv);
	if (AB)
		*nab += __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_sub_sat(v16,
				__builtin_bit_cast(sgh_u16x2, hi2)), __builtin_bit_cast(sgh_u16x2, k1)));
	const sgh_u16x2 tt = __builtin_elementwise_min(v16 - __builtin_bit_cast(sgh_u16x2, lo2), (sgh_u16x2){256, 256});
	const uint32_t t64 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(tt << (sgh_u16x2){6, 6}));
	const uint32_t t8 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(tt << (sgh_u16x2){3, 3}));
	const uint32_t a0 = __builtin_amdgcn_perm(t64, l4, 0x0c0c0500u), a1 = __builtin_amdgcn_perm(t64, l4, 0x0c0c0700u);
	const uint32_t i0 = 1u << (t8 & 31u), i1 = 1u << ((t8 >> 16) & 31u);
	atomicAdd((uint32_t *)((char *)h + a0), i0);
	atomicAdd((uint32_t *)((char *)h + sizeof(uint32_t) * SGH_HROWS * 64 + a1), i1);
	nonzero += __builtin_bit_cast(uint32_t, __builtin_elementwise_min(v16, __builtin_bit_cast(sgh_u16x2, k1)));
	nsat += __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(v16, __builtin_bit_cast(sgh_u16x2, ksat)));
#else
	(void)k1;
	(void)ksat;
	const uint32_t t = sgh_pk_min(sgh_pk_sub_wrap(vv, lo2), 0x01000100u);
	const uint32_t t64 = sgh_pk_shl(t, 6), t8 = sgh_pk_shl(t, 3);
	const uint32_t a0 = __builtin_amdgcn_perm(t64, l4, 0x0c0c0500u), a1 = __builtin_amdgcn_perm(t64, l4, 0x0c0c0700u);
	const uint32_t i0 = 1u << (t8 & 31u), i1 = 1u << ((t8 >> 16) & 31u);
	atomicAdd((uint32_t *)((char *)h + a0), i0);
	atomicAdd((uint32_t *)((char *)h + sizeof(uint32_t) * SGH_HROWS * 64 + a1), i1);
	/* plain u32 adds (no carry crosses the halves: a lane counts at most N / 4 frames), so
	 * the compiler folds the adds of consecutive frames into v_add3_u32 */
	nonzero += sgh_pk_min(vv, 0x00010001u);
	nsat += sgh_pk_sub_sat(vv, 0xFFFEFFFEu);
#endif
}

/* two frames of one pixel pair, their independent packed ops interleaved: a packed op that
 * reads the previous op's result needs a wait state (s_nop) on gfx950, the other frame's op
 * fills it */
template <bool AB = false>
__device__ __forceinline__ void sgh_bin_pair2(uint32_t *h, uint32_t l4, uint32_t lo2, uint32_t va, uint32_t vb,
		uint32_t &nonzero, uint32_t &nsat, uint32_t k1, uint32_t ksat, uint32_t *nab = nullptr, uint32_t hi2 = 0u) {
	const sgh_u16x2 a16 = __builtin_bit_cast(sgh_u16x2, va), b16 = __builtin_bit_cast(sgh_u16x2, vb);
	const sgh_u16x2 l16 = __builtin_bit_cast(sgh_u16x2, lo2), c256 = {256, 256};
	/* sched_barriers between the stages: the scheduler otherwise serialises the two frames again
	 * (it minimises live registers) and the wait states come back */
	const sgh_u16x2 da = a16 - l16, db = b16 - l16;
	__builtin_amdgcn_sched_barrier(0);
	const sgh_u16x2 ta = __builtin_elementwise_min(da, c256), tb = __builtin_elementwise_min(db, c256);
	__builtin_amdgcn_sched_barrier(0);
	const uint32_t a64 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(ta << (sgh_u16x2){6, 6}));
	const uint32_t b64 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(tb << (sgh_u16x2){6, 6}));
	const uint32_t a8 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(ta << (sgh_u16x2){3, 3}));
	const uint32_t b8 = __builtin_bit_cast(uint32_t, (sgh_u16x2)(tb << (sgh_u16x2){3, 3}));
	__builtin_amdgcn_sched_barrier(0);
	char *const h1 = (char *)h + sizeof(uint32_t) * SGH_HROWS * 64;
	atomicAdd((uint32_t *)((char *)h + __builtin_amdgcn_perm(a64, l4, 0x0c0c0500u)), 1u << (a8 & 31u));
	atomicAdd((uint32_t *)(h1 + __builtin_amdgcn_perm(a64, l4, 0x0c0c0700u)), 1u << ((a8 >> 16) & 31u));
	atomicAdd((uint32_t *)((char *)h + __builtin_amdgcn_perm(b64, l4, 0x0c0c0500u)), 1u << (b8 & 31u));
	atomicAdd((uint32_t *)(h1 + __builtin_amdgcn_perm(b64, l4, 0x0c0c0700u)), 1u << ((b8 >> 16) & 31u));
	const sgh_u16x2 k1v = __builtin_bit_cast(sgh_u16x2, k1), ksv = __builtin_bit_cast(sgh_u16x2, ksat);
	nonzero += __builtin_bit_cast(uint32_t, __builtin_elementwise_min(a16, k1v)) +
		__builtin_bit_cast(uint32_t, __builtin_elementwise_min(b16, k1v));
	nsat += __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(a16, ksv)) +
		__builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(b16, ksv));
	if (AB) {
		const sgh_u16x2 hv = __builtin_bit_cast(sgh_u16x2, hi2);
		*nab += __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_sub_sat(a16, hv), k1v)) +
			__builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_elementwise_sub_sat(b16, hv), k1v));
	}
}

/* normalised SIGMA / WINSORIZED builds: keep the value of an out-of-band sample other than 0 /
 * 65535 (a cosmic ray that the frame's scale moved off 65535, a cold pixel).  Such a sample
 * used to send its pixel to the redo list, whose kernel gathers the whole column again, one
 * scattered line per sample (1.2 % of the pixels under multiplicative scaling, 1.65 ms of
 * staging for 0.2 GB of data); with the few values known the finish writes the pixel's
 * sorted column itself (sgh_compact).  A rare branch: the test is four VALU ops per pair */
template <int NI>
__device__ __forceinline__ void sgh_capture(SghLds<NI> &L, int i, int lane, uint32_t lo2, uint32_t v, uint32_t k1,
		uint32_t ksat, uint32_t k255) {
	/* packed: sat(v - lo - 255) > 0 (outside the band) and min(v, 1) - sat(v - 65534) = 1 (not 0,
	 * not 65535); the last two are the build's own counter terms (shared after inlining) */
	const sgh_u16x2 v16 = __builtin_bit_cast(sgh_u16x2, v);
	const sgh_u16x2 d = __builtin_elementwise_sub_sat(v16 - __builtin_bit_cast(sgh_u16x2, lo2),
			__builtin_bit_cast(sgh_u16x2, k255));
	const sgh_u16x2 nrm = __builtin_elementwise_min(v16, __builtin_bit_cast(sgh_u16x2, k1)) -
		__builtin_elementwise_sub_sat(v16, __builtin_bit_cast(sgh_u16x2, ksat));
	const uint32_t g = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(d, nrm));
	if (__builtin_expect(g != 0u, 0)) {
		if (g & 0xFFFFu) {
			const int col = 128 * i + lane;
			const uint32_t k = atomicAdd(&L.ovn[col], 1u);
			if (k < SGH_OVK)
				L.ov[k][col] = (uint16_t)(v & 0xFFFFu);
		}
		if (g >> 16) {
			const int col = 128 * i + 64 + lane;
			const uint32_t k = atomicAdd(&L.ovn[col], 1u);
			if (k < SGH_OVK)
				L.ov[k][col] = (uint16_t)(v >> 16);
		}
	}
}

/* ------------------------------------------------------------------------------------
 * paired-lane finish: all 4 waves, 32 pixels per wave, the two lanes of a pair share one
 * pixel and split its work (prefix groups, the two medians, the two threshold queries and
 * their moments), exchanging results through DPP; both lanes carry identical loop state,
 * so a pair never diverges and the per-pixel instruction chain is about halved.
 * ------------------------------------------------------------------------------------ */
__device__ __forceinline__ uint32_t sgh_x(uint32_t v) {	/* value of the partner lane (quad_perm 1,0,3,2) */
	return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t sgh_x64(uint64_t v) {
	return (uint64_t)sgh_x((uint32_t)v) | ((uint64_t)sgh_x((uint32_t)(v >> 32)) << 32);
}

/* sum over the wave (all lanes active): row_shr 1, 2, 4, 8 with zero fill leave each 16-lane
 * row's total in its lane 15 */
__device__ __forceinline__ uint32_t sgh_wave_sum(uint32_t x) {
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
	x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
	return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) + (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
		(uint32_t)__builtin_amdgcn_readlane((int)x, 47) + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

/* value at global rank g (single rank) */
__device__ __forceinline__ int sgh_value_at1(const SghPix &P, int g) {
	const int r = g - P.nz;
	const bool in = r >= 0 && r < P.nb;
	const int grp = sgh_grp_of(P, r);
	uint32_t d[SGH_GRP];
	sgh_grp(P, grp, d);
	return in ? sgh_locate(P, grp, d, sgh_pre(P, P.pc, grp), (uint32_t)r) : (r < 0 ? 0 : 65535);
}

/* sigma = sqrt(num / (n (n - 1))) of the kept set (0 for num <= 0), as 2 num h with
 * h = 0.5 / sqrt(num n (n - 1)) refined twice from the hardware v_rsq_f64 (coupled Newton
 * steps on s ~ sqrt(x), h ~ 0.5 / sqrt(x): an initial relative error e becomes ~2 e^4, so a
 * few ulp in all), 8 dependent fp64 operations instead of the ~26 of an IEEE division and
 * square root.  The decisions keep a rounding band of 1e-13 relative (SGH_BAND), ~500 times
 * the error.  num < 2^53: num <= n^2 65535^2 / 4. */
__device__ __forceinline__ double sgh_sigma_fast(long long num, int n) {
	const double nd = (double)(num > 0 ? num : 1);
	const double x = nd * ((double)n * (double)(n - 1));
	const double y = __builtin_amdgcn_rsq(x);
	double h = 0.5 * y, s = x * y;
	double r = fma(-s, h, 0.5);
	s = fma(s, r, s);
	h = fma(h, r, h);
	r = fma(-s, h, 0.5);
	h = fma(h, r, h);
	const double sig = (nd + nd) * h;
	return num > 0 ? sig : 0.0;
}

/* a median rank query split in two: the group read is issued one pass ahead (the next
 * pass's ranks are known once the clip counts are), the locate runs when the value is needed */
struct SghMed {
	int r, grp;
	uint32_t d[SGH_GRP];
};
__device__ __forceinline__ void sgh_med_issue(const SghPix &P, int g, SghMed &m) {
	m.r = g - P.nz;
	m.grp = sgh_grp_of(P, m.r);
	sgh_grp(P, m.grp, m.d);
}
__device__ __forceinline__ int sgh_med_value(const SghPix &P, const SghMed &m) {
	const bool in = m.r >= 0 && m.r < P.nb;
	const int v = sgh_locate(P, m.grp, m.d, sgh_pre(P, P.pc, m.grp), (uint32_t)m.r);
	return in ? v : (m.r < 0 ? 0 : 65535);
}

/* the SIGMA loop (:1674-1695 + sigma_clipping :1148-1161) on the histogram, split over a lane
 * pair: half 0 owns the low side (median rank g1, threshold a - 1, M(A - 1)), half 1 the high
 * side (rank g2, threshold bt, M(B)).  The median's group read is issued during the previous
 * pass, sigma comes from sgh_sigma_fast, and the clamps and selects are straight-line code, so
 * a pass is one basic block (round 2: the loop's VALU count, not its dependency chain, is what
 * the kernel pays for; scripts/gpu_r2t.sh, gpu_r2w.sh). */
template <bool ZT, bool CAP = false>
__device__ __forceinline__ int sgh_sigma3(const SghPix &P, int N, double sl, double sh, int half, uint16_t *value,
		uint32_t *rlo_out, uint32_t *rhi_out, int &passes) {
	/* a query the below-band normalised zeros (ZT: additive normalisation) or the captured out-of-band
	 * samples (CAP) make undecidable here */
	auto zbad = [&](int v) { return ((ZT || CAP) && v >= 0 && v < P.zmax) || (CAP && v >= P.omin && v < 65535); };
	int A = 0, B = 65535, n = N, r = 0, nrem;
	SghM MA = {0, 0, 0}, MB = P.T;
	uint32_t rlo = 0, rhi = 0;
	SghMed md;
	sgh_med_issue(P, (int)((unsigned)(half ? N : N - 1) >> 1), md);
	do {
		const long long S = MB.s - MA.s;
		const unsigned long long SS = MB.ss - MA.ss;
		const long long num = (long long)n * (long long)SS - S * S;
		const bool exact0 = (num == 0);
		const double sigma = sgh_sigma_fast(num, n);
		/* n >= 4: the halvings as unsigned shifts; the median as (m1 + m2) * 0.5 (exact), with
		 * m2 = m1 for odd n, so no branch */
		const int mv = sgh_med_value(P, md);
		/* a median rank among below-band samples that are not all zeros, or among above-band ones that are
		 * not all 65535 */
		uint32_t zb = (((ZT || CAP) && P.zmax && md.r < 0) || (CAP && P.omin < 65535 && md.r >= P.nb)) ? 1u : 0u;
		const int mo = (int)sgh_x((uint32_t)mv);
		const int m1 = half ? mo : mv, m2 = (n & 1) ? m1 : (half ? mv : mo);
		const double median = (double)(m1 + m2) * 0.5;
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		const double tol = exact0 ? 0.0 : SGH_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
		int a = sgh_ceil_clamp(blo - tol);
		a = a < A ? A : a;
		int bt = sgh_floor_clamp(bhi + tol);
		bt = bt > B ? B : bt;
		SghQ q;
		sgh_q_load(P, half ? bt : a - 1, q);
		if (zbad(half ? bt : a - 1))
			zb = 1u;
		const int cm = sgh_q_count(P, q), co = (int)sgh_x((uint32_t)cm);
		const int cnt_a = half ? co : cm, cnt_bt = half ? cm : co;
		uint32_t amb = 0;
		if (!exact0) {
			if (!half) {
				int amb1 = sgh_floor_clamp(blo + tol);
				amb1 = amb1 > B ? B : amb1;
				amb = (a <= amb1 && sgh_cnt_le(P, amb1) - cnt_a > 0) ? 1u : 0u;
				if (a <= amb1 && zbad(amb1))
					zb = 1u;
			} else {
				int amb0 = sgh_ceil_clamp(bhi - tol);
				amb0 = amb0 < A ? A : amb0;
				amb = (amb0 <= bt && cnt_bt - sgh_cnt_le(P, amb0 - 1) > 0) ? 1u : 0u;
				if (amb0 <= bt && zbad(amb0 - 1))
					zb = 1u;
			}
		}
		amb |= zb;
		if (amb | sgh_x(amb))
			return 1;
		const int L = cnt_a - MA.c, H = MB.c - cnt_bt;
		if (L + H > n)
			return 1;
		/* `if (N - r <= 4) break;` inside the clipping loop (:1684) */
		const int need = n - 4 - r;
		int fb = -1;
		if (need <= 0)
			fb = 0;
		else if (L >= need)
			fb = need - 1;
		else if (L + H >= need)
			fb = (n - H) + (need - L) - 1;
		if (fb >= 0 && fb < n - 1)
			return 1;
		/* a pass that removes nothing is the last one: no next median, no moments (both lanes
		 * of a pair take the branch together, so the exchanges inside see an active partner) */
		if (L | H) {
			/* the next pass's median ranks: kept count n - L - H starting at rank cnt_a (or MA.c) */
			const int ca = L ? cnt_a : MA.c, nn = n - L - H;
			sgh_med_issue(P, ca + (int)((unsigned)(half ? nn : nn - 1) >> 1), md);
			/* moments of this lane's bound; field-wise selects (a select of whole structs
			 * becomes a scratch access) */
			const SghM Mq = sgh_q_moments(P, q);
			const bool mine = half ? (H != 0) : (L != 0);
			const int mc = mine ? Mq.c : (half ? MB.c : MA.c);
			const long long ms = mine ? Mq.s : (half ? MB.s : MA.s);
			const unsigned long long mss = mine ? Mq.ss : (half ? MB.ss : MA.ss);
			const int oc = (int)sgh_x((uint32_t)mc);
			const long long os = (long long)sgh_x64((uint64_t)ms);
			const unsigned long long oss = sgh_x64(mss);
			if (L) {
				A = a;
				MA.c = half ? oc : mc;
				MA.s = half ? os : ms;
				MA.ss = half ? oss : mss;
			}
			if (H) {
				B = bt;
				MB.c = half ? mc : oc;
				MB.s = half ? ms : os;
				MB.ss = half ? mss : oss;
			}
		}
		rlo += L;
		rhi += H;
		r += L + H;
		nrem = L + H;
		n -= nrem;
		passes++;
	} while (nrem > 0 && n > 3);
	const long long tot = (MB.s - MA.s) + (long long)n * P.lo;
	*value = sg_round_to_WORD((double)tot / (double)n);
	*rlo_out = rlo;
	*rhi_out = rhi;
	return SG_CLS_OK;
}

/* ------------------------------------------------------------------------------------
 * WINSORIZED (:1710-1749 + Winsorized :1163-1168) on the histogram, mirroring
 * reject_winsorized() of the sorted path decision for decision.  The kept set is the value
 * interval [A, B] (moments MA = M(A-1), MB = M(B), as in SIGMA); the Winsorized copy w of
 * the sorted kept samples is Lw copies of vlo, the kept samples with values in [IA, IB]
 * (the inner part, moments MI_A = M(IA-1), MI_B = M(IB)), Hw copies of vhi; clamping keeps
 * w sorted, so its median is a rank query and its moments are the inner moments plus the
 * clamped copies.  Both lanes of a pair run the same loop (no split); moments are relative
 * to lo, and sd is shift invariant.
 * ------------------------------------------------------------------------------------ */
__device__ __forceinline__ double sgh_sd_rel(int n, long long S, long long SS, bool *e0) {
	const long long num = (long long)n * SS - S * S;
	*e0 = (num == 0);
	return sgh_sigma_fast(num, n);
}
/* sqrt(x) for x > 0 from v_rsq_f64 and two coupled Newton steps (as sgh_sigma_fast) */
__device__ __forceinline__ double sgh_sqrt_fast(double x) {
	const double y = __builtin_amdgcn_rsq(x);
	double h = 0.5 * y, s = x * y;
	double r = fma(-s, h, 0.5);
	s = fma(s, r, s);
	h = fma(h, r, h);
	r = fma(-s, h, 0.5);
	return fma(s, r, s);
}
/* round_to_WORD(m) decision ambiguous (m within tol of 0, 65535 or a .5) */
__device__ __forceinline__ bool sgh_round_ambiguous(double m, double tol) {
	if (fabs(m) <= tol || fabs(m - 65535.0) <= tol)
		return true;
	if (m <= 0.0 || m > 65535.0)
		return false;
	const double t = m + 0.5;
	return fabs(t - rint(t)) <= tol;
}

/* # samples with value < thr (thr real) */
__device__ __forceinline__ int sgh_cnt_lt(const SghPix &P, double thr) {
	/* v < thr <=> v <= ceil(thr) - 1 */
	double c = ceil(thr) - 1.0;
	if (c < -1.0)
		c = -1.0;
	if (c > 65535.0)
		c = 65535.0;
	return sgh_cnt_le(P, (int)c);
}
/* # samples with value <= thr */
__device__ __forceinline__ int sgh_cnt_le_d(const SghPix &P, double thr) {
	double c = floor(thr);
	if (c < -1.0)
		c = -1.0;
	if (c > 65535.0)
		c = 65535.0;
	return sgh_cnt_le(P, (int)c);
}

__device__ __forceinline__ SghM sgh_M_le(const SghPix &P, int v) {
	SghQ q;
	sgh_q_load(P, v, q);
	return sgh_q_moments(P, q);
}

/* ------------------------------------------------------------------------------------
 * SIGMEDIAN (:1696-1709 + sigma_clipping :1148-1161) on the histogram, decision for decision
 * reject_sigmedian() of the sorted path: a clipped sample is replaced by round_to_WORD(median)
 * and N stays, so the pixel's multiset is the window of samples never replaced - the values in
 * [A, B], moments M(A - 1), M(B) as in SIGMA - plus up to SGH_SMG groups of equal replacement
 * values (gc = 0: a free slot; the groups are unordered, their ranks are counted).  sigma comes
 * from the exact moments of the whole multiset, decisions keep the rounding band, a decision
 * inside it, a fifth group, a pass that replaces samples by the values they hold (the
 * reference's loop never ends there) or 4096 passes go to the redo list (the sorted path takes
 * them and reports what the reference would do).  One lane per pixel.
 * ------------------------------------------------------------------------------------ */
#define SGH_SMG 4
__device__ __forceinline__ double sgh_sigma_num(long long S, unsigned long long SS, int n, bool &e0) {
	/* n SS - S^2 in 128 bits (relative moments: S^2 passes 2^63 for large N), then as sgh_sigma_fast */
	const __int128 num = (__int128)n * (__int128)SS - (__int128)S * (__int128)S;
	e0 = num == 0;
	if (num <= 0)
		return 0.0;
	const double nd = (double)num;
	const double x = nd * ((double)n * (double)(n - 1));
	const double y = __builtin_amdgcn_rsq(x);
	double h = 0.5 * y, s = x * y;
	double r = fma(-s, h, 0.5);
	s = fma(s, r, s);
	h = fma(h, r, h);
	r = fma(-s, h, 0.5);
	h = fma(h, r, h);
	return (nd + nd) * h;
}
__device__ int sgh_sigmedian(const SghPix &P, int N, double sl, double sh, uint16_t *value, uint32_t *rlo_out,
		uint32_t *rhi_out) {
	int A = 0, B = 65535;
	SghM MA = {0, 0, 0}, MB = P.T;
	uint32_t gv[SGH_SMG];
	int gc[SGH_SMG];
#pragma unroll
	for (int k = 0; k < SGH_SMG; k++) {
		gv[k] = 0u;
		gc[k] = 0;
	}
	long long S = P.T.s;			/* the multiset's moments, values relative to lo */
	unsigned long long SS = P.T.ss;
	uint32_t rlo = 0, rhi = 0;
	int iter = 0, n;
	/* window samples with value <= v (v integer) */
	auto wle = [&](int v) -> int {
		int c = sgh_cnt_le(P, v);
		c = c < MA.c ? MA.c : (c > MB.c ? MB.c : c);
		return c - MA.c;
	};
	/* multiset elements < t / <= t (t real) */
	auto cnt_lt = [&](double t) -> int {
		double cv = ceil(t) - 1.0;
		cv = cv < -1.0 ? -1.0 : (cv > 65535.0 ? 65535.0 : cv);
		int c = wle((int)cv);
#pragma unroll
		for (int k = 0; k < SGH_SMG; k++)
			c += (gc[k] && (double)gv[k] < t) ? gc[k] : 0;
		return c;
	};
	auto cnt_le = [&](double t) -> int {
		double cv = floor(t);
		cv = cv < -1.0 ? -1.0 : (cv > 65535.0 ? 65535.0 : cv);
		int c = wle((int)cv);
#pragma unroll
		for (int k = 0; k < SGH_SMG; k++)
			c += (gc[k] && (double)gv[k] <= t) ? gc[k] : 0;
		return c;
	};
	do {
		if (++iter > 4096)
			return SG_CLS_LITERAL;
		bool e0;
		const double sigma = sgh_sigma_num(S, SS, N, e0);
		/* median ranks: group k's copies start at rank st[k] = window samples < gv_k + the group
		 * copies of smaller values; a rank in no group's run is a window rank */
		int st[SGH_SMG];
#pragma unroll
		for (int k = 0; k < SGH_SMG; k++) {
			int b = 0;
#pragma unroll
			for (int j = 0; j < SGH_SMG; j++)
				b += (j != k && gc[j] && gv[j] < gv[k]) ? gc[j] : 0;
			st[k] = gc[k] ? wle((int)gv[k] - 1) + b : 0;
		}
		auto at = [&](int r) -> int {
			int before = 0, gval = -1;
#pragma unroll
			for (int k = 0; k < SGH_SMG; k++) {
				if (gc[k]) {
					if (r >= st[k] && r < st[k] + gc[k])
						gval = (int)gv[k];
					before += (st[k] + gc[k] <= r) ? gc[k] : 0;
				}
			}
			return gval >= 0 ? gval : sgh_value_at1(P, MA.c + (r - before));
		};
		const int g1 = (N - 1) / 2, g2 = N / 2;
		const int m1 = at(g1), m2 = g1 == g2 ? m1 : at(g2);
		const double median = g1 == g2 ? (double)m1 : (double)(m1 + m2) / 2.0;
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		double tlo = blo, thi = bhi;
		if (!e0) {
			const double tol = SGH_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
			if (cnt_lt(blo - tol) != cnt_le(blo + tol) || cnt_lt(bhi - tol) != cnt_le(bhi + tol))
				return SG_CLS_LITERAL;
			tlo = blo - tol;	/* no element lies within tol of either threshold */
			thi = bhi + tol;
		}
		const int L = cnt_lt(tlo), H = N - cnt_le(thi);
		if (L + H > N)
			return SG_CLS_LITERAL;	/* negative sigma factors: the else-if order matters */
		n = L + H;
		rlo += (uint32_t)L;
		rhi += (uint32_t)H;
		if (!n)
			break;
		/* the window's replaced ends, then the replaced groups */
		int A2 = sgh_ceil_clamp(tlo), B2 = sgh_floor_clamp(thi);
		A2 = A2 < A ? A : A2;
		B2 = B2 > B ? B : B2;
		SghM MA2 = A2 > A ? sgh_M_le(P, A2 - 1) : MA;
		SghM MB2 = B2 < B ? sgh_M_le(P, B2) : MB;
		if (MB2.c < MA2.c)	/* the whole window replaced */
			MB2 = MA2;
		long long rs = (MA2.s - MA.s) + (MB.s - MB2.s);
		unsigned long long rss = (MA2.ss - MA.ss) + (MB.ss - MB2.ss);
#pragma unroll
		for (int k = 0; k < SGH_SMG; k++) {
			if (gc[k] && ((double)gv[k] < tlo || (double)gv[k] > thi)) {
				const long long u = (long long)gv[k] - P.lo;
				rs += u * gc[k];
				rss += (unsigned long long)(u * u) * (unsigned long long)gc[k];
				gc[k] = 0;
			}
		}
		const uint32_t mw = sg_round_to_WORD(median);
		const long long um = (long long)mw - P.lo;
		if (rs == um * n && rss == (unsigned long long)(um * um) * (unsigned long long)n)
			return SG_CLS_LITERAL;	/* the next pass sees the same multiset: never ends */
		S += um * n - rs;
		SS += (unsigned long long)(um * um) * (unsigned long long)n - rss;
		/* the n replacements join the group of value mw, or a free slot */
		int slot = -1;
#pragma unroll
		for (int k = SGH_SMG - 1; k >= 0; k--)
			slot = (gc[k] == 0) ? k : slot;
#pragma unroll
		for (int k = SGH_SMG - 1; k >= 0; k--)
			slot = (gc[k] && gv[k] == mw) ? k : slot;
		if (slot < 0)
			return SG_CLS_LITERAL;
#pragma unroll
		for (int k = 0; k < SGH_SMG; k++) {
			if (k == slot) {
				gc[k] = (gc[k] && gv[k] == mw) ? gc[k] + n : n;
				gv[k] = mw;
			}
		}
		A = A2;
		B = B2;
		MA = MA2;
		MB = MB2;
	} while (n > 0 && N > 3);
	const long long tot = S + (long long)N * P.lo;
	*value = sg_round_to_WORD((double)tot / (double)N);
	*rlo_out = rlo;
	*rhi_out = rhi;
	return SG_CLS_OK;
}

/* One threshold query of the Winsorized loop: the samples <= v (count, and their moments
 * relative to lo as exact doubles) and the neighbouring sample value on one side, dir 0 the
 * smallest sample > v, dir 1 the largest sample <= v, from ONE read of the group holding v's
 * bin.  A clamp growth needs all three (the count decides the clamp, the moments leave the
 * inner part, the neighbour is the inner part's new end), which the round-2 loop formed with
 * three separate queries (sgh_cnt_le, sgh_M_le, sgh_value_at1: three group reads).  A
 * neighbour outside the group (or outside the band) comes from a rank query. */
struct SghX {
	int c;		/* samples <= v */
	double s, ss;	/* their sum and sum of squares of (value - lo) */
	int nb;		/* the neighbouring sample value, or a bound on it (sgh_qx) */
};
__device__ __forceinline__ SghX sgh_qx(const SghPix &P, int v, int dir) {
	int t = v - P.lo;
	t = t < -1 ? -1 : (t > SGH_BINS - 1 ? SGH_BINS - 1 : t);
	const int tc = t < 0 ? 0 : t;
	const int g = tc >> 5;
	/* the group's 8 dwords and the boundary dword (the one holding bin tc) read once more
	 * instead of selected (SghQ's trick).  The group prefixes stay in registers: kept in LDS
	 * (25 dwords per column) they grew a tile to 49.5 KB of LDS and cost 3.5 ms on configs[4] -
	 * at 36.7 KB a fourth tile fits a CU while other tiles' waves 2 / 3 have left after their
	 * build (profiles/r03_wins_ab.log) */
	uint32_t d[SGH_GRP];
	sgh_grp(P, g, d);
	const uint32_t bw = P.hb[((P.col >> 6) * SGH_HROWS + (tc >> 2)) * 64 + (P.col & 63)];
	const uint32_t pc = sgh_pre(P, P.pc, g), ps = sgh_pre(P, P.ps, g), pss = sgh_pre(P, P.pss, g);
	const int kb = (t >> 2) - g * SGH_GRP;	/* -1 for t = -1: nothing at or below v in the band */
	const uint32_t mt = t >= 0 ? 0xFFFFFFFFu >> (24 - 8 * (t & 3)) : 0u;	/* bins <= t of the boundary dword */
#pragma unroll
	for (int k = 0; k < SGH_GRP; k++)
		d[k] = k < kb ? d[k] : 0u;
	const uint32_t bd = bw & mt;
	uint32_t c = __builtin_amdgcn_sad_u8(bd, 0u, 0u), s = 0, ss = 0;
	sgh_grp_moments(d, c, s, ss);
	/* the boundary dword: bins j = 4 kq + b, j^2 = (4 kq)^2 + 2 (4 kq) b + b^2 */
	const uint32_t kq = (uint32_t)((tc >> 2) - g * SGH_GRP);
	const uint32_t cb = __builtin_amdgcn_sad_u8(bd, 0u, 0u);
	const uint32_t sb = __builtin_amdgcn_udot4(bd, 0x03020100u, 0u, false);
	const uint32_t qb = __builtin_amdgcn_udot4(bd, 0x09040100u, 0u, false);
	const uint32_t k4 = 4u * kq;
	ss += qb + __umul24(2u * k4, sb) + __umul24(__umul24(k4, k4), cb);
	s += sb + __umul24(k4, cb);
	const uint32_t b0 = (uint32_t)g * (4u * SGH_GRP);
	SghX x;
	x.c = P.nz + (int)(pc + c);
	x.s = P.zs + (double)(ps + s + __umul24(b0, c));
	x.ss = P.zss + (double)(pss + ss + __umul24(2u * b0, s) + __umul24(__umul24(b0, b0), c));
	if (v < 0) {
		x.c = 0;
		x.s = x.ss = 0.0;
	}
	if (v >= 65535) {
		x.c = P.T.c;
		x.s = (double)P.T.s;
		x.ss = (double)P.T.ss;
	}
	/* neighbour from the boundary dword only: up, the first non-empty bin above t in it (else
	 * a lower bound: the next dword's first bin, or v + 1); down, the last non-empty bin at or
	 * below t in it (else an upper bound: the dword's first bin - 1, or v).  Bounds are all
	 * the Winsorized loop asks of its inner-part ends (sgh_winsorized) */
	const int base = P.lo + 4 * (tc >> 2);
	const uint32_t wu = bw & ~mt, wd = bd;
	const int up = t < 0 ? v + 1 : base + 4;
	const int dn = t < 0 ? v : base - 1;
	const int vf = wu && v >= 0 ? base + (int)(__builtin_ctz(wu) >> 3) : (up > v + 1 ? up : v + 1);
	const int vl = wd && v < 65535 ? base + (int)((31 - __builtin_clz(wd)) >> 3) : (dn < v ? dn : v);
	x.nb = dir ? vl : vf;
	return x;
}

/* A/B probe build (-DSGH_WPROF): wave time per region of the Winsorized finish.  One active
 * lane (the first in EXEC) adds the cycles since the wave's previous checkpoint to the region
 * that ends here, so divergent control flow is counted once per wave; slot 0 = last stamp,
 * 1..7 regions, 8 inner iterations, 9 passes */
#ifdef SGH_WPROF
__device__ __forceinline__ void sgh_wp(uint64_t *w, int region, int cnt = 0) {
	const uint64_t now = __builtin_readcyclecounter();
	const uint64_t ex = __builtin_amdgcn_read_exec();
	if ((int)(threadIdx.x & 63) == __builtin_ctzll(ex)) {
		if (region >= 0)
			w[1 + region] += now - w[0];
		w[0] = now;
		if (cnt)
			w[7 + cnt]++;
	}
}
#define SGH_WP(r, c) sgh_wp(P.wp, r, c)
__device__ __forceinline__ void sgh_wpev(uint64_t *w, int k) {
	const uint64_t ex = __builtin_amdgcn_read_exec();
	if ((int)(threadIdx.x & 63) == __builtin_ctzll(ex))
		w[10 + k]++;
}
#define SGH_WPEV(k) sgh_wpev(P.wp, k)
#else
#define SGH_WP(r, c)
#define SGH_WPEV(k)
#endif

template <bool CAP = false>
__device__ int sgh_winsorized(const SghPix &P, int N, double sl, double sh, int cap, uint16_t *value, uint32_t *rlo_out,
		uint32_t *rhi_out) {
	/* CAP: the pixel's captured out-of-band samples (sgh_finish2, round 6) make a query at v in
	 * [0, zmax) or [omin, 65535), or a median rank among the out-of-band samples, undecidable here;
	 * the neighbour bounds of sgh_qx and the kept ends klo / khi stay bounds elsewhere */
	auto zbad = [&](int v) { return CAP && ((v >= 0 && v < P.zmax) || (v >= P.omin && v < 65535)); };
	auto rbad = [&](int g) { const int r = g - P.nz; return CAP && ((r < 0 && P.zmax > 0) || (r >= P.nb && P.omin < 65535)); };
	int A = 0, B = 65535, n = N, r = 0, nrem;
	SghM MA = {0, 0, 0}, MB = P.T;
	uint32_t rlo = 0, rhi = 0;
#ifdef SGH_WINS_ITERS
	*rlo_out = 0;
#endif
	/* smallest / largest kept sample at the start of a pass (a lower / an upper bound from the
	 * second pass on: the clip queries' neighbours, sgh_qx); the first pass's from two rank
	 * queries */
	int klo = sgh_value_at1(P, 0), khi = sgh_value_at1(P, N - 1);
	do {
		const long long S = MB.s - MA.s;
		const long long SS = (long long)(MB.ss - MA.ss);
		bool e0;
		double sigma = sgh_sd_rel(n, S, SS, &e0);
		const int g1 = MA.c + (n - 1) / 2, g2 = MA.c + n / 2;
		int km1, km2;	/* kept values at the median ranks: fixed for the whole pass */
		if (rbad(g1) || rbad(g2))
			return 1;
		sgh_value_at2(P, g1, g2, km1, km2);
		double median = (g1 == g2) ? (double)km1 : (double)(km1 + km2) / 2.0;
		SGH_WP(1, 2);
		/* inner loop.  The inner part of w is the kept ranks [Lw, n - Hw); ulo <= its smallest
		 * value and uhi >= its largest (bounds: sgh_qx does not leave a histogram group to find
		 * them), so a threshold outside [ulo, uhi) - the common case once the clamps have
		 * settled - needs no histogram query, and one inside it is counted by one sgh_qx, which
		 * also gives the moments that leave the inner part and its new end.  The median of w is
		 * vlo, vhi or km1 / km2 */
		int Lw = 0, Hw = 0, vlo = 0, vhi = 0;
		/* inner-part bounds: counts as int, moments as doubles (exact: |S| <= N 65535 and
		 * SS <= N 65535^2 stay below 2^53) */
		int ciA = MA.c, ciB = MB.c;
		double sA = (double)MA.s, ssA = (double)MA.ss, sB = (double)MB.s, ssB = (double)MB.ss;
		int ulo = klo, uhi = khi;
		const double inn = 1.0 / ((double)n * (double)(n - 1));
		bool sig_e0 = e0;
		for (int guard = 0;; guard++) {
			SGH_WP(4, 1);
			if (guard >= cap)
				return 1;	/* a long Winsorize (hundreds of iterations with several 0 / 65535
					 * samples) goes to the replay rather than holding its wave */
#ifdef SGH_WINS_ITERS	/* A/B probe build: inner iterations (low 16 bits) and outer passes (high) */
			(*rlo_out)++;
#endif
			const double m0 = median - 1.5 * sigma, m1d = median + 1.5 * sigma;
			const double tol = sig_e0 ? 0.0 : SGH_BAND * (fabs(median) + 1.5 * sigma + 1.0);
			const int nin = n - Lw - Hw;
			auto v_lt = [](double thr) {
				const double c = ceil(thr) - 1.0;
				return c < -1.0 ? -1 : (c > 65535.0 ? 65535 : (int)c);
			};
			auto v_le = [](double thr) {
				const double c = floor(thr);
				return c < -1.0 ? -1 : (c > 65535.0 ? 65535 : (int)c);
			};
			/* the common case as one floor per side: when m lies more than 2 t (t = the
			 * rounding check's band, >= tol) from every integer and from every half-integer,
			 * ceil(m - tol) - 1 = floor(m + tol) = floor(m), round_to_WORD(m) is decided and
			 * not ambiguous; otherwise the thresholds come from the general formulas.  Either
			 * way a1 = ceil(m0 - tol) - 1 and b1 = floor(m1 + tol): the clamp bounds IA - 1
			 * and IB of the round-2 loop, so a growth's moments are the query's own */
			const double t2 = 2.0 * (tol + 1e-9 * tol);
			const double fl0 = floor(m0), fr0 = m0 - fl0, fl1 = floor(m1d), fr1 = m1d - fl1;
			const bool fast0 = fr0 > t2 && fr0 < 1.0 - t2 && fabs(fr0 - 0.5) > t2;
			const bool fast1 = fr1 > t2 && fr1 < 1.0 - t2 && fabs(fr1 - 0.5) > t2;
			auto clampv = [](double c) { return c < -1.0 ? -1 : (c > 65535.0 ? 65535 : (int)c); };
			auto round_fast = [](double m, double fl, double fr) -> int {
				return m <= 0.0 ? 0 : (m > 65535.0 ? 65535 : (int)fl + (fr > 0.5 ? 1 : 0));
			};
			if (!fast0 || !fast1)
				SGH_WPEV(2);
			const int a1 = fast0 ? clampv(fl0) : v_lt(m0 - tol), a2 = fast0 ? a1 : v_le(m0 + tol);
			const int b1 = fast1 ? clampv(fl1) : v_le(m1d + tol), b2 = fast1 ? b1 : v_lt(m1d - tol);
			/* the growth queries of both sides through ONE query site: a lane runs its low query,
			 * then its high one, so a wave executes the query body max(queries per lane) times
			 * (the round-2 loop had six query sites, each run when any lane needed it) */
			const bool needL = nin > 0 && a1 >= ulo && a1 < uhi;
			const bool needH = nin > 0 && b1 >= ulo && b1 < uhi;
			/* a query writes its side's inner-part bound and moments straight into the state
			 * (a query that finds no growth returns the moments the state already holds: no
			 * sample lies between the last growth's threshold and this one, since a1 >= ulo); the
			 * count checks below use the values from before the queries */
			const int ciA0 = ciA, ciB0 = ciB, ulo0 = ulo, uhi0 = uhi;
			int cL = 0, cH = 0;
			int pend = (needL ? 1 : 0) | (needH ? 2 : 0);
			SGH_WP(2, 0);
#pragma clang loop unroll(disable)
			while (pend != 0) {
				SGH_WPEV(0);
				const int side = (pend & 1) ? 0 : 1;
				if (zbad(side ? b1 : a1))
					return 1;
				const SghX x = sgh_qx(P, side ? b1 : a1, side);
#ifdef SGH_QX_TWICE	/* A/B probe build: every query body runs twice (its price in the kernel time) */
				uint32_t z0;
				asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
				const int qx_extra = sgh_qx(P, (side ? b1 : a1) + (int)z0, side).c & (int)z0;
#else
				const int qx_extra = 0;
#endif
				if (side) {
					cH = x.c + qx_extra;
					sB = x.s;
					ssB = x.ss;
					uhi = x.nb;
				} else {
					cL = x.c;
					sA = x.s;
					ssA = x.ss;
					ulo = x.nb;
				}
				pend &= pend - 1;
			}
			SGH_WP(3, 0);
			/* # w elements <= v: the clamped copies plus the inner ones (v's count, when v lies
			 * in [ulo, uhi), is the query's; in the rare ambiguous cases a second threshold's
			 * count comes from a plain count query) */
			auto w_le = [&](int v, bool have, int cq) {
				int c = (Lw && vlo <= v) ? Lw : 0;
				if (nin > 0 && v >= ulo0) {
					if (v >= uhi0) {
						c += nin;
					} else {
						if (!have)
							SGH_WPEV(1);
						if (!have && zbad(v))
							return -1;
						int k = have ? cq : sgh_cnt_le(P, v);
						k = k < ciA0 ? ciA0 : (k > ciB0 ? ciB0 : k);
						c += k - ciA0;
					}
				}
				if (Hw && vhi <= v)
					c += Hw;
				return c;
			};
			const int clo = w_le(a1, true, cL);
			if (!sig_e0 && a2 != a1) {
				const int c2 = w_le(a2, false, 0);
				if (c2 < 0 || clo != c2)
					return 1;
			}
			const int chi = n - w_le(b1, true, cH);
			if (!sig_e0 && b2 != b1) {
				const int c2 = w_le(b2, false, 0);
				if (c2 < 0 || chi != n - c2)
					return 1;
			}
			if (clo + chi > n)
				return 1;
			if (clo > 0) {
				if (!fast0 && sgh_round_ambiguous(m0, tol + 1e-9 * tol))
					return 1;
				if (clo < Lw || clo > n - Hw)
					return 1;
				if (clo > Lw) {
					/* the inner samples below m0 join the clamped copies */
					if (!needL)
						return 1;	/* every inner sample clamped at once: the sorted path decides */
					SGH_WPEV(3);
					ciA = cL;
				}
				Lw = clo;
				vlo = fast0 ? round_fast(m0, fl0, fr0) : sg_round_to_WORD(m0);
			}
			if (chi > 0) {
				if (!fast1 && sgh_round_ambiguous(m1d, tol + 1e-9 * tol))
					return 1;
				if (chi < Hw || chi > n - Lw)
					return 1;
				if (chi > Hw) {
					if (!needH)
						return 1;
					SGH_WPEV(4);
					ciB = cH;
				}
				Hw = chi;
				vhi = fast1 ? round_fast(m1d, fl1, fr1) : sg_round_to_WORD(m1d);
			}
			if (ciB - ciA != n - Lw - Hw)
				return 1;	/* inner part and clamp counts disagree: leave it to the sorted path */
			/* median of w: the kept values at the median ranks unless clamped */
			{
				const int lhs = (n - 1) / 2, rhs = n / 2;
				const int wl = lhs < Lw ? vlo : (lhs >= n - Hw ? vhi : km1);
				const int wr = rhs < Lw ? vlo : (rhs >= n - Hw ? vhi : km2);
				median = (lhs == rhs) ? (double)wl : (double)(wl + wr) / 2.0;
			}
			/* with N <= 1448 every Winsorized moment is an integer under 2^53, so the double
			 * arithmetic is exact and the iteration needs no 64-bit integer multiplies
			 * (quarter-rate v_mul_lo / v_mad_u64) */
			const double Sin = sB - sA, SSin = ssB - ssA;
			double num;
			if (N <= SGH_WIN_DBL_MAXN) {
				const double dl = (double)(vlo - P.lo), dh = (double)(vhi - P.lo);
				const double Lf = (double)Lw, Hf = (double)Hw;
				const double Sw = fma(dh, Hf, fma(dl, Lf, Sin));
				const double SSw = fma(dh * dh, Hf, fma(dl * dl, Lf, SSin));
				num = (double)n * SSw - Sw * Sw;
			} else {
				const long long dl = (long long)vlo - P.lo, dh = (long long)vhi - P.lo;
				const long long Sw = (long long)Sin + dl * Lw + dh * Hw;
				const long long SSw = (long long)SSin + dl * dl * Lw + dh * dh * Hw;
				num = (double)((long long)n * SSw - Sw * Sw);
			}
			const double sigma0 = sigma;
			const bool e00 = sig_e0;
			const bool we0 = (num == 0.0);
			sigma = 1.134 * (num > 0.0 ? sgh_sqrt_fast(num * inn) : 0.0);
			sig_e0 = we0;
			if (e00) {
				SGH_WPEV(5);
				if (we0)
					break;	/* 0/0 = NaN: the loop exits */
				continue;	/* x/0 = inf > 0.0005 */
			}
			/* |sigma - sigma0| / sigma0 > 0.0005 as the sign of d = |sigma - sigma0| -
			 * 0.0005 sigma0 (sigma0 > 0 here): no division; |d| <= 7e-13 sigma0 covers the
			 * band |q - 0.0005| <= 5e-13 + 1e-13 (1 + q) of the divided form near q = 0.0005 */
			const double d = fabs(sigma - sigma0) - 0.0005 * sigma0;
			if (fabs(d) <= 7e-13 * sigma0)
				return 1;
			if (!(d > 0.0))
				break;
		}
		SGH_WP(4, 0);
		/* clip pass on the kept set with the Winsorized sigma / median (:1731-1747) */
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		const double tol = sig_e0 ? 0.0 : SGH_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
		int a = sgh_ceil_clamp(blo - tol);
		if (a < A)
			a = A;
		int bt = sgh_floor_clamp(bhi + tol);
		if (bt > B)
			bt = B;
		/* the clip counts, moments and the next pass's kept ends (exact doubles: relative to lo,
		 * SS <= 65535^3 < 2^53) */
		if (zbad(a - 1) || zbad(bt))
			return 1;
		const SghX xa = sgh_qx(P, a - 1, 0), xb = sgh_qx(P, bt, 1);
		const int cnt_a = xa.c, cnt_bt = xb.c;
		if (!sig_e0) {
			int amb1 = sgh_floor_clamp(blo + tol);
			if (amb1 > B)
				amb1 = B;
			if (a <= amb1 && (zbad(amb1) || sgh_cnt_le(P, amb1) - cnt_a > 0))
				return 1;
			int amb0 = sgh_ceil_clamp(bhi - tol);
			if (amb0 < A)
				amb0 = A;
			if (amb0 <= bt && (zbad(amb0 - 1) || cnt_bt - sgh_cnt_le(P, amb0 - 1) > 0))
				return 1;
		}
		const int L = cnt_a - MA.c, H = MB.c - cnt_bt;
		if (L + H > n)
			return 1;
		const int need = n - 4 - r;
		int fb = -1;
		if (need <= 0)
			fb = 0;
		else if (L >= need)
			fb = need - 1;
		else if (L + H >= need)
			fb = (n - H) + (need - L) - 1;
		if (fb >= 0 && fb < n - 1)
			return 1;
		if (L) {
			A = a;
			MA.c = xa.c;
			MA.s = (long long)xa.s;
			MA.ss = (unsigned long long)xa.ss;
			klo = xa.nb;
		}
		if (H) {
			B = bt;
			MB.c = xb.c;
			MB.s = (long long)xb.s;
			MB.ss = (unsigned long long)xb.ss;
			khi = xb.nb;
		}
		rlo += L;
		rhi += H;
		r += L + H;
		nrem = L + H;
		n -= nrem;
		SGH_WP(5, 0);
	} while (nrem > 0 && n > 3);
	const long long tot = (MB.s - MA.s) + (long long)n * P.lo;
	*value = sg_round_to_WORD((double)tot / (double)n);
#ifndef SGH_WINS_ITERS
	*rlo_out = rlo;
#endif
	*rhi_out = rhi;
	return SG_CLS_OK;
}

/*
 * stack_median's pixel (src/stacking/stacking.c:746-767, REJ 8) and PERCENTILE rejection
 * (:1660-1673 + percentile_clipping :1130-1143, REJ 1) from the column histogram.  Both are
 * rank queries on the sorted column: the median is gsl_stats_ushort_median_from_sorted_data
 * (odd N: a[N/2]; even: (a[(N-1)/2] + a[N/2]) / 2.0), which stack_median truncates to WORD
 * (:766-767).  PERCENTILE rejects a sample p as low when (median - p) / median > sig[0], else
 * as high when (p - median) / median > sig[1], both evaluated in the reference's double
 * arithmetic (median is a half-integer, median - p is exact, the division correctly rounded
 * and monotone in p): the low set is {p <= L}, the high set {p >= Uh}, found at the bound
 * estimate and stepped to the exact predicate edge, so no rounding band is needed.  The kept
 * samples are the values in (L, Uh); their exact sum / count is round_to_WORD'ed (:1790-1794).
 * The removal loop keeps its last sample when every one is rejected (`N > 1`, :1667-1672):
 * the largest.  With this row's normalised zeros among the below-band samples (ZT) a rank or
 * a count landing among them is not decided here (redo).
 */
template <int REJ, bool ZT>
__device__ __forceinline__ int sgh_median_pct(const SghPix &P, int N, double sl, double sh, int nbl, bool cleanB,
		bool cleanA, uint16_t *value, uint32_t *rlo, uint32_t *rhi) {
	/* nbl samples lie below the band (cleanB: all of them zeros, or this row's normalised
	 * zeros under ZT), N - nbl - nb above it (cleanA: all 65535).  A rank among the below- or
	 * above-band samples is decided here only when they are clean (a normalised-zero rank
	 * never: those values are not in the histogram) */
	auto rank_ok = [&](int g) {
		return g >= nbl ? (g < nbl + P.nb || cleanA) : (cleanB && !(ZT && P.zmax > 0));
	};
	auto value_at = [&](int g, int &v1) {	/* single rank, the band group read once */
		int x2;
		sgh_value_at2n(P, nbl, g, g, v1, x2);
	};
	const int g1 = (N - 1) / 2, g2 = N / 2;
	if (!rank_ok(g1) || !rank_ok(g2))
		return SG_CLS_LITERAL;
	int m1, m2;
	sgh_value_at2n(P, nbl, g1, g2, m1, m2);
	if (REJ == 8) {
		*value = (uint16_t)((m1 + m2) >> 1);	/* (WORD)((a + b) / 2.0): truncation of a half-integer */
		return SG_CLS_OK;
	}
	const double median = g1 == g2 ? (double)m1 : ((double)m1 + (double)m2) / 2.0;
	auto plo = [&](int v) { return (median - (double)v) / median > sl; };
	auto phi = [&](int v) { return ((double)v - median) / median > sh; };
	/* L: the largest sample value rejected low (-1: none); Uh: the smallest rejected high
	 * (65536: none) and not low (the reference tests low first) */
	int L = sgh_ceil_clamp(median - sl * median) - 1;	/* NaN -> -1 */
	L = L > 65535 ? 65535 : L;
	while (L < 65535 && plo(L + 1))
		L++;
	while (L >= 0 && !plo(L))
		L--;
	int U = sgh_floor_clamp(median + sh * median) + 1;	/* NaN -> 65536 */
	U = U < 0 ? 0 : U;
	while (U > 0 && phi(U - 1))
		U--;
	while (U <= 65535 && !phi(U))
		U++;
	const int Uh = U > L + 1 ? U : L + 1;
	/* the counts at L and Uh - 1 and the kept samples' sum are exact when no below-band sample
	 * of unknown value can be kept or counted apart (L >= lo - 1, or the below-band samples are
	 * clean) and likewise above the band; normalised zeros straddling a threshold are not */
	if ((!cleanB && L < P.lo - 1) || (!cleanA && Uh - 1 > P.lo + 255))
		return SG_CLS_LITERAL;
	if (ZT && P.zmax > 0 && ((L >= 0 && L < P.zmax) || (Uh - 1 >= 0 && Uh - 1 < P.zmax)))
		return SG_CLS_LITERAL;
	SghQ qa, qb;
	sgh_q_load(P, L, qa);
	sgh_q_load(P, Uh - 1, qb);
	auto count = [&](const SghQ &q) {
		return q.v < 0 ? 0 : (q.v >= 65535 ? N : nbl + (int)(sgh_pre(P, P.pc, q.g) + q.cp));
	};
	const int nlow = count(qa), nle = count(qb);
	const int nhigh = N - nle, kept = nle - nlow;
	*rlo = (uint32_t)nlow;
	*rhi = (uint32_t)nhigh;
	if (kept == 0) {	/* every sample rejected: the removal stops at the last one */
		if (!rank_ok(N - 1))
			return SG_CLS_LITERAL;
		int mx;
		value_at(N - 1, mx);
		*value = (uint16_t)mx;
		return SG_CLS_OK;
	}
	/* the moments at L and Uh - 1 both hold the below-band samples (their difference cancels
	 * them unless L = -1, where they are kept and clean) */
	const SghM ma = sgh_q_moments(P, qa), mb = sgh_q_moments(P, qb);
	const long long sum = (mb.s - ma.s) + (long long)kept * P.lo;	/* exact: below 2^32 */
	*value = sg_round_to_WORD((double)sum / (double)kept);
	return SG_CLS_OK;
}

/* the compact redo (normalised SIGMA / WINSORIZED): every lane with `want` set owns a pixel
 * whose samples are all known to the tile, the histogram's band, its zeros and 65535s and the
 * k <= SGH_OVK captured out-of-band values.  The whole wave writes each such pixel's sorted
 * column to p.cmp_cols[slot] (N u16: zeros, the captured values below the band, the band
 * expanded bin by bin, those above it, 65535s) and its pixel to p.cmp_list[slot];
 * k_stack_sorted<., true> then stages the column with coalesced loads instead of N scattered
 * ones.  A pixel past p.cmp_cap goes to the redo list as before.  Wave-uniform control flow */
template <int NI>
__device__ __forceinline__ void sgh_compact(const SgStackParams &p, const SghLds<NI> &L, bool want, int col, int lo,
		unsigned int pix, int nzl, int nsl, int kl, unsigned int *__restrict__ redo_count,
		unsigned int *__restrict__ redo_list) {
	const int lane = threadIdx.x & 63;
	const int N = p.N;
	uint64_t m = __ballot(want);
	if (!m)
		return;
	/* one slot reservation for all of the wave's pixels (a returning global atomic per pixel
	 * serialised the loop on its latency) */
	unsigned int base = 0;
	if (lane == 0)
		base = atomicAdd(p.cmp_count, (unsigned int)__popcll(m));
	base = (unsigned int)__builtin_amdgcn_readfirstlane((int)base);
	for (unsigned int slot = base; m; slot++) {
		const int src = __builtin_ctzll(m);
		m &= m - 1;
		const int cs = __builtin_amdgcn_readlane(col, src), ls = __builtin_amdgcn_readlane(lo, src);
		const unsigned int ps = (unsigned int)__builtin_amdgcn_readlane((int)pix, src);
		if (slot >= p.cmp_cap) {
			if (lane == 0)
				redo_list[atomicAdd(redo_count, 1u)] = ps;
			continue;
		}
		uint16_t *dst = p.cmp_cols + (size_t)slot * (size_t)N;
		const int nz = __builtin_amdgcn_readlane(nzl, src), ns = __builtin_amdgcn_readlane(nsl, src);
		const int k = __builtin_amdgcn_readlane(kl, src);	/* <= SGH_OVK: checked by the caller */
		/* the captured values: lane t < k holds value t; below the band or above it */
		const int ov = lane < k ? (int)L.ov[lane < SGH_OVK ? lane : 0][cs] : 0;
		const bool below = lane < k && ov < ls;
		const int nbelow = __popcll(__ballot(below)), nabove = k - nbelow;
		if (lane < k) {
			/* rank among the captured values on the same side (ties by index) */
			int r = 0;
#pragma unroll
			for (int t = 0; t < SGH_OVK; t++) {
				const int u = __shfl(ov, t, 64);
				if (t < k && t != lane && ((u < ls) == below) && (u < ov || (u == ov && t < lane)))
					r++;
			}
			dst[below ? nz + r : N - ns - nabove + r] = (uint16_t)ov;
		}
		/* the band: lane l expands dword l (values lo + 4 l .. lo + 4 l + 3) after the exclusive
		 * prefix of the lanes before it */
		const uint32_t d = L.h[cs >> 6][lane][cs & 63];
		const int c0 = (int)(d & 0xFFu), c1 = (int)((d >> 8) & 0xFFu), c2 = (int)((d >> 16) & 0xFFu), c3 = (int)(d >> 24);
		const int tot = c0 + c1 + c2 + c3;
		int inc = tot;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const int y = __shfl_up(inc, o, 64);
			if (lane >= o)
				inc += y;
		}
		int pos = nz + nbelow + inc - tot;
		const int v0 = ls + 4 * lane;
		const int cnt[4] = {c0, c1, c2, c3};
#pragma unroll
		for (int b = 0; b < 4; b++) {
			for (int r = 0; r < cnt[b]; r++)
				dst[pos + r] = (uint16_t)(v0 + b);
			pos += cnt[b];
		}
		for (int r = lane; r < nz; r += 64)
			dst[r] = 0;
		for (int r = N - ns + lane; r < N; r += 64)
			dst[r] = 65535;
		if (lane == 0)
			p.cmp_list[slot] = ps;
	}
}

/* pixel column `col` of the tile (x its image column); PAIR: lane pair half `half`, else one
 * lane per column (half = 0); CAP: normalised SIGMA / WINSORIZED kernel (captured out-of-band
 * values, sgh_compact) */
template <int REJ, bool PAIR, int NI, bool ZT = false, bool CAP = false, class LT = SghLds<NI>>
__device__ __forceinline__ void sgh_finish2(const SgStackParams &p, LT &L, int col, int half, int lo, int R, int c, int x,
		unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list, bool zrow = false) {
	const int lane = threadIdx.x & 63;
	const int N = p.N;
	const uint32_t *hc = &L.h[col >> 6][0][col & 63];	/* dword j at hc[64 j] */
	if (SG_DBG(p) == 2 || SG_DBG(p) == 3) {
		if (x < p.W && !half)
			p.out[((int64_t)c * p.H + R) * p.W + x] = (uint16_t)(hc[0] + L.nz[col]);
		return;
	}
	/* A/B timeline (dbg 11): cycles of the prefix and of the pass loop, passes per wave */
	const uint64_t c0 = SG_DBG(p) == 11 ? __builtin_readcyclecounter() : 0;
#ifdef SGH_WPROF
	if (REJ == 4 && lane == 0) {
		uint64_t *w = L.wp[threadIdx.x >> 6];
		for (int k = 1; k < 16; k++)
			w[k] = 0;
		w[0] = __builtin_readcyclecounter();
	}
#endif
	int passes = 0;
	/* prefix: this lane's 4 groups, then the partner's 4 (PAIR), or all 8 */
	constexpr int NG = PAIR ? SGH_NGRP / 2 : SGH_NGRP;
	uint32_t gc[NG], gs[NG], gss[NG];
#pragma unroll
	for (int k = 0; k < NG; k++) {
		const int g = PAIR ? (SGH_NGRP / 2) * half + k : k;
		uint32_t d[SGH_GRP], cc = 0, s = 0, ss = 0;
#pragma unroll
		for (int j = 0; j < SGH_GRP; j++)
			d[j] = hc[64 * (g * SGH_GRP + j)];
		sgh_grp_moments(d, cc, s, ss);
		/* 24-bit multiplies (v_mul_u32_u24, full rate): b0 <= 224, cc <= 32 * 255, s < 2^18 */
		const uint32_t b0 = (uint32_t)g * (4u * SGH_GRP);
		gc[k] = cc;
		gs[k] = s + __umul24(b0, cc);
		gss[k] = ss + __umul24(2u * b0, s) + __umul24(__umul24(b0, b0), cc);
	}
	SghPix P;
	uint32_t cum = 0, s32 = 0, ss32 = 0;	/* band totals */
	if constexpr (PAIR) {
		/* exclusive prefix of the lane's own 4 groups, offset by the low half's totals in the
		 * high half; the partner's 4 entries follow at index 4..7 (SghPix::hx) */
		uint32_t oc = 0, os = 0, oss = 0;
#pragma unroll
		for (int k = 0; k < NG; k++) {
			P.pc[k] = oc;
			P.ps[k] = os;
			P.pss[k] = oss;
			oc += gc[k];
			os += gs[k];
			oss += gss[k];
		}
		const uint32_t xc = sgh_x(oc), xs = sgh_x(os), xss = sgh_x(oss);
		const uint32_t fc = half ? xc : 0u, fs = half ? xs : 0u, fss = half ? xss : 0u;
#pragma unroll
		for (int k = 0; k < NG; k++) {
			P.pc[k] += fc;
			P.ps[k] += fs;
			P.pss[k] += fss;
		}
#pragma unroll
		for (int k = 0; k < NG; k++) {
			P.pc[NG + k] = sgh_x(P.pc[k]);
			P.ps[NG + k] = sgh_x(P.ps[k]);
			P.pss[NG + k] = sgh_x(P.pss[k]);
		}
		cum = oc + xc;
		s32 = os + xs;
		ss32 = oss + xss;
		P.hx = half ? NG : 0;
	} else {
#pragma unroll
		for (int g = 0; g < SGH_NGRP; g++) {
			P.pc[g] = cum;
			P.ps[g] = s32;
			P.pss[g] = ss32;
			cum += gc[g];
			s32 += gs[g];
			ss32 += gss[g];
		}
		P.hx = 0;
	}
	const int oob = (int)hc[64 * SGH_DW];
	/* ZT (SIGMA with additive normalisation): this row's normalised zeros of frames shifted out
	 * of it, from the host's border-row table (SgStackParams::ztab).  Interior tiles only
	 * (zrow): at the image edges a frame shifted out in both directions gives 0 instead (the x
	 * shift's zero is not normalised, :1628-1632), and the sample count alone cannot tell one
	 * such frame from an unrelated out-of-band sample */
	int zc = 0, zmax = 0;
	long long zs = 0, zss = 0;
	if (ZT && (REJ == 2 || REJ == 4) && zrow && p.ztab) {
		const int t = R < p.ztab_k1 ? R : (R >= p.H - p.ztab_k2 ? p.ztab_k1 + (R - (p.H - p.ztab_k2)) : -1);
		if (t >= 0) {
			const int *e = p.ztab + 8 * t;
			zc = e[0];
			zs = (long long)(uint32_t)e[1] | ((long long)e[6] << 32);
			zss = (long long)(uint32_t)e[2] | ((long long)e[3] << 32);
			zmax = e[5];
		}
	}
	P.zmax = 0;
	P.omin = 65535;
	P.lo = lo;
	P.nz = (int)L.nz[col];
	P.ns = (int)L.ns[col];
	P.nb = (int)cum;
	P.col = col;
	P.hb = &L.h[0][0][0];
#ifdef SGH_WPROF
	P.wp = L.wp[threadIdx.x >> 6];
	SGH_WP(0, 0);
#endif
	int cls = SG_CLS_OK;
	uint16_t value = 0;
	uint32_t rlo = 0, rhi = 0;
	bool cmp = false;	/* CAP: the pixel's sorted column goes out through sgh_compact */
	const uint64_t c1 = SG_DBG(p) == 11 ? __builtin_readcyclecounter() : 0;
	if (x < p.W) {
		/* CAP SIGMA (round 6): up to SGH_OVK out-of-band samples other than 0 / 65535, every one captured
		 * (their values in L.ov: a scaled cosmic ray, a dead pixel moved off 0), join the pixel as known
		 * samples (counts and moments below or above the band) instead of sending it to the compact list;
		 * a query or median rank among them is undecidable here (zbad) and redoes the pixel */
		int kx = 0;
		if constexpr (CAP && (REJ == 2 || REJ == 4)) {
			const int k = oob - P.nz - P.ns;
			if (P.nb + oob == N && zc == 0 && k > 0 && k <= SGH_OVK && (int)L.ovn[col] == k)
				kx = k;
		}
		if (SG_DBG(p) == 1) {
			value = (uint16_t)(s32 + ss32);
		} else if (P.nb + oob != N || (zc && zmax >= lo) || (REJ != 1 && REJ != 8 && oob != P.nz + P.ns + zc + kx)) {
			cls = 1;	/* out-of-band sample other than 0 / 65535 (or than this row's normalised
				 * zeros), or a wrapped u8 counter */
			if constexpr (CAP) {
				if (p.cmp_cols) {	/* every sample known: no wrap, no row zeros, all captured */
					const int k = oob - P.nz - P.ns;
					cmp = P.nb + oob == N && zc == 0 && k > 0 && k <= SGH_OVK && (int)L.ovn[col] == k;
				}
			}
		} else {
			const long long dz = -(long long)lo, ds = 65535 - (long long)lo;
			P.Z.c = P.nz;
			P.Z.s = dz * P.nz;
			P.Z.ss = (unsigned long long)(dz * dz) * (unsigned long long)P.nz;
			if (zc) {	/* the normalised zeros join the below-band samples */
				const long long l = lo;
				P.Z.c += zc;
				P.Z.s += zs - (long long)zc * l;
				P.Z.ss += (unsigned long long)(zss - 2 * l * zs + (long long)zc * l * l);
				P.nz += zc;
				P.zmax = zmax;
			}
			P.T.c = N;
			P.T.s = (long long)s32 + P.Z.s + ds * P.ns;
			P.T.ss = (unsigned long long)ss32 + P.Z.ss + (unsigned long long)(ds * ds) * (unsigned long long)P.ns;
			if constexpr (CAP && (REJ == 2 || REJ == 4)) {
				if (kx) {
#pragma unroll
					for (int k = 0; k < SGH_OVK; k++) {
						if (k < kx) {
							const int v = (int)L.ov[k][col];
							const long long d = (long long)v - lo;
							const unsigned long long d2 = (unsigned long long)(d * d);
							P.T.s += d;
							P.T.ss += d2;
							if (v < lo) {	/* below the band: with the zeros (counts, moments, ranks) */
								P.Z.c++;
								P.Z.s += d;
								P.Z.ss += d2;
								P.nz++;
								P.zmax = v > P.zmax ? v : P.zmax;
							} else {
								P.omin = v < P.omin ? v : P.omin;
							}
						}
					}
				}
			}
			if (REJ == 1 || REJ == 8) {
				/* out-of-band samples of any value: below the band nbl of them, above na */
				const int na = (int)L.na[col], nbl = oob - na;
				cls = sgh_median_pct<REJ, ZT>(P, N, p.sig0, p.sig1, nbl, nbl == P.nz, na == P.ns, &value, &rlo, &rhi);
			} else if (REJ == 3) {
				cls = sgh_sigmedian(P, N, p.sig0, p.sig1, &value, &rlo, &rhi);
			} else if (REJ == 4 || !PAIR) {
				/* zeros (and captured samples below the band): their moments, exact as doubles
				 * (dz = -lo, dz^2 nz < 2^53) */
				P.zs = (double)P.Z.s;
				P.zss = (double)P.Z.ss;
				cls = sgh_winsorized<CAP>(P, N, p.sig0, p.sig1, p.wins_cap, &value, &rlo, &rhi);
				if constexpr (CAP && REJ == 4)
					cmp = cls != SG_CLS_OK && kx && p.cmp_cols;	/* every sample known: the sorted column */
#ifdef SGH_WINS_ITERS
				value = (uint16_t)rlo;	/* A/B probe build: the image holds the inner iteration counts */
				cls = SG_CLS_OK;
				rlo = rhi = 0;
#endif
#ifdef SGH_WINS_FEAT	/* A/B probe build: the image holds min(zeros, 255) << 8 | min(65535s, 255) */
				value = (uint16_t)(((P.nz < 255 ? P.nz : 255) << 8) | (P.ns < 255 ? P.ns : 255));
				cls = SG_CLS_OK;
				rlo = rhi = 0;
#endif
			} else {
				cls = sgh_sigma3<ZT, CAP>(P, N, p.sig0, p.sig1, half, &value, &rlo, &rhi, passes);
				if constexpr (CAP && REJ == 2)
					cmp = cls != SG_CLS_OK && kx && p.cmp_cols;	/* every sample known: the sorted column */
#ifdef SGH_SIGMA_PASSES	/* A/B probe build: the image holds the pass counts */
				value = (uint16_t)passes;
				cls = SG_CLS_OK;
				rlo = rhi = 0;
#endif
			}
		}
		const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
		if (!half) {
			if (cls == SG_CLS_OK) {
#ifndef SGH_WPROF
				if (SG_DBG(p) != 11)	/* the timeline A/B keeps its stamps in the output buffer */
					p.out[pix] = value;
#endif
			} else if (!cmp) {
#ifndef SGH_WPROF
				const unsigned int slot = atomicAdd(redo_count, 1u);
				redo_list[slot] = (unsigned int)pix;
#endif
			}
		}
		if (cls != SG_CLS_OK || half)
			rlo = rhi = 0;
	}
	if (SG_DBG(p) == 11 && NI == 2) {
		const uint64_t c2 = __builtin_readcyclecounter();
		int pmax = passes, psum = passes;
		for (int o = 32; o > 0; o >>= 1) {
			pmax = max(pmax, __shfl_xor(pmax, o, 64));
			psum += __shfl_xor(psum, o, 64);
		}
		if (lane == 0) {
			uint64_t *tw = (uint64_t *)p.out + (size_t)blockIdx.x * 32 + 4 + 3 * (threadIdx.x >> 6);
			tw[0] = c1 - c0;
			tw[1] = c2 - c1;
			tw[2] = (uint64_t)pmax | ((uint64_t)psum << 16);
		}
	}
	/* wave sums of the rejection counts (each lane's count <= N, so a wave's sum of 32 pixel
	 * counts fits 32 bits for any N the kernel takes): DPP row sums + 4 readlanes instead of
	 * six dependent ds_bpermute rounds */
#ifdef SGH_WPROF
	if (REJ == 4) {
		sgh_wp(L.wp[threadIdx.x >> 6], 6);
		if (lane == 0) {
			const uint64_t *w = L.wp[threadIdx.x >> 6];
			unsigned long long *g = (unsigned long long *)p.out;
			for (int k = 1; k < 16; k++)
				atomicAdd(g + k, (unsigned long long)w[k]);
			atomicAdd(g, 1ull);	/* finishing waves */
		}
	}
#endif
	if constexpr (CAP)
		sgh_compact<NI>(p, L, cmp && !half && x < p.W, col, lo, (unsigned int)(((int64_t)c * p.H + R) * p.W + x),
				(int)L.nz[col], (int)L.ns[col], oob - (int)L.nz[col] - (int)L.ns[col], redo_count, redo_list);
	const unsigned long long a = sgh_wave_sum(rlo), b = sgh_wave_sum(rhi);
	if (lane == 0 && (a | b)) {
		unsigned long long *sh = p.rej + ((size_t)((blockIdx.x * 8 + (col >> 5)) % SG_REJ_SHARDS) * 6 + c * 2);
		atomicAdd(sh, a);
		atomicAdd(sh + 1, b);
	}
}

/* clear the tile's histogram and counters with 16-byte stores (called after the first frame
 * loads are issued, so their latency covers it; the build's start barrier orders it before
 * the first atomic) */
struct SghWgBarrier {
	__device__ __forceinline__ void operator()() const { __syncthreads(); }
	__device__ __forceinline__ void wait_prev() const { __syncthreads(); }
};
template <int NI, int BW = SghCfg<NI>::WAVES, class BAR = SghWgBarrier>
__device__ __forceinline__ void sgh_clear(SghLds<NI> &L, bool wait_prev, const BAR &bar = BAR()) {
	if (wait_prev)
		bar.wait_prev();	/* the previous tile's finish is done with L */
	constexpr int NH = 2 * NI * SGH_HROWS * 64 / 4, NC = 128 * NI / 4, T = 64 * BW;
	uint4 *h = (uint4 *)&L.h[0][0][0];
	const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
	for (int k = 0; k < (NH + T - 1) / T; k++) {
		const int i = (int)threadIdx.x + k * T;
		if (i < NH)
			h[i] = z;
	}
	if ((int)threadIdx.x < NC) {
		((uint4 *)L.nz)[threadIdx.x] = z;
		((uint4 *)L.ns)[threadIdx.x] = z;
		((uint4 *)L.na)[threadIdx.x] = z;
		((uint4 *)L.ovn)[threadIdx.x] = z;
	}
}

/* one wave's share of the tile's histogram build: 16-frame blocks, wave w bins blocks w,
 * w+WAVES, w+2 WAVES, ... in order, with NBUF named register buffers: a buffer is refilled with
 * the wave's block NBUF steps ahead right after it has been binned, so NBUF-1 blocks stay in
 * flight during the binning; the shift table of that block is fetched (scalar loads) before
 * the binning.  No block is loaded twice.  Frames 0..15 (wave 0's first block) are the centre
 * sample: wave 0 sorts them and publishes the band starts through LDS while the other waves'
 * first blocks are in flight (one barrier, which also covers the clear). */
template <bool EDGE, int NBUF, int NORM, int NI>
__device__ __forceinline__ void sgh_build(const SgStackParams &p, const SghRo &ro, SghLds<NI> &L, const SghFrame &F,
		int wave, int lane,
		uint32_t (&lo2)[NI], uint32_t (&nonzero)[NI], uint32_t (&nsat)[NI], int &counted, bool wait_prev) {
	constexpr int M = 16;		/* frames per block */
	constexpr int WAVES = SghCfg<NI>::WAVES;
	constexpr int STEP = M * WAVES;
	constexpr int AHEAD = NBUF * STEP;
	const int N = p.N;
	uint32_t *const h = &L.h[0][0][0];
	const uint32_t l4 = (uint32_t)lane * 4u;
	uint32_t buf[NBUF][M][NI], fix[NBUF][NI];
	SghTab16 T;
	auto loadblk = [&](int f0, uint32_t (&dst)[M][NI], uint32_t (&fx)[NI]) {
		if (f0 + M <= N)
			sgh_loadblk<true, EDGE, NI>(F, T, N, f0, dst, fx);
		else
			sgh_loadblk<false, EDGE, NI>(F, T, N, f0, dst, fx);
	};
	int f[NBUF];
#pragma unroll
	for (int k = 0; k < NBUF; k++) {
		f[k] = M * wave + k * STEP;
#pragma unroll
		for (int i = 0; i < NI; i++)
			fix[k][i] = 0;
		if (f[k] < N) {
			sgh_tab16(ro, f[k], T);
			loadblk(f[k], buf[k], fix[k]);
		}
	}
	sgh_clear(L, wait_prev);
	if (wave == 0) {
#pragma unroll
		for (int i = 0; i < NI; i++) {
			uint32_t p16[SGH_CENTER];
#pragma unroll
			for (int m = 0; m < SGH_CENTER; m++) {
				p16[m] = sgh_fixup<EDGE>(buf[0][m][i], fix[0][i], m);
				if (NORM) {
					double a, b;
					sgh_coef(ro, m, a, b);
					p16[m] = sgh_norm_pair<NORM, EDGE>(p16[m], a, b, fix[0][i], m);
				}
			}
			int la, lb;
			sgh_centre2(p16, la, lb);
			L.lo2[i][lane] = (uint32_t)la | ((uint32_t)lb << 16);
		}
	}
	__syncthreads();	/* histogram cleared, band starts published */
#pragma unroll
	for (int i = 0; i < NI; i++)
		lo2[i] = L.lo2[i][lane];
	const bool loads_only = SG_DBG(p) == 3;
	auto binblk = [&](int f0, const uint32_t (&raw)[M][NI], const uint32_t (&fx)[NI]) {
		if (loads_only) {
#pragma unroll
			for (int m = 0; m < M; m++)
#pragma unroll
				for (int i = 0; i < NI; i++)
					nonzero[i] ^= raw[m][i];
		} else {
#pragma unroll
			for (int m = 0; m < M; m++) {
				if (f0 + M <= N || f0 + m < N) {
					double a = 0.0, b = 0.0;
					if (NORM)
						sgh_coef(ro, f0 + m, a, b);
#pragma unroll
					for (int i = 0; i < NI; i++) {
						uint32_t v = sgh_fixup<EDGE>(raw[m][i], fx[i], m);
						if (NORM)
							v = sgh_norm_pair<NORM, EDGE>(v, a, b, fx[i], m);
						sgh_bin_pair(h + i * (2 * SGH_HROWS * 64), l4, lo2[i], v, nonzero[i], nsat[i]);
					}
				}
			}
		}
		counted += (N - f0 < M ? N - f0 : M);
	};
	if (f[0] + AHEAD < N)
		sgh_tab16(ro, f[0] + AHEAD, T);
	while (f[0] < N) {
#pragma unroll
		for (int k = 0; k < NBUF; k++) {
			if (f[k] >= N)
				break;
			binblk(f[k], buf[k], fix[k]);
			const int nf = f[k] + AHEAD;
			if (nf < N)
				loadblk(nf, buf[k], fix[k]);	/* T = table of nf */
			f[k] = nf;
			const int kn = (k + 1) % NBUF;
			const int tn = f[kn] + AHEAD;	/* the next buffer's refill */
			if (f[kn] < N && tn < N)
				sgh_tab16(ro, tn, T);
		}
	}
}

/* the same build with 8-frame half blocks (the default for NI = 1, SGH_HALF1; NI = 2 loads
 * two dwords per lane and frame):
 * wave w bins the 16-frame blocks w, w + WAVES, ... in order, each as two halves; NB blocks
 * (2 NB half buffers) are in flight, so while one half is binned 2 NB - 1 halves keep
 * loading (with two 8-wave workgroups per CU, one workgroup's loads must carry the CU while
 * the other runs its finish).  The shift table of a block is fetched once for both halves.
 * Wave 0's first block (frames 0..15) is the centre sample. */
#ifndef SGH_NB
#define SGH_NB 1	/* 2: 4.85 vs 4.62 ms (NI = 2, scripts/gpu_r2i.sh) */
#endif
/* NI = 1 also streams half blocks (scripts/gpu_r2u.sh, two alternating rounds on one box:
 * 4.111-4.119 ms against 4.179-4.186 for the 16-frame build, NB = 1 and 2 equal; the 16-frame
 * build with a third buffer 4.23-4.24): the straight-line steady loop with sched_barriers keeps
 * every refill right behind its binning */
#ifndef SGH_HALF1
#define SGH_HALF1 1
#endif
/* band centre from the first half blocks of waves 0 and 1 (frames 0..7, 16..23) instead of
 * wave 0's whole first block: 3.88 -> 3.74 ms (scripts/gpu_r3n.sh), the start barrier no
 * longer waits for a second half block to land (8 frames alone: 3.64 ms but a noisier centre
 * sends 35 k pixels to the redo list, scripts/gpu_r3m.sh) */
#ifndef SGH_CENTER2W
#define SGH_CENTER2W 1
#endif
#ifndef SGH_WINS_ORDER
#define SGH_WINS_ORDER 1	/* WINSORIZED finish: columns with zeros / 65535s first (sgh_tile) */
#endif

template <bool EDGE, int NORM, int NI, int NB, int BW = SghCfg<NI>::WAVES, class BAR = SghWgBarrier, bool AB = false>
__device__ __forceinline__ void sgh_build_half(const SgStackParams &p, const SghRo &ro, SghLds<NI> &L, const SghFrame &F,
		int wave, int lane, uint32_t (&lo2)[NI], uint32_t (&nonzero)[NI], uint32_t (&nsat)[NI], int &counted,
		bool wait_prev, const BAR &bar = BAR(), uint32_t *nab = nullptr) {
	constexpr int MB = 8;
	constexpr int WAVES = BW;	/* the waves building the tile */
	constexpr int STEP = 16 * WAVES;	/* frames between a wave's consecutive blocks */
	const int N = p.N;
	uint32_t *const h = &L.h[0][0][0];
	const uint32_t l4 = (uint32_t)lane * 4u;
	const uint32_t k1 = sgh_opaque(0x00010001u), ksat = sgh_opaque(0xFFFEFFFEu);
	const uint32_t k255 = NORM && !AB ? sgh_opaque(0x00FF00FFu) : 0u;
	uint32_t buf[NB][2][MB][NI], fix[NB][2][NI];
	SghTab16 T;
	/* half hh (frames f16 + 8 hh ..) of the block at f16, bounds-checked unless whole */
	auto loadh = [&](int f16, int hh, uint32_t (&dst)[MB][NI], uint32_t (&fx)[NI]) {
		if (f16 + 16 <= N) {
			if (hh == 0)
				sgh_loadblk<true, EDGE, NI, MB, 0>(F, T, N, f16, dst, fx);
			else
				sgh_loadblk<true, EDGE, NI, MB, 8>(F, T, N, f16 + 8, dst, fx);
		} else {
			if (hh == 0)
				sgh_loadblk<false, EDGE, NI, MB, 0>(F, T, N, f16, dst, fx);
			else
				sgh_loadblk<false, EDGE, NI, MB, 8>(F, T, N, f16 + 8, dst, fx);
		}
	};
	int f16 = 16 * wave;
#pragma unroll
	for (int b = 0; b < NB; b++) {
		const int fb = f16 + b * STEP;
#pragma unroll
		for (int i = 0; i < NI; i++)
			fix[b][0][i] = fix[b][1][i] = 0;
		if (fb < N) {
			sgh_tab16(ro, fb, T);
			loadh(fb, 0, buf[b][0], fix[b][0]);
			loadh(fb, 1, buf[b][1], fix[b][1]);
		}
	}
	sgh_clear<NI, BW>(L, wait_prev, bar);
	const bool nocentre = SG_DBG(p) == 15;	/* A/B: loads only, no centre and no start barrier */
	static_assert(!SGH_CENTER2W || SGH_CENTER == 2 * MB, "two half blocks make the centre sample");
	if (SGH_CENTER2W && !nocentre) {
		/* the centre sample is the first half block of wave 0 (frames 0..7) and of wave 1
		 * (frames 16..23): both land with the kernel's first loads, so the start barrier does
		 * not wait for a second half block */
		if (wave == 1) {
#pragma unroll
			for (int i = 0; i < NI; i++)
#pragma unroll
				for (int m = 0; m < MB; m++) {
					uint32_t v = sgh_fixup<EDGE>(buf[0][0][m][i], fix[0][0][i], m);
					if (NORM) {
						double a, b;
						sgh_coef(ro, f16 + m, a, b);
						v = sgh_norm_pair<NORM, EDGE>(v, a, b, fix[0][0][i], m);
					}
					L.cs[i][m][lane] = v;
				}
		}
		bar();
		if (wave == 0) {
#pragma unroll
			for (int i = 0; i < NI; i++) {
				uint32_t p16[SGH_CENTER];
#pragma unroll
				for (int m = 0; m < MB; m++) {
					p16[m] = sgh_fixup<EDGE>(buf[0][0][m][i], fix[0][0][i], m);
					if (NORM) {
						double a, b;
						sgh_coef(ro, m, a, b);
						p16[m] = sgh_norm_pair<NORM, EDGE>(p16[m], a, b, fix[0][0][i], m);
					}
					p16[MB + m] = L.cs[i][m][lane];
				}
				int la, lb;
				sgh_centre2(p16, la, lb);
				L.lo2[i][lane] = (uint32_t)la | ((uint32_t)lb << 16);
			}
		}
	} else if (wave == 0 && !nocentre) {
#pragma unroll
		for (int i = 0; i < NI; i++) {
			uint32_t p16[SGH_CENTER];
#pragma unroll
			for (int m = 0; m < SGH_CENTER; m++) {
				const int mm = m & (MB - 1), hh = m / MB;
				p16[m] = sgh_fixup<EDGE>(buf[0][hh][mm][i], fix[0][hh][i], mm);
				if (NORM) {
					double a, b;
					sgh_coef(ro, m, a, b);
					p16[m] = sgh_norm_pair<NORM, EDGE>(p16[m], a, b, fix[0][hh][i], mm);
				}
			}
			int la, lb;
			sgh_centre2(p16, la, lb);
			L.lo2[i][lane] = (uint32_t)la | ((uint32_t)lb << 16);
		}
	}
	if (!nocentre)
		bar();	/* histogram cleared, band starts published */
#pragma unroll
	for (int i = 0; i < NI; i++)
		lo2[i] = nocentre ? 0u : L.lo2[i][lane];
	uint32_t hi2[NI];	/* AB: lo + 255 per half (lo <= 65279: no carry between the halves) */
#pragma unroll
	for (int i = 0; i < NI; i++)
		hi2[i] = lo2[i] + 0x00FF00FFu;
	const bool loads_only = SG_DBG(p) == 3 || nocentre;
	/* bin one half (frames f0 .. f0 + 7), per-frame bounds when it is not whole */
	auto binh = [&](int f0, const uint32_t (&raw)[MB][NI], const uint32_t (&fx)[NI], bool whole) {
		if (loads_only) {
#pragma unroll
			for (int m = 0; m < MB; m++)
#pragma unroll
				for (int i = 0; i < NI; i++)
					nonzero[i] ^= raw[m][i];
		} else if (SGH_BIN2 && !NORM && !EDGE && whole) {
#pragma unroll
			for (int m = 0; m < MB; m += 2)
#pragma unroll
				for (int i = 0; i < NI; i++)
					sgh_bin_pair2<AB>(h + i * (2 * SGH_HROWS * 64), l4, lo2[i], raw[m][i], raw[m + 1][i], nonzero[i],
							nsat[i], k1, ksat, AB ? nab + i : nullptr, hi2[i]);
		} else {
#pragma unroll
			for (int m = 0; m < MB; m++) {
				if (whole || f0 + m < N) {
					double a = 0.0, b = 0.0;
					if (NORM)
						sgh_coef(ro, f0 + m, a, b);
#pragma unroll
					for (int i = 0; i < NI; i++) {
						uint32_t v = sgh_fixup<EDGE>(raw[m][i], fx[i], m);
						if (NORM)
							v = sgh_norm_pair<NORM, EDGE>(v, a, b, fx[i], m);
						sgh_bin_pair<AB>(h + i * (2 * SGH_HROWS * 64), l4, lo2[i], v, nonzero[i], nsat[i], k1, ksat,
								AB ? nab + i : nullptr, hi2[i]);
						if (NORM && !AB)
							sgh_capture(L, i, lane, lo2[i], v, k1, ksat, k255);
					}
				}
			}
		}
		const int nf = N - f0;
		counted += whole ? MB : (nf < 0 ? 0 : (nf < MB ? nf : MB));
	};
	/* steady state, straight-line: the NB blocks in hand and their refills all whole.
	 * sched_barrier keeps each refill right after the binning of its buffer (the scheduler
	 * otherwise hoists the next half's binning above the refill, and its vmcnt waits then
	 * drain every load before any new one issues) */
	while (f16 + (2 * NB - 1) * STEP + 16 <= N) {
#pragma unroll
		for (int b = 0; b < NB; b++) {
			const int fb = f16 + b * STEP, nx = fb + NB * STEP;
			sgh_tab16(ro, nx, T);
			binh(fb, buf[b][0], fix[b][0], true);
			__builtin_amdgcn_sched_barrier(0);
			sgh_loadblk<true, EDGE, NI, MB, 0>(F, T, N, nx, buf[b][0], fix[b][0]);
			__builtin_amdgcn_sched_barrier(0);
			binh(fb + 8, buf[b][1], fix[b][1], true);
			__builtin_amdgcn_sched_barrier(0);
			sgh_loadblk<true, EDGE, NI, MB, 8>(F, T, N, nx + 8, buf[b][1], fix[b][1]);
			__builtin_amdgcn_sched_barrier(0);
		}
		f16 += NB * STEP;
	}
	/* the remaining blocks, in order, with bounds */
	while (f16 < N) {
#pragma unroll
		for (int b = 0; b < NB; b++) {
			const int fb = f16 + b * STEP, nx = fb + NB * STEP;
			if (fb >= N)
				break;
			if (nx < N)
				sgh_tab16(ro, nx, T);
			binh(fb, buf[b][0], fix[b][0], fb + 16 <= N);
			if (nx < N)
				loadh(nx, 0, buf[b][0], fix[b][0]);
			binh(fb + 8, buf[b][1], fix[b][1], fb + 16 <= N);
			if (nx < N)
				loadh(nx, 1, buf[b][1], fix[b][1]);
		}
		f16 += NB * STEP;
	}
}

/* REJ 2 = SIGMA, 4 = WINSORIZED; NORM 0 none, 1 additive, 2 multiplicative; NI pixel pairs
 * per lane (tile of 128 NI pixels, 4 NI waves).  Two 8-wave workgroups (69 KB of LDS each)
 * or four 4-wave ones (34.5 KB) per CU: 16 waves, at most 128 VGPRs. */
/* one tile: bid = its index in (channel, row, 128 NI-column tile) order; wait_prev: a tile after
 * the first one of this workgroup, whose first frame loads may be issued while other waves of
 * the workgroup still finish the previous tile (the clear waits for them) */
template <int REJ, int NORM, int NI>
__device__ __forceinline__ void sgh_tile(const SgStackParams &p, const SghRo &ro, SghLds<NI> &L, int bid, bool wait_prev,
		unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list, int load = 0) {
	constexpr int WAVES = SghW<REJ, NI>::WAVES, COLS = 128 * NI;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int ntx = (p.W + COLS - 1) / COLS;
	const int nrows = p.row_end - p.row_begin;
	/* (the divisions are off the critical path: shifts instead measured equal, scripts/gpu_r3r.sh) */
	const int xt = bid % ntx;
	bid /= ntx;
	const int R = p.row_begin + (bid % nrows);
	const int c = bid / nrows;
	const int x0 = xt * COLS;
	bool interior = x0 >= p.hist_maxsx && x0 + COLS + p.hist_maxsx <= p.W;
	if (SG_DBG(p) == 4)		/* A/B: every full tile on the dword path (wrong edges) */
		interior = x0 + COLS <= p.W;
	if (SG_DBG(p) == 5 && !interior)	/* A/B: skip the edge tiles */
		return;
	SghFrame F;
	F.plane0 = (const char *)(p.frames + (int64_t)c * p.plane_stride);
	F.fstride2 = p.frame_stride * 2;
	F.plane_bytes = (uint32_t)p.H * (uint32_t)p.W * 2u;
	F.w2 = p.W * 2;
	F.rw2 = R * p.W * 2;
	F.xa2 = (uint32_t)(x0 + 2 * lane) * 2u;
	F.x02 = (uint32_t)x0 * 2u;

	/* the histogram and the zero / 65535 counters are cleared by the build right after it has
	 * issued its first frame loads (sgh_clear), and its start barrier covers the clear */
	/* A/B timeline (SG_HIST_DBG=11, NI = 2): per tile, s_memrealtime (100 MHz) at entry,
	 * after the build barrier and at the end of every wave's finish, written into the
	 * output buffer as u64 [tile][4] (the image is garbage in this mode) */
	uint64_t *const tl = (uint64_t *)p.out + (size_t)blockIdx.x * 32;
	const bool timeline = NI == 2 && SG_DBG(p) == 11;
	if (timeline && tid == 0) {
		tl[0] = __builtin_amdgcn_s_memrealtime();
		tl[3] = 0;
	}

	uint32_t nonzero[NI], nsat[NI], lo2[NI], nab[NI];
	constexpr bool AB = REJ == 1 || REJ == 8;	/* stack_median / PERCENTILE: count the samples above the band */
#pragma unroll
	for (int i = 0; i < NI; i++)
		nonzero[i] = nsat[i] = nab[i] = 0;
	int counted = 0;
	/* the loading phase at a raised wave priority (SgStackParams::prio, default 1), so the
	 * waves that keep loads in flight issue ahead of other tiles' finish phases on the same
	 * SIMD: 4.73 -> 4.58 ms on configs[2]; 2 (priority 3) and 3 (finish raised instead) are
	 * A/B alternatives, both slower */
	if (p.prio == 1)
		__builtin_amdgcn_s_setprio(1);
	else if (p.prio == 2)
		__builtin_amdgcn_s_setprio(3);
	/* NORM 1..3, load 1: the build loads through the single-rounding pairs (NORM 4 / 5), load 2
	 * (additive, scale 1) through the integer offsets (NORM 6); the finish is the same (so are the
	 * normalised samples) */
	constexpr int NF = NORM == 2 ? 5 : 4;
	constexpr bool NORMI = NORM == 1 || NORM == 3;
	const bool fma = NORM >= 1 && NORM <= 3 && load == 1;
	SghRo rf = ro;
	rf.norm = ro.norm + ro.npad;
	SghRo ri = ro;
	ri.norm = ro.norm + 2 * ro.npad + 1;
	if (NORMI && load == 2 && NI == 1 && !SGH_HALF1 && !AB) {
		if (interior)
			sgh_build<false, SGH_NBUF, 6, NI>(p, ri, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
		else
			sgh_build<true, SGH_NBUF, 6, NI>(p, ri, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
	} else if (NORMI && load == 2) {
		if (interior)
			sgh_build_half<false, 6, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, ri, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
		else
			sgh_build_half<true, 6, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, ri, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
	} else if (NORM >= 1 && NORM <= 3 && fma && NI == 1 && !SGH_HALF1 && !AB) {
		if (interior)
			sgh_build<false, SGH_NBUF, NF, NI>(p, rf, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
		else
			sgh_build<true, SGH_NBUF, NF, NI>(p, rf, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
	} else if (NORM >= 1 && NORM <= 3 && fma) {
		if (interior)
			sgh_build_half<false, NF, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, rf, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
		else
			sgh_build_half<true, NF, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, rf, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
	} else if (NI == 1 && !SGH_HALF1 && !AB) {
		if (interior)
			sgh_build<false, SGH_NBUF, NORM, NI>(p, ro, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
		else
			sgh_build<true, SGH_NBUF, NORM, NI>(p, ro, L, F, wave, lane, lo2, nonzero, nsat, counted, wait_prev);
	} else {
		if (interior)
			sgh_build_half<false, NORM, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, ro, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
		else
			sgh_build_half<true, NORM, NI, NI == 1 ? SGH_NB : SGH_NB2, WAVES, SghWgBarrier, AB>(p, ro, L, F, wave, lane,
					lo2, nonzero, nsat, counted, wait_prev, SghWgBarrier(), nab);
	}
	if (counted) {
#pragma unroll
		for (int i = 0; i < NI; i++) {
			atomicAdd(&L.nz[128 * i + lane], (uint32_t)counted - (nonzero[i] & 0xFFFFu));
			atomicAdd(&L.nz[128 * i + 64 + lane], (uint32_t)counted - (nonzero[i] >> 16));
			atomicAdd(&L.ns[128 * i + lane], nsat[i] & 0xFFFFu);
			atomicAdd(&L.ns[128 * i + 64 + lane], nsat[i] >> 16);
			if (AB) {
				atomicAdd(&L.na[128 * i + lane], nab[i] & 0xFFFFu);
				atomicAdd(&L.na[128 * i + 64 + lane], nab[i] >> 16);
			}
		}
	}
	__syncthreads();
	if (timeline && tid == 0)
		tl[1] = __builtin_amdgcn_s_memrealtime();
	if (p.prio == 3)
		__builtin_amdgcn_s_setprio(1);	/* A/B: the finish raised instead */
	else if (p.prio)
		__builtin_amdgcn_s_setprio(0);
	/* column col = 64 g + l of the tile: pixel pair i = g >> 1 of lane l, half g & 1, i.e.
	 * image column x0 + 128 i + 2 l + (g & 1); its band start is the half of lo2[i][l] */
	auto col_x = [&](int col) { return x0 + 128 * (col >> 7) + 2 * (col & 63) + ((col >> 6) & 1); };
	auto col_lo = [&](int col) { return (int)((L.lo2[col >> 7][col & 63] >> (16 * ((col >> 6) & 1))) & 0xFFFFu); };
	if (REJ == 4) {
		/* WINSORIZED: the finish is VALU-bound and both lanes of a pair would run the same
		 * loop, so half of the waves take one pixel column per lane and the others leave
		 * their SIMD slots to other tiles.  A wave runs the inner loop as often as its slowest
		 * pixel needs, and a pixel holding a zero or a 65535 sample needs ~10 iterations against
		 * ~3 (scripts/wins_predict.py, profiles/r02z_wins_predict.log), so those columns are
		 * finished by wave 0 first and the rest after them (the sum of the two waves' maxima
		 * 26.4 -> 21.5 iterations per tile on configs[4]'s data) */
		if (NORM == 0 && NI == 1 && p.wx) {
			/* SG_WINS_EXPORT: a column holding a zero or a 65535 sample needs ~10 inner iterations
			 * against ~3 and holds its wave for them; it leaves the tile as its histogram (a slot per
			 * column, one atomic per wave) and k_hist_slow finishes it among columns of its own kind.
			 * The tile's waves finish the rest (a column without a slot is finished here) */
			if (wave >= 2)
				return;
			const int col = 64 * wave + lane;
			const int x = col_x(col);
			const uint32_t nout = L.nz[col] + L.ns[col];
			const bool slow = x < p.W && nout != 0u && nout <= (uint32_t)p.wx_kmax;
			const uint64_t m = __ballot(slow);
			unsigned int base = 0;
			if (m) {
				if (lane == 0)
					base = atomicAdd(p.wx_count, (unsigned int)__popcll(m));
				base = (unsigned int)__builtin_amdgcn_readfirstlane((int)base);
			}
			const unsigned int slot = base + (unsigned int)__popcll(m & ((1ull << lane) - 1ull));
			const bool out = slow && slot < p.wx_cap;
			if (out) {
				const uint32_t *hc = &L.h[col >> 6][0][col & 63];
				const size_t cap = p.wx_cap;
#pragma unroll 5
				for (int j = 0; j < SGH_HROWS; j++)
					p.wx[(size_t)j * cap + slot] = hc[64 * j];
				p.wx[(size_t)SGH_HROWS * cap + slot] = (uint32_t)col_lo(col);
				p.wx[(size_t)(SGH_HROWS + 1) * cap + slot] = L.nz[col] | (L.ns[col] << 16);
				p.wx[(size_t)(SGH_HROWS + 2) * cap + slot] = (uint32_t)(((int64_t)c * p.H + R) * p.W + x);
			}
			sgh_finish2<REJ, false, NI, false, false>(p, L, col, 0, col_lo(col), R, c, out ? p.W : x, redo_count,
					redo_list);
			return;
		}
		if (SGH_WINS_ORDER && NI == 1) {
			if (wave == 0) {
				const int ca = lane, cb = 64 + lane;
				const bool sa = (L.nz[ca] | L.ns[ca]) != 0u, sb = (L.nz[cb] | L.ns[cb]) != 0u;
				const uint64_t ma = __ballot(sa), mb = __ballot(sb);
				const uint64_t lt = (1ull << lane) - 1ull;
				const int na = __popcll(ma), ns = na + __popcll(mb);
				const int ra = __popcll(ma & lt), rb = __popcll(mb & lt);
				L.perm[sa ? ra : ns + (lane - ra)] = (uint8_t)ca;
				L.perm[sb ? na + rb : ns + (64 - na) + (lane - rb)] = (uint8_t)cb;
			}
			__syncthreads();
			if (wave >= 2)
				return;
			const int col = L.perm[64 * wave + lane];
			sgh_finish2<REJ, false, NI, NORM == 1 || NORM == 3, NORM != 0>(p, L, col, 0, col_lo(col), R, c, col_x(col),
					redo_count, redo_list, interior);
			return;
		}
		for (int col = 64 * wave + lane; col < COLS; col += 64 * WAVES)
			sgh_finish2<REJ, false, NI, NORM == 1 || NORM == 3, NORM != 0>(p, L, col, 0, col_lo(col), R, c, col_x(col),
					redo_count, redo_list, interior);
		return;
	}
	if (REJ == 3) {	/* SIGMEDIAN: one lane per column (waves 0 and 1) */
		for (int col = 64 * wave + lane; col < COLS; col += 64 * WAVES)
			sgh_finish2<REJ, false, NI, false, false>(p, L, col, 0, col_lo(col), R, c, col_x(col), redo_count, redo_list);
		return;
	}
	/* every wave finishes 32 pixel columns, a lane pair per column */
	const int half = lane & 1;
	int col = 32 * wave + (lane >> 1);
	for (; col < COLS; col += 32 * WAVES)
		sgh_finish2<REJ, true, NI, NORM == 1 || NORM == 3 || NORM == 4, NORM != 0 && REJ == 2>(p, L, col, half, col_lo(col), R, c,
				col_x(col), redo_count, redo_list, interior);
	if (timeline && lane == 0) {
		const uint64_t t = __builtin_amdgcn_s_memrealtime();
		if (wave == 0)
			tl[2] = t;
		atomicMax((unsigned long long *)&tl[3], (unsigned long long)t);
	}
}

/* REJ 2 = SIGMA, 4 = WINSORIZED; NORM 0 none, 1 additive, 2 multiplicative, 3 additive with the
 * folded + 0.5; NI pixel pairs per lane (tile of 128 NI pixels, 4 NI waves).  Two 8-wave
 * workgroups (69 KB of LDS each) or four 4-wave ones (36 KB) per CU: 16 waves, at most 128
 * VGPRs. */
#ifndef SGH_WINS_WPE
#define SGH_WINS_WPE 2	/* WINSORIZED: waves per SIMD the register budget is sized for (2-wave tiles: 4 tiles per CU, the LDS limit; 4 waves per SIMD = 128 VGPRs spill) */
#endif
template <int REJ, int NORM, int NI>
__global__ void __launch_bounds__((64 * SghW<REJ, NI>::WAVES), ((REJ == 4 && NI == 1) ? SGH_WINS_WPE : SghCfg<NI>::WPE))
k_stack_hist(SgStackParams p, const int *__restrict__ tab, const int4 *__restrict__ norm,
		unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list) {
	SghRo ro;
	ro.tab = tab;
	ro.norm = norm;
	ro.npad = p.hist_npad;
	__shared__ SghLds<NI> L;
	/* XCD-aware tile order: the dispatcher deals workgroups round-robin to the 8 XCDs, so
	 * XCD k gets a contiguous run of tiles (whole rows: neighbouring tiles share the 128-B
	 * lines their shifted rows straddle in that XCD's L2, and the slower image-edge tiles
	 * spread evenly instead of all landing on XCDs 0 and 7) */
	const int nblk = (int)gridDim.x, xcd = (int)blockIdx.x & 7, q = nblk >> 3, rem = nblk & 7;
	const int vb = xcd * q + (xcd < rem ? xcd : rem) + ((int)blockIdx.x >> 3);
	const int ntiles = ((p.W + 128 * NI - 1) / (128 * NI)) * (p.row_end - p.row_begin) * p.C;
	/* one tile per workgroup: stacking 2 or 4 consecutive tiles per workgroup (the next
	 * tile's first loads overlapping the previous finish) measured 5.0 / 4.9 ms against 3.58
	 * (scripts/gpu_r3p.sh; the tile loop also costs registers: 128 VGPRs + scratch) */
	if (vb >= ntiles)
		return;
	/* normalised: the single-rounding load when k_norm_fma_check found it exact for every frame (its
	 * flag word behind the pairs stays 0; the host stages 1 when the check is not run) */
	const unsigned int verdict = NORM >= 1 && NORM <= 3 ? ((const unsigned int *)(norm + 2 * ro.npad))[0] : 3u;
	/* 1: single rounding (fma), 2: integer offset (additive, scale 1), 0: the reference's operations */
	const int load = (NORM == 1 || NORM == 3) && !(verdict & 2u) ? 2 : (!(verdict & 1u) ? 1 : 0);
	sgh_tile<REJ, NORM, NI>(p, ro, L, vb, false, redo_count, redo_list, load);
}

/* k_norm_fma_check: may the normalising load use one fma per sample?  The reference normalises
 * a sample x in two or three roundings (:1642-1651, round_to_WORD utils.c:68-74): additive
 * fl(fl(x scale) - offset) (+ 0.5), multiplicative fl(fl(x scale) mul) + 0.5.  The candidate is
 * fma(x, a, b) with {a, b} = {scale, -(offset - 0.5)} (mode 3: the folded offset), {scale,
 * fl(0.5 - offset)} (mode 1) or {fl(scale mul), 0.5} (mode 2).  Both go through the kernels'
 * conversion (v_cvt_u32_f64, then the pack's clamp to 65535) for every u16 x of every frame; one
 * difference anywhere sets the flag word and the call keeps the reference's operations.
 * pairs: the {scale, offset - 0.5 | offset | mul} pairs of the histogram kernels; the candidates go
 * npad pairs further, the flag word (staged 0 when the check runs; bit 0: the fma differs, bit 1: the
 * integer form differs) 2 npad pairs further.  Additive with scale 1 also tries clamp(x - K, 0, 65535)
 * (two packed saturating u16 ops per pixel pair, NORM 6), written 2 npad + 1 pairs further.  Grid (16, N) x 256 threads,
 * 16 values per thread. */
__global__ void __launch_bounds__(256)
k_norm_fma_check(double *__restrict__ pairs, int N, int npad, int mode, unsigned int *__restrict__ verdict) {
	const int f = blockIdx.y;
	if (f >= N)
		return;
	const double a = pairs[2 * f], b = pairs[2 * f + 1];
	const double A = mode == 2 ? a * b : a;
	const double B = mode == 2 ? 0.5 : (mode == 3 ? -b : 0.5 - b);
	/* additive with scale 1: clamp(x - K, 0, 65535), K = ceil(offset - 0.5) clamped to +-65535 */
	const bool icand = mode != 2 && a == 1.0;
	const double kc = ceil(mode == 3 ? b : b - 0.5);
	const int K = icand ? (kc > 65535.0 ? 65535 : (kc < -65535.0 ? -65535 : (int)kc)) : 0;
	auto cvt = [](double y) -> uint32_t {
		uint32_t r;
		asm volatile("v_cvt_u32_f64 %0, %1" : "=v"(r) : "v"(y));
		return r < 65535u ? r : 65535u;
	};
	bool bad = false, ibad = !icand;
	const int x0 = blockIdx.x * 4096 + threadIdx.x;
#pragma unroll 4
	for (int k = 0; k < 16; k++) {
		const int xi = x0 + 256 * k;
		const double x = (double)xi;
		const double t = x * a;
		const double yr = mode == 3 ? t - b : (mode == 1 ? t - b : t * b) + 0.5;
		const uint32_t r = cvt(yr);
		bad |= r != cvt(__builtin_fma(x, A, B));
		const int yi = xi - K;
		ibad |= r != (uint32_t)(yi < 0 ? 0 : (yi > 65535 ? 65535 : yi));
	}
	const unsigned int flags = (__ballot(bad) ? 1u : 0u) | (__ballot(ibad) ? 2u : 0u);
	if (flags && (threadIdx.x & 63) == 0) {
		atomicOr((unsigned int *)(pairs + 4 * (size_t)npad), flags);
		atomicOr(verdict, flags);	/* counter block: read back with the counters (sg_stack_stats::norm_fma) */
	}
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		pairs[2 * ((size_t)npad + f)] = A;
		pairs[2 * ((size_t)npad + f) + 1] = B;
		/* the integer pair (int4 2 npad + 1 + f): {kpos, kneg} in both u16 halves */
		const uint32_t kp = (uint32_t)(K > 0 ? K : 0), kn = (uint32_t)(K < 0 ? -K : 0);
		int *ip = (int *)(pairs + 4 * (size_t)npad + 2 + 2 * (size_t)f);
		ip[0] = (int)(kp | kp << 16);
		ip[1] = (int)(kn | kn << 16);
	}
}

/* k_hist_slow: the exported WINSORIZED columns (SgStackParams::wx), 64 per wave, each lane's
 * histogram column back in LDS in the tile's layout, finished by the tile's own code (sgh_finish2:
 * the same queries, decisions, redo list and counters).  Waves of exported columns only: their
 * inner-iteration counts are alike, and no build shares the CU's LDS with them. */
struct SghSlowLds {
	uint32_t h[1][SGH_HROWS][64];
	uint32_t nz[64], ns[64], na[64];
};
#ifndef SGH_SLOW_WPE
#define SGH_SLOW_WPE 2
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SGH_SLOW_WPE)))
k_hist_slow(SgStackParams p, unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list) {
	__shared__ SghSlowLds L;
	const int lane = threadIdx.x & 63;
	const unsigned int cnt = *(volatile const unsigned int *)p.wx_count;
	const unsigned int n = cnt < p.wx_cap ? cnt : p.wx_cap;
	const size_t cap = p.wx_cap;
	for (unsigned int s0 = blockIdx.x * 64u; s0 < n; s0 += gridDim.x * 64u) {
		const unsigned int slot = s0 + (unsigned int)lane;
		const bool v = slot < n;
#pragma unroll 5
		for (int j = 0; j < SGH_HROWS; j++)
			L.h[0][j][lane] = v ? p.wx[(size_t)j * cap + slot] : 0u;
		const uint32_t lo = v ? p.wx[(size_t)SGH_HROWS * cap + slot] : 1u;
		const uint32_t zs = v ? p.wx[(size_t)(SGH_HROWS + 1) * cap + slot] : 0u;
		const uint32_t pix = v ? p.wx[(size_t)(SGH_HROWS + 2) * cap + slot] : 0u;
		L.nz[lane] = zs & 0xFFFFu;
		L.ns[lane] = zs >> 16;
		L.na[lane] = 0u;
		const uint32_t W = (uint32_t)p.W, t = pix / W;
		const int x = v ? (int)(pix - t * W) : p.W;
		const int R = (int)(t % (uint32_t)p.H), c = (int)(t / (uint32_t)p.H);
		/* each lane reads only its own column: no barrier */
		sgh_finish2<4, false, 1, false, false, SghSlowLds>(p, L, lane, 0, (int)lo, R, c, x, redo_count, redo_list);
	}
}

template __global__ void k_stack_hist<2, 0, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<2, 1, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<2, 2, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<2, 3, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<4, 3, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<4, 0, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<4, 1, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<4, 2, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<1, 0, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<1, 1, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<1, 2, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<1, 3, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<3, 0, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<3, 1, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<3, 2, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<3, 3, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<8, 0, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<8, 1, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<8, 2, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<8, 3, 1>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<2, 0, 2>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);
template __global__ void k_stack_hist<4, 0, 2>(SgStackParams, const int *, const int4 *, unsigned int *,
		unsigned int *);

/* threads per histogram workgroup (the host's launch shape) */
int sgh_block_threads(int ni, int rej) {
	if (rej == 4)
		return ni == 2 ? 64 * SghW<4, 2>::WAVES : 64 * SghW<4, 1>::WAVES;
	return ni == 2 ? 64 * SghCfg<2>::WAVES : 64 * SghCfg<1>::WAVES;
}
