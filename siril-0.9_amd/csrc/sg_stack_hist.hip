/*
 * sg_stack_hist.hip - gfx950 fast path of stack_mean_with_rejection, SIGMA rejection
 * (src/stacking/stacking.c:1674-1695 + sigma_clipping :1148-1161), without sorting.
 *
 * Why: the reference sorts every pixel column (quicksort_s) on every clipping pass.  A
 * sort of N = 512 u16 per pixel costs ~O(N log^2 N) compare-exchanges on a GPU, far more
 * VALU than the N*2 bytes the pixel reads from HBM can hide.  But every quantity a
 * sigma-clip pass needs is a function of the column's value HISTOGRAM:
 *   - the kept set after any number of passes is {v : A <= v <= B} (low clips remove the
 *     lowest values, high clips the highest; the set stays a value interval);
 *   - median of the kept set = value at a rank, counts below/above a threshold = ranks;
 *   - sigma comes from exact integer moments n, S, SS of the kept set.
 * So each 64-pixel tile builds, per pixel, an exact histogram of 256 unit-wide bins
 * [lo, lo+255] around the median of the first 16 frames (u8 counts packed 4 per dword),
 * plus counters of the samples below / above the band and of the zeros / 65535s among
 * them (out-of-frame zero fill, dead pixels, saturation, cosmics).  4 waves stream the
 * N frames into it: per-frame buffer descriptors give 128-byte coalesced row loads whose
 * out-of-frame lanes read 0 from the hardware bounds check (shift + zero fill of
 * :1535-1654 for free), two frames share a VGPR (16-bit halves) and are binned with
 * packed u16 arithmetic and branch-free LDS atomics.  Wave 0 then prefix-sums the bins
 * once and runs the reference's pass loop as O(log) histogram queries.
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
#define SGH_WAVES 4
#define SGH_CENTER 16		/* frames used for the centre estimate */
#define SGH_BAND 1e-11		/* same rounding band as the sorted path (SG_BAND) */

typedef unsigned short sgh_u16x2 __attribute__((ext_vector_type(2)));

/* hist[0]          : samples below the band (u32)
 * hist[1 + j] byte b: count of value lo + 4j + b
 * hist[1 + SGH_DW]  : samples above the band (u32) */
struct SghLds {
	uint32_t hist[SGH_DW + 2][64];
	uint16_t cum16[SGH_DW / 4][64];		/* band samples in bins < 16(j+1) */
	uint32_t nz[64], ns[64];		/* zeros / 65535s (all of them lie outside the band) */
};

struct SghPix {
	int lo;			/* value of bin 0, 1 <= lo <= 65279 */
	int nz, ns, nb;		/* zeros, 65535s, band samples (nz + nb + ns == N) */
	int lane;
	const SghLds *L;
};

/* # band samples with bin index <= t (t in [-1, 255]) */
__device__ __forceinline__ int sgh_band_le(const SghPix &P, int t) {
	if (t < 0)
		return 0;
	if (t > SGH_BINS - 1)
		t = SGH_BINS - 1;
	const int j16 = t >> 4, jd = t >> 2;
	int base = j16 ? (int)P.L->cum16[j16 - 1][P.lane] : 0;
	for (int k = 4 * j16; k < jd; k++)
		base += (int)__builtin_amdgcn_sad_u8(P.L->hist[1 + k][P.lane], 0u, 0u);
	const uint32_t d = P.L->hist[1 + jd][P.lane];
	const int sh = ((t & 3) + 1) * 8;
	const uint32_t m = sh >= 32 ? 0xFFFFFFFFu : ((1u << sh) - 1u);
	return base + (int)__builtin_amdgcn_sad_u8(d & m, 0u, 0u);
}

/* # samples with value <= v, v in [-1, 65535] */
__device__ __forceinline__ int sgh_cnt_le(const SghPix &P, int v) {
	if (v < 0)
		return 0;
	if (v < P.lo)
		return P.nz;
	if (v < P.lo + SGH_BINS)
		return P.nz + sgh_band_le(P, v - P.lo);
	if (v < 65535)
		return P.nz + P.nb;
	return P.nz + P.nb + P.ns;
}

/* value at global rank g (0-based) */
__device__ int sgh_value_at(const SghPix &P, int g) {
	if (g < P.nz)
		return 0;
	g -= P.nz;
	if (g >= P.nb)
		return 65535;
	/* smallest j with cum16[j] > g, then walk its 4 dwords */
	int a = 0, b = SGH_DW / 4 - 1;
	while (a < b) {
		const int m = (a + b) >> 1;
		if ((int)P.L->cum16[m][P.lane] > g)
			b = m;
		else
			a = m + 1;
	}
	int base = a ? (int)P.L->cum16[a - 1][P.lane] : 0;
	int k = 4 * a;
	uint32_t d = P.L->hist[1 + k][P.lane];
	for (; k < 4 * a + 3; k++) {
		const int bs = (int)__builtin_amdgcn_sad_u8(d, 0u, 0u);
		if (base + bs > g)
			break;
		base += bs;
		d = P.L->hist[2 + k][P.lane];
	}
	int i = 0;
	for (; i < 3; i++) {
		base += (int)((d >> (8 * i)) & 0xFF);
		if (base > g)
			break;
	}
	return P.lo + 4 * k + i;
}

/* count, sum and sum of squares of (v - lo) over samples with v1 <= v <= v2 */
__device__ void sgh_range_moments(const SghPix &P, int v1, int v2, long long &s, unsigned long long &ss) {
	s = 0;
	ss = 0;
	if (v1 > v2)
		return;
	if (P.nz && v1 <= 0 && 0 <= v2) {
		const long long d = -P.lo;
		s += d * P.nz;
		ss += (unsigned long long)(d * d) * (unsigned long long)P.nz;
	}
	if (P.ns && v1 <= 65535 && 65535 <= v2) {
		const long long d = 65535 - P.lo;
		s += d * P.ns;
		ss += (unsigned long long)(d * d) * (unsigned long long)P.ns;
	}
	int b1 = v1 - P.lo, b2 = v2 - P.lo;
	if (b1 < 0)
		b1 = 0;
	if (b2 > SGH_BINS - 1)
		b2 = SGH_BINS - 1;
	if (b1 > b2)
		return;
	uint32_t s32 = 0, ss32 = 0;
	for (int j = b1 >> 2; j <= (b2 >> 2); j++) {
		uint32_t d = P.L->hist[1 + j][P.lane];
		const int first = 4 * j, last = 4 * j + 3;
		if (first < b1)
			d &= 0xFFFFFFFFu << (8 * (b1 - first));
		if (last > b2)
			d &= 0xFFFFFFFFu >> (8 * (last - b2));
		const uint32_t bs = __builtin_amdgcn_sad_u8(d, 0u, 0u);
		const uint32_t d1 = __builtin_amdgcn_udot4(d, 0x03020100u, 0u, false);
		const uint32_t d2 = __builtin_amdgcn_udot4(d, 0x09040100u, 0u, false);
		const uint32_t jj = (uint32_t)j;
		s32 += 4u * jj * bs + d1;
		ss32 += 16u * jj * jj * bs + 8u * jj * d1 + d2;
	}
	s += (long long)s32;
	ss += (unsigned long long)ss32;
}

__device__ __forceinline__ int sgh_ceil_clamp(double x) {
	if (!(x > 0.0))
		return 0;
	if (x > 65536.0)
		return 65536;
	return (int)ceil(x);
}
__device__ __forceinline__ int sgh_floor_clamp(double x) {
	if (!(x < 65535.0))
		return 65535;
	if (x < -1.0)
		return -1;
	return (int)floor(x);
}

/* the reference's SIGMA loop on the histogram; returns SG_CLS_OK or 1 (redo in the
 * sorted kernel).  Decision logic mirrors clip_pass() of the sorted path. */
__device__ int sgh_sigma(const SghPix &P, int N, double sl, double sh, long long S, unsigned long long SS,
		uint16_t *value, uint32_t *rlo_out, uint32_t *rhi_out) {
	/* kept set = samples with A <= v <= B; cntA = # samples < A, cntB = # samples <= B */
	int A = 0, B = 65535, n = N, r = 0, nrem, cntA = 0, cntB = N;
	uint32_t rlo = 0, rhi = 0;
	do {
		const long long num = (long long)n * (long long)SS - S * S;
		const bool exact0 = (num == 0);
		const double sigma = num <= 0 ? 0.0 : sqrt((double)num / ((double)n * (double)(n - 1)));
		const int g1 = cntA + (n - 1) / 2, g2 = cntA + n / 2;
		const int m1 = sgh_value_at(P, g1);
		const int m2 = (g2 == g1) ? m1 : sgh_value_at(P, g2);
		const double median = (g1 == g2) ? (double)m1 : (double)(m1 + m2) / 2.0;
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		const double tol = exact0 ? 0.0 : SGH_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
		/* low: v < blo - tol rejected; v in [blo - tol, blo + tol] ambiguous */
		int a = sgh_ceil_clamp(blo - tol);
		if (a < A)
			a = A;
		int bt = sgh_floor_clamp(bhi + tol);
		if (bt > B)
			bt = B;
		const int cnt_a = a > A ? sgh_cnt_le(P, a - 1) : cntA;	/* # < a */
		const int cnt_bt = bt < B ? sgh_cnt_le(P, bt) : cntB;	/* # <= bt */
		if (!exact0) {
			int amb1 = sgh_floor_clamp(blo + tol);
			if (amb1 > B)
				amb1 = B;
			if (a <= amb1 && sgh_cnt_le(P, amb1) - cnt_a > 0)
				return 1;
			int amb0 = sgh_ceil_clamp(bhi - tol);
			if (amb0 < A)
				amb0 = A;
			if (amb0 <= bt && cnt_bt - sgh_cnt_le(P, amb0 - 1) > 0)
				return 1;
		}
		const int L = cnt_a - cntA, H = cntB - cnt_bt;
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
		if (L) {
			long long s;
			unsigned long long ss;
			sgh_range_moments(P, A, a - 1, s, ss);
			S -= s;
			SS -= ss;
			A = a;
			cntA = cnt_a;
		}
		if (H) {
			long long s;
			unsigned long long ss;
			sgh_range_moments(P, bt + 1, B, s, ss);
			S -= s;
			SS -= ss;
			B = bt;
			cntB = cnt_bt;
		}
		rlo += L;
		rhi += H;
		r += L + H;
		nrem = L + H;
		n -= nrem;
	} while (nrem > 0 && n > 3);
	const long long tot = S + (long long)n * P.lo;
	*value = sg_round_to_WORD((double)tot / (double)n);
	*rlo_out = rlo;
	*rhi_out = rhi;
	return SG_CLS_OK;
}

/* centre estimate from 16 samples: median of those that are neither 0 nor 65535 (the
 * out-of-frame zero fill of edge pixels must not drag the band away), bitonic network */
__device__ __forceinline__ uint32_t sgh_median16(const uint32_t (&in)[SGH_CENTER]) {
	uint32_t v[SGH_CENTER];
#pragma unroll
	for (int i = 0; i < SGH_CENTER; i++)
		v[i] = in[i];
#pragma unroll
	for (int k = 2; k <= SGH_CENTER; k <<= 1) {
#pragma unroll
		for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
			for (int i = 0; i < SGH_CENTER; i++) {
				const int l = i ^ j;
				if (l > i) {
					const bool up = (i & k) == 0;
					const uint32_t a = v[i], b = v[l];
					const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
					v[i] = up ? lo : hi;
					v[l] = up ? hi : lo;
				}
			}
		}
	}
	int z = 0, sat = 0;
#pragma unroll
	for (int i = 0; i < SGH_CENTER; i++) {
		z += v[i] == 0;
		sat += v[i] == 65535;
	}
	int idx = z + (SGH_CENTER - z - sat) / 2;
	if (idx > SGH_CENTER - 1)
		idx = SGH_CENTER - 1;
	uint32_t r = v[0];
#pragma unroll
	for (int i = 1; i < SGH_CENTER; i++)
		r = (i == idx) ? v[i] : r;
	return r;
}

/* per-frame load context: each frame gets its own buffer descriptor (num_records = one
 * plane) so that any offset outside the plane reads 0 through the hardware bounds check */
struct SghFrame {
	const char *plane0;		/* channel plane of frame 0 */
	int64_t fstride2;		/* bytes between frames */
	uint32_t plane_bytes;
	int rw2;			/* R * W * 2 */
	int w2;				/* W * 2 */
	uint32_t x2;			/* 2 * x (per lane) */
};

/* one sample: c1 = shifty*W*2 + 2*shiftx, sx2 = 2*shiftx (per-frame table, read from LDS
 * as wave-uniform VGPR values); byte offset (R - sy) W 2 + 2 (x - sx): a row outside the
 * frame gives a negative (huge) or past-the-plane offset -> 0 (the zero rows of
 * :1550-1577); the column check forces an out-of-range offset (the x shift writes 0,
 * :1628-1632) */
__device__ __forceinline__ unsigned short sgh_load(const SghFrame &F, const char *base, uint32_t nrec, int c1, int sx2) {
	const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nrec, 0x00020000);
	const uint32_t sc2 = F.x2 - (uint32_t)sx2;
	const uint32_t voff = sc2 < (uint32_t)F.w2 ? (uint32_t)(F.rw2 - c1) + F.x2 : 0x80000000u;
	return __builtin_amdgcn_raw_buffer_load_b16(rsrc, (int)voff, 0, 0);
}

/* shift table of the 16 frames f0..f0+15 (f0 % 16 == 0): c1 (one s_load_dwordx16) and the
 * int16 sx2 (one s_load_dwordx8), wave-uniform values in SGPRs; the table is padded to a
 * multiple of 16 frames with zeros */
struct SghTab16 {
	int c1[16];
	uint32_t sx2p[8];
};
__device__ __forceinline__ void sgh_tab16(const SgStackParams &p, int f0, SghTab16 &T) {
	const int4 *q = (const int4 *)(p.hist_tab + f0);
	const int4 *r = (const int4 *)(p.hist_tab + p.hist_npad + f0 / 2);
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

/* 16 frames f0..f0+15, one sample per register (packing at load time would make the
 * compiler wait for each load right after issuing it); frames >= N get num_records = 0
 * (every lane reads 0; never binned) */
template <bool FULL>
__device__ __forceinline__ void sgh_loadblk(const SghFrame &F, const SghTab16 &T, int N, int f0, uint32_t (&dst)[16]) {
	const char *b = F.plane0 + (int64_t)f0 * F.fstride2;
#pragma unroll
	for (int m = 0; m < 8; m++) {
		const uint32_t na = (FULL || f0 + 2 * m < N) ? F.plane_bytes : 0u;
		const uint32_t nb = (FULL || f0 + 2 * m + 1 < N) ? F.plane_bytes : 0u;
		const int sxa = (int)(int16_t)(T.sx2p[m] & 0xFFFFu), sxb = (int)T.sx2p[m] >> 16;
		dst[2 * m] = sgh_load(F, b, na, T.c1[2 * m], sxa);
		b += F.fstride2;
		dst[2 * m + 1] = sgh_load(F, b, nb, T.c1[2 * m + 1], sxb);
		b += F.fstride2;
	}
}

/* bin a pair of samples (two frames of this lane's pixel, 16-bit halves of vv) */
__device__ __forceinline__ void sgh_bin_pair(SghLds &L, uint32_t laneaddr, uint32_t lo1x2, uint32_t vv,
		uint32_t &nonzero, uint32_t &nsat, int dbg) {
	const sgh_u16x2 v = __builtin_bit_cast(sgh_u16x2, vv);
	if (dbg == 3) {		/* A/B: loads only */
		nonzero += vv;
		return;
	}
	const sgh_u16x2 l1 = __builtin_bit_cast(sgh_u16x2, lo1x2);
	sgh_u16x2 t = __builtin_elementwise_sub_sat(v, l1);	/* 0 below the band, 1..256 inside */
	t = __builtin_elementwise_min(t, (sgh_u16x2){257, 257});
	/* 0 below (dword 0, a u32 counter), 4..259 band, 260 above (dword 65, u32) */
	t = t + __builtin_elementwise_min(t, (sgh_u16x2){1, 1}) * (sgh_u16x2){3, 3};
	const uint32_t tt = __builtin_bit_cast(uint32_t, t);
	const uint32_t t3 = tt << 3;
	const uint32_t a0 = (__builtin_amdgcn_ubfe(tt, 2, 8) << 8) + laneaddr;
	const uint32_t a1 = (__builtin_amdgcn_ubfe(tt, 18, 8) << 8) + laneaddr;
	const uint32_t i0 = 1u << (t3 & 24u);
	const uint32_t i1 = 1u << __builtin_amdgcn_ubfe(t3, 16, 5);
	uint32_t *h = &L.hist[0][0];
	atomicAdd(h + (a0 >> 2), i0);
	atomicAdd(h + (a1 >> 2), i1);
	/* nonzero samples and 65535 samples of the pair */
	const sgh_u16x2 nzv = __builtin_elementwise_min(v, (sgh_u16x2){1, 1});
	const sgh_u16x2 sv = __builtin_elementwise_sub_sat(v, (sgh_u16x2){65534, 65534});
	nonzero = __builtin_amdgcn_udot2(nzv, (sgh_u16x2){1, 1}, nonzero, false);
	nsat = __builtin_amdgcn_udot2(sv, (sgh_u16x2){1, 1}, nsat, false);
}

__global__ void __launch_bounds__(64 * SGH_WAVES)
k_stack_hist(SgStackParams p, unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list) {
	__shared__ SghLds L;
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int ntx = (p.W + SG_TILE_W - 1) / SG_TILE_W;
	const int nrows = p.row_end - p.row_begin;
	int bid = blockIdx.x;
	const int xt = bid % ntx;
	bid /= ntx;
	const int R = p.row_begin + (bid % nrows);
	const int c = bid / nrows;
	const int x = xt * SG_TILE_W + lane;
	const int N = p.N;
	const int Npad = (N + 15) & ~15;
	SghFrame F;
	F.plane0 = (const char *)(p.frames + (int64_t)c * p.plane_stride);
	F.fstride2 = p.frame_stride * 2;
	F.plane_bytes = (uint32_t)p.H * (uint32_t)p.W * 2u;
	F.w2 = p.W * 2;
	F.rw2 = R * p.W * 2;
	F.x2 = (uint32_t)x * 2u;

	for (int i = tid; i < (SGH_DW + 2) * 64; i += 64 * SGH_WAVES)
		(&L.hist[0][0])[i] = 0;
	if (tid < 64) {
		L.nz[tid] = 0;
		L.ns[tid] = 0;
	}
	__syncthreads();

	constexpr int M = 16, MP = M / 2;	/* frames per block, packed pairs per block */
	auto loadblk = [&](int f0, const SghTab16 &T, uint32_t (&dst)[M]) {
		if (f0 + M <= N)
			sgh_loadblk<true>(F, T, N, f0, dst);
		else
			sgh_loadblk<false>(F, T, N, f0, dst);
	};
	/* 16-frame blocks: wave w bins blocks w, w+4, ...; frames 0..15 (block 0) are the
	 * centre sample every wave loads.  Two named buffers keep the next block's loads in
	 * flight while the current one is binned; the shift table of the block after that is
	 * fetched (scalar loads) before binning. */
	uint32_t p16[SGH_CENTER], bufA[M], bufB[M];
	SghTab16 T;
	sgh_tab16(p, 0, T);
	sgh_loadblk<true>(F, T, N, 0, p16);
	int fb = M * wave;
	if (fb >= SGH_CENTER && fb < N) {
		sgh_tab16(p, fb, T);
		loadblk(fb, T, bufA);
	}
	constexpr int STEP = M * SGH_WAVES;
	sgh_tab16(p, fb + STEP < N ? fb + STEP : (fb < Npad ? fb : 0), T);
	/* centre: median of the first 16 samples */
	uint32_t v16[SGH_CENTER];
#pragma unroll
	for (int k = 0; k < SGH_CENTER; k++)
		v16[k] = p16[k];
	int lo = (int)sgh_median16(v16) - SGH_BINS / 2;
	if (lo < 1)
		lo = 1;
	if (lo > 65535 - SGH_BINS)
		lo = 65535 - SGH_BINS;
	if (fb < SGH_CENTER) {
#pragma unroll
		for (int m = 0; m < M; m++)
			bufA[m] = p16[m];
	}

	const uint32_t laneaddr = (uint32_t)lane * 4u;
	const uint32_t lo1x2 = (uint32_t)(lo - 1) * 0x10001u;
	uint32_t nonzero = 0, nsat = 0, counted = 0;
	auto binblk = [&](int f0, const uint32_t (&raw)[M]) {
		uint32_t src[MP];
#pragma unroll
		for (int m = 0; m < MP; m++)
			src[m] = raw[2 * m] | (raw[2 * m + 1] << 16);
		if (f0 + M <= N) {
#pragma unroll
			for (int m = 0; m < MP; m++)
				sgh_bin_pair(L, laneaddr, lo1x2, src[m], nonzero, nsat, p.dbg);
			counted += M;
		} else {
			/* partial last block: a lone frame is paired with a 65535 sample whose count
			 * is taken back below */
			for (int m = 0; m < MP; m++) {
				const int fa = f0 + 2 * m;
				if (fa >= N)
					break;
				const uint32_t vv = fa + 1 < N ? src[m] : ((src[m] & 0xFFFFu) | 0xFFFF0000u);
				sgh_bin_pair(L, laneaddr, lo1x2, vv, nonzero, nsat, p.dbg);
				counted += 2;
				if (fa + 1 >= N) {
					atomicSub(&L.hist[SGH_DW + 1][lane], 1u);	/* the padding 65535 */
					nsat--;
					nonzero--;
					counted--;
				}
			}
		}
	};
	/* invariant: T = table of block nx(fb) = the block loaded next */
	auto nx = [&](int f) { return f + STEP < N ? f + STEP : f; };
	while (fb < N) {
		loadblk(nx(fb), T, bufB);
		sgh_tab16(p, nx(nx(fb)), T);
		binblk(fb, bufA);
		fb += STEP;
		if (fb >= N)
			break;
		loadblk(nx(fb), T, bufA);
		sgh_tab16(p, nx(nx(fb)), T);
		binblk(fb, bufB);
		fb += STEP;
	}
	if (counted) {
		atomicAdd(&L.nz[lane], counted - nonzero);
		atomicAdd(&L.ns[lane], nsat);
	}
	__syncthreads();
	if (wave != 0)
		return;

	if (p.dbg >= 2) {
		if (x < p.W)
			p.out[((int64_t)c * p.H + R) * p.W + x] = (uint16_t)(L.hist[1][lane] + nonzero);
		return;
	}
	/* wave 0: prefix counts + band moments (relative to lo) */
	uint32_t cum = 0, s32 = 0, ss32 = 0;
#pragma unroll 16
	for (int j = 0; j < SGH_DW; j++) {
		const uint32_t d = L.hist[1 + j][lane];
		const uint32_t bs = __builtin_amdgcn_sad_u8(d, 0u, 0u);
		const uint32_t d1 = __builtin_amdgcn_udot4(d, 0x03020100u, 0u, false);
		const uint32_t d2 = __builtin_amdgcn_udot4(d, 0x09040100u, 0u, false);
		const uint32_t jj = (uint32_t)j;
		s32 += 4u * jj * bs + d1;
		ss32 += 16u * jj * jj * bs + 8u * jj * d1 + d2;
		cum += bs;
		if ((j & 3) == 3)
			L.cum16[j >> 2][lane] = (uint16_t)cum;
	}
	const int below = (int)L.hist[0][lane];
	const int above = (int)L.hist[SGH_DW + 1][lane];
	SghPix P;
	P.lo = lo;
	P.nz = (int)L.nz[lane];
	P.ns = (int)L.ns[lane];
	P.nb = (int)cum;
	P.lane = lane;
	P.L = &L;
	int cls = SG_CLS_OK;
	uint16_t value = 0;
	uint32_t rlo = 0, rhi = 0;
	if (x < p.W) {
		/* every out-of-band sample must be a 0 or a 65535, and no counter may have wrapped */
		if (p.dbg == 1) {
			value = (uint16_t)(s32 + ss32);
		} else if (below + P.nb + above != N || below != P.nz || above != P.ns) {
			cls = 1;
		} else {
			const long long dz = -(long long)lo, ds = 65535 - (long long)lo;
			const long long S = (long long)s32 + dz * P.nz + ds * P.ns;
			const unsigned long long SS = (unsigned long long)ss32 +
				(unsigned long long)(dz * dz) * (unsigned long long)P.nz +
				(unsigned long long)(ds * ds) * (unsigned long long)P.ns;
			cls = sgh_sigma(P, N, p.sig0, p.sig1, S, SS, &value, &rlo, &rhi);
		}
		const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
		if (cls == SG_CLS_OK) {
			p.out[pix] = value;
		} else {
			const unsigned int slot = atomicAdd(redo_count, 1u);
			redo_list[slot] = (unsigned int)pix;
			rlo = rhi = 0;
		}
	}
	unsigned long long a = rlo, b = rhi;
	for (int o = 32; o > 0; o >>= 1) {
		a += __shfl_down(a, o, 64);
		b += __shfl_down(b, o, 64);
	}
	if (lane == 0 && (a | b)) {
		unsigned long long *sh = p.rej + ((size_t)(blockIdx.x % SG_REJ_SHARDS) * 6 + c * 2);
		atomicAdd(sh, a);
		atomicAdd(sh + 1, b);
	}
}
