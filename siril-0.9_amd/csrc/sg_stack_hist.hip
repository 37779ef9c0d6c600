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
 * around a centre c (median of the first 16 frames), u8 counts packed 4 per dword,
 * plus explicit lists of the (rare) values outside the band.  4 waves stream the N
 * frames into it with coalesced 128-byte row loads (shift + zero fill applied at load,
 * :1535-1654); wave 0 then prefix-sums the bins once and runs the reference's pass loop
 * as O(log) histogram queries.
 *
 * Exactness: decisions use exact moments; a pixel whose decision falls within a rounding
 * band of a threshold (GSL's long-double sd vs exact), whose loop would hit the
 * reference's early `break` (N - r <= 4, :1684, stale rejected[]), whose median falls
 * outside the band, whose tail list overflows or whose u8 bins overflow (detected: the
 * byte sum must equal the band count) is appended to a redo list and recomputed by the
 * sorted kernel (k_stack_sorted<.., true>), which in turn hands knife-edge pixels to the
 * literal (fp80) path.  Output is therefore bit-identical to the sorted path.
 */
#include "sg_common.hpp"

#define SGH_BINS 256
#define SGH_DW (SGH_BINS / 4)	/* dwords per pixel histogram */
#define SGH_T 16		/* tail capacity per side per pixel */
#define SGH_WAVES 4
#define SGH_CENTER 16		/* frames used for the centre estimate */
#define SGH_BAND 1e-11		/* same rounding band as the sorted path (SG_BAND) */

struct SghLds {
	uint32_t hist[SGH_DW][64];		/* byte b of hist[j][px] = count of bin 4j+b */
	uint16_t cumdw[SGH_DW][64];		/* band samples in bins < 4(j+1) */
	uint16_t tails[2][SGH_T][64];		/* low / high out-of-band values */
	uint32_t ntail[2][64];
	uint32_t nband[64];
	uint32_t nzero[64], nsat[64];		/* out-of-band samples equal to 0 / 65535 (not listed) */
	unsigned long long tsum[64], tsq[64];	/* tail moments relative to lo (two's complement sum) */
};

struct SghPix {
	int lo;			/* value of bin 0 */
	int nlo, nhi, nb;	/* samples below / above / inside the band (nlo, nhi include nz, ns) */
	int nz, ns;		/* out-of-band zeros / 65535s (counted, not listed) */
	int nll, nhl;		/* listed low / high tail values */
	int lane;
	const SghLds *L;
};

/* # band samples with bin index <= t (t in [-1, 255]) */
__device__ __forceinline__ int sgh_band_le(const SghPix &P, int t) {
	if (t < 0)
		return 0;
	if (t > SGH_BINS - 1)
		t = SGH_BINS - 1;
	const int j = t >> 2;
	const int base = j ? (int)P.L->cumdw[j - 1][P.lane] : 0;
	const uint32_t d = P.L->hist[j][P.lane];
	const int sh = ((t & 3) + 1) * 8;
	const uint32_t m = sh >= 32 ? 0xFFFFFFFFu : ((1u << sh) - 1u);
	return base + (int)__builtin_amdgcn_sad_u8(d & m, 0u, 0u);
}

/* # samples (all frames) with value <= v, v in [-1, 65535] */
__device__ int sgh_cnt_le(const SghPix &P, int v) {
	if (v < 0)
		return 0;
	if (v < P.lo) {
		int c = P.nz;
		for (int k = 0; k < P.nll; k++)
			c += (int)P.L->tails[0][k][P.lane] <= v;
		return c;
	}
	if (v < P.lo + SGH_BINS)
		return P.nlo + sgh_band_le(P, v - P.lo);
	int c = P.nlo + P.nb + (v >= 65535 ? P.ns : 0);
	for (int k = 0; k < P.nhl; k++)
		c += (int)P.L->tails[1][k][P.lane] <= v;
	return c;
}

/* value at global rank g (0-based) if it lies in the band or on a counted 0 / 65535
 * tail, else -1 (listed tails are unsorted) */
__device__ int sgh_value_at(const SghPix &P, int g) {
	if (g < P.nz)
		return 0;
	if (g >= P.nlo + P.nb + P.nhl)
		return 65535;
	g -= P.nlo;
	if (g < 0 || g >= P.nb)
		return -1;
	/* smallest j with cumdw[j] > g */
	int a = 0, b = SGH_DW - 1;
	while (a < b) {
		const int m = (a + b) >> 1;
		if ((int)P.L->cumdw[m][P.lane] > g)
			b = m;
		else
			a = m + 1;
	}
	int base = a ? (int)P.L->cumdw[a - 1][P.lane] : 0;
	const uint32_t d = P.L->hist[a][P.lane];
	int i = 0;
	for (; i < 3; i++) {
		base += (int)((d >> (8 * i)) & 0xFF);
		if (base > g)
			break;
	}
	return P.lo + 4 * a + i;
}

/* count, sum and sum of squares of (v - lo) over samples with v1 <= v <= v2 */
__device__ void sgh_range_moments(const SghPix &P, int v1, int v2, int &cnt, long long &s, unsigned long long &ss) {
	cnt = 0;
	s = 0;
	ss = 0;
	if (v1 > v2)
		return;
	if (P.nz && v1 <= 0 && 0 <= v2) {
		const long long d = -P.lo;
		cnt += P.nz;
		s += d * P.nz;
		ss += (unsigned long long)(d * d) * (unsigned long long)P.nz;
	}
	if (P.ns && v1 <= 65535 && 65535 <= v2) {
		const long long d = 65535 - P.lo;
		cnt += P.ns;
		s += d * P.ns;
		ss += (unsigned long long)(d * d) * (unsigned long long)P.ns;
	}
	for (int k = 0; k < P.nll; k++) {
		const int v = P.L->tails[0][k][P.lane];
		if (v >= v1 && v <= v2) {
			const long long d = v - P.lo;
			cnt++;
			s += d;
			ss += (unsigned long long)(d * d);
		}
	}
	for (int k = 0; k < P.nhl; k++) {
		const int v = P.L->tails[1][k][P.lane];
		if (v >= v1 && v <= v2) {
			const long long d = v - P.lo;
			cnt++;
			s += d;
			ss += (unsigned long long)(d * d);
		}
	}
	int b1 = v1 - P.lo, b2 = v2 - P.lo;
	if (b1 < 0)
		b1 = 0;
	if (b2 > SGH_BINS - 1)
		b2 = SGH_BINS - 1;
	if (b1 > b2)
		return;
	uint32_t c32 = 0, s32 = 0, ss32 = 0;
	for (int j = b1 >> 2; j <= (b2 >> 2); j++) {
		uint32_t d = P.L->hist[j][P.lane];
		const int first = 4 * j, last = 4 * j + 3;
		if (first < b1)
			d &= 0xFFFFFFFFu << (8 * (b1 - first));
		if (last > b2)
			d &= 0xFFFFFFFFu >> (8 * (last - b2));
		const uint32_t bs = __builtin_amdgcn_sad_u8(d, 0u, 0u);
		const uint32_t d1 = __builtin_amdgcn_udot4(d, 0x03020100u, 0u, false);
		const uint32_t d2 = __builtin_amdgcn_udot4(d, 0x09040100u, 0u, false);
		const uint32_t jj = (uint32_t)j;
		c32 += bs;
		s32 += 4u * jj * bs + d1;
		ss32 += 16u * jj * jj * bs + 8u * jj * d1 + d2;
	}
	cnt += (int)c32;
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
 * sorted kernel) */
__device__ int sgh_sigma(const SghPix &P, int N, double sl, double sh, long long S, unsigned long long SS,
		uint16_t *value, uint32_t *rlo_out, uint32_t *rhi_out) {
	int A = 0, B = 65535, n = N, r = 0, nrem;
	uint32_t rlo = 0, rhi = 0;
	do {
		const long long num = (long long)n * (long long)SS - S * S;
		const bool exact0 = (num == 0);
		const double sigma = num <= 0 ? 0.0 : sqrt((double)num / ((double)n * (double)(n - 1)));
		const int below = sgh_cnt_le(P, A - 1);
		const int g1 = below + (n - 1) / 2, g2 = below + n / 2;
		const int m1 = sgh_value_at(P, g1);
		const int m2 = (g2 == g1) ? m1 : sgh_value_at(P, g2);
		if (m1 < 0 || m2 < 0)
			return 1;
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
		if (!exact0) {
			int amb1 = sgh_floor_clamp(blo + tol);
			if (amb1 > B)
				amb1 = B;
			if (a <= amb1 && sgh_cnt_le(P, amb1) - sgh_cnt_le(P, a - 1) > 0)
				return 1;
			int amb0 = sgh_ceil_clamp(bhi - tol);
			if (amb0 < A)
				amb0 = A;
			if (amb0 <= bt && sgh_cnt_le(P, bt) - sgh_cnt_le(P, amb0 - 1) > 0)
				return 1;
		}
		int L = 0, H = 0;
		if (a > A)
			L = sgh_cnt_le(P, a - 1) - below;
		if (bt < B)
			H = sgh_cnt_le(P, B) - sgh_cnt_le(P, bt);
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
			int c;
			long long s;
			unsigned long long ss;
			sgh_range_moments(P, A, a - 1, c, s, ss);
			S -= s;
			SS -= ss;
			A = a;
		}
		if (H) {
			int c;
			long long s;
			unsigned long long ss;
			sgh_range_moments(P, bt + 1, B, c, s, ss);
			S -= s;
			SS -= ss;
			B = bt;
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

/* median of 16 values (the 9th smallest), bitonic network */
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
	return v[SGH_CENTER / 2];
}

__device__ __forceinline__ void sgh_add(SghLds &L, int lane, int lo, uint32_t v, uint32_t &nb,
		long long &ts, unsigned long long &tq) {
	const uint32_t b = v - (uint32_t)lo;
	if (b < SGH_BINS) {
		atomicAdd(&L.hist[b >> 2][lane], 1u << ((b & 3) * 8));
		nb++;
	} else {
		if (v == 0) {
			atomicAdd(&L.nzero[lane], 1u);
		} else if (v == 65535) {
			atomicAdd(&L.nsat[lane], 1u);
		} else {
			const int side = (int)v < lo ? 0 : 1;
			const uint32_t slot = atomicAdd(&L.ntail[side][lane], 1u);
			if (slot < SGH_T)
				L.tails[side][slot][lane] = (uint16_t)v;
		}
		const long long d = (long long)v - lo;
		ts += d;
		tq += (unsigned long long)(d * d);
	}
}

/* sample of frame f at (c, R, x) without normalisation (NO_NORM fast path): the y
 * shifted band read leaves zero rows, the x shift writes 0 (:1550-1577, :1628-1632).
 * f and sh (packed shift (shiftx & 0xffff) | shifty << 16) are wave-uniform: the row
 * address is scalar, the column offset per lane; out-of-frame samples load a valid
 * address and are masked to 0 (no divergent branch, so the loads stay in flight). */
__device__ __forceinline__ uint32_t sgh_load(const SgStackParams &p, const uint16_t *plane0, int f, int sh,
		int R, int x) {
	const int sx = (int)(int16_t)(sh & 0xFFFF);
	const int sy = sh >> 16;
	const int sr = R - sy;
	const bool rowok = (unsigned)sr < (unsigned)p.H;
	const uint16_t *rowp = plane0 + (int64_t)f * p.frame_stride + (int64_t)sr * p.W;
	const int sc = x - sx;
	const bool ok = rowok && (unsigned)sc < (unsigned)p.W;
	/* invalid samples read a zero page instead of being masked after the load */
	const uint16_t *a = ok ? rowp + sc : p.zeros + (threadIdx.x & 63);
	return *a;
}

__device__ __forceinline__ int sgh_shift(const SgStackParams &p, int f) {
	return p.use_shift ? __builtin_amdgcn_readfirstlane(p.shiftxy[f]) : 0;
}

/* packed shifts of 16 consecutive frames f0..f0+15 (f0 % 16 == 0; the table is padded
 * to a multiple of 16 entries and 64-byte aligned): 4 scalar dwordx4 loads */
__device__ __forceinline__ void sgh_shift16(const SgStackParams &p, int f0, int (&sh)[16]) {
	if (!p.use_shift) {
#pragma unroll
		for (int m = 0; m < 16; m++)
			sh[m] = 0;
		return;
	}
	const int4 *q = (const int4 *)(p.shiftxy + f0);
#pragma unroll
	for (int i = 0; i < 4; i++) {
		const int4 t = q[i];
		sh[4 * i] = __builtin_amdgcn_readfirstlane(t.x);
		sh[4 * i + 1] = __builtin_amdgcn_readfirstlane(t.y);
		sh[4 * i + 2] = __builtin_amdgcn_readfirstlane(t.z);
		sh[4 * i + 3] = __builtin_amdgcn_readfirstlane(t.w);
	}
}

__global__ void __launch_bounds__(64 * SGH_WAVES)
k_stack_hist(SgStackParams p, unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list) {
	__shared__ SghLds L;
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int ntx = (p.W + SG_TILE_W - 1) / SG_TILE_W;
	const int nrows = p.row_end - p.row_begin;
	int bid = blockIdx.x;
	const int xt = bid % ntx;
	bid /= ntx;
	const int R = p.row_begin + (bid % nrows);
	const int c = bid / nrows;
	const int x = xt * SG_TILE_W + lane;
	const int N = p.N;
	const uint16_t *plane0 = p.frames + (int64_t)c * p.plane_stride;

	/* zero the histograms and counters */
	for (int i = tid; i < SGH_DW * 64; i += 64 * SGH_WAVES)
		(&L.hist[0][0])[i] = 0;
	if (tid < 64) {
		L.ntail[0][tid] = 0;
		L.ntail[1][tid] = 0;
		L.nband[tid] = 0;
		L.nzero[tid] = 0;
		L.nsat[tid] = 0;
		L.tsum[tid] = 0;
		L.tsq[tid] = 0;
	}
	/* centre: median of the first 16 samples (every wave computes it identically) */
	uint32_t v16[SGH_CENTER];
#pragma unroll
	for (int k = 0; k < SGH_CENTER; k++)
		v16[k] = sgh_load(p, plane0, k, sgh_shift(p, k), R, x);
	int lo = (int)sgh_median16(v16) - SGH_BINS / 2;
	if (lo < 0)
		lo = 0;
	if (lo > 65536 - SGH_BINS)
		lo = 65536 - SGH_BINS;
	__syncthreads();

	uint32_t nb = 0;
	long long ts = 0;
	unsigned long long tq = 0;
	/* frames in chunks of 64: wave w bins frames [g0 + 16w, g0 + 16w + 16); the next
	 * chunk's 16 loads are issued before the current 16 samples are binned.  Frames
	 * 0..15 are wave 0's first block (already loaded for the centre). */
	constexpr int M = 16;
	const int wave_u = __builtin_amdgcn_readfirstlane(wave);
	auto load16 = [&](int f0, uint32_t(&dst)[M]) {
		int sh[M];
		sgh_shift16(p, f0, sh);
#pragma unroll
		for (int m = 0; m < M; m++) {
			const int f = f0 + m < N ? f0 + m : N - 1;
			dst[m] = sgh_load(p, plane0, f, sh[m], R, x);
		}
	};
	auto add16 = [&](int f0, const uint32_t(&src)[M]) {
#pragma unroll
		for (int m = 0; m < M; m++)
			if (f0 + m < N)
				sgh_add(L, lane, lo, src[m], nb, ts, tq);
	};
	/* two named buffers: the loads of block k+1 are in flight while block k is binned */
	uint32_t bufA[M], bufB[M];
	int fb = M * wave_u;
	if (fb == 0) {
#pragma unroll
		for (int m = 0; m < M; m++)
			bufA[m] = v16[m];
	} else if (fb < N) {
		load16(fb, bufA);
	}
	/* the prefetch is unconditional (the last block re-loads itself) so no register
	 * merge forces the compiler to wait for it before binning */
	while (fb < N) {
		load16(fb + 64 < N ? fb + 64 : fb, bufB);
		add16(fb, bufA);
		fb += 64;
		if (fb >= N)
			break;
		load16(fb + 64 < N ? fb + 64 : fb, bufA);
		add16(fb, bufB);
		fb += 64;
	}
	atomicAdd(&L.nband[lane], nb);
	if (ts)
		atomicAdd(&L.tsum[lane], (unsigned long long)ts);
	if (tq)
		atomicAdd(&L.tsq[lane], tq);
	__syncthreads();
	if (wave != 0)
		return;

	/* wave 0: prefix counts + band moments (relative to lo) */
	uint32_t cum = 0, s32 = 0, ss32 = 0;
	for (int j = 0; j < SGH_DW; j++) {
		const uint32_t d = L.hist[j][lane];
		const uint32_t bs = __builtin_amdgcn_sad_u8(d, 0u, 0u);
		const uint32_t d1 = __builtin_amdgcn_udot4(d, 0x03020100u, 0u, false);
		const uint32_t d2 = __builtin_amdgcn_udot4(d, 0x09040100u, 0u, false);
		const uint32_t jj = (uint32_t)j;
		s32 += 4u * jj * bs + d1;
		ss32 += 16u * jj * jj * bs + 8u * jj * d1 + d2;
		cum += bs;
		L.cumdw[j][lane] = (uint16_t)cum;
	}
	SghPix P;
	P.lo = lo;
	P.nll = (int)L.ntail[0][lane];
	P.nhl = (int)L.ntail[1][lane];
	P.nz = (int)L.nzero[lane];
	P.ns = (int)L.nsat[lane];
	P.nlo = P.nll + P.nz;
	P.nhi = P.nhl + P.ns;
	P.nb = (int)L.nband[lane];
	P.lane = lane;
	P.L = &L;
	int cls = SG_CLS_OK;
	uint16_t value = 0;
	uint32_t rlo = 0, rhi = 0;
	if (x < p.W) {
		if ((int)cum != P.nb || P.nll > SGH_T || P.nhl > SGH_T)
			cls = 1;	/* u8 bin overflow or tail overflow */
		else
			cls = sgh_sigma(P, N, p.sig0, p.sig1, (long long)s32 + (long long)L.tsum[lane],
					(unsigned long long)ss32 + L.tsq[lane], &value, &rlo, &rhi);
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
