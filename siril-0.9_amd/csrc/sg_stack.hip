/*
 * sg_stack.hip - gfx950 stacking kernels for the Siril 0.9 hot path.
 *
 * k_stack_sorted<NREG>  : median (stacking.c:362-816) and mean-with-rejection for
 *                         PERCENTILE / SIGMA / WINSORIZED (stacking.c:1189-1858).
 *   1. stage a 64-pixel x N-frame tile of one row into LDS (shift + zero fill +
 *      normalisation fused into the gather, :1535-1654);
 *   2. each wave sorts two pixel columns at once: the N samples (padded to 64*NREG
 *      with 65535) live in NREG packed-u16 VGPRs per lane and go through a bitonic
 *      network (v_pk_min_u16 / v_pk_max_u16 inside a lane, __shfl_xor across lanes);
 *      the sorted columns are written back in place;
 *   3. one lane per pixel runs the reference's iteration on the sorted column with
 *      exact integer moments (S, SS) instead of GSL's long-double recurrences.  Every
 *      threshold comparison is made against a rounding band; a pixel whose decision
 *      falls inside the band, or whose loop hits the reference's early `break`
 *      (N - r <= 4, :1684) before the last sample, is queued for the literal path.
 * k_stack_literal       : the queued pixels, one thread each, replaying the reference
 *                         loop literally (frame order, GSL sd via soft x87 fp80,
 *                         stale rejected[] state carried between pixels in the
 *                         reference's OpenMP thread order for first-pass breaks).
 * k_stack_reduce        : SUM (:196-355), MAX (:824-972), MIN (:979-1128) and MEAN
 *                         with NO_REJEC: streaming per-pixel reductions.
 */
#include "sg_common.hpp"
#include "sg_f80.h"

typedef unsigned short sg_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) {
	sg_u16x2 x = __builtin_bit_cast(sg_u16x2, a), y = __builtin_bit_cast(sg_u16x2, b);
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b) {
	sg_u16x2 x = __builtin_bit_cast(sg_u16x2, a), y = __builtin_bit_cast(sg_u16x2, b);
	return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

/* ascending bitonic sort of 64*NREG packed pairs; element e = lane*NREG + r */
template <int NREG>
__device__ __forceinline__ void bitonic_sort_packed(uint32_t (&v)[NREG], int lane) {
	constexpr int NPAD = 64 * NREG;
#pragma unroll
	for (int k = 2; k <= NPAD; k <<= 1) {
		/* first stage of each merge: compare e with e ^ (k-1) (mirror), all ascending */
		if (k <= NREG) {
#pragma unroll
			for (int r = 0; r < NREG; r++) {
				const int q = r ^ (k - 1);
				if (q > r) {
					uint32_t a = v[r], b = v[q];
					v[r] = pk_min(a, b);
					v[q] = pk_max(a, b);
				}
			}
		} else {
			const int m = k / NREG - 1;
			const bool lower = (lane & (k / (2 * NREG))) == 0;
			uint32_t t[NREG];
#pragma unroll
			for (int r = 0; r < NREG; r++)
				t[r] = (uint32_t)__shfl_xor((int)v[NREG - 1 - r], m, 64);
#pragma unroll
			for (int r = 0; r < NREG; r++)
				v[r] = lower ? pk_min(v[r], t[r]) : pk_max(v[r], t[r]);
		}
		/* half cleaners */
#pragma unroll
		for (int j = k >> 2; j > 0; j >>= 1) {
			if (j < NREG) {
#pragma unroll
				for (int r = 0; r < NREG; r++) {
					const int q = r ^ j;
					if (q > r) {
						uint32_t a = v[r], b = v[q];
						v[r] = pk_min(a, b);
						v[q] = pk_max(a, b);
					}
				}
			} else {
				const int m = j / NREG;
				const bool lower = (lane & m) == 0;
#pragma unroll
				for (int r = 0; r < NREG; r++) {
					uint32_t t = (uint32_t)__shfl_xor((int)v[r], m, 64);
					v[r] = lower ? pk_min(v[r], t) : pk_max(v[r], t);
				}
			}
		}
	}
}

/* ----------------------------------------------------------------------------------
 * exact-moment rejection on a sorted column
 * ---------------------------------------------------------------------------------- */
struct SgCol {
	const uint16_t *base;	/* LDS, element e at base[e * SG_STAGE_STRIDE] */
	__device__ __forceinline__ uint32_t operator()(int e) const { return base[e * SG_STAGE_STRIDE]; }
};

/* # of elements in [lo,hi) with value < thr */
__device__ __forceinline__ int col_count_lt(const SgCol &A, int lo, int hi, double thr) {
	int a = lo, b = hi;
	while (a < b) {
		int m = (a + b) >> 1;
		if ((double)A(m) < thr)
			a = m + 1;
		else
			b = m;
	}
	return a - lo;
}
/* # of elements in [lo,hi) with value <= thr */
__device__ __forceinline__ int col_count_le(const SgCol &A, int lo, int hi, double thr) {
	int a = lo, b = hi;
	while (a < b) {
		int m = (a + b) >> 1;
		if ((double)A(m) <= thr)
			a = m + 1;
		else
			b = m;
	}
	return a - lo;
}

/* gsl_stats_ushort_median_from_sorted_data on [lo, lo+n) */
__device__ __forceinline__ double col_median(const SgCol &A, int lo, int n) {
	const int lhs = (n - 1) / 2, rhs = n / 2;
	if (lhs == rhs)
		return (double)A(lo + lhs);
	return (double)(A(lo + lhs) + A(lo + rhs)) / 2.0;
}

/* sample sd from exact moments: sqrt(num / (n (n-1))), num = n*SS - S^2 */
__device__ __forceinline__ double exact_sd(int n, uint64_t S, uint64_t SS, bool *exact0) {
	int64_t num = (int64_t)n * (int64_t)SS - (int64_t)(S * S);
	*exact0 = (num == 0);
	if (num <= 0)
		return 0.0;
	return sqrt((double)num / ((double)n * (double)(n - 1)));
}

/* relative rounding band around every continuous threshold (relative to the median's
 * magnitude): GSL's long double mean recurrence is off by <= n 2^-64 |mean| ~ 3e-17 |mean|
 * for n = 512, which moves sd by about the same absolute amount; the double operations
 * after it add a few ulp (~1e-16).  1e-13 leaves a margin of ~1000 */
#define SG_BAND 1e-13

/* A/B diagnostics (SG_HIST_DBG=12): why pixels leave the sorted path */
__device__ unsigned int g_sg_why[32];
/* k_stack_replay timing (SG_HIST_DBG=12): max cycles of a pixel (total, gather, sort), pixels,
 * fp80 sd recomputations, passes (sums) */
__device__ unsigned long long g_sg_rprof[16];
/* the replay's per-pixel timing / counting (cycle counter reads, LDS bookkeeping) only in a
 * probe build (make EXTRA=-DSG_REPLAY_PROF, read by SG_HIST_DBG=12); production builds carry none */
#ifdef SG_REPLAY_PROF
#define SG_RPROF(...) __VA_ARGS__
#else
#define SG_RPROF(...)
#endif
#define SG_WHY(k) (atomicAdd(&g_sg_why[k], 1u), SG_CLS_LITERAL)

struct SgRejState {
	int lo, hi;
	uint64_t S, SS;
	int r, iter;
	uint32_t rlo, rhi;
};

/* one clipping pass (:1679-1693 / :1731-1747) with given sigma / median on the sorted
 * window.  Returns SG_CLS_*; *n = samples removed. */
__device__ int clip_pass(const SgCol &A, SgRejState &st, double sigma, bool exact0,
		double median, double sl, double sh, int N0, int *n_removed) {
	const int N = st.hi - st.lo;
	const double tl = sl * sigma, th = sh * sigma;
	const double blo = median - tl, bhi = median + th;
	int L, H;
	if (exact0) {
		L = col_count_lt(A, st.lo, st.hi, blo);
		H = N - col_count_le(A, st.lo, st.hi, bhi);
	} else {
		const double tol = SG_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
		const int L1 = col_count_lt(A, st.lo, st.hi, blo - tol);
		const int L2 = col_count_le(A, st.lo, st.hi, blo + tol);
		if (L1 != L2)
			return SG_WHY(1);
		const int H1 = N - col_count_le(A, st.lo, st.hi, bhi + tol);
		const int H2 = N - col_count_lt(A, st.lo, st.hi, bhi - tol);
		if (H1 != H2)
			return SG_WHY(2);
		L = L1;
		H = H1;
	}
	if (L + H > N)
		return SG_WHY(3);	/* negative sigma factors: else-if order matters */
	/* where does `if (N - r <= 4) break;` fire?  r counts rejections cumulatively */
	const int need = N - 4 - st.r;
	int fb = -1;
	if (need <= 0)
		fb = 0;
	else if (L >= need)
		fb = need - 1;
	else if (L + H >= need)
		fb = (N - H) + (need - L) - 1;
	if (fb >= 0 && fb < N - 1) {
		/* entries after fb keep stale values */
		if (st.iter == 1) {
			if (N0 > 4)
				return (atomicAdd(&g_sg_why[20], 1u), SG_CLS_CHAIN);	/* stale values of the previous pixel */
			/* N0 <= 4: only entry 0 is ever written, the rest stay calloc zero (:1497) */
			const int low0 = (L >= 1);
			const int high0 = (!low0) && (H == N);
			if (low0)
				st.rlo++;
			if (high0)
				st.rhi++;
			const int n = low0 || high0;
			if (n) {
				const uint32_t v = A(st.lo);
				st.S -= v;
				st.SS -= (uint64_t)v * v;
				st.lo++;
			}
			st.r += n;
			*n_removed = n;
			return SG_CLS_OK;
		}
		return SG_WHY(4);	/* stale values of this pixel's previous pass */
	}
	st.rlo += L;
	st.rhi += H;
	for (int i = 0; i < L; i++) {
		const uint32_t v = A(st.lo + i);
		st.S -= v;
		st.SS -= (uint64_t)v * v;
	}
	for (int i = 0; i < H; i++) {
		const uint32_t v = A(st.hi - 1 - i);
		st.S -= v;
		st.SS -= (uint64_t)v * v;
	}
	st.lo += L;
	st.hi -= H;
	st.r += L + H;
	*n_removed = L + H;
	return SG_CLS_OK;
}

__device__ int reject_sigma(const SgCol &A, SgRejState &st, double sl, double sh, int N0) {
	int n;
	do {
		st.iter++;
		const int N = st.hi - st.lo;
		bool e0;
		const double sigma = exact_sd(N, st.S, st.SS, &e0);
		const double median = col_median(A, st.lo, N);
		const int rc = clip_pass(A, st, sigma, e0, median, sl, sh, N0, &n);
		if (rc != SG_CLS_OK)
			return rc;
	} while (n > 0 && (st.hi - st.lo) > 3);
	return SG_CLS_OK;
}

/* SIGMEDIAN (:1696-1709): a rejected sample is replaced by round_to_WORD(median) and N stays,
 * so the pixel's multiset is the sorted window A[lo, hi) of samples never replaced plus a few
 * groups of equal replacement values (one new group per pass at most, ascending by value).
 * st.S / st.SS hold the whole multiset's exact moments; sigma and the decisions take the SIGMA
 * path's rounding band, a decision inside it goes to the literal kernel. */
#define SG_SMG 4	/* replacement groups a pixel may collect before it goes to the literal kernel */
struct SgSmed {
	int ng;
	uint32_t gv[SG_SMG];
	int gc[SG_SMG];
};
/* # multiset elements < t (le: <= t) */
__device__ __forceinline__ int smed_count(const SgCol &A, const SgRejState &st, const SgSmed &g, double t, bool le) {
	int c = le ? col_count_le(A, st.lo, st.hi, t) : col_count_lt(A, st.lo, st.hi, t);
	for (int k = 0; k < g.ng; k++)
		c += (le ? (double)g.gv[k] <= t : (double)g.gv[k] < t) ? g.gc[k] : 0;
	return c;
}
/* the r-th smallest element (0-based) of the multiset */
__device__ __forceinline__ uint32_t smed_at(const SgCol &A, const SgRejState &st, const SgSmed &g, int r) {
	int before = 0;	/* group elements ranked before r */
	for (int k = 0; k < g.ng; k++) {
		const int start = col_count_lt(A, st.lo, st.hi, (double)g.gv[k]) + before;
		if (r < start)
			break;
		if (r < start + g.gc[k])
			return g.gv[k];
		before += g.gc[k];
	}
	return A(st.lo + r - before);
}
__device__ int reject_sigmedian(const SgCol &A, SgRejState &st, double sl, double sh, int N0) {
	SgSmed g;
	g.ng = 0;
	int n;
	do {
		/* the reference has no cap: a pass whose replacements hold the values they replace
		 * repeats forever (e.g. {0, 0, 1, 1} with sig[1] < 0.87: median 0.5, both 1s clipped and
		 * set to round_to_WORD(0.5) = 1); such a pixel, or one past 4096 passes, fails the call */
		if (++st.iter > 4096)
			return SG_CLS_NOTERM;
		bool e0;
		const double sigma = exact_sd(N0, st.S, st.SS, &e0);
		const int g1 = (N0 - 1) / 2, g2 = N0 / 2;
		const uint32_t m1 = smed_at(A, st, g, g1), m2 = g1 == g2 ? m1 : smed_at(A, st, g, g2);
		const double median = g1 == g2 ? (double)m1 : (double)(m1 + m2) / 2.0;
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		/* low: median - v > tl, else high: v - median > th (median - v is exact) */
		double tlo = blo, thi = bhi;
		if (!e0) {
			const double tol = SG_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
			if (smed_count(A, st, g, blo - tol, false) != smed_count(A, st, g, blo + tol, true))
				return SG_WHY(21);
			if (smed_count(A, st, g, bhi - tol, false) != smed_count(A, st, g, bhi + tol, true))
				return SG_WHY(22);
			tlo = blo - tol;	/* no element lies within tol of either threshold */
			thi = bhi + tol;
		}
		const int L = smed_count(A, st, g, tlo, false), H = N0 - smed_count(A, st, g, thi, true);
		if (L + H > N0)
			return SG_WHY(23);	/* negative sigma factors: the else-if order matters */
		n = L + H;
		st.rlo += (uint32_t)L;
		st.rhi += (uint32_t)H;
		if (!n)
			break;
		/* the window's rejected prefix and suffix, then the rejected groups */
		const int wl = col_count_lt(A, st.lo, st.hi, tlo);
		const int wh = (st.hi - st.lo) - col_count_le(A, st.lo, st.hi, thi);
		uint64_t rs = 0, rss = 0;	/* moments of the replaced samples */
		for (int i = 0; i < wl; i++) {
			const uint64_t v = A(st.lo + i);
			rs += v;
			rss += v * v;
		}
		for (int i = 0; i < wh; i++) {
			const uint64_t v = A(st.hi - 1 - i);
			rs += v;
			rss += v * v;
		}
		st.lo += wl;
		st.hi -= wh;
		int ng = 0;
		for (int k = 0; k < g.ng; k++) {
			const double v = (double)g.gv[k];
			if (v < tlo || v > thi) {
				const uint64_t u = g.gv[k];
				rs += u * (uint64_t)g.gc[k];
				rss += u * u * (uint64_t)g.gc[k];
			} else {
				g.gv[ng] = g.gv[k];
				g.gc[ng] = g.gc[k];
				ng++;
			}
		}
		g.ng = ng;
		/* the n replacements round_to_WORD(median), kept ascending */
		const uint32_t mw = sg_round_to_WORD(median);
		/* every replaced sample already equal to mw (equal sums and sums of squares): the next
		 * pass sees the same array */
		if (rs == (uint64_t)mw * n && rss == (uint64_t)mw * mw * n)
			return SG_CLS_NOTERM;
		st.S += (uint64_t)mw * (uint64_t)n - rs;
		st.SS += (uint64_t)mw * mw * (uint64_t)n - rss;
		int k = 0;
		while (k < g.ng && g.gv[k] < mw)
			k++;
		if (k < g.ng && g.gv[k] == mw) {
			g.gc[k] += n;
		} else {
			if (g.ng == SG_SMG)
				return SG_WHY(24);
			for (int j = g.ng; j > k; j--) {
				g.gv[j] = g.gv[j - 1];
				g.gc[j] = g.gc[j - 1];
			}
			g.gv[k] = mw;
			g.gc[k] = n;
			g.ng++;
		}
	} while (n > 0 && N0 > 3);
	return SG_CLS_OK;
}

/* gsl_fit_linear's x-only recurrences for x = 0 .. N - 1: m_x (the mean) and m_dx2 depend on N
 * alone, so they are tabulated once per call (tab[2 N], tab[2 N + 1]) with the same double
 * operations in the same order (GSL fit/linear.c, as k_stack_literal runs them) */
__global__ void __launch_bounds__(64)
k_linfit_tables(double *__restrict__ tab, int nmax) {
	const int n = blockIdx.x * 64 + threadIdx.x;
	if (n < 1 || n > nmax)
		return;
	double m_x = 0.0, m_dx2 = 0.0;
	for (int i = 0; i < n; i++)
		m_x += ((double)i - m_x) / (i + 1.0);
	for (int i = 0; i < n; i++) {
		const double dx = (double)i - m_x;
		m_dx2 += (dx * dx - m_dx2) / (i + 1.0);
	}
	tab[2 * n] = m_x;
	tab[2 * n + 1] = m_dx2;
}

/* the smallest double t with (t / sigma) > s (line_clipping's test, :1174-1181): the rounded
 * quotient is monotone in t for sigma > 0, so the test of every frame is one compare against this
 * threshold instead of a division.  Returns false (the caller divides) outside the tame range
 * where the search is known to end within a few ulps. */
__device__ __forceinline__ bool sg_div_gt_threshold(double sigma, double s, double &thr) {
	if (!(sigma > 1e-200 && sigma < 1e200) || !(fabs(s) < 1e100) || s != s)
		return false;
	double c = s * sigma;
	if (!(fabs(c) < 1e250))
		return false;
	int guard = 0;
	while ((c / sigma) > s) {	/* down to a t that fails */
		c = nextafter(c, -HUGE_VAL);
		if (++guard > 64)
			return false;
	}
	while (!((c / sigma) > s)) {	/* up to the first t that passes */
		c = nextafter(c, HUGE_VAL);
		if (++guard > 128)
			return false;
	}
	thr = c;
	return true;
}

/* LINEARFIT (:1750-1784) on the lane's sorted column in LDS (element e at col[e * SG_STAGE_STRIDE]),
 * bit-identical to the literal replay: gsl_fit_linear's y recurrences (m_y, m_dxdy) in double per
 * pixel, its x-only ones from the per-N table (tab), the mean absolute residual, line_clipping with
 * rejected[] by position (one bit per entry in LDS, rb[(j / 32) * 64], written a word at a time;
 * the entries after the `N - r <= 4` break keep this pixel's previous pass), its two divisions
 * replaced by thresholds (sg_div_gt_threshold), and the order-preserving removal as one compaction
 * (the reference's loop visits old index j = 0 .. N - 1 and drops the flagged ones, :1767-1773; a
 * sorted array stays sorted, so quicksort_s is the identity).  A first pass that breaks early
 * needs the previous pixel's stale entries and goes to the literal kernel. */
__device__ int reject_linearfit(uint16_t *col, uint32_t *rb, int N0, double sl, double sh, SgRejState &st,
		const double *__restrict__ tab) {
	auto at = [&](int e) -> uint32_t { return col[e * SG_STAGE_STRIDE]; };
	int N = N0, r = 0, n, pass = 0;
	do {
		const double m_x = tab[2 * N], m_dx2 = tab[2 * N + 1];
		double m_y = 0;
		for (int i = 0; i < N; i++)
			m_y += ((double)at(i) - m_y) / (i + 1.0);
		double m_dxdy = 0;
		for (int i = 0; i < N; i++) {
			const double dx = (double)i - m_x;
			const double dy = (double)at(i) - m_y;
			m_dxdy += (dx * dy - m_dxdy) / (i + 1.0);
		}
		const double a = m_dxdy / m_dx2;
		const double b = m_y - m_x * a;
		double sigma = 0.0;
		for (int f = 0; f < N; f++)
			sigma += (fabs((double)at(f) - (a * (double)f + b)));
		sigma /= (double)N;
		double tlo = 0.0, thi = 0.0;
		const bool fast = sg_div_gt_threshold(sigma, sl, tlo) && sg_div_gt_threshold(sigma, sh, thi);
		n = 0;
		int frame;
		uint32_t bits = 0;
		for (frame = 0; frame < N; frame++) {
			const double y = (double)at(frame), af = a * (double)frame;
			int v = 0;
			const double t1 = af + b - y, t2 = y - af - b;
			if (fast ? t1 >= tlo : (t1 / sigma) > sl) {
				st.rlo++;
				v = -1;
			} else if (fast ? t2 >= thi : (t2 / sigma) > sh) {
				st.rhi++;
				v = 1;
			}
			if (v != 0) {
				bits |= 1u << (frame & 31);
				r++;
			}
			if ((frame & 31) == 31) {
				rb[(frame >> 5) * 64] = bits;
				bits = 0;
			}
			if (N - r <= 4)
				break;
		}
		{	/* the word holding the last entry written: its entries above it keep their old bits */
			const int last = frame < N ? frame : N - 1;
			if ((last & 31) != 31) {
				const uint32_t m = (2u << (last & 31)) - 1u;
				uint32_t &w = rb[(last >> 5) * 64];
				w = (w & ~m) | (bits & m);
			}
		}
		if (pass++ == 0 && frame < N - 1)
			return SG_CLS_LITERAL;
		int w = 0;
		for (int j = 0; j < N; j++) {
			if ((rb[(j >> 5) * 64] >> (j & 31)) & 1u)
				n++;
			else
				col[(w++) * SG_STAGE_STRIDE] = col[j * SG_STAGE_STRIDE];
		}
		N -= n;
	} while (n > 0 && N > 3);
	uint64_t S = 0;
	for (int e = 0; e < N; e++)
		S += at(e);
	st.S = S;
	st.lo = 0;
	st.hi = N;
	return SG_CLS_OK;
}

/* element i of the Winsorized copy w = [vlo x Lw] ++ A[lo+Lw, hi-Hw) ++ [vhi x Hw] */
struct SgWins {
	int Lw, Hw;
	uint32_t vlo, vhi;
	uint64_t Sin, SSin;	/* moments of the inner (unclamped) part */
};

__device__ __forceinline__ uint32_t wins_at(const SgCol &A, const SgRejState &st, const SgWins &w, int i) {
	const int N = st.hi - st.lo;
	if (i < w.Lw)
		return w.vlo;
	if (i >= N - w.Hw)
		return w.vhi;
	return A(st.lo + i);
}

/* # of w elements < thr (w sorted) */
__device__ __forceinline__ int wins_count_lt(const SgCol &A, const SgRejState &st, const SgWins &w, double thr) {
	const int N = st.hi - st.lo;
	int c = 0;
	if (w.Lw && (double)w.vlo < thr)
		c += w.Lw;
	c += col_count_lt(A, st.lo + w.Lw, st.hi - w.Hw, thr);
	if (w.Hw && (double)w.vhi < thr)
		c += w.Hw;
	(void)N;
	return c;
}
__device__ __forceinline__ int wins_count_le(const SgCol &A, const SgRejState &st, const SgWins &w, double thr) {
	int c = 0;
	if (w.Lw && (double)w.vlo <= thr)
		c += w.Lw;
	c += col_count_le(A, st.lo + w.Lw, st.hi - w.Hw, thr);
	if (w.Hw && (double)w.vhi <= thr)
		c += w.Hw;
	return c;
}

/* round_to_WORD(m) decision is ambiguous if m sits within tol of 0, 65535 or a .5 */
__device__ __forceinline__ bool round_ambiguous(double m, double tol) {
	if (fabs(m) <= tol || fabs(m - 65535.0) <= tol)
		return true;
	if (m <= 0.0 || m > 65535.0)
		return false;
	const double t = m + 0.5;
	return fabs(t - rint(t)) <= tol;
}

__device__ int reject_winsorized(const SgCol &A, SgRejState &st, double sl, double sh, int N0) {
	int n;
	do {
		st.iter++;
		const int N = st.hi - st.lo;
		bool e0;
		double sigma = exact_sd(N, st.S, st.SS, &e0);
		double median = col_median(A, st.lo, N);
		SgWins w = {0, 0, 0, 0, st.S, st.SS};
		bool sig_e0 = e0;
		int guard = 0;
		for (;;) {
			if (++guard > 4096)
				return SG_WHY(5);
			const double m0 = median - 1.5 * sigma;
			const double m1 = median + 1.5 * sigma;
			const double tol = sig_e0 ? 0.0 : SG_BAND * (fabs(median) + 1.5 * sigma + 1.0);
			/* clamp: w < m0 -> round(m0); else w > m1 -> round(m1) */
			int clo = wins_count_lt(A, st, w, m0 - tol);
			if (!sig_e0 && clo != wins_count_le(A, st, w, m0 + tol))
				return SG_WHY(6);
			int chi = N - wins_count_le(A, st, w, m1 + tol);
			if (!sig_e0 && chi != N - wins_count_lt(A, st, w, m1 - tol))
				return SG_WHY(7);
			if (clo + chi > N)
				return SG_WHY(8);
			if (clo > 0) {
				if (round_ambiguous(m0, tol + 1e-9 * tol))
					return SG_WHY(9);
				if (clo < w.Lw || clo > N - w.Hw)
					return SG_WHY(10);
				for (int i = w.Lw; i < clo; i++) {
					const uint32_t v = A(st.lo + i);
					w.Sin -= v;
					w.SSin -= (uint64_t)v * v;
				}
				w.Lw = clo;
				w.vlo = sg_round_to_WORD(m0);
			}
			if (chi > 0) {
				if (round_ambiguous(m1, tol + 1e-9 * tol))
					return SG_WHY(11);
				if (chi < w.Hw || chi > N - w.Lw)
					return SG_WHY(12);
				for (int i = w.Hw; i < chi; i++) {
					const uint32_t v = A(st.hi - 1 - i);
					w.Sin -= v;
					w.SSin -= (uint64_t)v * v;
				}
				w.Hw = chi;
				w.vhi = sg_round_to_WORD(m1);
			}
			/* median and 1.134 * sd of w (w stays sorted: see DESIGN.md) */
			{
				const int lhs = (N - 1) / 2, rhs = N / 2;
				if (lhs == rhs)
					median = (double)wins_at(A, st, w, lhs);
				else
					median = (double)(wins_at(A, st, w, lhs) + wins_at(A, st, w, rhs)) / 2.0;
			}
			const uint64_t Sw = w.Sin + (uint64_t)w.vlo * w.Lw + (uint64_t)w.vhi * w.Hw;
			const uint64_t SSw = w.SSin + (uint64_t)w.vlo * w.vlo * w.Lw + (uint64_t)w.vhi * w.vhi * w.Hw;
			const double sigma0 = sigma;
			const bool e00 = sig_e0;
			bool we0;
			sigma = 1.134 * exact_sd(N, Sw, SSw, &we0);
			sig_e0 = we0;
			/* while ((fabs(sigma - sigma0) / sigma0) > 0.0005) */
			if (e00) {
				if (we0)
					break;	/* 0/0 = NaN: the loop exits */
				continue;	/* x/0 = inf > 0.0005 */
			}
			const double q = fabs(sigma - sigma0) / sigma0;
			if (fabs(q - 0.0005) <= 1e-9 * 0.0005 + SG_BAND * (1.0 + q))
				return SG_WHY(13);
			if (!(q > 0.0005))
				break;
		}
		const int rc = clip_pass(A, st, sigma, sig_e0, median, sl, sh, N0, &n);
		if (rc != SG_CLS_OK)
			return rc;
	} while (n > 0 && (st.hi - st.lo) > 3);
	return SG_CLS_OK;
}

/* PERCENTILE (:1660-1673, percentile_clipping :1130-1143): pure double arithmetic, the
 * same expressions are evaluated here, so no band is needed */
__device__ int reject_percentile(const SgCol &A, SgRejState &st, double plow, double phigh) {
	const int N = st.hi - st.lo;
	const double median = col_median(A, st.lo, N);
	/* low predicate is monotone decreasing in x for median >= 0 */
	int a = 0, b = N;
	while (a < b) {
		int m = (a + b) >> 1;
		if ((median - (double)A(st.lo + m)) / median > plow)
			a = m + 1;
		else
			b = m;
	}
	const int L = a;
	/* high predicate monotone increasing; evaluated only where low is false */
	a = L;
	b = N;
	while (a < b) {
		int m = (a + b) >> 1;
		if (((double)A(st.lo + m) - median) / median > phigh)
			b = m;
		else
			a = m + 1;
	}
	const int H = N - a;
	st.rlo += L;
	st.rhi += H;
	int keep_lo, keep_hi;
	if (L + H <= N - 1) {
		keep_lo = L;
		keep_hi = N - H;
	} else {	/* removals stop at N == 1: the last sample survives */
		keep_lo = N - 1;
		keep_hi = N;
	}
	for (int i = 0; i < keep_lo; i++) {
		const uint32_t v = A(st.lo + i);
		st.S -= v;
		st.SS -= (uint64_t)v * v;
	}
	for (int i = keep_hi; i < N; i++) {
		const uint32_t v = A(st.lo + i);
		st.S -= v;
		st.SS -= (uint64_t)v * v;
	}
	st.hi = st.lo + keep_hi;
	st.lo = st.lo + keep_lo;
	return SG_CLS_OK;
}

/* ----------------------------------------------------------------------------------
 * main sorted kernel
 * ---------------------------------------------------------------------------------- */
template <int NREG, bool LISTED>
__global__ void __launch_bounds__(SG_SORT_THREADS)
k_stack_sorted(SgStackParams p, const unsigned int *__restrict__ list, const unsigned int *__restrict__ list_count) {
	extern __shared__ __attribute__((aligned(16))) uint16_t stage[];
	__shared__ int slot_c[SG_TILE_W], slot_R[SG_TILE_W], slot_x[SG_TILE_W];
	uint32_t *stage32 = (uint32_t *)stage;
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const int N = p.N;
	/* LISTED: the redo / compact list, slots of 64 pixels dealt to the blocks in a grid-stride
	 * loop, so one fixed grid takes any list length the device produced (no host round trip);
	 * otherwise one tile of one image row per block */
	unsigned int count = 0;
	if (LISTED) {
		count = *list_count;
		if (p.cmp_src && count > p.cmp_cap)	/* the compact list: slots past the capacity went to the redo list */
			count = p.cmp_cap;
		if (!p.cmp_src && p.list_minn && count <= p.list_minn)
			return;	/* a short list: k_stack_replay takes it */
	}
	for (unsigned int vb = blockIdx.x;; vb += gridDim.x) {
	int c0 = 0;
	if (LISTED) {
		if (vb * SG_TILE_W >= count)
			break;
		if (tid < SG_TILE_W) {
			const unsigned int k = vb * SG_TILE_W + tid;
			if (k < count) {
				const unsigned int pix = list[k];
				const int xx = (int)(pix % (unsigned)p.W);
				const unsigned int cr = pix / (unsigned)p.W;
				slot_x[tid] = xx;
				slot_R[tid] = (int)(cr % (unsigned)p.H);
				slot_c[tid] = (int)(cr / (unsigned)p.H);
			} else {
				slot_x[tid] = -1;
				slot_R[tid] = 0;
				slot_c[tid] = 0;
			}
		}
	} else {
		const int ntx = (p.W + SG_TILE_W - 1) / SG_TILE_W;
		const int nrows = p.row_end - p.row_begin;
		int b = (int)vb;
		const int xt = b % ntx;
		b /= ntx;
		const int R = p.row_begin + (b % nrows);
		c0 = b / nrows;
		if (tid < SG_TILE_W) {
			const int xx = xt * SG_TILE_W + tid;
			slot_x[tid] = xx < p.W ? xx : -1;
			slot_R[tid] = R;
			slot_c[tid] = c0;
		}
	}
	__syncthreads();

	if (LISTED && p.cmp_src) {
		/* the compact redo list (sg_stack_hist.hip sgh_compact): slot k's sorted column is
		 * cmp_src[k][0 .. N), read by a wave per slot with coalesced loads; no gather, no sort */
		const unsigned int k0 = vb * SG_TILE_W;
		for (int sl = wave; sl < SG_TILE_W; sl += SG_SORT_THREADS / 64) {
			if (slot_x[sl] < 0)
				continue;
			const uint16_t *col = p.cmp_src + (size_t)(k0 + sl) * (size_t)N;
			for (int e = lane; e < N; e += 64)
				stage[e * SG_STAGE_STRIDE + sl] = col[e];
		}
		__syncthreads();
	} else {
		/* 1. stage the tile: frame f, slot -> stage[f][slot].  Lane = slot (its pixel fixed), wave w
		 * takes frames w, w + 4, ...: a frame's shift and normalisation coefficients are wave-uniform
		 * (scalar loads), where the flat idx loop loaded them per sample (the redo lists of
		 * normalised stacks, ~200 k pixels, spent most of their time here) */
		{
			const int xx = slot_x[lane], cc = slot_c[lane], RR = slot_R[lane];
			constexpr int NW = SG_SORT_THREADS / 64, NB = 8;
			const uint16_t *plane = p.frames + (int64_t)cc * p.plane_stride;
			/* NB frames per wave in flight: every lane loads from a clamped (always valid) address,
			 * the sample is then selected (sg_gather's rules: an x-shifted sample is 0 and not
			 * normalised, a y-shifted row reads 0 and is normalised) */
			for (int f0 = __builtin_amdgcn_readfirstlane(wave); f0 < N; f0 += NW * NB) {
				uint16_t raw[NB];
				bool xin[NB];
#pragma unroll
				for (int k = 0; k < NB; k++) {
					const int f = f0 + k * NW < N ? f0 + k * NW : N - 1;
					const int sx = p.use_shift ? p.shiftx[f] : 0, sy = p.use_shift ? p.shifty[f] : 0;
					const int sr = RR - sy, sc = xx - sx;
					const bool yin = (unsigned)sr < (unsigned)p.H;
					xin[k] = xx >= 0 && (unsigned)sc < (unsigned)p.W;
					const int r = yin ? sr : 0, c = xin[k] ? sc : 0;
					const uint16_t v = plane[(int64_t)f * p.frame_stride + (int64_t)r * p.W + c];
					raw[k] = yin ? v : (uint16_t)0;
				}
#pragma unroll
				for (int k = 0; k < NB; k++) {
					const int f = f0 + k * NW;
					if (f < N)
						stage[f * SG_STAGE_STRIDE + lane] = xin[k] ? sg_normalize(p, f, raw[k]) : (uint16_t)0;
				}
			}
		}
		__syncthreads();

		/* 2. sort column pairs (2q, 2q+1) */
		for (int q = wave; q < SG_TILE_W / 2; q += SG_SORT_THREADS / 64) {
			uint32_t v[NREG];
#pragma unroll
			for (int r = 0; r < NREG; r++) {
				const int f = r * 64 + lane;
				v[r] = (f < N) ? stage32[f * (SG_STAGE_STRIDE / 2) + q] : 0xFFFFFFFFu;
			}
			bitonic_sort_packed<NREG>(v, lane);
			/* write back sorted element e = lane*NREG + r into row e (only e < N) */
#pragma unroll
			for (int r = 0; r < NREG; r++) {
				const int e = lane * NREG + r;
				if (e < N)
					stage32[e * (SG_STAGE_STRIDE / 2) + q] = v[r];
			}
		}
		__syncthreads();
	}

	/* 3. per-pixel rejection, one lane per pixel */
	const int sl = tid;
	uint32_t my_rlo = 0, my_rhi = 0;
	if (tid < SG_TILE_W) {
		const int x = slot_x[sl];
		const int c = slot_c[sl];
		const int R = slot_R[sl];
		if (x >= 0) {
			SgCol A = {stage + sl};
			uint16_t value = 0;
			int cls = SG_CLS_OK;
			if (p.method == 2) {	/* stack_median: implicit double -> WORD truncation */
				value = (uint16_t)col_median(A, 0, N);
			} else {
				SgRejState st;
				st.lo = 0;
				st.hi = N;
				st.r = 0;
				st.iter = 0;
				st.rlo = st.rhi = 0;
				uint64_t S = 0, SS = 0;
				for (int e = 0; e < N; e++) {
					const uint32_t a = A(e);
					S += a;
					SS += (uint64_t)a * a;
				}
				st.S = S;
				st.SS = SS;
				switch (p.rejection) {
				case 1:
					cls = reject_percentile(A, st, p.sig0, p.sig1);
					break;
				case 2:
					cls = reject_sigma(A, st, p.sig0, p.sig1, N);
					break;
				case 4:
					cls = reject_winsorized(A, st, p.sig0, p.sig1, N);
					break;
				case 3:
					cls = reject_sigmedian(A, st, p.sig0, p.sig1, N);
					if (cls == SG_CLS_NOTERM) {
						*p.loop_fault = 1u;
						cls = SG_CLS_OK;
					}
					break;
				case 5:
					cls = reject_linearfit(stage + sl, (uint32_t *)(stage + (size_t)N * SG_STAGE_STRIDE) + sl, N,
							p.sig0, p.sig1, st, p.linfit_tab);
					break;
				case 0:
					break;
				default:	/* SIGMEDIAN past its groups etc. never come here: unknown codes go literal */
					cls = SG_CLS_LITERAL;
				}
				if (cls == SG_CLS_OK) {
					/* SIGMEDIAN keeps all N samples (the replaced ones in st.S) */
					value = sg_round_to_WORD((double)st.S / (double)(p.rejection == 3 ? N : st.hi - st.lo));
					my_rlo = st.rlo;
					my_rhi = st.rhi;
				}
			}
			const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
			if (cls == SG_CLS_OK) {
				p.out[pix] = value;
			} else {
				sg_flag_set(p, pix, cls);
				const unsigned int slot = atomicAdd(p.flag_count, 1u);
				if (slot < p.flag_cap)
					p.flag_list[slot] = (unsigned int)pix;
			}
		}
		/* rejection counters */
		if (p.method != 2) {
			if (LISTED) {
				if (my_rlo | my_rhi) {
					unsigned long long *sh = p.rej + ((size_t)(sl % SG_REJ_SHARDS) * 6 + c * 2);
					atomicAdd(sh, (unsigned long long)my_rlo);
					atomicAdd(sh + 1, (unsigned long long)my_rhi);
				}
			} else {
				/* wave reduce, one sharded atomic per tile */
				unsigned long long lo = my_rlo, hi = my_rhi;
				for (int o = 32; o > 0; o >>= 1) {
					lo += __shfl_down(lo, o, 64);
					hi += __shfl_down(hi, o, 64);
				}
				if (tid == 0 && (lo | hi)) {
					unsigned long long *sh = p.rej + ((size_t)(vb % SG_REJ_SHARDS) * 6 + c0 * 2);
					atomicAdd(sh, lo);
					atomicAdd(sh + 1, hi);
				}
			}
		}
	}
	if (!LISTED)
		break;
	__syncthreads();	/* the slot tables and the stage are rewritten by the next list tile */
	}
}

template __global__ void k_stack_sorted<1, false>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<1, true>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<2, false>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<2, true>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<4, false>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<4, true>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<8, false>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<8, true>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<16, false>(SgStackParams, const unsigned int *, const unsigned int *);
template __global__ void k_stack_sorted<16, true>(SgStackParams, const unsigned int *, const unsigned int *);


/* ----------------------------------------------------------------------------------
 * streaming reductions: SUM / MAX / MIN / MEAN(NO_REJEC)
 * ---------------------------------------------------------------------------------- */
__global__ void __launch_bounds__(256)
k_stack_reduce(SgStackParams p) {
	const int x = blockIdx.x * 256 + threadIdx.x;
	const int R = p.row_begin + blockIdx.y;
	const int c = blockIdx.z;
	const bool live = x < p.W;
	const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
	const uint16_t *plane = p.frames + (int64_t)c * p.plane_stride;
	const int N = p.N;
	/* frames in batches of 16: every load of a batch is issued before any is used (an
	 * out-of-frame sample loads a valid dummy address and is masked), so each wave keeps 16
	 * row reads in flight */
	uint32_t acc = (p.method == 4) ? 65535u : 0u;
	/* the dummy address: a resident row of frame 0 (the base may be biased to a band) */
	const int64_t dummy = (int64_t)p.res_begin * p.W;
	for (int f0 = 0; f0 < N; f0 += 16) {
		uint32_t v[16], xin = 0, ok = 0;
#pragma unroll
		for (int m = 0; m < 16; m++) {
			const int f = f0 + m < N ? f0 + m : N - 1;
			const int sx = p.use_shift ? p.shiftx[f] : 0;
			const int sy = p.use_shift ? p.shifty[f] : 0;
			const int nx = x - sx, ny = R - sy;
			const bool xi = (unsigned)nx < (unsigned)p.W, yi = (unsigned)ny < (unsigned)p.H;
			bool ld = live && f0 + m < N && xi && yi;
			if (p.method != 1 && nx == 0 && ny == 0)
				ld = false;	/* `ii > 0`: source pixel 0 is never used (:307) */
			const int64_t off = ld ? (int64_t)f * p.frame_stride + (int64_t)ny * p.W + nx : dummy;
			v[m] = plane[off];
			v[m] = ld ? v[m] : 0u;
			xin |= (uint32_t)(xi && f0 + m < N) << m;
			ok |= (uint32_t)ld << m;
		}
#pragma unroll
		for (int m = 0; m < 16; m++) {
			if (p.method == 1) {	/* mean, NO_REJEC: the gather of sg_gather (shift, zero fill, norm) */
				if ((xin >> m) & 1u)
					acc += p.normalize ? sg_normalize(p, f0 + m, (uint16_t)v[m]) : v[m];
			} else if ((ok >> m) & 1u) {
				if (p.method == 0)
					acc += v[m];
				else if (p.method == 3)
					acc = v[m] > acc ? v[m] : acc;
				else
					acc = v[m] < acc ? v[m] : acc;
			}
		}
	}
	unsigned int blockmax = 0;
	if (live) {
		if (p.method == 1) {
			p.out[pix] = sg_round_to_WORD((double)acc / (double)N);
		} else if (p.method == 0) {
			p.sum_buf[pix] = acc;
			blockmax = acc;
		} else {
			p.out[pix] = (uint16_t)acc;
		}
	}
	if (p.method == 0) {
		for (int o = 32; o > 0; o >>= 1) {
			unsigned int t = (unsigned int)__shfl_down((int)blockmax, o, 64);
			blockmax = t > blockmax ? t : blockmax;
		}
		if ((threadIdx.x & 63) == 0 && blockmax)
			atomicMax(p.maxim, blockmax);
	}
}

/* The same reductions with a pixel PAIR per lane: one 4-byte buffer load per frame at the
 * shifted (2-byte aligned) address, 256 B per wave instruction instead of 128 B of u16
 * loads.  Each frame gets a buffer resource spanning its plane, so a row shifted out of the
 * frame reads 0 from the bounds check; at the left / right image edge, where one pixel of
 * the pair leaves the image, the load moves by one sample and the pair is fixed up.  Rows
 * and pixels are then masked exactly as k_stack_reduce does (xin / ok).  Host: plane bytes
 * < 2^31. */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sg_plane_rsrc(const uint16_t *base, uint32_t nrec) {
	return __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)nrec, 0x00020000);
}

/* the per-lane pixel-pair loop of the general path: any shift, the image edges, the masks of
 * every method */
__device__ __forceinline__ void sg_reduce_pairs(const SgStackParams &p, int x, int R, int c, uint32_t &acc_a,
		uint32_t &acc_b) {
	const bool live_a = x < p.W, live_b = x + 1 < p.W;
	const uint16_t *plane = p.frames + (int64_t)c * p.plane_stride;
	const uint32_t nrec = (uint32_t)p.H * (uint32_t)p.W * 2u;
	const int N = p.N;
	/* shifts of 64 frames at a time: one vector load per wave (lane l = frame f0 + l), read
	 * back per frame with readlane, so a batch's sample loads do not wait on 32 scalar loads */
	int vsx = 0, vsy = 0;
	const int lane = threadIdx.x & 63;
	for (int f0 = 0; f0 < N; f0 += 16) {
		if ((f0 & 63) == 0 && p.use_shift) {
			const int fl = f0 + lane < N ? f0 + lane : N - 1;
			vsx = p.shiftx[fl];
			vsy = p.shifty[fl];
		}
		uint32_t v[16];
		int nxs[16];
		bool yis[16], y0s[16];
#pragma unroll
		for (int m = 0; m < 16; m++) {
			const int f = f0 + m < N ? f0 + m : N - 1;
			const int sx = p.use_shift ? __builtin_amdgcn_readlane(vsx, (f0 & 63) + m) : 0;
			const int sy = p.use_shift ? __builtin_amdgcn_readlane(vsy, (f0 & 63) + m) : 0;
			const int nx = x - sx, ny = R - sy;
			nxs[m] = nx;
			yis[m] = (unsigned)ny < (unsigned)p.H && f0 + m < N;
			y0s[m] = ny == 0;
			/* the dword holding (nx, nx + 1), moved inside the row at the image edges */
			const int lx = nx < 0 ? nx + 1 : (nx + 1 >= p.W ? nx - 1 : nx);
			const uint32_t off = yis[m] ? (uint32_t)(ny * p.W + lx) * 2u : 0x80000000u;
			v[m] = __builtin_amdgcn_raw_buffer_load_b32(sg_plane_rsrc(plane + (int64_t)f * p.frame_stride, nrec),
					(int)off, 0, 0);
		}
#pragma unroll
		for (int m = 0; m < 16; m++) {
			const int nx = nxs[m];
			const bool yi = yis[m];
			/* samples of pixel a (source column nx) and b (nx + 1) */
			uint32_t a, b;
			if (nx < 0) {
				a = 0u;
				b = v[m] & 0xFFFFu;
			} else if (nx + 1 >= p.W) {
				a = v[m] >> 16;
				b = 0u;
			} else {
				a = v[m] & 0xFFFFu;
				b = v[m] >> 16;
			}
			const bool in = f0 + m < N;
			const bool xa = live_a && in && (unsigned)nx < (unsigned)p.W;
			const bool xb = live_b && in && (unsigned)(nx + 1) < (unsigned)p.W;
			if (p.method == 1) {	/* mean, NO_REJEC: y-shifted rows are zeros (normalised), x-shifted are skipped */
				if (xa)
					acc_a += p.normalize ? sg_normalize(p, f0 + m, (uint16_t)(yi ? a : 0u)) : (yi ? a : 0u);
				if (xb)
					acc_b += p.normalize ? sg_normalize(p, f0 + m, (uint16_t)(yi ? b : 0u)) : (yi ? b : 0u);
			} else {
				/* `ii > 0`: source pixel 0 is never used (:307) */
				const bool oka = xa && yi && !(nx == 0 && y0s[m]);
				const bool okb = xb && yi && !(nx + 1 == 0 && y0s[m]);
				if (p.method == 0) {
					acc_a += oka ? a : 0u;
					acc_b += okb ? b : 0u;
				} else if (p.method == 3) {
					acc_a = (oka && a > acc_a) ? a : acc_a;
					acc_b = (okb && b > acc_b) ? b : acc_b;
				} else {
					acc_a = (oka && a < acc_a) ? a : acc_a;
					acc_b = (okb && b < acc_b) ? b : acc_b;
				}
			}
		}
	}
}

/* the pair's results: MEAN round_to_WORD(sum / N) (:1790-1794), SUM raw sums + the maximum
 * (scaled by k_sum_finalize, :328-342), MAX / MIN the extremum */
__device__ __forceinline__ void sg_reduce_store(const SgStackParams &p, int x, int R, int c, uint32_t acc_a,
		uint32_t acc_b) {
	const bool live_a = x < p.W, live_b = x + 1 < p.W;
	unsigned int blockmax = 0;
	const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
	for (int k = 0; k < 2; k++) {
		if (!(k ? live_b : live_a))
			continue;
		const uint32_t acc = k ? acc_b : acc_a;
		if (p.method == 1) {
			p.out[pix + k] = sg_round_to_WORD((double)acc / (double)p.N);
		} else if (p.method == 0) {
			p.sum_buf[pix + k] = acc;
			blockmax = acc > blockmax ? acc : blockmax;
		} else {
			p.out[pix + k] = (uint16_t)acc;
		}
	}
	if (p.method == 0) {
		for (int o = 32; o > 0; o >>= 1) {
			unsigned int t = (unsigned int)__shfl_down((int)blockmax, o, 64);
			blockmax = t > blockmax ? t : blockmax;
		}
		if ((threadIdx.x & 63) == 0 && blockmax)
			atomicMax(p.maxim, blockmax);
	}
}

__global__ void __launch_bounds__(256)
k_stack_reduce2(SgStackParams p) {
	const int x = 2 * (blockIdx.x * 256 + threadIdx.x);
	const int R = p.row_begin + blockIdx.y;
	const int c = blockIdx.z;
	uint32_t acc_a = (p.method == 4) ? 65535u : 0u, acc_b = acc_a;
	sg_reduce_pairs(p, x, R, c, acc_a, acc_b);
	sg_reduce_store(p, x, R, c, acc_a, acc_b);
}

/*
 * k_stack_reduce3: the same reductions with the loads of k_stack_hist.  A workgroup of 4 waves
 * takes a 512-pixel segment of one row (a lane a pixel pair, a wave 128 pixels); workgroups are dealt XCD-aware
 * (each XCD gets contiguous whole rows, so the 128-B lines a shifted row segment straddles are
 * fetched once into that XCD's L2 and shared by the neighbouring segment).  In an interior
 * segment (no shifted column can leave the image, and none reaches source pixel 0) a frame's
 * shifted row segment start is one SGPR offset, (R W + x0) 2 - c1[f] with c1 = shifty W 2 +
 * 2 shiftx from the call's shift table (scalar loads), so a load costs no VALU; a row shifted
 * out of the frame reads 0 from the buffer bounds check (gfx950 checks voffset + soffset
 * unsigned, so a negative start is out of range too).  SUM and MEAN add 0 for such rows (the
 * reference's zero fill, normalised for MEAN), MAX ignores them, MIN skips them (a uniform
 * test of the frame's shifty).  Two 16-frame register buffers per lane.  Other segments take the
 * general per-lane loop (sg_reduce_pairs).  M: 0 SUM, 1 MEAN, 2 normalised MEAN, 3 MAX, 4 MIN.
 */
template <int M, int SEG>
__global__ void __launch_bounds__(256)
k_stack_reduce3(SgStackParams p, const int *__restrict__ tab, const int *__restrict__ shifty) {
	/* SEG 256-byte segments per wave (a wave 128 SEG pixels, a workgroup 512 SEG), MB = 16 / SEG
	 * frames per register buffer (the bytes in flight per wave stay).  The loads-only probe reads
	 * 512 x 4096^2 in 3.28 ms at 256 B, 3.00 at 512 B, 2.99 at 1 KiB per frame row
	 * (tools/bw_probe4.hip, profiles/r05c_probe5.log), but this kernel measured 3.52 / 3.59 / 4.33
	 * ms at SEG 1 / 2 / 4 (profiles/r05g: twice the edge waves on the general path, half the
	 * frames per buffer), so SEG = 1 is the default (SG_REDUCE_SEG, A/B) */
	constexpr int MB = 16 / SEG, PXW = 128 * SEG, PXG = 4 * PXW;
	const int nblk = (int)gridDim.x, xcd = (int)blockIdx.x & 7, q = nblk >> 3, rem = nblk & 7;
	const int vb = xcd * q + (xcd < rem ? xcd : rem) + ((int)blockIdx.x >> 3);
	const int bpr = (p.W + PXG - 1) / PXG;
	const int nrows = p.row_end - p.row_begin;
	const int xt = vb % bpr, rr = vb / bpr;
	const int R = p.row_begin + rr % nrows, c = rr / nrows;
	/* each wave its own segment: only the segments at the image edges take the general loop */
	const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	const int x0 = xt * PXG + PXW * wave;
	uint32_t acc_a[SEG], acc_b[SEG];
#pragma unroll
	for (int k = 0; k < SEG; k++)
		acc_a[k] = acc_b[k] = M == 4 ? 65535u : 0u;
	const bool interior = x0 > p.hist_maxsx && x0 + PXW + p.hist_maxsx <= p.W;
	if (!interior) {
#pragma unroll
		for (int k = 0; k < SEG; k++) {
			const int x = x0 + 128 * k + 2 * lane;
			sg_reduce_pairs(p, x, R, c, acc_a[k], acc_b[k]);
			sg_reduce_store(p, x, R, c, acc_a[k], acc_b[k]);
		}
		return;
	}
	const int N = p.N;
	const char *plane = (const char *)(p.frames + (int64_t)c * p.plane_stride);
	const uint32_t nrec = (uint32_t)p.H * (uint32_t)p.W * 2u;
	const int rowb = (R * p.W + x0) * 2;
	const int vofs = lane * 4;
	uint32_t mm[SEG];	/* MAX / MIN: both pixels packed */
#pragma unroll
	for (int k = 0; k < SEG; k++)
		mm[k] = M == 4 ? 0xFFFFFFFFu : 0u;
	const int64_t fstride2 = p.frame_stride * 2;
	int vsy = 0;	/* MIN: shifty of frames f0 + lane (64 at a time), read back with readlane */
	/* MB frames: their c1 (scalar loads; the table is zero padded to a multiple of 16 frames),
	 * then SEG loads per frame; frames past N read nothing */
	auto loadb = [&](int f0, uint32_t (&v)[MB][SEG]) {
		int c1[MB];
		const int *t = tab + __builtin_amdgcn_readfirstlane(f0);
#pragma unroll
		for (int i = 0; i < MB; i++)
			c1[i] = t[i];
		const char *fb = plane + (int64_t)f0 * fstride2;
#pragma unroll
		for (int m = 0; m < MB; m++) {
			const uint32_t n = f0 + m < N ? nrec : 0u;
#pragma unroll
			for (int k = 0; k < SEG; k++)
				v[m][k] = __builtin_amdgcn_raw_buffer_load_b32(
						sg_plane_rsrc((const uint16_t *)(fb + (int64_t)m * fstride2), n), vofs + 256 * k,
						rowb - c1[m], 0);
		}
	};
	auto accb = [&](int f0, const uint32_t (&v)[MB][SEG], bool full) {
		if (M == 4 && p.use_shift && (f0 & 63) == 0)
			vsy = shifty[f0 + lane < N ? f0 + lane : N - 1];
#pragma unroll
		for (int m = 0; m < MB; m++) {
			const int f = f0 + m;
			if (!full && f >= N)
				continue;
			int sy = 0;
			if (M == 4)
				sy = p.use_shift ? __builtin_amdgcn_readlane(vsy, (f0 & 63) + m) : 0;
#pragma unroll
			for (int k = 0; k < SEG; k++) {
				const uint32_t a = v[m][k] & 0xFFFFu, b = v[m][k] >> 16;
				if (M == 0 || M == 1) {	/* SUM; MEAN without normalisation: the sum (the divisor is N) */
					acc_a[k] += a;
					acc_b[k] += b;
				} else if (M == 2) {	/* normalised MEAN: the zero fill of a row shifted out is normalised too */
					acc_a[k] += sg_normalize(p, f, (uint16_t)a);
					acc_b[k] += sg_normalize(p, f, (uint16_t)b);
				} else if (M == 3) {
					mm[k] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(sg_u16x2, mm[k]),
							__builtin_bit_cast(sg_u16x2, v[m][k])));
				} else if ((unsigned)(R - sy) < (unsigned)p.H) {
					mm[k] = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(sg_u16x2, mm[k]),
							__builtin_bit_cast(sg_u16x2, v[m][k])));
				}
			}
		}
	};
	/* two register buffers: the next block's loads are issued before this block is accumulated;
	 * the steady loop is straight-line code with sched_barriers (the compiler otherwise
	 * interleaves the accumulation with the loads, and conditional loads make its vmcnt waits
	 * drain the block in flight) */
	uint32_t bufa[MB][SEG], bufb[MB][SEG];
	loadb(0, bufa);
	int f0 = 0;
	while (f0 + 3 * MB <= N) {
		loadb(f0 + MB, bufb);
		__builtin_amdgcn_sched_barrier(0);
		accb(f0, bufa, true);
		__builtin_amdgcn_sched_barrier(0);
		loadb(f0 + 2 * MB, bufa);
		__builtin_amdgcn_sched_barrier(0);
		accb(f0 + MB, bufb, true);
		__builtin_amdgcn_sched_barrier(0);
		f0 += 2 * MB;
	}
	/* the last one to three blocks, with bounds */
	if (f0 + MB < N)
		loadb(f0 + MB, bufb);
	accb(f0, bufa, f0 + MB <= N);
	if (f0 + MB < N) {
		if (f0 + 2 * MB < N)
			loadb(f0 + 2 * MB, bufa);
		accb(f0 + MB, bufb, f0 + 2 * MB <= N);
		if (f0 + 2 * MB < N)
			accb(f0 + 2 * MB, bufa, f0 + 3 * MB <= N);
	}
#pragma unroll
	for (int k = 0; k < SEG; k++) {
		if (M == 3 || M == 4) {
			acc_a[k] = mm[k] & 0xFFFFu;
			acc_b[k] = mm[k] >> 16;
		}
		sg_reduce_store(p, x0 + 128 * k + 2 * lane, R, c, acc_a[k], acc_b[k]);
	}
}
#define SG_R3(M)                                                                               \
	template __global__ void k_stack_reduce3<M, 1>(SgStackParams, const int *, const int *);   \
	template __global__ void k_stack_reduce3<M, 2>(SgStackParams, const int *, const int *);   \
	template __global__ void k_stack_reduce3<M, 4>(SgStackParams, const int *, const int *);
SG_R3(0)
SG_R3(1)
SG_R3(2)
SG_R3(3)
SG_R3(4)
#undef SG_R3

/* SUM finalisation: out = round_to_WORD(sum) or round_to_WORD(sum * 65535/maxim) (:328-342) */
__global__ void __launch_bounds__(256)
k_sum_finalize(SgStackParams p) {
	const int x = blockIdx.x * 256 + threadIdx.x;
	const int R = p.row_begin + blockIdx.y;
	const int c = blockIdx.z;
	if (x >= p.W)
		return;
	const int64_t pix = ((int64_t)c * p.H + R) * p.W + x;
	const unsigned int maxim = *p.maxim;
	const double ratio = (maxim > 65535u) ? 65535.0 / (double)maxim : 1.0;
	const uint32_t s = p.sum_buf[pix];
	p.out[pix] = (ratio == 1.0) ? sg_round_to_WORD((double)s) : sg_round_to_WORD((double)s * ratio);
}

/* ----------------------------------------------------------------------------------
 * literal path (one thread per queued pixel)
 * ---------------------------------------------------------------------------------- */
struct SgChainTables {
	const int *blk_of_row;		/* [C][H] top-down row -> block index */
	const int *blk_channel, *blk_start, *blk_end, *blk_first;	/* per block; first block of its thread chunk */
	int nblocks;
};

__device__ void shellsort_u16(uint16_t *a, int n) {
	const int gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
	for (int g = 0; g < 8; g++) {
		const int gap = gaps[g];
		for (int i = gap; i < n; i++) {
			uint16_t t = a[i];
			int j = i;
			for (; j >= gap && a[j - gap] > t; j -= gap)
				a[j] = a[j - gap];
			a[j] = t;
		}
	}
}

__device__ __forceinline__ double lit_median(const uint16_t *s, int n) {
	const int lhs = (n - 1) / 2, rhs = n / 2;
	if (n == 0)
		return 0.0;
	if (lhs == rhs)
		return (double)s[lhs];
	return (s[lhs] + s[rhs]) / 2.0;
}

__device__ __forceinline__ double lit_sd(const uint16_t *s, int n) {
	/* the double-double evaluation of the x87 recurrences (sg_f80.h; soft sg_f80 steps only near
	 * a rounding midpoint) */
	const double mean = f80dd_gsl_mean_u16(s, n);
	const double var = f80dd_gsl_variance_m_u16(s, n, mean);
	return sqrt(var * ((double)n / (double)(n - 1)));
}

__device__ __forceinline__ int lit_sigma_clip(uint16_t px, double sl, double sh, double sigma,
		double median, uint32_t *rej) {
	if (median - (double)px > sl * sigma) {
		rej[0]++;
		return -1;
	} else if ((double)px - median > sh * sigma) {
		rej[1]++;
		return 1;
	}
	return 0;
}

__device__ __forceinline__ void lit_remove(uint16_t *a, int i, int n) {
	for (int k = i; k < n - 1; k++)
		a[k] = a[k + 1];
}

/* the reference loop of :1656-1794 on `stack` (frame order) with the carried `rejected` */
__device__ uint16_t literal_pixel(uint16_t *stack, int8_t *rejected, uint16_t *wst, int nb_frames,
		int type, double sl, double sh, uint32_t *crej, int *first_break) {
	int N = nb_frames;
	double median, sigma;
	int n, j, r = 0, frame, pass = 0;
	*first_break = 0;
	switch (type) {
	case 1:
		shellsort_u16(stack, N);
		median = lit_median(stack, N);
		for (frame = 0; frame < N; frame++) {
			int v = 0;
			if ((median - (double)stack[frame]) / median > sl) {
				crej[0]++;
				v = -1;
			} else if (((double)stack[frame] - median) / median > sh) {
				crej[1]++;
				v = 1;
			}
			rejected[frame] = (int8_t)v;
		}
		for (frame = 0, j = 0; frame < N; frame++, j++) {
			if (rejected[j] != 0 && N > 1) {
				lit_remove(stack, frame, N);
				frame--;
				N--;
			}
		}
		break;
	case 2:
	case 4:
		do {
			sigma = lit_sd(stack, N);
			shellsort_u16(stack, N);
			median = lit_median(stack, N);
			if (type == 4) {
				double sigma0;
				for (int jj = 0; jj < N; jj++)
					wst[jj] = stack[jj];
				int guard = 0;
				do {
					const double m0 = median - 1.5 * sigma;
					const double m1 = median + 1.5 * sigma;
					for (int jj = 0; jj < N; jj++) {
						if (wst[jj] < m0)
							wst[jj] = sg_round_to_WORD(m0);
						else if (wst[jj] > m1)
							wst[jj] = sg_round_to_WORD(m1);
					}
					shellsort_u16(wst, N);
					median = lit_median(wst, N);
					sigma0 = sigma;
					sigma = 1.134 * lit_sd(wst, N);
				} while ((fabs(sigma - sigma0) / sigma0) > 0.0005 && ++guard < 100000);
			}
			n = 0;
			for (frame = 0; frame < N; frame++) {
				rejected[frame] = (int8_t)lit_sigma_clip(stack[frame], sl, sh, sigma, median, crej);
				if (rejected[frame])
					r++;
				if (N - r <= 4)
					break;
			}
			if (pass++ == 0 && frame < N - 1)
				*first_break = 1;
			for (frame = 0, j = 0; frame < N - n; frame++, j++) {
				if (rejected[j] != 0) {
					lit_remove(stack, frame, N - n);
					n++;
					frame--;
				}
			}
			N = N - n;
		} while (n > 0 && N > 3);
		break;
	case 3: {
		/* a pass whose replacements change nothing repeats forever in the reference (see
		 * reject_sigmedian): *first_break = 2 reports it, as does a pixel past 4096 passes */
		int guard = 0;
		do {
			sigma = lit_sd(stack, N);
			shellsort_u16(stack, N);
			median = lit_median(stack, N);
			n = 0;
			bool changed = false;
			for (frame = 0; frame < N; frame++) {
				if (lit_sigma_clip(stack[frame], sl, sh, sigma, median, crej)) {
					const uint16_t mw = sg_round_to_WORD(median);
					changed |= stack[frame] != mw;
					stack[frame] = mw;
					n++;
				}
			}
			if (n > 0 && N > 3 && (!changed || ++guard >= 4096)) {
				*first_break = 2;
				break;
			}
		} while (n > 0 && N > 3);
		break;
	}
	case 5:
		do {
			shellsort_u16(stack, N);
			/* gsl_fit_linear(x = 0..N-1, y = stack): b = intercept, a = slope */
			double m_x = 0, m_y = 0, m_dx2 = 0, m_dxdy = 0;
			for (int i = 0; i < N; i++) {
				m_x += ((double)i - m_x) / (i + 1.0);
				m_y += ((double)stack[i] - m_y) / (i + 1.0);
			}
			for (int i = 0; i < N; i++) {
				const double dx = (double)i - m_x;
				const double dy = (double)stack[i] - m_y;
				m_dx2 += (dx * dx - m_dx2) / (i + 1.0);
				m_dxdy += (dx * dy - m_dxdy) / (i + 1.0);
			}
			const double a = m_dxdy / m_dx2;
			const double b = m_y - m_x * a;
			sigma = 0.0;
			for (frame = 0; frame < N; frame++)
				sigma += (fabs((double)stack[frame] - (a * (double)frame + b)));
			sigma /= (double)N;
			n = 0;
			for (frame = 0; frame < N; frame++) {
				int v = 0;
				if (((a * (double)frame + b - (double)stack[frame]) / sigma) > sl) {
					crej[0]++;
					v = -1;
				} else if ((((double)stack[frame] - a * (double)frame - b) / sigma) > sh) {
					crej[1]++;
					v = 1;
				}
				rejected[frame] = (int8_t)v;
				if (v != 0)
					r++;
				if (N - r <= 4)
					break;
			}
			if (pass++ == 0 && frame < N - 1)
				*first_break = 1;
			for (frame = 0, j = 0; frame < N - n; frame++, j++) {
				if (rejected[j] != 0) {
					lit_remove(stack, frame, N - n);
					frame--;
					n++;
				}
			}
			N = N - n;
		} while (n > 0 && N > 3);
		break;
	default:
		break;
	}
	double sum = 0.0;
	for (frame = 0; frame < N; ++frame)
		sum += stack[frame];
	return sg_round_to_WORD(sum / (double)N);
}

/* predecessor / successor in the reference's per-OpenMP-thread pixel order:
 * blocks of the thread's static chunk in order, rows top-down, x ascending */
__device__ int64_t chain_pred(const SgStackParams &p, const SgChainTables &t, int64_t pix) {
	const int x = (int)(pix % p.W);
	const int64_t cr = pix / p.W;
	const int R = (int)(cr % p.H), c = (int)(cr / p.H);
	if (x > 0)
		return pix - 1;
	const int trow = p.H - 1 - R;
	const int b = t.blk_of_row[(int64_t)c * p.H + trow];
	if (trow > t.blk_start[b])
		return ((int64_t)c * p.H + (R + 1)) * p.W + (p.W - 1);
	if (b > t.blk_first[b]) {
		const int pb = b - 1;
		const int pR = p.H - 1 - t.blk_end[pb];
		return ((int64_t)t.blk_channel[pb] * p.H + pR) * p.W + (p.W - 1);
	}
	return -1;
}

__device__ int64_t chain_succ(const SgStackParams &p, const SgChainTables &t, int64_t pix) {
	const int x = (int)(pix % p.W);
	const int64_t cr = pix / p.W;
	const int R = (int)(cr % p.H), c = (int)(cr / p.H);
	if (x < p.W - 1)
		return pix + 1;
	const int trow = p.H - 1 - R;
	const int b = t.blk_of_row[(int64_t)c * p.H + trow];
	if (trow < t.blk_end[b])
		return ((int64_t)c * p.H + (R - 1)) * p.W;
	const int nb = b + 1;
	if (nb < t.nblocks && t.blk_first[nb] == t.blk_first[b]) {
		const int nR = p.H - 1 - t.blk_start[nb];
		return ((int64_t)t.blk_channel[nb] * p.H + nR) * p.W;
	}
	return -1;
}

__device__ __forceinline__ bool chain_in_band(const SgStackParams &p, int64_t pix) {
	const int R = (int)((pix / p.W) % p.H);
	return R >= p.row_begin && R < p.row_end;
}

/* every frame row pixel `pix` reads (R - shifty, clipped to the frame) is resident */
__device__ __forceinline__ bool chain_resident(const SgStackParams &p, int64_t pix) {
	const int R = (int)((pix / p.W) % p.H);
	const int lo = max(0, R - p.sy_max), hi = min(p.H - 1, R - p.sy_min);
	return lo > hi || (lo >= p.res_begin && hi < p.res_end);
}

__device__ __forceinline__ void gather_stack(const SgStackParams &p, int64_t pix, uint16_t *stack) {
	const int x = (int)(pix % p.W);
	const int64_t cr = pix / p.W;
	const int R = (int)(cr % p.H), c = (int)(cr / p.H);
	for (int f = 0; f < p.N; f++)
		stack[f] = sg_gather(p, f, c, R, x);
}

/* ----------------------------------------------------------------------------------
 * exact wave-per-pixel replay (SIGMA / WINSORIZED queued pixels)
 * ---------------------------------------------------------------------------------- */
/*
 * k_stack_replay: one wave per queued pixel replays the reference loop (:1674-1749)
 * literally in structure - the stack array in frame order, quicksort, the rejected[]
 * array by POSITION, the `if (N - r <= 4) break;` with the entries after the break keeping
 * this pixel's previous-pass values, the order-preserving removal - but with exact
 * integer moments instead of GSL's long double sums.  Every continuous decision gets the
 * same rounding band as the sorted path; a decision inside the band switches the pixel to
 * exact mode (GSL's sd in soft fp80 on lane 0 from then on, no band).  Only a pixel whose
 * FIRST pass breaks early (its stale entries belong to the previous pixel of the OpenMP
 * thread) stays queued for k_stack_literal.  This takes the early-break and near-tie
 * pixels (e.g. image-edge columns half filled by the shift zero fill under WINSORIZED) off
 * the one-thread fp80 path.  The stack is sorted once: after the first pass the removal keeps
 * it sorted, and quicksort_s of a sorted array is the identity; the Winsorized copy stays
 * sorted under clamping.
 */
#define SG_REPLAY_FASTN 512	/* SIGMA fast passes (replay_sigma_fast) up to this many frames */
#ifndef SG_REPLAY_WFAST
#define SG_REPLAY_WFAST 1	/* WINSORIZED passes on the same fast path (replay_winsor_inner) */
#endif
/* per-wave LDS of the replay, sized for up to NM frames: k_stack_replay<SG_REPLAY_FASTN> for
 * N <= 512 holds 10.6 KB per wave instead of 24.8 KB, so 7 two-wave workgroups fit a CU
 * instead of 3 (the replay is latency-bound: one wave per pixel) */
template <int NM>
struct SgReplayLdsT {
	uint16_t stack[NM];
	uint16_t w[NM];
	uint16_t wprev[NM];	/* w before the current clamp (exact-mode recomputation) */
	uint16_t orig[NM];	/* the first pass's stack in frame order */
	int8_t rej[NM];
	uint32_t p1[SG_REPLAY_FASTN + 1];	/* prefix sums of the sorted stack (SIGMA fast passes) */
	unsigned long long p2[SG_REPLAY_FASTN + 1];
	int nsd, npass, handover;	/* fp80 recomputations, passes, fast-path handovers (SG_HIST_DBG=12 timing) */
	unsigned long long t_sort, t_fast;
};

__device__ __forceinline__ int wave_excl_scan(int v, int lane) {
	int x = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const int t = __shfl_up(x, o, 64);
		if (lane >= o)
			x += t;
	}
	return x - v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

__device__ __forceinline__ int wave_or(int v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v |= __shfl_xor(v, o, 64);
	return v;
}

__device__ __forceinline__ void replay_moments(const uint16_t *a, int n, int lane, uint64_t &S, uint64_t &SS) {
	uint64_t s = 0, ss = 0;
	for (int j = lane; j < n; j += 64) {
		const uint64_t v = a[j];
		s += v;
		ss += v * v;
	}
	S = wave_sum_u64(s);
	SS = wave_sum_u64(ss);
}

/* ascending bitonic sort of a[0..n) (padded with 65535 up to a power of two; the pad lies
 * inside the array's capacity and is never read as data) */
__device__ void replay_sort(uint16_t *a, int n, int lane) {
	int P = 1;
	while (P < n)
		P <<= 1;
	for (int j = n + lane; j < P; j += 64)
		a[j] = 0xFFFF;
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	for (int k = 2; k <= P; k <<= 1)
		for (int j = k >> 1; j > 0; j >>= 1) {
			for (int i = lane; i < P; i += 64) {
				const int l = i ^ j;
				if (l > i) {
					const uint16_t x = a[i], y = a[l];
					const bool up = (i & k) == 0;
					if ((x > y) == up) {
						a[i] = y;
						a[l] = x;
					}
				}
			}
			__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		}
}

/* the same sort with the array in registers: element e = 64 k + lane in x[k]; partners 64 or
 * more apart are in the lane's own registers, closer ones one lane shuffle away, so a stage is
 * KM independent compare-exchanges instead of KM dependent LDS round trips (the LDS version
 * above dominated the replay of a 512-frame pixel).  The sorted array is unique for u16 keys,
 * so the result is the same array. */
template <int KM, int JR>
__device__ __forceinline__ void replay_cx_reg(uint32_t (&x)[KM], int kk, int lane) {
#pragma unroll
	for (int k = 0; k < KM; k++) {
		if ((k & JR) == 0 && (k | JR) < KM) {
			const bool up = ((64 * k + lane) & kk) == 0;
			const uint32_t u = x[k], v = x[k | JR];
			const uint32_t mn = u < v ? u : v, mx = u < v ? v : u;
			x[k] = up ? mn : mx;
			x[k | JR] = up ? mx : mn;
		}
	}
}
template <int KM>
__device__ __forceinline__ void replay_sort_reg(uint16_t *a, int n, int lane) {
	constexpr int P = 64 * KM;
	uint32_t x[KM];
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int e = 64 * k + lane;
		x[k] = e < n ? a[e] : 0xFFFFu;
	}
	/* the stage loops stay loops (the kernel runs once per call, its code cold in the
	 * instruction cache: a fully unrolled network is ~2 K instructions); only the per-register
	 * work of a stage is unrolled */
#pragma unroll 1
	for (int kk = 2; kk <= P; kk <<= 1) {
#pragma unroll 1
		for (int j = kk >> 1; j > 0; j >>= 1) {
			if (j >= 64) {
				if (j == 64)
					replay_cx_reg<KM, 1>(x, kk, lane);
				else if (j == 128)
					replay_cx_reg<KM, 2>(x, kk, lane);
				else if (j == 256)
					replay_cx_reg<KM, 4>(x, kk, lane);
				else if (j == 512)
					replay_cx_reg<KM, 8>(x, kk, lane);
				else
					replay_cx_reg<KM, 16>(x, kk, lane);
			} else {
				const bool lower = (lane & j) == 0;
#pragma unroll
				for (int k = 0; k < KM; k++) {
					const bool up = ((64 * k + lane) & kk) == 0;
					const uint32_t y = (uint32_t)__shfl_xor((int)x[k], j, 64);
					const uint32_t mn = x[k] < y ? x[k] : y, mx = x[k] < y ? y : x[k];
					x[k] = (lower == up) ? mn : mx;
				}
			}
		}
	}
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int e = 64 * k + lane;
		if (e < n)
			a[e] = (uint16_t)x[k];
	}
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ void replay_sort_any(uint16_t *a, int n, int lane) {
	if (n <= 512)	/* one instance: smaller stacks sort padded (less code to fetch) */
		replay_sort_reg<8>(a, n, lane);
	else
		replay_sort(a, n, lane);
}

__device__ __forceinline__ double replay_median(const uint16_t *a, int n) {
	const int lhs = (n - 1) / 2, rhs = n / 2;
	if (lhs == rhs)
		return (double)a[lhs];
	return (double)(a[lhs] + a[rhs]) / 2.0;
}

/* GSL's sd (long double recurrences in soft fp80) of a[0..n), computed on lane 0 and
 * broadcast: the reference's gsl_stats_sd, as lit_sd */
__device__ __forceinline__ double replay_gsl_sd(const uint16_t *a, int n, int lane) {
	double v = 0.0;
	if (lane == 0)
		v = lit_sd(a, n);
	return __shfl(v, 0, 64);
}
template <class LDS>
__device__ __forceinline__ double replay_gsl_sd(LDS &L, const uint16_t *a, int n, int lane) {
	SG_RPROF(if (lane == 0) L.nsd++;)
	return replay_gsl_sd(a, n, lane);
}

/* sg_gather of a pixel's N <= SG_REPLAY_FASTN samples with every load in flight at once: the
 * shifts of all 8 frames of a lane first, then all 8 samples (the plain loop waits for two
 * dependent loads per frame) */
__device__ __forceinline__ void replay_gather_batched(const SgStackParams &p, uint16_t *dst, int c, int R, int x,
		int lane) {
	constexpr int KM = SG_REPLAY_FASTN / 64;
	int sx[KM], sy[KM];
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int f = 64 * k + lane;
		sx[k] = sy[k] = 0;
		if (p.use_shift && f < p.N) {
			sx[k] = p.shiftx[f];
			sy[k] = p.shifty[f];
		}
	}
	uint16_t v[KM];
	bool colok[KM];
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int f = 64 * k + lane;
		const int sr = R - sy[k], sc = x - sx[k];
		colok[k] = (unsigned)sc < (unsigned)p.W;
		v[k] = 0;
		if (f < p.N && colok[k] && (unsigned)sr < (unsigned)p.H)
			v[k] = p.frames[(int64_t)f * p.frame_stride + (int64_t)c * p.plane_stride + (int64_t)sr * p.W + sc];
	}
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int f = 64 * k + lane;
		if (f < p.N)
			dst[f] = colok[k] ? sg_normalize(p, f, v[k]) : (uint16_t)0;
	}
}

__device__ __forceinline__ unsigned long long wave_excl_scan_u64(unsigned long long v, int lane) {
	unsigned long long x = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const unsigned long long t = __shfl_up(x, o, 64);
		if (lane >= o)
			x += t;
	}
	return x - v;
}

/* SIGMA passes on the sorted stack while no decision is ambiguous and no early break fires:
 * the stack is sorted, low clips are its smallest values and high clips its largest, so
 * without a break every pass trims a prefix and a suffix and the kept set stays the
 * contiguous range [lo, hi) of the sorted array.  Moments come from prefix sums formed once,
 * the median is two reads, the clip counts are ballots; decisions are the general loop's, in
 * the same double arithmetic with the same band.  rejected[] is written as the general loop
 * leaves it (this pass's decisions by position), so the loop can hand a pass it cannot decide
 * (returns 0: ambiguous, or an early break) to the general loop with the state it expects:
 * the range is compacted to the front and N, r, passes and counters carry over.
 * Returns 1 when the pixel is finished (value and counters set). */
/* WINSORIZED inner loop of one pass (:1710-1729 + Winsorized :1163-1168) on the sorted kept
 * range [lo, hi), mirroring replay_pixel's type-4 loop decision for decision: the clamped copy w
 * is kept as Lw copies of vlo, the range's own values [lo + Lw, hi - Hw), Hw copies of vhi (a
 * clamp either re-clamps all earlier copies of a side or none of them, so one value per side
 * suffices); its moments come from the prefix sums, its median from two positions, the
 * counts below m0 / above m1 from ballots.  Returns 0 where the general loop would recompute
 * a sigma the reference's way (ambiguous clamp or convergence decision) or give up (guard):
 * the pass then goes to the general loop.  On 1, median / sigma / e0 are the pass's
 * Winsorized values. */
template <class LDS>
__device__ int replay_winsor_inner(LDS &L, const uint32_t (&xs)[SG_REPLAY_FASTN / 64], int lo, int hi,
		int lane, double &median, double &sigma, bool &e0) {
	constexpr int KM = SG_REPLAY_FASTN / 64;
	const int n = hi - lo;
	int Lw = 0, Hw = 0;
	uint32_t vlo = 0, vhi = 0;
	bool sig_e0 = e0;
	auto w_at = [&](int k) -> double {	/* element k of the sorted w */
		return (double)(k < Lw ? vlo : (k >= n - Hw ? vhi : (uint32_t)L.stack[lo + k]));
	};
	for (int guard = 0;; guard++) {
		if (guard > 100000)
			return 0;
		const double m0 = median - 1.5 * sigma, m1 = median + 1.5 * sigma;
		const double tol = sig_e0 ? 0.0 : SG_BAND * (fabs(median) + 1.5 * sigma + 1.0);
		/* inner values below m0 / above m1, ambiguity over every element of w */
		int amb = 0, nlo = 0, nhi = 0;
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = 64 * k + lane;
			const bool in = e >= lo + Lw && e < hi - Hw;
			const double x = (double)xs[k];
			if (in && !sig_e0 && ((x >= m0 - tol && x <= m0 + tol) || (x >= m1 - tol && x <= m1 + tol)))
				amb = 1;
			nlo += (int)__popcll(__ballot(in && x < m0));
			nhi += (int)__popcll(__ballot(in && !(x < m0) && x > m1));
		}
		amb = __ballot(amb) != 0ull;	/* one instruction instead of six lane shuffles */
		const double xl = (double)vlo, xh = (double)vhi;
		if (Lw && !sig_e0 && ((xl >= m0 - tol && xl <= m0 + tol) || (xl >= m1 - tol && xl <= m1 + tol)))
			amb = 1;
		if (Hw && !sig_e0 && ((xh >= m0 - tol && xh <= m0 + tol) || (xh >= m1 - tol && xh <= m1 + tol)))
			amb = 1;
		const bool lo_c = Lw && xl < m0, hi_c = Hw && !(xh < m0) && xh > m1;
		const bool clamped_lo = nlo > 0 || lo_c, clamped_hi = nhi > 0 || hi_c;
		if (amb || (clamped_lo && round_ambiguous(m0, tol + 1e-9 * tol)) ||
				(clamped_hi && round_ambiguous(m1, tol + 1e-9 * tol)))
			return 0;
		/* the copies of a side either all move (their value is past the new bound) or stay */
		if (Lw && !lo_c && xl > m1)
			return 0;	/* (cannot happen: vlo < vhi; kept for safety) */
		if (Hw && !hi_c && xh < m0)
			return 0;
		const uint32_t nvlo = sg_round_to_WORD(m0), nvhi = sg_round_to_WORD(m1);
		if (clamped_lo) {
			if (Lw && !lo_c)
				return 0;	/* inner values below m0 while the old copies are not: w leaves this form */
			Lw += nlo;
			vlo = nvlo;
		}
		if (clamped_hi) {
			if (Hw && !hi_c)
				return 0;
			Hw += nhi;
			vhi = nvhi;
		}
		if (Lw + Hw > n)
			return 0;
		median = (n & 1) ? w_at((n - 1) / 2) : (w_at((n - 1) / 2) + w_at(n / 2)) / 2.0;
		const uint64_t Sw = (uint64_t)Lw * vlo + (uint64_t)Hw * vhi + (uint64_t)(L.p1[hi - Hw] - L.p1[lo + Lw]);
		const uint64_t SSw = (uint64_t)Lw * vlo * vlo + (uint64_t)Hw * vhi * vhi + (L.p2[hi - Hw] - L.p2[lo + Lw]);
		const double sigma0 = sigma;
		const bool e00 = sig_e0;
		bool we0;
		sigma = 1.134 * exact_sd(n, Sw, SSw, &we0);
		sig_e0 = we0;
		if (e00) {
			if (we0)
				break;	/* 0/0 = NaN: the loop exits */
			continue;	/* x/0 = inf > 0.0005 */
		}
		const double q = fabs(sigma - sigma0) / sigma0;
		if (fabs(q - 0.0005) <= 1e-9 * 0.0005 + SG_BAND * (1.0 + q))
			return 0;
		if (!(q > 0.0005))
			break;
	}
	e0 = sig_e0;
	return 1;
}

template <class LDS>
__device__ int replay_sigma_fast(LDS &L, int &N, int &r, int &iter, double sl, double sh, int lane,
		uint32_t &clo, uint32_t &chi, uint16_t *value, int type = 2) {
	constexpr int KM = SG_REPLAY_FASTN / 64;
	{	/* prefix sums over the sorted stack, 8 consecutive samples per lane */
		uint32_t a = 0;
		unsigned long long b = 0;
		uint32_t v[KM];
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = KM * lane + k;
			v[k] = e < N ? L.stack[e] : 0u;
			a += v[k];
			b += (unsigned long long)v[k] * v[k];
		}
		uint32_t ea = (uint32_t)wave_excl_scan((int)a, lane);
		unsigned long long eb = wave_excl_scan_u64(b, lane);
		if (lane == 0) {
			L.p1[0] = 0;
			L.p2[0] = 0;
		}
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = KM * lane + k;
			ea += v[k];
			eb += (unsigned long long)v[k] * v[k];
			if (e < N) {
				L.p1[e + 1] = ea;
				L.p2[e + 1] = eb;
			}
		}
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	}
	/* the sorted stack in registers (element 64 k + lane in xs[k]): the passes below do not
	 * move it, so every pass and Winsorize iteration reads registers instead of LDS */
	uint32_t xs[KM];
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const int e = 64 * k + lane;
		xs[k] = e < N ? (uint32_t)L.stack[e] : 0u;
	}
	int lo = 0, hi = N;
	uint32_t fl = 0, fh = 0;	/* clip counts of the fast passes (wave-uniform) */
	bool handover = false;
	for (;;) {
		const int n = hi - lo;
		const uint64_t S = (uint64_t)(L.p1[hi] - L.p1[lo]), SS = L.p2[hi] - L.p2[lo];
		bool e0;
		double sigma = exact_sd(n, S, SS, &e0);
		double median = replay_median(L.stack + lo, n);
		if (type == 4 && !replay_winsor_inner(L, xs, lo, hi, lane, median, sigma, e0)) {
			handover = true;
			break;
		}
		const double tl = sl * sigma, th = sh * sigma;
		const double blo = median - tl, bhi = median + th;
		const double tol = e0 ? 0.0 : SG_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
		int amb = 0, cl = 0, ch = 0;
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = 64 * k + lane;
			const bool in = e >= lo && e < hi;
			const double x = (double)xs[k];
			if (in && tol > 0.0 && ((x >= blo - tol && x <= blo + tol) || (x >= bhi - tol && x <= bhi + tol)))
				amb = 1;
			const bool low = in && (median - x > tl), high = in && !low && (x - median > th);
			cl += (int)__popcll(__ballot(low));
			ch += (int)__popcll(__ballot(high));
		}
		if (__ballot(amb) != 0ull) {
			handover = true;
			break;
		}
		/* the general loop's first frame fb with n - (r + rejections in [0, fb]) <= 4 */
		const int need = n - 4 - r;
		int fb = n - 1;
		if (need <= 0)
			fb = 0;
		else if (cl >= need)
			fb = need - 1;
		else if (cl + ch >= need)
			fb = (n - ch) + (need - cl) - 1;
		if (fb < n - 1) {
			handover = true;
			break;
		}
		iter++;
		SG_RPROF(if (lane == 0) L.npass++;)
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int j = 64 * k + lane;
			if (j < n)
				L.rej[j] = j < cl ? (int8_t)-1 : (j >= n - ch ? (int8_t)1 : (int8_t)0);
		}
		r += cl + ch;
		fl += (uint32_t)cl;
		fh += (uint32_t)ch;
		lo += cl;
		hi -= ch;
		if (!(cl + ch > 0 && hi - lo > 3))
			break;
	}
	if (!handover) {
		N = hi - lo;
		*value = sg_round_to_WORD((double)(L.p1[hi] - L.p1[lo]) / (double)N);
		clo = fl;	/* totals */
		chi = fh;
		return 1;
	}
	/* the general loop keeps per-lane partial counts and sums them over the wave at the end */
	clo = lane == 0 ? fl : 0u;
	chi = lane == 0 ? fh : 0u;
	/* compact [lo, hi) to the front for the general loop */
	const int n = hi - lo;
	if (lo > 0) {
		uint16_t kv[KM];
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = 64 * k + lane;
			kv[k] = e < n ? L.stack[lo + e] : 0;
		}
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const int e = 64 * k + lane;
			if (e < n)
				L.stack[e] = kv[k];
		}
	}
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	N = n;
	return 0;
}

/* returns 1 on success (value / counters set), 0 = leave the pixel to the literal path
 * (first pass broken early, or the Winsorize guard).  Each sigma comes from exact integer
 * moments; when a decision that uses it falls inside the rounding band, that sigma is
 * recomputed the reference's way (replay_gsl_sd, on the same array in the same order) and
 * the decision is evaluated in the reference's double arithmetic with no band (`sx`: the
 * current sigma is the reference's own value).  Every sigma is a function of an integer
 * array, and the arrays depend on earlier sigmas only through discrete decisions, so the
 * next sigma starts from exact moments again. */
/* PMAX: positions per lane of the general loop's per-lane chunks (8 for N <= 512, so the chunk
 * arrays d[] / kv[] are indexed statically and stay in registers; 32 up to SG_REPLAY_MAXN,
 * where they live in scratch) */
template <int PMAX, class LDS>
__device__ int replay_pixel(LDS &L, int N0, int type, double sl, double sh, int lane, uint16_t *value,
		uint32_t *rlo, uint32_t *rhi) {
	int N = N0, r = 0, n, iter = 0;
	uint32_t clo = 0, chi = 0;
	if (N0 <= SG_REPLAY_FASTN) {
#pragma unroll
		for (int k = 0; k < SG_REPLAY_FASTN / 64; k++) {
			const int j = 64 * k + lane;
			if (j < N0) {
				L.rej[j] = 0;
				L.orig[j] = L.stack[j];	/* frame order: the first pass's sd input */
			}
		}
	} else {
		for (int j = lane; j < N0; j += 64) {
			L.rej[j] = 0;
			L.orig[j] = L.stack[j];
		}
	}
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	replay_sort_any(L.stack, N, lane);	/* the quicksort_s of the first pass; later passes keep it sorted */
	SG_RPROF(if (lane == 0) L.t_sort = __builtin_readcyclecounter();)
	if ((type == 2 || (type == 4 && SG_REPLAY_WFAST)) && N <= SG_REPLAY_FASTN) {
		const int done = replay_sigma_fast(L, N, r, iter, sl, sh, lane, clo, chi, value, type);
		SG_RPROF(if (lane == 0) {
			L.t_fast = __builtin_readcyclecounter();
			L.handover = !done;
		})
		if (done) {
			*rlo = clo;
			*rhi = chi;
			return 1;
		}
	}
	do {
		iter++;
		SG_RPROF(if (lane == 0) L.npass++;)
		uint64_t S, SS;
		replay_moments(L.stack, N, lane, S, SS);
		bool e0;
		double sigma = exact_sd(N, S, SS, &e0);
		bool sx = false;
		const uint16_t *src = iter == 1 ? L.orig : L.stack;	/* this pass's sd input (sorted after pass 1) */
		double median = replay_median(L.stack, N);
		if (type == 4) {
			for (int j = lane; j < N; j += 64)
				L.w[j] = L.stack[j];
			__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
			bool sig_e0 = e0;
			bool from_w = false;	/* sigma's input: the pass-level array, or w */
			for (int guard = 0;; guard++) {
				if (guard > 100000)
					return 0;
				double m0 = median - 1.5 * sigma, m1 = median + 1.5 * sigma;
				if (!sx) {
					const double tol = sig_e0 ? 0.0 : SG_BAND * (fabs(median) + 1.5 * sigma + 1.0);
					int amb = 0, clamped_lo = 0, clamped_hi = 0;
					for (int j = lane; j < N; j += 64) {
						const double x = (double)L.w[j];
						if (!sig_e0 && ((x >= m0 - tol && x <= m0 + tol) || (x >= m1 - tol && x <= m1 + tol)))
							amb = 1;
						if (x < m0)
							clamped_lo = 1;
						else if (x > m1)
							clamped_hi = 1;
					}
					amb = wave_or(amb);
					clamped_lo = wave_or(clamped_lo);
					clamped_hi = wave_or(clamped_hi);
					if (amb || (clamped_lo && round_ambiguous(m0, tol + 1e-9 * tol)) ||
							(clamped_hi && round_ambiguous(m1, tol + 1e-9 * tol))) {
						sx = true;
						sigma = from_w ? 1.134 * replay_gsl_sd(L, L.w, N, lane) : replay_gsl_sd(L, src, N, lane);
						m0 = median - 1.5 * sigma;
						m1 = median + 1.5 * sigma;
					}
				}
				if (!sx && from_w) {
					for (int j = lane; j < N; j += 64)
						L.wprev[j] = L.w[j];	/* sigma's input, for a later recomputation */
				}
				const uint16_t vlo = sg_round_to_WORD(m0), vhi = sg_round_to_WORD(m1);
				for (int j = lane; j < N; j += 64) {
					const double x = (double)L.w[j];
					if (x < m0)
						L.w[j] = vlo;
					else if (x > m1)
						L.w[j] = vhi;
				}
				__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
				median = replay_median(L.w, N);
				uint64_t Sw, SSw;
				replay_moments(L.w, N, lane, Sw, SSw);
				const double sigma0 = sigma;
				const bool e00 = sig_e0, s0x = sx, prev_from_w = from_w;
				bool we0;
				sigma = 1.134 * exact_sd(N, Sw, SSw, &we0);
				sig_e0 = we0;
				sx = false;
				from_w = true;
				if (e00) {
					if (we0)
						break;	/* 0/0 = NaN: the loop exits */
					continue;	/* x/0 = inf > 0.0005 */
				}
				const double q = fabs(sigma - sigma0) / sigma0;
				if (fabs(q - 0.0005) <= 1e-9 * 0.0005 + SG_BAND * (1.0 + q)) {
					const double s0 = s0x ? sigma0
							      : prev_from_w ? 1.134 * replay_gsl_sd(L, L.wprev, N, lane)
									    : replay_gsl_sd(L, src, N, lane);
					sigma = 1.134 * replay_gsl_sd(L, L.w, N, lane);
					sx = true;
					if (!((fabs(sigma - s0) / s0) > 0.0005))
						break;
					continue;
				}
				if (!(q > 0.0005))
					break;
			}
			e0 = sig_e0;
		}
		/* decisions, frame order, with the early break */
		const int per = (N + 63) / 64, j0 = lane * per;
		int cnt = 0;
		int8_t d[PMAX];
		for (int attempt = 0; attempt < 2; attempt++) {
			const double tl = sl * sigma, th = sh * sigma;
			const double blo = median - tl, bhi = median + th;
			const double tol = (e0 || sx) ? 0.0 : SG_BAND * (fabs(median) + fabs(tl) + fabs(th) + 1.0);
			int amb = 0;
			cnt = 0;
#pragma unroll
			for (int k = 0; k < PMAX && k < per; k++) {
				const int j = j0 + k;
				int8_t v = 0;
				if (j < N) {
					const double x = (double)L.stack[j];
					if (tol > 0.0 && ((x >= blo - tol && x <= blo + tol) || (x >= bhi - tol && x <= bhi + tol)))
						amb = 1;
					v = (median - x > tl) ? -1 : ((x - median > th) ? 1 : 0);
				}
				d[k] = v;
				cnt += v != 0;
			}
			if (!wave_or(amb))
				break;
			/* recompute this pass's sigma the reference's way and decide again, exactly */
			sx = true;
			sigma = type == 4 ? 1.134 * replay_gsl_sd(L, L.w, N, lane) : replay_gsl_sd(L, src, N, lane);
		}
		/* first frame fb with N - (r + #rejections in [0, fb]) <= 4 */
		const int before = wave_excl_scan(cnt, lane);
		int fb_lane = N;
		{
			int c = r + before;
			bool found = false;
#pragma unroll
			for (int k = 0; k < PMAX; k++) {	/* no early exit, so the loop unrolls */
				const int j = j0 + k;
				if (k < per && j < N && !found) {
					c += d[k] != 0;
					if (N - c <= 4) {
						fb_lane = j;
						found = true;
					}
				}
			}
		}
		int fb = fb_lane;
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) {
			const int t = __shfl_xor(fb, o, 64);
			fb = t < fb ? t : fb;
		}
		if (fb > N - 1)
			fb = N - 1;
		if (iter == 1 && fb < N - 1)
			return 0;	/* stale entries of the previous pixel */
		int nrej = 0;
#pragma unroll
		for (int k = 0; k < PMAX && k < per; k++) {
			const int j = j0 + k;
			if (j <= fb) {
				L.rej[j] = d[k];
				nrej += d[k] != 0;
				clo += d[k] < 0;
				chi += d[k] > 0;
			}
		}
		r += (int)wave_sum_u64((uint64_t)nrej);
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		/* order-preserving removal of every position j < N with rejected[j] != 0 */
		int keep = 0;
		uint16_t kv[PMAX];
#pragma unroll
		for (int k = 0; k < PMAX && k < per; k++) {
			const int j = j0 + k;
			kv[k] = j < N ? L.stack[j] : 0;
			keep += (j < N && L.rej[j] == 0);
		}
		int pos = wave_excl_scan(keep, lane);
		const int kept = (int)wave_sum_u64((uint64_t)keep);
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
		for (int k = 0; k < PMAX && k < per; k++) {
			const int j = j0 + k;
			if (j < N && L.rej[j] == 0)
				L.stack[pos++] = kv[k];
		}
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		n = N - kept;
		N = kept;
	} while (n > 0 && N > 3);
	uint64_t S, SS;
	replay_moments(L.stack, N, lane, S, SS);
	*value = sg_round_to_WORD((double)S / (double)N);
	*rlo = (uint32_t)wave_sum_u64((uint64_t)clo);
	*rhi = (uint32_t)wave_sum_u64((uint64_t)chi);
	return 1;
}

/* ---------------------------------------------------------------------------------------
 * LINEARFIT, decision-exact (:1750-1784).  The reference fits y = a i + b to the sorted kept
 * stack with gsl_fit_linear's double recurrences (m_x, m_y, m_dx2, m_dxdy, then b = m_dxdy /
 * m_dx2, a = m_y - m_x b), takes sigma = mean |y_i - (a i + b)| and clips with line_clipping.
 * Its decisions only depend on those rounded values through comparisons, so this path takes the
 * fit from exact integer sums (S_y = sum y, S_iy = sum i y over the kept sorted ranks i, and the
 * closed forms of x = 0 .. N-1: slope = (12 S_iy - 6 (N-1) S_y) / (N (N^2 - 1))), and decides
 * every test against a bound on how far the reference's rounded recurrences can be from the
 * exact fit:
 *   |m_x err| <= 2 N^2 u, |m_y err| <= 2 N u Y, |m_dx2 err| <= 6 N^3 u, |m_dxdy err| <= 6 N^2 u Y
 * (u = 2^-53, Y = the kept maximum; each recurrence step m += (v - m)/(k+1) adds at most
 * 2u|v - m|/(k+1) + u|m| and damps the carried error by k/(k+1)), propagated through the slope,
 * intercept, residuals, sigma and the division (LINEARFIT round 5), each taken 4x.
 * A test closer to its threshold than that, a sigma within the bound of 0, a pass that would
 * reach the `N - r <= 4` break (its rejected[] entries after the break are stale state) or any
 * other corner sends the pixel to the redo list (the sorted kernel's reject_linearfit, which
 * replays the recurrences bit for bit, and the literal kernel for first-pass breaks).
 *
 * One workgroup per 64 pixels of a row: the N frames' 128-B row segments (shifted, normalised
 * as sg_gather) land in LDS as per-pixel columns; each wave then takes a pixel at a time with its
 * column in registers (element 64 k + lane in x[k]), sorts it (bitonic, replay_cx_reg), and runs
 * the passes with ballots for the ranks and wave sums for S_y, S_iy and sigma. */
/* lane exchanges on the VALU (DPP / swizzle instead of ds_bpermute round trips): the partner
 * lane ^ J of every lane */
template <int J>
__device__ __forceinline__ uint32_t lfx_xor(uint32_t v, int lane) {
	if (J == 1)
		return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);	/* quad_perm [1,0,3,2] */
	if (J == 2)
		return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);	/* quad_perm [2,3,0,1] */
	if (J == 4 || J == 8) {	/* row_shl:J for the lower half of each 2J group, row_shr:J for the upper */
		const uint32_t up = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x100 + J, 0xF, 0xF, false);
		const uint32_t dn = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x110 + J, 0xF, 0xF, false);
		return (lane & J) ? dn : up;
	}
	if (J == 16)	/* swizzle bit mode within 32 lanes: and 0x1F, xor 0x10 */
		return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x401F);
	return (uint32_t)__shfl_xor((int)v, J, 64);
}

/* compare-exchanges on two pixels' columns at once: element e of pixel A in the low half of
 * x[k], of pixel B in the high half (the network does not depend on the data), by packed u16
 * min / max */
__device__ __forceinline__ uint32_t lfx_pk_min(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
}
__device__ __forceinline__ uint32_t lfx_pk_max(uint32_t a, uint32_t b) {
	uint32_t r;
	asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
	return r;
}
template <int KM, int J>
__device__ __forceinline__ void lfx_cx_lanes(uint32_t (&x)[KM], int kk, int lane) {
	const bool lower = (lane & J) == 0;
	/* ((64 k + lane) & kk) == 0 splits into a lane part (kk < 64) and a uniform k part (kk >= 64) */
	const bool lane_up = (lane & kk) == 0;
#pragma unroll
	for (int k = 0; k < KM; k++) {
		const bool up = ((64 * k) & kk) == 0 && lane_up;
		const uint32_t y = lfx_xor<J>(x[k], lane);
		/* both computed, then selected (an asm call inside the ?: became a divergent branch) */
		const uint32_t mn = lfx_pk_min(x[k], y), mx = lfx_pk_max(x[k], y);
		x[k] = (lower == up) ? mn : mx;
	}
}
template <int KM, int JR>
__device__ __forceinline__ void lfx_cx_reg(uint32_t (&x)[KM], int kk, int lane) {
	(void)lane;	/* kk >= 128 here: the direction is uniform per register */
#pragma unroll
	for (int k = 0; k < KM; k++) {
		if ((k & JR) == 0 && (k | JR) < KM) {
			const bool up = ((64 * k) & kk) == 0;
			const uint32_t u = x[k], v = x[k | JR];
			const uint32_t mn = lfx_pk_min(u, v), mx = lfx_pk_max(u, v);
			x[k] = up ? mn : mx;
			x[k | JR] = up ? mx : mn;
		}
	}
}

template <int KM>
__device__ __forceinline__ void lfx_sort(uint32_t (&x)[KM], int lane) {
	constexpr int P = 64 * KM;
#pragma unroll 1
	for (int kk = 2; kk <= P; kk <<= 1) {
#pragma unroll 1
		for (int j = kk >> 1; j > 0; j >>= 1) {
			switch (j) {
			case 1: lfx_cx_lanes<KM, 1>(x, kk, lane); break;
			case 2: lfx_cx_lanes<KM, 2>(x, kk, lane); break;
			case 4: lfx_cx_lanes<KM, 4>(x, kk, lane); break;
			case 8: lfx_cx_lanes<KM, 8>(x, kk, lane); break;
			case 16: lfx_cx_lanes<KM, 16>(x, kk, lane); break;
			case 32: lfx_cx_lanes<KM, 32>(x, kk, lane); break;
			case 64: lfx_cx_reg<KM, 1>(x, kk, lane); break;
			case 128: lfx_cx_reg<KM, 2>(x, kk, lane); break;
			case 256: lfx_cx_reg<KM, 4>(x, kk, lane); break;
			default: lfx_cx_reg<KM, 8>(x, kk, lane); break;
			}
		}
	}
}

/* wave totals by the DPP inclusive-scan sequence (row_shr 1..3, 4, 8, row_bcast 15 / 31: the
 * last lane holds the total), read from lane 63; no LDS round trips */
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int lfx_dpp(int v) {
	return __builtin_amdgcn_update_dpp(0, v, CTRL, RM, BM, true);
}
__device__ __forceinline__ uint32_t lfx_sum_u32(uint32_t v0) {
	const int v = (int)v0;
	int t = v + lfx_dpp<0x111, 0xF, 0xF>(v);
	t += lfx_dpp<0x112, 0xF, 0xF>(v);
	t += lfx_dpp<0x113, 0xF, 0xF>(v);
	t += lfx_dpp<0x114, 0xF, 0xE>(t);
	t += lfx_dpp<0x118, 0xF, 0xC>(t);
	t += lfx_dpp<0x142, 0xA, 0xF>(t);
	t += lfx_dpp<0x143, 0xC, 0xF>(t);
	return (uint32_t)__builtin_amdgcn_readlane(t, 63);
}
__device__ __forceinline__ uint32_t lfx_max_u32(uint32_t v) {
	auto mx = [](uint32_t a, int b) { return a > (uint32_t)b ? a : (uint32_t)b; };
	uint32_t t = mx(v, lfx_dpp<0x111, 0xF, 0xF>((int)v));
	t = mx(t, lfx_dpp<0x112, 0xF, 0xF>((int)v));
	t = mx(t, lfx_dpp<0x113, 0xF, 0xF>((int)v));
	t = mx(t, lfx_dpp<0x114, 0xF, 0xE>((int)t));
	t = mx(t, lfx_dpp<0x118, 0xF, 0xC>((int)t));
	t = mx(t, lfx_dpp<0x142, 0xA, 0xF>((int)t));
	t = mx(t, lfx_dpp<0x143, 0xC, 0xF>((int)t));
	return (uint32_t)__builtin_amdgcn_readlane((int)t, 63);
}
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double lfx_dppd(double x) {
	const int lo = lfx_dpp<CTRL, RM, BM>(__double2loint(x)), hi = lfx_dpp<CTRL, RM, BM>(__double2hiint(x));
	return __hiloint2double(hi, lo);
}
/* exact for the integer-valued sums used here (every partial < 2^53); the residual sum's order
 * only enters its error bound */
__device__ __forceinline__ double lfx_sum_f64(double v) {
	double t = v + lfx_dppd<0x111, 0xF, 0xF>(v);
	t += lfx_dppd<0x112, 0xF, 0xF>(v);
	t += lfx_dppd<0x113, 0xF, 0xF>(v);
	t += lfx_dppd<0x114, 0xF, 0xE>(t);
	t += lfx_dppd<0x118, 0xF, 0xC>(t);
	t += lfx_dppd<0x142, 0xA, 0xF>(t);
	t += lfx_dppd<0x143, 0xC, 0xF>(t);
	return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(t), 63),
			__builtin_amdgcn_readlane(__double2loint(t), 63));
}

/* one pixel's passes; x[] sorted ascending (pads 0xFFFF at elements >= N0).  Returns 1 with the
 * value and counters, 0 when the pixel goes to the redo list.  The kept set is one 64-bit lane
 * mask per register (uniform, SGPRs): the ranks come from mbcnt on the mask, the rejection
 * counts and the removal are mask operations, and a lane's tests are compares whose results are
 * the masks themselves; one margin serves both tests (the larger of the two sides'; per-lane bit
 * fields and two margins took 303 ms against 261, profiles/r05z4_*, r05ad_*). */
template <int KM>
__device__ int lfx_pixel_m(const uint32_t (&x)[KM], int N0, double sl, double sh, int lane, uint16_t &value,
		uint32_t &rlo, uint32_t &rhi) {
	constexpr double u = 1.1102230246251565e-16;
	unsigned long long km[KM];
#pragma unroll
	for (int k = 0; k < KM; k++)
		km[k] = __ballot(64 * k + lane < N0);
	int N = N0, r = 0;
	uint32_t clo = 0, chi = 0;
	double Sy = 0.0;
	double xd[KM];
#pragma unroll
	for (int k = 0; k < KM; k++)
		xd[k] = (double)x[k];
	const double asl = fabs(sl), ash = fabs(sh), amx = asl > ash ? asl : ash;
	for (int pass = 0; pass < 4096; pass++) {
		double rank[KM];
		int base = 0;
		uint32_t sy = 0, ymax = 0, siy = 0;
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const bool kp = (km[k] >> lane) & 1ull;
			const int rk = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km[k] >> 32),
					__builtin_amdgcn_mbcnt_lo((unsigned)km[k], 0u));
			base += __popcll(km[k]);
			rank[k] = (double)rk;
			const uint32_t xk = kp ? x[k] : 0u;
			sy += xk;
			siy += (uint32_t)rk * xk;
			ymax = xk > ymax ? xk : ymax;
		}
		if (N < 8)
			return 0;
		Sy = (double)lfx_sum_u32(sy);
		/* S_iy < 2^36: two integer wave sums of its 16-bit halves (a lane's siy < 2^30) */
		const double Siy = (double)lfx_sum_u32(siy & 0xFFFFu) + 65536.0 * (double)lfx_sum_u32(siy >> 16);
		ymax = lfx_max_u32(ymax);
		const double n = (double)N, Y = (double)ymax, inv_n = 1.0 / n;
		const double Pn = 12.0 * Siy - 6.0 * (n - 1.0) * Sy;
		const double slope = Pn / (n * (n * n - 1.0));
		const double b0 = Sy * inv_n - 0.5 * (n - 1.0) * slope;
		double dv[KM];
		double sres = 0.0;
#pragma unroll
		for (int k = 0; k < KM; k++) {
			dv[k] = fma(slope, rank[k], b0) - xd[k];
			sres += ((km[k] >> lane) & 1ull) ? fabs(dv[k]) : 0.0;
		}
		const double sigma = lfx_sum_f64(sres) * inv_n;
		/* the bounds above (the LINEARFIT comment) in closed form, before one 4x safety factor on
		 * each test's margin (8 <= n <= 1024: mdx2 - dmdx2 >= 0.75 mdx2 and 1 / mdx2 <= 12.2 / n^2):
		 * dS = (6 n^2 u Y + |s| 6 n^3 u) 16.3 / n^2 + 4 u |s| rounded up to 98 u (Y + (n + 1) |s|);
		 * dB = 2 n u Y + 2 n^2 u |s| + n dS / 2 + 8 u Rm.  (Each level took its own 4x until round 5:
		 * 16-64x on a test, 10.5 k redo pixels.) */
		const double as = fabs(slope), nas = n * as;
		const double dS = 98.0 * u * (Y + nas + as);
		const double Rm = Y + nas + fabs(b0) + 1.0;
		const double dB = 2.0 * u * n * (Y + nas) + 0.5 * n * dS + 8.0 * u * Rm;
		const double dline = n * dS + dB + 32.0 * u * Rm;
		const double dsig = dline + 2.0 * (n + 2.0) * u * Rm;
		if (!(sigma > 4.0 * dsig) || !(sl == sl) || !(sh == sh) || !(sl > 0.0) || !(sh > 0.0))
			return 0;	/* non-positive factors: the else-if order matters, the general path decides */
		const double tL = sl * sigma, tH = sh * sigma;
		const double e1 = 4.0 * dS;
		const double eM = 4.0 * (dB + 32.0 * u * Rm + amx * dsig + 4.0 * u * (Rm + amx * sigma));
		/* with sl, sh > 0 a sample is at most one of low (line - y > tL) and high (y - line > tH) */
		unsigned long long amb = 0;
		int nl = 0, nh = 0;
#pragma unroll
		for (int k = 0; k < KM; k++) {
			const double e = fma(e1, rank[k], eM);
			const double a = dv[k] - tL, b = dv[k] + tH;
			const unsigned long long lo = __ballot(a > e) & km[k], hi = __ballot(b < -e) & km[k];
			amb |= __ballot(fabs(a) <= e || fabs(b) <= e) & km[k];
			nl += __popcll(lo);
			nh += __popcll(hi);
			km[k] &= ~(lo | hi);
		}
		if (amb)
			return 0;
		const int nrej = nl + nh;
		if (r + nrej >= N - 4)
			return 0;
		clo += nl;
		chi += nh;
		r += nrej;
		N -= nrej;
		if (!(nrej > 0 && N > 3)) {
			if (nrej > 0) {
				uint32_t s2 = 0;
#pragma unroll
				for (int k = 0; k < KM; k++)
					s2 += ((km[k] >> lane) & 1ull) ? x[k] : 0u;
				Sy = (double)lfx_sum_u32(s2);
			}
			value = sg_round_to_WORD(Sy / (double)N);
			rlo = clo;
			rhi = chi;
			return 1;
		}
	}
	return 0;
}

/* the passes of BOTH pixels of a packed sorted pair (pixel 0 in the low u16 of x2[k], pixel 1 in
 * the high one) in lockstep (round 6): per pixel the arithmetic and decisions of
 * lfx_pixel_m, step for step; the two pixels' wave reductions and fp64 chains are independent work
 * in one basic block, so each hides the other's latency (lfx_pixel_m is a serial chain of wave
 * reductions per pass).  Per-element doubles (rank, sample, residual) are recomputed where used
 * instead of held in arrays, which keeps two pixels in about one pixel's registers.  A pixel that
 * has finished rides along (its results are not committed) until the other one finishes.
 * ok[h]: 1 value and counters, 0 redo list. */
template <int KM>
__device__ void lfx_pixel2_m(const uint32_t (&x2)[KM], int N0, double sl, double sh, int lane, uint16_t (&value)[2],
		uint32_t (&rlo)[2], uint32_t (&rhi)[2], int (&ok)[2]) {
	constexpr double u = 1.1102230246251565e-16;
	unsigned long long km[2][KM];
#pragma unroll
	for (int k = 0; k < KM; k++)
		km[0][k] = km[1][k] = __ballot(64 * k + lane < N0);
	int N[2] = {N0, N0}, r[2] = {0, 0}, st[2] = {0, 0};	/* st: 0 running, 1 value, 2 redo */
	uint32_t clo[2] = {0, 0}, chi[2] = {0, 0};
	const double asl = fabs(sl), ash = fabs(sh), amx = asl > ash ? asl : ash;
	auto xv = [&](int h, int k) -> uint32_t { return h ? (x2[k] >> 16) : (x2[k] & 0xFFFFu); };
	for (int pass = 0; pass < 4096 && (st[0] == 0 || st[1] == 0); pass++) {
		uint32_t sy[2], siy[2], ymax[2];
#pragma unroll
		for (int h = 0; h < 2; h++) {
			int base = 0;
			sy[h] = siy[h] = ymax[h] = 0;
#pragma unroll
			for (int k = 0; k < KM; k++) {
				const bool kp = (km[h][k] >> lane) & 1ull;
				const int rk = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km[h][k] >> 32),
						__builtin_amdgcn_mbcnt_lo((unsigned)km[h][k], 0u));
				base += __popcll(km[h][k]);
				const uint32_t xk = kp ? xv(h, k) : 0u;
				sy[h] += xk;
				siy[h] += (uint32_t)rk * xk;
				ymax[h] = xk > ymax[h] ? xk : ymax[h];
			}
		}
		double Sy[2], Siy[2], Y[2];
#pragma unroll
		for (int h = 0; h < 2; h++) {
			Sy[h] = (double)lfx_sum_u32(sy[h]);
			Siy[h] = (double)lfx_sum_u32(siy[h] & 0xFFFFu) + 65536.0 * (double)lfx_sum_u32(siy[h] >> 16);
			Y[h] = (double)lfx_max_u32(ymax[h]);
		}
		double slope[2], b0[2], sres[2], inv_n[2];
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const double n = (double)N[h];
			inv_n[h] = 1.0 / n;
			const double Pn = 12.0 * Siy[h] - 6.0 * (n - 1.0) * Sy[h];
			slope[h] = Pn / (n * (n * n - 1.0));
			b0[h] = Sy[h] * inv_n[h] - 0.5 * (n - 1.0) * slope[h];
			int base = 0;
			double sr = 0.0;
#pragma unroll
			for (int k = 0; k < KM; k++) {
				const int rk = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km[h][k] >> 32),
						__builtin_amdgcn_mbcnt_lo((unsigned)km[h][k], 0u));
				base += __popcll(km[h][k]);
				const double dv = fma(slope[h], (double)rk, b0[h]) - (double)xv(h, k);
				sr += ((km[h][k] >> lane) & 1ull) ? fabs(dv) : 0.0;
			}
			sres[h] = sr;
		}
		double sigma[2];
#pragma unroll
		for (int h = 0; h < 2; h++)
			sigma[h] = lfx_sum_f64(sres[h]) * inv_n[h];
#pragma unroll
		for (int h = 0; h < 2; h++) {
			if (st[h] != 0)
				continue;
			if (N[h] < 8) {
				st[h] = 2;
				continue;
			}
			const double n = (double)N[h];
			/* lfx_pixel_m's closed-form bounds and 4x margins */
			const double as = fabs(slope[h]), nas = n * as;
			const double dS = 98.0 * u * (Y[h] + nas + as);
			const double Rm = Y[h] + nas + fabs(b0[h]) + 1.0;
			const double dB = 2.0 * u * n * (Y[h] + nas) + 0.5 * n * dS + 8.0 * u * Rm;
			const double dline = n * dS + dB + 32.0 * u * Rm;
			const double dsig = dline + 2.0 * (n + 2.0) * u * Rm;
			if (!(sigma[h] > 4.0 * dsig) || !(sl == sl) || !(sh == sh) || !(sl > 0.0) || !(sh > 0.0)) {
				st[h] = 2;
				continue;
			}
			const double tL = sl * sigma[h], tH = sh * sigma[h];
			const double e1 = 4.0 * dS;
			const double eM = 4.0 * (dB + 32.0 * u * Rm + amx * dsig + 4.0 * u * (Rm + amx * sigma[h]));
			unsigned long long amb = 0, rm[KM];
			int nl = 0, nh = 0, base = 0;
#pragma unroll
			for (int k = 0; k < KM; k++) {
				const int rk = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km[h][k] >> 32),
						__builtin_amdgcn_mbcnt_lo((unsigned)km[h][k], 0u));
				base += __popcll(km[h][k]);
				const double dv = fma(slope[h], (double)rk, b0[h]) - (double)xv(h, k);
				const double e = fma(e1, (double)rk, eM);
				const double a = dv - tL, b = dv + tH;
				const unsigned long long lo = __ballot(a > e) & km[h][k], hi = __ballot(b < -e) & km[h][k];
				amb |= __ballot(fabs(a) <= e || fabs(b) <= e) & km[h][k];
				nl += __popcll(lo);
				nh += __popcll(hi);
				rm[k] = lo | hi;
			}
			if (amb) {
				st[h] = 2;
				continue;
			}
			const int nrej = nl + nh;
			if (r[h] + nrej >= N[h] - 4) {
				st[h] = 2;
				continue;
			}
#pragma unroll
			for (int k = 0; k < KM; k++)
				km[h][k] &= ~rm[k];
			clo[h] += nl;
			chi[h] += nh;
			r[h] += nrej;
			N[h] -= nrej;
			if (!(nrej > 0 && N[h] > 3)) {
				double S = Sy[h];
				if (nrej > 0) {
					uint32_t s2 = 0;
#pragma unroll
					for (int k = 0; k < KM; k++)
						s2 += ((km[h][k] >> lane) & 1ull) ? xv(h, k) : 0u;
					S = (double)lfx_sum_u32(s2);
				}
				value[h] = sg_round_to_WORD(S / (double)N[h]);
				rlo[h] = clo[h];
				rhi[h] = chi[h];
				st[h] = 1;
			}
		}
	}
	ok[0] = st[0] == 1;
	ok[1] = st[1] == 1;
}

template <int KM, int NW, bool PAIR = false>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu((PAIR && KM == 8) ? 4 : 1)))	/* pair: 4 waves per SIMD */
k_stack_linfit(SgStackParams p, unsigned int *__restrict__ redo_count, unsigned int *__restrict__ redo_list) {
	extern __shared__ uint16_t lfx_cols[];
	constexpr int LS = 64 * KM + 2;	/* column stride: an odd dword count (conflict-free stores) */
	const int tid = threadIdx.x, lane = tid & 63;
	const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int N = p.N;
	const int ntx = (p.W + 63) / 64, nrows = p.row_end - p.row_begin;
	int bid = blockIdx.x;
	const int xt = bid % ntx;
	bid /= ntx;
	const int R = p.row_begin + (bid % nrows), c = bid / nrows;
	const int x0 = xt * 64;
	/* the tile: frame f's row segment by wave f % NW, sample of pixel px at lfx_cols[px LS + f] */
	{
		const int px = lane, x = x0 + px;
		uint16_t *dst = lfx_cols + px * LS;
		const uint16_t *plane = p.frames + (int64_t)c * p.plane_stride;
#pragma unroll 8
		for (int f = wave; f < N; f += NW) {
			int sx = 0, sy = 0;
			if (p.use_shift) {
				sx = p.shiftx[f];
				sy = p.shifty[f];
			}
			const int sr = R - sy, sc = x - sx;
			const bool colok = (unsigned)sc < (unsigned)p.W;
			uint16_t v = 0;
			if (colok && (unsigned)sr < (unsigned)p.H)
				v = plane[(int64_t)f * p.frame_stride + (int64_t)sr * p.W + sc];
			dst[f] = colok ? sg_normalize(p, f, v) : (uint16_t)0;
		}
		for (int f = N + wave; f < 64 * KM; f += NW)
			dst[f] = 0xFFFF;
	}
	__syncthreads();
	const int np = min(64, p.W - x0);
	/* pixel pairs (q, q + NW) of wave q % NW sorted together (packed halves).  The fit passes are
	 * a serial chain of wave reductions: NW waves per tile (8: four per SIMD at KM = 8) hide it */
	for (int q0 = wave; q0 < np; q0 += 2 * NW) {
		uint32_t v2[KM];
#pragma unroll
		for (int k = 0; k < KM; k++)
			v2[k] = (uint32_t)lfx_cols[q0 * LS + 64 * k + lane] |
				((uint32_t)lfx_cols[(q0 + NW < 64 ? q0 + NW : q0) * LS + 64 * k + lane] << 16);
		lfx_sort<KM>(v2, lane);
		if (PAIR) {	/* both pixels' passes in lockstep (lfx_pixel2_m) */
			uint16_t value[2] = {0, 0};
			uint32_t rl[2] = {0, 0}, rh[2] = {0, 0};
			int ok[2] = {0, 0};
			lfx_pixel2_m<KM>(v2, N, p.sig0, p.sig1, lane, value, rl, rh, ok);
			for (int h = 0; h < 2; h++) {
				const int q = q0 + NW * h;
				if (q >= np)
					break;
				const int64_t pix = ((int64_t)c * p.H + R) * p.W + x0 + q;
				if (lane == 0) {
					if (ok[h]) {
						p.out[pix] = value[h];
						unsigned long long *sh = p.rej + ((size_t)(blockIdx.x % SG_REJ_SHARDS) * 6 + c * 2);
						if (rl[h])
							atomicAdd(sh, (unsigned long long)rl[h]);
						if (rh[h])
							atomicAdd(sh + 1, (unsigned long long)rh[h]);
					} else {
						redo_list[atomicAdd(redo_count, 1u)] = (unsigned int)pix;
					}
				}
			}
			continue;
		}
#pragma unroll 1
		for (int h = 0; h < 2; h++) {
			const int q = q0 + NW * h;
			if (q >= np)
				break;
			uint32_t v[KM];
#pragma unroll
			for (int k = 0; k < KM; k++)
				v[k] = h ? v2[k] >> 16 : v2[k] & 0xFFFFu;
			const int64_t pix = ((int64_t)c * p.H + R) * p.W + x0 + q;
			uint16_t value = 0;
			uint32_t rl = 0, rh = 0;
			const int ok = lfx_pixel_m<KM>(v, N, p.sig0, p.sig1, lane, value, rl, rh);
			if (lane == 0) {
				if (ok) {
					p.out[pix] = value;
					unsigned long long *sh = p.rej + ((size_t)(blockIdx.x % SG_REJ_SHARDS) * 6 + c * 2);
					if (rl)
						atomicAdd(sh, (unsigned long long)rl);
					if (rh)
						atomicAdd(sh + 1, (unsigned long long)rh);
				} else {
					redo_list[atomicAdd(redo_count, 1u)] = (unsigned int)pix;
				}
			}
		}
	}
}
template __global__ void k_stack_linfit<8, 8, true>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<8, 4, true>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<16, 8, true>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<16, 4, true>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<8, 4>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<8, 8>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<8, 16>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<16, 4>(SgStackParams, unsigned int *, unsigned int *);
template __global__ void k_stack_linfit<16, 8>(SgStackParams, unsigned int *, unsigned int *);

/* the histogram path's redo list queued for k_stack_replay / k_stack_literal: class
 * LITERAL, appended to the flag list the sorted kernel would have appended them to.  The
 * count is read on the device; a list longer than maxn is left to the sorted kernel. */
__global__ void __launch_bounds__(256)
k_redo_to_literal(SgStackParams p, const unsigned int *__restrict__ list, const unsigned int *__restrict__ count,
		unsigned int maxn) {
	const unsigned int n = *count;
	if (n > maxn)
		return;
	for (unsigned int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
		const unsigned int pix = list[i];
		sg_flag_set(p, pix, SG_CLS_LITERAL);
		const unsigned int slot = atomicAdd(p.flag_count, 1u);
		if (slot < p.flag_cap)
			p.flag_list[slot] = pix;
	}
}

/* every pixel of the band (all channels) queued for k_stack_literal: the route of stacks with no
 * histogram path beyond the sorted kernel's 1024 frames */
__global__ void __launch_bounds__(256)
k_list_all(SgStackParams p) {
	const int64_t nb = (int64_t)(p.row_end - p.row_begin) * p.W, total = nb * p.C;
	for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
		const int64_t c = i / nb, r = i - c * nb;
		const int64_t pix = (c * p.H + p.row_begin) * p.W + r;
		sg_flag_set(p, pix, SG_CLS_LITERAL);
		p.flag_list[i] = (unsigned int)pix;
	}
	if (blockIdx.x == 0 && threadIdx.x == 0)
		*p.flag_count = (unsigned int)total;
}

template <int NM>
__global__ void __launch_bounds__(64 * SG_REPLAY_WAVES)
k_stack_replay(SgStackParams p) {
	__shared__ SgReplayLdsT<NM> Ls[SG_REPLAY_WAVES];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	SgReplayLdsT<NM> &L = Ls[wv];
	unsigned int count = *p.flag_count;
	if (count > p.flag_cap)
		count = p.flag_cap;
	if ((p.rejection != 2 && p.rejection != 4) || p.N > NM)
		return;
	/* items [0, nr): the histogram path's redo list (when short enough), then the flag list (the
	 * sorted kernel's queued pixels); a redo pixel the replay cannot finish joins the flag list as
	 * LITERAL (appended past `count`: the literal kernel's phase 1 takes it) */
	unsigned int nr = p.rp_list ? *p.rp_count : 0;
	if (nr > p.rp_maxn)
		nr = 0;
	const unsigned int nw = gridDim.x * SG_REPLAY_WAVES;
	for (unsigned int i = blockIdx.x * SG_REPLAY_WAVES + wv; i < nr + count; i += nw) {
		const bool direct = i < nr;
		const int64_t pix = direct ? p.rp_list[i] : p.flag_list[i - nr];
		if (!direct && sg_flag_get(p, pix) != SG_CLS_LITERAL)
			continue;
		const int x = (int)(pix % p.W);
		const int64_t cr = pix / p.W;
		const int R = (int)(cr % p.H), c = (int)(cr / p.H);
		SG_RPROF(const unsigned long long t0 = __builtin_readcyclecounter();)
		if (p.N <= SG_REPLAY_FASTN)
			replay_gather_batched(p, L.stack, c, R, x, lane);
		else
			for (int f = lane; f < p.N; f += 64)
				L.stack[f] = sg_gather(p, f, c, R, x);
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		SG_RPROF(const unsigned long long t1 = __builtin_readcyclecounter();
		if (lane == 0) {
			L.nsd = 0;
			L.npass = 0;
			L.handover = 0;
			L.t_sort = t1;
			L.t_fast = t1;
		})
		uint16_t v;
		uint32_t rl, rh;
		const int ok = p.N <= SG_REPLAY_FASTN ? replay_pixel<SG_REPLAY_FASTN / 64>(L, p.N, p.rejection, p.sig0, p.sig1,
									     lane, &v, &rl, &rh)
						     : replay_pixel<NM / 64>(L, p.N, p.rejection, p.sig0, p.sig1,
									     lane, &v, &rl, &rh);
#ifdef SG_REPLAY_PROF
		if (SG_DBG(p) == 12 && lane == 0) {
			const unsigned long long t2 = __builtin_readcyclecounter();
			atomicMax(&g_sg_rprof[0], t2 - t0);
			atomicMax(&g_sg_rprof[1], t1 - t0);
			atomicMax(&g_sg_rprof[2], L.t_sort - t1);
			atomicAdd(&g_sg_rprof[3], 1ull);
			atomicAdd(&g_sg_rprof[4], (unsigned long long)L.nsd);
			atomicAdd(&g_sg_rprof[5], (unsigned long long)L.npass);
			atomicMax(&g_sg_rprof[6], (unsigned long long)L.nsd);
			if (L.nsd == 0)
				atomicMax(&g_sg_rprof[7], t2 - t0);
			atomicAdd(&g_sg_rprof[8], t2 - t0);
			atomicAdd(&g_sg_rprof[9], t1 - t0);
			atomicAdd(&g_sg_rprof[10], L.t_sort - t1);
			atomicAdd(&g_sg_rprof[11], L.t_fast - L.t_sort);
			atomicAdd(&g_sg_rprof[12], (unsigned long long)L.handover);
			atomicMax(&g_sg_rprof[13], L.t_fast - L.t_sort);
			atomicMax(&g_sg_rprof[14], (unsigned long long)L.npass);
		}
#endif
		if (!ok) {
			if (direct && lane == 0) {	/* to the literal kernel, as k_redo_to_literal queues */
				sg_flag_set(p, pix, SG_CLS_LITERAL);
				const unsigned int slot = atomicAdd(p.flag_count, 1u);
				if (slot < p.flag_cap)
					p.flag_list[slot] = (unsigned int)pix;
			}
			continue;
		}
		if (lane == 0) {
			p.out[pix] = v;
			sg_flag_set(p, pix, SG_CLS_DONE);
			unsigned long long *sh = p.rej + ((size_t)(i % SG_REJ_SHARDS) * 6 + c * 2);
			if (rl)
				atomicAdd(sh, (unsigned long long)rl);
			if (rh)
				atomicAdd(sh + 1, (unsigned long long)rh);
		}
	}
}
template __global__ void k_stack_replay<SG_REPLAY_FASTN>(SgStackParams);
template __global__ void k_stack_replay<SG_REPLAY_MAXN>(SgStackParams);

/* phase 1: queued pixels (class LITERAL) replayed with an all-zero incoming rejected[];
 * a pixel whose first pass breaks early with N > 4 read its predecessor's stale entries
 * and is promoted to class CHAIN (no output).  phase 2: class CHAIN pixels replay the
 * chain from the last self-determined predecessor in reference thread order.  Only pixels
 * of the band [row_begin, row_end) were classified; a predecessor outside it is classified
 * here (replayed from a zero rejected[]: a first pass without an early break writes every
 * entry, so its final state is its own), and one whose rows are not resident stops the
 * pixel with walk_fault set (the call then fails). */
__global__ void __launch_bounds__(64)
k_stack_literal(SgStackParams p, SgChainTables t, unsigned int count, uint8_t *scratch, int phase) {
	const unsigned int nthreads = gridDim.x * blockDim.x;
	const unsigned int gid = blockIdx.x * blockDim.x + threadIdx.x;
	uint16_t *stack = (uint16_t *)(scratch + (size_t)gid * (((size_t)p.N * 5 + 15) & ~(size_t)15));
	uint16_t *wst = stack + p.N;
	int8_t *rejected = (int8_t *)(wst + p.N);
	if (!count) {	/* 0: take the queue length from the device counter */
		count = *p.flag_count;
		if (count > p.flag_cap)
			count = p.flag_cap;
	}
	for (unsigned int i = gid; i < count; i += nthreads) {
		const int64_t pix = p.flag_list[i];
		const int cls = sg_flag_get(p, pix);
		if (cls != (phase == 1 ? SG_CLS_LITERAL : SG_CLS_CHAIN))
			continue;	/* SG_CLS_DONE: finished by k_stack_replay */
		uint32_t crej[2] = {0, 0};
		int fbrk;
		if (p.method == 2) {	/* stack_median's pixel (:746-767): redo list of the histogram path */
			gather_stack(p, pix, stack);
			shellsort_u16(stack, p.N);
			p.out[pix] = (uint16_t)lit_median(stack, p.N);
			sg_flag_set(p, pix, SG_CLS_DONE);
			continue;
		}
		if (phase == 1) {
			for (int k = 0; k < p.N; k++)
				rejected[k] = 0;
		} else {
			/* walk back to the last pixel whose final rejected[] is self-determined */
			int64_t q = chain_pred(p, t, pix);
			bool fault = false;
			while (q >= 0) {
				if (chain_in_band(p, q)) {
					if (sg_flag_get(p, q) != SG_CLS_CHAIN && sg_flag_get(p, q) != SG_CLS_CHAIN_DONE)
						break;
				} else {
					if (!chain_resident(p, q)) {
						fault = true;
						break;
					}
					uint32_t dummy[2] = {0, 0};
					for (int k = 0; k < p.N; k++)
						rejected[k] = 0;
					gather_stack(p, q, stack);
					literal_pixel(stack, rejected, wst, p.N, p.rejection, p.sig0, p.sig1, dummy, &fbrk);
					if (!(fbrk == 1 && p.N > 4))
						break;
				}
				q = chain_pred(p, t, q);
			}
			if (fault) {
				*p.walk_fault = 1u;
				continue;
			}
			for (int k = 0; k < p.N; k++)
				rejected[k] = 0;
			int64_t cur;
			if (q >= 0) {
				uint32_t dummy[2] = {0, 0};
				gather_stack(p, q, stack);
				literal_pixel(stack, rejected, wst, p.N, p.rejection, p.sig0, p.sig1, dummy, &fbrk);
				cur = chain_succ(p, t, q);
			} else {
				/* start of the emulated thread's work: calloc'ed rejected[] */
				cur = pix;
				int64_t pr = chain_pred(p, t, cur);
				while (pr >= 0) {
					cur = pr;
					pr = chain_pred(p, t, cur);
				}
			}
			while (cur >= 0 && cur != pix) {
				uint32_t dummy[2] = {0, 0};
				gather_stack(p, cur, stack);
				literal_pixel(stack, rejected, wst, p.N, p.rejection, p.sig0, p.sig1, dummy, &fbrk);
				cur = chain_succ(p, t, cur);
			}
		}
		gather_stack(p, pix, stack);
		const uint16_t v = literal_pixel(stack, rejected, wst, p.N, p.rejection, p.sig0, p.sig1, crej, &fbrk);
		if (p.rejection == 3 && fbrk == 2)
			*p.loop_fault = 1u;
		if (phase == 1 && fbrk == 1 && p.N > 4) {
			sg_flag_set(p, pix, SG_CLS_CHAIN);
			continue;
		}
		p.out[pix] = v;
		/* finished: a second tail launch (after the host's late redo launch) skips it; a phase-2
		 * pixel stays a chain link for the other walks of this phase */
		sg_flag_set(p, pix, phase == 1 ? SG_CLS_DONE : SG_CLS_CHAIN_DONE);
		const int c = (int)(pix / ((int64_t)p.W * p.H));
		unsigned long long *sh = p.rej + ((size_t)(i % SG_REJ_SHARDS) * 6 + c * 2);
		if (crej[0])
			atomicAdd(sh, (unsigned long long)crej[0]);
		if (crej[1])
			atomicAdd(sh + 1, (unsigned long long)crej[1]);
	}
}

/* ----------------------------------------------------------------------------------
 * call plumbing without DMA: a stack call's inputs come from its pinned (host-mapped) staging
 * block and its counters go back into a host-mapped slot through these two kernels (an SDMA
 * copy's start-up cost ~20 us each way per call, profiles/r05b_band8)
 * ---------------------------------------------------------------------------------- */
__global__ void __launch_bounds__(256)
k_stage_copy(uint4 *__restrict__ dst, const uint4 *__restrict__ src, unsigned int n16) {
	for (unsigned int i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256)
		dst[i] = src[i];
}

/* host slot: rejection sums [3][2] u64 at 0, the flag block (flag / walk-fault / redo / compact
 * counts, loop fault, the SUM maximum at word 16) at byte 64; the device shards and flag words
 * 0..15 are zeroed for the slot's next call (the SUM maximum stays: a streamed SUM keeps it) */
__global__ void __launch_bounds__(256)
k_ctr_finalize(unsigned long long *__restrict__ ctr, unsigned long long *__restrict__ host) {
	__shared__ unsigned long long part[6][256];
	const int t = threadIdx.x;
	unsigned long long a[6] = {0, 0, 0, 0, 0, 0};
	for (int k = t; k < SG_REJ_SHARDS; k += 256)
#pragma unroll
		for (int j = 0; j < 6; j++) {
			a[j] += ctr[(size_t)k * 6 + j];
			ctr[(size_t)k * 6 + j] = 0ull;
		}
#pragma unroll
	for (int j = 0; j < 6; j++)
		part[j][t] = a[j];
	__syncthreads();
	for (int o = 128; o > 0; o >>= 1) {
		if (t < o)
#pragma unroll
			for (int j = 0; j < 6; j++)
				part[j][t] += part[j][t + o];
		__syncthreads();
	}
	unsigned int *fl = (unsigned int *)(ctr + (size_t)SG_REJ_SHARDS * 6);
	unsigned int *hf = (unsigned int *)(host + 8);
	if (t < 6)
		host[t] = part[t][0];
	if (t < 32) {
		const unsigned int v = fl[t];
		hf[t] = v;
		if (t < 16)
			fl[t] = 0u;
	}
}

/* ----------------------------------------------------------------------------------
 * synthetic generator (include/sg_synth.h) on the device
 * ---------------------------------------------------------------------------------- */
#include "../../include/sg_synth.h"

__global__ void __launch_bounds__(256)
k_synth_fill(uint16_t *frames, int first_frame, int nframes, int C, int H, int W, int row_begin, int row_end,
		uint64_t seed, int maxshift, int64_t frame_stride, int64_t plane_stride) {
	const int nrows = row_end - row_begin;
	const int64_t total = (int64_t)nframes * C * nrows * W;
	for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
			i += (int64_t)gridDim.x * blockDim.x) {
		const int x = (int)(i % W);
		int64_t t = i / W;
		const int rr = (int)(t % nrows);
		t /= nrows;
		const int c = (int)(t % C);
		const int f = (int)(t / C);
		const int R = row_begin + rr;
		frames[(int64_t)f * frame_stride + (int64_t)c * plane_stride + (int64_t)R * W + x] =
			sg_synth_pixel(seed, first_frame + f, c, R, x, maxshift);
	}
}

/* A/B diagnostics: print and clear the reason counters (SG_HIST_DBG=12) */
void sg_dbg_why_dump(hipStream_t s) {
	unsigned int h[32];
	if (hipMemcpyFromSymbolAsync(h, HIP_SYMBOL(g_sg_why), sizeof h, 0, hipMemcpyDeviceToHost, s) != hipSuccess)
		return;
	if (hipStreamSynchronize(s) != hipSuccess)
		return;
	fprintf(stderr, "sg why:");
	for (int k = 0; k < 32; k++)
		if (h[k])
			fprintf(stderr, " %d:%u", k, h[k]);
	fprintf(stderr, "\n");
	memset(h, 0, sizeof h);
	(void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sg_why), h, sizeof h, 0, hipMemcpyHostToDevice, s);
	unsigned long long r[16];
	if (hipMemcpyFromSymbolAsync(r, HIP_SYMBOL(g_sg_rprof), sizeof r, 0, hipMemcpyDeviceToHost, s) != hipSuccess ||
			hipStreamSynchronize(s) != hipSuccess)
		return;
	fprintf(stderr, "replay: %llu pixels, max cycles %llu (gather %llu, sort %llu), fp80 sd %llu (max %llu per pixel), "
			"passes %llu, max cycles without fp80 %llu\n", r[3], r[0], r[1], r[2], r[4], r[6], r[5], r[7]);
	if (r[3])
		fprintf(stderr, "replay means: total %llu gather %llu sort %llu fast %llu (max %llu), handovers %llu, max passes %llu\n",
				r[8] / r[3], r[9] / r[3], r[10] / r[3], r[11] / r[3], r[13], r[12], r[14]);
	memset(r, 0, sizeof r);
	(void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_sg_rprof), r, sizeof r, 0, hipMemcpyHostToDevice, s);
}
