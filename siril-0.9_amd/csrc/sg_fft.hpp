/*
 * sg_fft.hpp - device FFT building blocks of the DFT registration (sg_register.hip: power-of-
 * two sides, sg_register_gen.hip: any side): complex double arithmetic, in-register small DFTs,
 * Stockham auto-sort passes in LDS, the fused memory-in / memory-out transform, and the top-2
 * arg-max used to detect near ties of the correlation maximum.
 */
#pragma once
#include "sg_common.hpp"
#include <math.h>
#include <type_traits>

typedef double2 sg_c64;

__device__ __forceinline__ int sg_bitrev(int x, int logn) {
	return (int)(__brev((unsigned)x) >> (32 - logn));
}

/* ------------------------------------------------------------------------------------
 * nb independent length-n FFTs held in LDS (transform b at buf + b*bstride), natural order
 * in and out: Stockham auto-sort passes of radix 8 (then 4 / 2 for the remaining factor),
 * each thread taking whole radix-R butterflies in registers (a 2048-point transform is 4
 * LDS round trips instead of 11).  tw: see sg_twiddle; the inverse uses
 * conjugate twiddles (unnormalised, FFTW_BACKWARD).
 * ------------------------------------------------------------------------------------ */
/* LDS element index with one pad slot per 8 elements: the Stockham stores of the first
 * passes (stride 8 and 64 elements between neighbouring threads) would otherwise hit the
 * same banks 8- to 32-fold */
__device__ __forceinline__ int sg_pad(int i) {
	return i + (i >> 3);
}
#define SG_PADN(n) ((n) + ((n) >> 3))
/* element stride between the columns of a column-strip kernel (k_reg_cols, k_reg_cols_xpower):
 * float2 strips +4 so that the batch-minor passes (4 columns x 8 consecutive elements per 32-lane
 * group: the last FFT pass, the cross power, the inverse's first pass) and the first pass's
 * stores fall on distinct banks -- a bank model of the S = 2048 pass (64 banks for ds_read_b64,
 * 32 for ds_write_b64, MI355X_MICROARCH.md LDS) gives 1.54x the conflict-free LDS cycles against
 * 2.62x at +1, and SQ_LDS_BANK_CONFLICT of the pass was 2.05x its active LDS cycles
 * (profiles/r04r_sq_register_1.txt); double2 strips keep +1 */
template <class C>
__host__ __device__ constexpr int sg_col_stride(int S) {
	return SG_PADN(S) + (sizeof(C) == 8 ? 4 : 1);
}

/* complex arithmetic for C = double2 (the default, every path) or float2 (the fp32 power-of-two
 * passes, whose near ties are re-run in fp64) */
template <class C> struct SgReal;
template <> struct SgReal<double2> { typedef double T; };
template <> struct SgReal<float2> { typedef float T; };
template <class C>
__device__ __forceinline__ C sg_mk(typename SgReal<C>::T x, typename SgReal<C>::T y) {
	C r;
	r.x = x;
	r.y = y;
	return r;
}
template <class C>
__device__ __forceinline__ C sg_cmul(C a, C b) {
	return sg_mk<C>(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
template <class C>
__device__ __forceinline__ C sg_cadd(C a, C b) {
	return sg_mk<C>(a.x + b.x, a.y + b.y);
}
template <class C>
__device__ __forceinline__ C sg_csub(C a, C b) {
	return sg_mk<C>(a.x - b.x, a.y - b.y);
}
/* multiply by -i (forward) or +i (inverse) */
template <class C>
__device__ __forceinline__ C sg_mul_mi(C a, bool inv) {
	return inv ? sg_mk<C>(-a.y, a.x) : sg_mk<C>(a.y, -a.x);
}

/* in-register DFT of R = 2, 4, 8 points (natural order in and out) */
template <int R, int RV, class C>
__device__ __forceinline__ void sg_dft_small(C (&v)[RV], bool inv) {
	typedef typename SgReal<C>::T T;
	if constexpr (R == 2) {
		const C a = v[0], b = v[1];
		v[0] = sg_cadd(a, b);
		v[1] = sg_csub(a, b);
		return;
	}
	else if constexpr (R == 4) {
		const C a0 = sg_cadd(v[0], v[2]), a1 = sg_csub(v[0], v[2]);
		const C b0 = sg_cadd(v[1], v[3]), b1 = sg_mul_mi(sg_csub(v[1], v[3]), inv);
		v[0] = sg_cadd(a0, b0);
		v[2] = sg_csub(a0, b0);
		v[1] = sg_cadd(a1, b1);
		v[3] = sg_csub(a1, b1);
		return;
	} else {
	/* R = 8: radix-2 DIF into two 4-point DFTs */
	const T h = (T)0.70710678118654752440;
	C e[4], o[4];
#pragma unroll
	for (int k = 0; k < 4; k++) {
		e[k] = sg_cadd(v[k], v[k + 4]);
		o[k] = sg_csub(v[k], v[k + 4]);
	}
	/* o[k] *= W8^k */
	o[1] = inv ? sg_mk<C>(h * (o[1].x - o[1].y), h * (o[1].x + o[1].y))
		   : sg_mk<C>(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));
	o[2] = sg_mul_mi(o[2], inv);
	o[3] = inv ? sg_mk<C>(-h * (o[3].x + o[3].y), h * (o[3].x - o[3].y))
		   : sg_mk<C>(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));
	sg_dft_small<4>(e, inv);
	sg_dft_small<4>(o, inv);
	const C *E = e, *O = o;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		v[2 * k] = E[k];
		v[2 * k + 1] = O[k];
	}
	}
}

/* tw holds the full circle twice: tw[k] = exp(-2 pi i k / n) and tw[n + k] = its conjugate
 * (the inverse), k < n, built on the host from the half-circle values by exact negation /
 * conjugation, so a twiddle is one load with no select (the direction is uniform) */
template <class C>
__device__ __forceinline__ C sg_twiddle(const C *__restrict__ tw, int n, int k, bool inv) {
	return (inv ? tw + n : tw)[k];
}

/* log2 of a power of two (a uniform value: scalar code); the batched transforms of this file
 * have power-of-two n, batch counts nb and strides, so item indices split with shifts and masks
 * instead of the integer divisions (v_rcp / v_mul_hi sequences) a runtime divisor costs */
__device__ __forceinline__ int sg_log2(int x) {
	return __builtin_ctz((unsigned)x);
}

template <int R, int EPT = 8, class C>
__device__ __forceinline__ void sg_stockham_pass(C *buf, int n, int nb, int bstride, int Ns,
		const C *__restrict__ tw, bool inv) {
	constexpr int MAXI = EPT / R;	/* work items per thread: nb * n <= EPT * blockDim (host-sized launches) */
	const int per = n / R, items = nb * per, lper = sg_log2(per), lks = sg_log2(n / (Ns * R));
	C v[MAXI][R], w[MAXI][R];
	const bool twiddled = Ns > 1;	/* the first pass (Ns = 1) multiplies by w^0 = 1 only */
	/* load every item's R inputs before anyone stores (in-place pass); the twiddles are
	 * fetched here too, so their latency overlaps the barrier wait */
#pragma unroll
	for (int it = 0; it < MAXI; it++) {
		const int t = threadIdx.x + it * blockDim.x;
		if (t < items) {
			const int b = t >> lper, j = t & (per - 1);
			const C *x = buf + b * bstride;
#pragma unroll
			for (int r = 0; r < R; r++)
				v[it][r] = x[sg_pad(j + r * per)];
			if (twiddled) {
				const int jm = j & (Ns - 1);
				const int kstep = jm << lks;
#pragma unroll
				for (int r = 1; r < R; r++)
					w[it][r] = sg_twiddle(tw, n, r * kstep, inv);
			}
		}
	}
	__syncthreads();
#pragma unroll
	for (int it = 0; it < MAXI; it++) {
		const int t = threadIdx.x + it * blockDim.x;
		if (t < items) {
			const int b = t >> lper, j = t & (per - 1);
			const int jm = j & (Ns - 1);
			if (twiddled) {
#pragma unroll
				for (int r = 1; r < R; r++)
					v[it][r] = sg_cmul(v[it][r], w[it][r]);
			}
			sg_dft_small<R, R>(v[it], inv);
			C *y = buf + b * bstride;
			const int base = (j - jm) * R + jm;
#pragma unroll
			for (int r = 0; r < R; r++)
				y[sg_pad(base + r * Ns)] = v[it][r];
		}
	}
	__syncthreads();
}

template <int EPT = 8, class C>
__device__ __forceinline__ void sg_lds_fft(C *buf, int n, int logn, int nb, int bstride, const C *__restrict__ tw,
		bool inverse) {
	(void)logn;
	__syncthreads();
	int Ns = 1;
	while (Ns < n) {
		const int rem = n / Ns;
		if (rem >= 8) {
			sg_stockham_pass<8, EPT>(buf, n, nb, bstride, Ns, tw, inverse);
			Ns *= 8;
		} else if (rem == 4) {
			sg_stockham_pass<4, EPT>(buf, n, nb, bstride, Ns, tw, inverse);
			Ns *= 4;
		} else {
			sg_stockham_pass<2, EPT>(buf, n, nb, bstride, Ns, tw, inverse);
			Ns *= 2;
		}
	}
}

/* The same transform with its first pass reading the input straight from memory and its
 * last pass writing the output straight to memory (ld(b, i) / st(b, i, v): element i of
 * transform b): two LDS round trips and four barriers fewer than staging through LDS.
 * Work items of these two passes are batch-minor (item t -> b = t % nb), so neighbouring
 * lanes of a column strip touch neighbouring columns of one row (64-B row segments).
 * The arithmetic is that of sg_lds_fft, operation for operation (n < 16, a single pass:
 * staged through LDS). */
/* LDS_IN: ld reads this same LDS buffer (element i of transform b at its padded slot), so
 * the first pass loads everything before anyone stores.  A st that writes element i back
 * to its own slot is race-free as is: the last pass's thread reads exactly the slots it
 * writes. */
template <int EPT, class C, class ST>
__device__ __forceinline__ void sg_fft_io_regs(C *buf, int n, int nb, int bstride, const C *__restrict__ tw,
		bool inv, C (&v)[EPT / 8][8], ST st);
template <bool LDS_IN = false, int EPT = 8, class C, class LD, class ST>
__device__ __forceinline__ void sg_fft_io(C *buf, int n, int nb, int bstride, const C *__restrict__ tw,
		bool inv, LD ld, ST st) {
	if (n < 16) {
		for (int t = threadIdx.x; t < nb * n; t += blockDim.x)
			buf[(size_t)(t % nb) * bstride + sg_pad(t / nb)] = ld(t % nb, t / nb);
		sg_lds_fft<EPT>(buf, n, 0, nb, bstride, tw, inv);
		for (int t = threadIdx.x; t < nb * n; t += blockDim.x)
			st(t % nb, t / nb, buf[(size_t)(t % nb) * bstride + sg_pad(t / nb)]);
		return;
	}
	/* first pass: radix 8, Ns = 1 (no twiddles); EPT / 8 items per thread, all loaded before
	 * any is stored */
	constexpr int FI = EPT / 8;
	C v[FI][8];
	{
		const int per = n >> 3, items = nb * per, lnb = sg_log2(nb);
#pragma unroll
		for (int it = 0; it < FI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			if (t < items) {
				const int b = t & (nb - 1), j = t >> lnb;
#pragma unroll
				for (int r = 0; r < 8; r++)
					v[it][r] = ld(b, j + r * per);
			}
		}
	}
	if (LDS_IN)
		__syncthreads();
	sg_fft_io_regs<EPT>(buf, n, nb, bstride, tw, inv, v, st);
}

/* sg_fft_io from its first pass's inputs already in registers (n >= 16): v[it][r] = element
 * j + r n / 8 of transform b, item t = threadIdx.x + it blockDim, b = t % nb, j = t / nb; a
 * caller that loads them ahead (the next row's, during this row's transform) hides the load
 * latency */
template <int EPT, class C, class ST>
__device__ __forceinline__ void sg_fft_io_regs(C *buf, int n, int nb, int bstride, const C *__restrict__ tw,
		bool inv, C (&v)[EPT / 8][8], ST st) {
	{
		constexpr int FI = EPT / 8;
		const int per = n >> 3, items = nb * per, lnb = sg_log2(nb);
#pragma unroll
		for (int it = 0; it < FI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			if (t < items) {
				const int b = t & (nb - 1), j = t >> lnb;
				sg_dft_small<8, 8>(v[it], inv);
				C *y = buf + b * bstride;
#pragma unroll
				for (int r = 0; r < 8; r++)
					y[sg_pad(j * 8 + r)] = v[it][r];
			}
		}
	}
	__syncthreads();
	int Ns = 8;
	/* middle passes in LDS (sg_lds_fft's radix sequence: 8 while n / Ns >= 8, then 4 or 2),
	 * leaving the last one */
	while (n / Ns > 8) {
		sg_stockham_pass<8, EPT>(buf, n, nb, bstride, Ns, tw, inv);
		Ns *= 8;
	}
	const int rl = n / Ns;
	auto last = [&](auto RC) {
		constexpr int R = decltype(RC)::value;
		constexpr int MAXI = EPT / R;
		const int per = n / R, items = nb * per, lnb = sg_log2(nb);
#pragma unroll
		for (int it = 0; it < MAXI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			if (t < items) {
				const int b = t & (nb - 1), j = t >> lnb;
				const C *x = buf + b * bstride;
				C v[R];
#pragma unroll
				for (int r = 0; r < R; r++)
					v[r] = x[sg_pad(j + r * per)];
#pragma unroll
				for (int r = 1; r < R; r++)
					v[r] = sg_cmul(v[r], sg_twiddle(tw, n, r * j, inv));
				sg_dft_small<R, R>(v, inv);
#pragma unroll
				for (int r = 0; r < R; r++)
					st(b, j + r * per, v[r]);
			}
		}
	};
	if (rl == 8)
		last(std::integral_constant<int, 8>());
	else if (rl == 4)
		last(std::integral_constant<int, 4>());
	else
		last(std::integral_constant<int, 2>());
}


/* ---------------------------------------------------------------------------------------
 * top-2 arg-max: the best (value, index) -- larger value, ties -> lower index, the
 * reference's first strict maximum (registration.c:337-343) -- and the best value at any
 * OTHER index.  Partials cover disjoint index sets, so merging keeps both exact.
 * ------------------------------------------------------------------------------------- */
struct SgTop2 {
	double v, v2;
	int i, pad;
};

__device__ __forceinline__ void sg_top2_init(SgTop2 &t) {
	t.v = -INFINITY;
	t.v2 = -INFINITY;
	t.i = 0x7fffffff;
	t.pad = 0;
}

__device__ __forceinline__ void sg_top2_merge(SgTop2 &a, double v, double v2, int i) {
	if (v > a.v || (v == a.v && i < a.i)) {
		a.v2 = fmax(a.v, v2);
		a.v = v;
		a.i = i;
	} else {
		a.v2 = fmax(a.v2, v);
	}
}

__device__ __forceinline__ void sg_top2_add(SgTop2 &a, double v, int i) {
	sg_top2_merge(a, v, -INFINITY, i);
}

__device__ __forceinline__ void sg_top2_wave(SgTop2 &a) {
	for (int o = 32; o > 0; o >>= 1) {
		const double v = __shfl_down(a.v, o, 64), v2 = __shfl_down(a.v2, o, 64);
		const int i = __shfl_down(a.i, o, 64);
		sg_top2_merge(a, v, v2, i);
	}
}

/* a thread's own top-2 in the precision of its transform (float for the fp32 passes: the
 * comparisons are those of the exactly converted doubles), branch-free: the update of
 * sg_top2_add as selects instead of a divergent branch per element; widened to SgTop2 for the
 * block reduction */
template <class T> struct SgTop2T {
	T v, v2;
	int i;
};
template <class T>
__device__ __forceinline__ void sg_top2t_init(SgTop2T<T> &t) {
	t.v = -INFINITY;
	t.v2 = -INFINITY;
	t.i = 0x7fffffff;
}
template <class T>
__device__ __forceinline__ void sg_top2t_add(SgTop2T<T> &a, T v, int i) {
	const bool nb = v > a.v || (v == a.v && i < a.i);
	a.v2 = nb ? a.v : fmax(a.v2, v);
	a.v = nb ? v : a.v;
	a.i = nb ? i : a.i;
}
/* the same for a thread that visits its indices in increasing order: an equal value never
 * carries a lower index, so the index tie-break drops out */
template <class T>
__device__ __forceinline__ void sg_top2t_add_inc(SgTop2T<T> &a, T v, int i) {
	const bool nb = v > a.v;
	a.v2 = nb ? a.v : fmax(a.v2, v);
	a.v = nb ? v : a.v;
	a.i = nb ? i : a.i;
}
/* sg_top2_merge / sg_top2_wave in the transform's precision (float: 3 dword shuffles per step
 * instead of 5; the same comparisons as on the exactly widened doubles) */
template <class T>
__device__ __forceinline__ void sg_top2t_merge(SgTop2T<T> &a, T v, T v2, int i) {
	const bool nb = v > a.v || (v == a.v && i < a.i);
	a.v2 = nb ? fmax(a.v, v2) : fmax(a.v2, v);
	a.v = nb ? v : a.v;
	a.i = nb ? i : a.i;
}
template <class T>
__device__ __forceinline__ void sg_top2t_wave(SgTop2T<T> &a) {
	for (int o = 32; o > 0; o >>= 1) {
		const T v = __shfl_down(a.v, o, 64), v2 = __shfl_down(a.v2, o, 64);
		const int i = __shfl_down(a.i, o, 64);
		sg_top2t_merge(a, v, v2, i);
	}
}
template <class T>
__device__ __forceinline__ SgTop2 sg_top2t_wide(const SgTop2T<T> &a) {
	SgTop2 t;
	t.v = (double)a.v;
	t.v2 = (double)a.v2;
	t.i = a.i;
	t.pad = 0;
	return t;
}

/* per-pair arg-max partial of the two frames a (real part) and b (imaginary part) */
struct SgBest {
	SgTop2 a, b;
};

/* block reduction of a and b; thread 0 returns the block's result in (a, b).  `sh` holds 16
 * waves' partials. */
__device__ __forceinline__ void sg_best_block(SgTop2 &a, SgTop2 &b, SgBest *sh) {
	sg_top2_wave(a);
	sg_top2_wave(b);
	const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		sh[wave].a = a;
		sh[wave].b = b;
	}
	__syncthreads();
	if (threadIdx.x == 0)
		for (int w = 1; w < nw; w++) {
			sg_top2_merge(a, sh[w].a.v, sh[w].a.v2, sh[w].a.i);
			sg_top2_merge(b, sh[w].b.v, sh[w].b.v2, sh[w].b.i);
		}
}

/* sum of squares of one row of a (and b) into the frames' energies */
__device__ __forceinline__ void sg_energy_add(unsigned long long ea, unsigned long long eb, int fa, int fb,
		unsigned long long *energy) {
	__shared__ unsigned long long se[2][16];
	for (int o = 32; o > 0; o >>= 1) {
		ea += __shfl_down(ea, o, 64);
		eb += __shfl_down(eb, o, 64);
	}
	const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		se[0][wave] = ea;
		se[1][wave] = eb;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < nw; w++) {
			ea += se[0][w];
			eb += se[1][w];
		}
		atomicAdd(energy + fa, ea);
		if (fb >= 0)
			atomicAdd(energy + fb, eb);
	}
}


/* candidates of a near tie: the indices whose FFT correlation reaches max - tol, for an exact
 * integer recomputation (k_reg_exact); capped, an overflow leaves the frame unresolved */
#define SG_CAND_CAP 64
struct SgCand {
	unsigned int count;
	int idx[SG_CAND_CAP];
	long long exact[SG_CAND_CAP];
};

__device__ __forceinline__ void sg_cand_push(SgCand *c, double v, double thr, int idx) {
	if (v >= thr) {
		const unsigned int k = atomicAdd(&c->count, 1u);
		if (k < SG_CAND_CAP)
			c->idx[k] = idx;
	}
}
