/*
 * sg_register.hip - gfx950 DFT registration (replaces register_shift_dft,
 * src/registration/registration.c:182-400) and the planetary quality estimate it records
 * (QualityEstimate, src/algos/quality.c:46-349; normalizeQualityData registration.c:163-176).
 *
 * Per frame the reference computes, with FFTW in complex double,
 *     c = IFFT2( FFT2(ref) * conj(FFT2(img)) )      (unnormalised, FFTW_BACKWARD)
 * and takes the first strict maximum of creal(c) in row-major order (:337-351).  Here:
 *   - frames go through the 2-D FFT two at a time, packed as a + i b (both are real), and
 *     their spectra are separated with F_a(k) = (Z(k) + conj Z(-k))/2,
 *     F_b(k) = (Z(k) - conj Z(-k))/2i;
 *   - the two cross-power spectra are packed back as P = R conj F_a + i R conj F_b, whose
 *     inverse is c_a + i c_b (both correlations are real): one forward and one inverse
 *     complex 2-D FFT per PAIR of frames;
 *   - FFTs are radix-2 in LDS in double precision (rows: one workgroup per row; columns:
 *     one workgroup per strip of CW columns), twiddles from a host table;
 *   - the inverse row pass fuses the per-row arg-max (first index on ties), a tiny kernel
 *     reduces the rows in order.
 * Only the arg-max leaves the device, so results equal the reference wherever the top two
 * correlation values are separated by more than the FFT rounding of either side (the exact
 * correlations are integers; FFTW's own choice between exactly tied integers is not
 * specified — "parity unpinned" there).  S must be a power of two.
 */
#include "sg_common.hpp"
#include "sg_ctx.hpp"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include <vector>

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

__device__ __forceinline__ sg_c64 sg_cmul(sg_c64 a, sg_c64 b) {
	return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ sg_c64 sg_cadd(sg_c64 a, sg_c64 b) {
	return make_double2(a.x + b.x, a.y + b.y);
}
__device__ __forceinline__ sg_c64 sg_csub(sg_c64 a, sg_c64 b) {
	return make_double2(a.x - b.x, a.y - b.y);
}
/* multiply by -i (forward) or +i (inverse) */
__device__ __forceinline__ sg_c64 sg_mul_mi(sg_c64 a, bool inv) {
	return inv ? make_double2(-a.y, a.x) : make_double2(a.y, -a.x);
}

/* in-register DFT of R = 2, 4, 8 points (natural order in and out) */
template <int R, int RV>
__device__ __forceinline__ void sg_dft_small(sg_c64 (&v)[RV], bool inv) {
	if constexpr (R == 2) {
		const sg_c64 a = v[0], b = v[1];
		v[0] = sg_cadd(a, b);
		v[1] = sg_csub(a, b);
		return;
	}
	else if constexpr (R == 4) {
		const sg_c64 a0 = sg_cadd(v[0], v[2]), a1 = sg_csub(v[0], v[2]);
		const sg_c64 b0 = sg_cadd(v[1], v[3]), b1 = sg_mul_mi(sg_csub(v[1], v[3]), inv);
		v[0] = sg_cadd(a0, b0);
		v[2] = sg_csub(a0, b0);
		v[1] = sg_cadd(a1, b1);
		v[3] = sg_csub(a1, b1);
		return;
	} else {
	/* R = 8: radix-2 DIF into two 4-point DFTs */
	const double h = 0.70710678118654752440;
	sg_c64 e[4], o[4];
#pragma unroll
	for (int k = 0; k < 4; k++) {
		e[k] = sg_cadd(v[k], v[k + 4]);
		o[k] = sg_csub(v[k], v[k + 4]);
	}
	/* o[k] *= W8^k */
	o[1] = inv ? make_double2(h * (o[1].x - o[1].y), h * (o[1].x + o[1].y))
		   : make_double2(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));
	o[2] = sg_mul_mi(o[2], inv);
	o[3] = inv ? make_double2(-h * (o[3].x + o[3].y), h * (o[3].x - o[3].y))
		   : make_double2(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));
	sg_dft_small<4>(e, inv);
	sg_dft_small<4>(o, inv);
	const sg_c64 *E = e, *O = o;
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
__device__ __forceinline__ sg_c64 sg_twiddle(const sg_c64 *__restrict__ tw, int n, int k, bool inv) {
	return (inv ? tw + n : tw)[k];
}

template <int R>
__device__ __forceinline__ void sg_stockham_pass(sg_c64 *buf, int n, int nb, int bstride, int Ns,
		const sg_c64 *__restrict__ tw, bool inv) {
	constexpr int MAXI = 8 / R;	/* work items per thread: nb * n <= 8 * blockDim (host-sized launches) */
	const int per = n / R, items = nb * per;
	sg_c64 v[MAXI][R], w[MAXI][R];
	const bool twiddled = Ns > 1;	/* the first pass (Ns = 1) multiplies by w^0 = 1 only */
	/* load every item's R inputs before anyone stores (in-place pass); the twiddles are
	 * fetched here too, so their latency overlaps the barrier wait */
#pragma unroll
	for (int it = 0; it < MAXI; it++) {
		const int t = threadIdx.x + it * blockDim.x;
		if (t < items) {
			const int b = t / per, j = t - b * per;
			const sg_c64 *x = buf + (size_t)b * bstride;
#pragma unroll
			for (int r = 0; r < R; r++)
				v[it][r] = x[sg_pad(j + r * per)];
			if (twiddled) {
				const int jm = j & (Ns - 1);
				const int kstep = jm * (n / (Ns * R));
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
			const int b = t / per, j = t - b * per;
			const int jm = j & (Ns - 1);
			if (twiddled) {
#pragma unroll
				for (int r = 1; r < R; r++)
					v[it][r] = sg_cmul(v[it][r], w[it][r]);
			}
			sg_dft_small<R, R>(v[it], inv);
			sg_c64 *y = buf + (size_t)b * bstride;
			const int base = (j - jm) * R + jm;
#pragma unroll
			for (int r = 0; r < R; r++)
				y[sg_pad(base + r * Ns)] = v[it][r];
		}
	}
	__syncthreads();
}

__device__ __forceinline__ void sg_lds_fft(sg_c64 *buf, int n, int logn, int nb, int bstride, const sg_c64 *__restrict__ tw,
		bool inverse) {
	(void)logn;
	__syncthreads();
	int Ns = 1;
	while (Ns < n) {
		const int rem = n / Ns;
		if (rem >= 8) {
			sg_stockham_pass<8>(buf, n, nb, bstride, Ns, tw, inverse);
			Ns *= 8;
		} else if (rem == 4) {
			sg_stockham_pass<4>(buf, n, nb, bstride, Ns, tw, inverse);
			Ns *= 4;
		} else {
			sg_stockham_pass<2>(buf, n, nb, bstride, Ns, tw, inverse);
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
template <bool LDS_IN = false, class LD, class ST>
__device__ __forceinline__ void sg_fft_io(sg_c64 *buf, int n, int nb, int bstride, const sg_c64 *__restrict__ tw,
		bool inv, LD ld, ST st) {
	if (n < 16) {
		for (int t = threadIdx.x; t < nb * n; t += blockDim.x)
			buf[(size_t)(t % nb) * bstride + sg_pad(t / nb)] = ld(t % nb, t / nb);
		sg_lds_fft(buf, n, 0, nb, bstride, tw, inv);
		for (int t = threadIdx.x; t < nb * n; t += blockDim.x)
			st(t % nb, t / nb, buf[(size_t)(t % nb) * bstride + sg_pad(t / nb)]);
		return;
	}
	/* first pass: radix 8, Ns = 1 (no twiddles) */
	{
		const int per = n >> 3, items = nb * per;
		const int t = threadIdx.x;
		const bool act = t < items;
		const int b = act ? t % nb : 0, j = act ? t / nb : 0;
		sg_c64 v[8];
		if (act) {
#pragma unroll
			for (int r = 0; r < 8; r++)
				v[r] = ld(b, j + r * per);
		}
		if (LDS_IN)
			__syncthreads();
		if (act) {
			sg_dft_small<8, 8>(v, inv);
			sg_c64 *y = buf + (size_t)b * bstride;
#pragma unroll
			for (int r = 0; r < 8; r++)
				y[sg_pad(j * 8 + r)] = v[r];
		}
	}
	__syncthreads();
	int Ns = 8;
	/* middle passes in LDS (sg_lds_fft's radix sequence: 8 while n / Ns >= 8, then 4 or 2),
	 * leaving the last one */
	while (n / Ns > 8) {
		sg_stockham_pass<8>(buf, n, nb, bstride, Ns, tw, inv);
		Ns *= 8;
	}
	const int rl = n / Ns;
	auto last = [&](auto RC) {
		constexpr int R = decltype(RC)::value;
		constexpr int MAXI = 8 / R;
		const int per = n / R, items = nb * per;
#pragma unroll
		for (int it = 0; it < MAXI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			if (t < items) {
				const int b = t % nb, j = t / nb;
				const sg_c64 *x = buf + (size_t)b * bstride;
				sg_c64 v[R];
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

/* row pass of the forward transform of a + i b (b = -1: zero imaginary part) */
__global__ void __launch_bounds__(512)
k_reg_rows_fwd(const uint16_t *__restrict__ sel, const int *__restrict__ fa, const int *__restrict__ fb,
		int S, int logS, const sg_c64 *__restrict__ tw, sg_c64 *__restrict__ work) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	const int row = blockIdx.x, pair = blockIdx.y;
	const size_t plane = (size_t)S * S;
	const uint16_t *pa = sel + (size_t)fa[pair] * plane + (size_t)row * S;
	const int b = fb[pair];
	const uint16_t *pb = b >= 0 ? sel + (size_t)b * plane + (size_t)row * S : nullptr;
	sg_c64 *out = work + (size_t)pair * plane + (size_t)row * S;
	(void)logS;
	sg_fft_io(buf, S, 1, S, tw, false,
			[&](int, int i) { return make_double2((double)pa[i], pb ? (double)pb[i] : 0.0); },
			[&](int, int i, sg_c64 v) { out[i] = v; });
}

/* strip of workgroup `id` out of n: the dispatcher deals workgroups round-robin over the 8
 * XCDs, so neighbouring strips (which share 128-B lines: a strip row is 64 B) would be
 * fetched by two L2s; give each XCD a contiguous range of strips instead (PMC FETCH_SIZE
 * of the column passes halves) */
__device__ __forceinline__ int sg_xcd_strip(int id, int n, int xcdmap) {
	if (!xcdmap || (n & 7))
		return id;
	return (id & 7) * (n >> 3) + (id >> 3);
}

/* column pass (forward or inverse) over strips of CW adjacent columns */
__global__ void __launch_bounds__(1024)
k_reg_cols(sg_c64 *__restrict__ work, int S, int logS, int CW, const sg_c64 *__restrict__ tw, int inverse,
		int xcdmap) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	const int x0 = sg_xcd_strip(blockIdx.x, gridDim.x, xcdmap) * CW, pair = blockIdx.y;
	const int bstride = SG_PADN(S) + 1;
	sg_c64 *base = work + (size_t)pair * S * S + x0;
	(void)logS;
	sg_fft_io(buf, S, CW, bstride, tw, inverse != 0, [&](int c, int r) { return base[(size_t)r * S + c]; },
			[&](int c, int r, sg_c64 v) { base[(size_t)r * S + c] = v; });
}

/* one term of the packed cross-power spectrum at (ky, kx): zk = Z(ky, kx),
 * zm = Z(-ky, -kx), rk = R(ky, kx).  F_a = (zk + conj zm) / 2, F_b = (zk - conj zm) / 2i;
 * result R conj F_a + i R conj F_b.  The term at (-ky, -kx) is this function with zk and
 * zm swapped (the negated differences are exact, products and sums commute), so every
 * element is formed by the same expression. */
__device__ __forceinline__ sg_c64 sg_xpower_at(sg_c64 zk, sg_c64 zm, sg_c64 rk) {
	const double ar = 0.5 * (zk.x + zm.x), ai = 0.5 * (zk.y - zm.y);
	const double br = 0.5 * (zk.y + zm.y), bi = -0.5 * (zk.x - zm.x);
	const double pr = rk.x * ar + rk.y * ai, pi = rk.y * ar - rk.x * ai;
	const double qr = rk.x * br + rk.y * bi, qi = rk.y * br - rk.x * bi;
	return make_double2(pr - qi, pi + qr);
}

/* separate the packed spectra and form the packed cross-power spectrum, in place:
 * each (k, -k) pair is handled by the thread of the smaller linear index */
__global__ void __launch_bounds__(256)
k_reg_xpower(sg_c64 *__restrict__ work, const sg_c64 *__restrict__ spec, int S) {
	const size_t plane = (size_t)S * S;
	sg_c64 *Z = work + (size_t)blockIdx.y * plane;
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < plane; i += (size_t)gridDim.x * blockDim.x) {
		const int ky = (int)(i / S), kx = (int)(i - (size_t)ky * S);
		const int my = (S - ky) & (S - 1), mx = (S - kx) & (S - 1);
		const size_t m = (size_t)my * S + mx;
		if (m < i)
			continue;
		const sg_c64 zk = Z[i], zm = Z[m];
		/* F_a(k) = (Z(k) + conj Z(-k))/2, F_b(k) = (Z(k) - conj Z(-k))/(2i) */
		const double ar = 0.5 * (zk.x + zm.x), ai = 0.5 * (zk.y - zm.y);
		const double br = 0.5 * (zk.y + zm.y), bi = -0.5 * (zk.x - zm.x);
		const sg_c64 rk = spec[i], rm = spec[m];
		/* P(k) = R(k) conj F_a(k) + i R(k) conj F_b(k) */
		{
			const double pr = rk.x * ar + rk.y * ai, pi = rk.y * ar - rk.x * ai;	/* R conj(Fa) */
			const double qr = rk.x * br + rk.y * bi, qi = rk.y * br - rk.x * bi;	/* R conj(Fb) */
			Z[i] = make_double2(pr - qi, pi + qr);
		}
		if (m != i) {
			/* F_a(-k) = conj F_a(k), F_b(-k) = conj F_b(k): P(-k) = R(-k) F_a + i R(-k) F_b */
			const double pr = rm.x * ar - rm.y * ai, pi = rm.x * ai + rm.y * ar;
			const double qr = rm.x * br - rm.y * bi, qi = rm.x * bi + rm.y * br;
			Z[m] = make_double2(pr - qi, pi + qr);
		}
	}
}

/* cross-power fused into the inverse ROW pass: workgroup (ky, pair) transforms rows ky
 * and -ky (mod S) together (the rows whose cross-power terms need each other): the first
 * FFT pass forms each term from the forward spectrum and the reference spectrum as it
 * reads them (sg_xpower_at), the last writes the inverse rows back in place.  The
 * inverse column pass then only reads (k_reg_cols_inv_argmax). */
__global__ void __launch_bounds__(1024)
k_reg_xpower_rows_inv(sg_c64 *__restrict__ work, const sg_c64 *__restrict__ spec, int S, int logS,
		const sg_c64 *__restrict__ tw) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	const int ky = blockIdx.x, pair = blockIdx.y;
	const int my = (S - ky) & (S - 1);
	const bool self = my == ky;
	sg_c64 *Z = work + (size_t)pair * S * S;
	const sg_c64 *Rs = spec;
	(void)logS;
	/* element i of row `row` (its mirror row `mrow`): the cross-power term as
	 * sg_xpower_at forms it, read straight from memory by the first FFT pass */
	sg_fft_io(buf, S, self ? 1 : 2, SG_PADN(S), tw, true,
			[&](int b, int i) {
				const int rw = b ? my : ky, mr = b ? ky : my;
				return sg_xpower_at(Z[(size_t)rw * S + i], Z[(size_t)mr * S + ((S - i) & (S - 1))],
						Rs[(size_t)rw * S + i]);
			},
			[&](int b, int i, sg_c64 v) { Z[(size_t)(b ? my : ky) * S + i] = v; });
}

/* better (value, index): larger value, ties -> lower index (first strict max, :337-343) */
__device__ __forceinline__ void sg_argmax_merge(double &v, int &i, double v2, int i2) {
	if (v2 > v || (v2 == v && i2 < i)) {
		v = v2;
		i = i2;
	}
}

struct SgBest {
	double va, vb;
	int ia, ib;
};

/* inverse row pass fused with the per-row arg-max of the real (frame a) and imaginary
 * (frame b) parts */
__global__ void __launch_bounds__(512)
k_reg_rows_inv_argmax(const sg_c64 *__restrict__ work, int S, int logS, const sg_c64 *__restrict__ tw,
		SgBest *__restrict__ best) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	__shared__ double rv[2][8];
	__shared__ int ri[2][8];
	const int row = blockIdx.x, pair = blockIdx.y;
	const sg_c64 *in = work + (size_t)pair * S * S + (size_t)row * S;
	double va = -INFINITY, vb = -INFINITY;
	int ia = 0x7fffffff, ib = 0x7fffffff;
	(void)logS;
	sg_fft_io(buf, S, 1, S, tw, true, [&](int, int j) { return in[j]; },
			[&](int, int j, sg_c64 c) {
				const int idx = row * S + j;
				sg_argmax_merge(va, ia, c.x, idx);
				sg_argmax_merge(vb, ib, c.y, idx);
			});
	for (int o = 32; o > 0; o >>= 1) {
		const double va2 = __shfl_down(va, o, 64), vb2 = __shfl_down(vb, o, 64);
		const int ia2 = __shfl_down(ia, o, 64), ib2 = __shfl_down(ib, o, 64);
		sg_argmax_merge(va, ia, va2, ia2);
		sg_argmax_merge(vb, ib, vb2, ib2);
	}
	const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		rv[0][wave] = va;
		ri[0][wave] = ia;
		rv[1][wave] = vb;
		ri[1][wave] = ib;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < nw; w++) {
			sg_argmax_merge(va, ia, rv[0][w], ri[0][w]);
			sg_argmax_merge(vb, ib, rv[1][w], ri[1][w]);
		}
		SgBest r;
		r.va = va;
		r.ia = ia;
		r.vb = vb;
		r.ib = ib;
		best[(size_t)pair * S + row] = r;
	}
}

/* inverse column pass fused with the arg-max of the real (frame a) and imaginary (frame b)
 * parts over the strip: nothing is written back */
__global__ void __launch_bounds__(1024)
k_reg_cols_inv_argmax(const sg_c64 *__restrict__ work, int S, int logS, int CW, const sg_c64 *__restrict__ tw,
		SgBest *__restrict__ best, int xcdmap) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	__shared__ double rv[2][16];
	__shared__ int ri[2][16];
	const int strip = sg_xcd_strip(blockIdx.x, gridDim.x, xcdmap);
	const int x0 = strip * CW, pair = blockIdx.y;
	const int bstride = SG_PADN(S) + 1;
	const sg_c64 *base = work + (size_t)pair * S * S + x0;
	double va = -INFINITY, vb = -INFINITY;
	int ia = 0x7fffffff, ib = 0x7fffffff;
	(void)logS;
	sg_fft_io(buf, S, CW, bstride, tw, true, [&](int c, int r) { return base[(size_t)r * S + c]; },
			[&](int c, int r, sg_c64 v) {
				const int lin = r * S + x0 + c;
				sg_argmax_merge(va, ia, v.x, lin);
				sg_argmax_merge(vb, ib, v.y, lin);
			});
	for (int o = 32; o > 0; o >>= 1) {
		const double va2 = __shfl_down(va, o, 64), vb2 = __shfl_down(vb, o, 64);
		const int ia2 = __shfl_down(ia, o, 64), ib2 = __shfl_down(ib, o, 64);
		sg_argmax_merge(va, ia, va2, ia2);
		sg_argmax_merge(vb, ib, vb2, ib2);
	}
	const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		rv[0][wave] = va;
		ri[0][wave] = ia;
		rv[1][wave] = vb;
		ri[1][wave] = ib;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < nw; w++) {
			sg_argmax_merge(va, ia, rv[0][w], ri[0][w]);
			sg_argmax_merge(vb, ib, rv[1][w], ri[1][w]);
		}
		SgBest r;
		r.va = va;
		r.ia = ia;
		r.vb = vb;
		r.ib = ib;
		best[(size_t)pair * gridDim.x + strip] = r;
	}
}

/* ---------------------------------------------------------------------------------------
 * Half-spectrum pass order (default): three plane passes per pair instead of four.
 *   1. k_reg_rows_fwd_half: row FFT of a + i b, separated per row into the row spectra of
 *      the two real frames, A(kx) = (z(kx) + conj z(-kx))/2, B(kx) = (z(kx) - conj z(-kx))/2i,
 *      of which kx in [0, S/2] is kept (Hermitian rows).  A(0) and A(S/2) are real, so
 *      column 0 packs A(0) + i A(S/2).  Layout of a pair plane row: [A' | B'], S/2 + S/2.
 *   2. k_reg_cols_xpower: per column (of A' or B'), forward column FFT, cross-power with
 *      the reference's column (R conj F), inverse column FFT: the cross-power needs no
 *      mirrored column any more, so the forward and inverse column passes fuse.  Column 0
 *      of each half holds two real sequences and is separated / re-packed over (ky, -ky),
 *      which lie in the same column.
 *   3. k_reg_rows_inv_half_argmax: the inverse column output is Hermitian in kx (the
 *      correlation is real), so each row's full spectrum is rebuilt from kx <= S/2, the
 *      two frames packed as Qa + i Qb, inverse row FFT -> c_a + i c_b, arg-max fused.
 * Same unnormalised FFTW_BACKWARD result as the full complex transforms; plane traffic per
 * pair 84 B per pixel instead of 116.
 * ------------------------------------------------------------------------------------- */
__global__ void __launch_bounds__(512)
k_reg_rows_fwd_half(const uint16_t *__restrict__ sel, const int *__restrict__ fa, const int *__restrict__ fb,
		int S, const sg_c64 *__restrict__ tw, sg_c64 *__restrict__ work) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	const int row = blockIdx.x, pair = blockIdx.y, H = S >> 1;
	const size_t plane = (size_t)S * S;
	const uint16_t *pa = sel + (size_t)fa[pair] * plane + (size_t)row * S;
	const int b = fb[pair];
	const uint16_t *pb = b >= 0 ? sel + (size_t)b * plane + (size_t)row * S : nullptr;
	sg_c64 *out = work + (size_t)pair * plane + (size_t)row * S;
	sg_fft_io(buf, S, 1, S, tw, false,
			[&](int, int i) { return make_double2((double)pa[i], pb ? (double)pb[i] : 0.0); },
			[&](int, int i, sg_c64 v) { buf[sg_pad(i)] = v; });
	__syncthreads();
	for (int k = threadIdx.x; k < H; k += blockDim.x) {
		const sg_c64 zk = buf[sg_pad(k)], zm = buf[sg_pad(k ? S - k : H)];
		sg_c64 A, B;
		if (k == 0) {
			A = make_double2(zk.x, zm.x);	/* A(0) + i A(S/2) */
			B = make_double2(zk.y, zm.y);
		} else {
			A = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
			B = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
		}
		out[k] = A;
		out[H + k] = B;
	}
}

/* R conj F */
__device__ __forceinline__ sg_c64 sg_rconj(sg_c64 r, sg_c64 f) {
	return make_double2(r.x * f.x + r.y * f.y, r.y * f.x - r.x * f.y);
}

/* The reference-spectrum loads of all 8 cross-power items of a thread are issued together
 * (launches are sized so that CW * S = 8 * blockDim, thr_for).  Issuing them before the
 * forward FFT instead spills (128 VGPRs at 4 waves per SIMD). */
__global__ void __launch_bounds__(1024)
k_reg_cols_xpower(sg_c64 *__restrict__ work, const sg_c64 *__restrict__ spec, int S, int CW,
		const sg_c64 *__restrict__ tw, int xcdmap, int pb) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	int x0 = sg_xcd_strip(blockIdx.x, gridDim.x, xcdmap) * CW, pair = blockIdx.y;
	/* pb > 1: blocks of pb pairs per strip dispatched back to back on one XCD (strip-major
	 * inside a pair block), so the strip's reference-spectrum columns are read from HBM once per
	 * block and from that XCD's L2 by the block's other pairs, while neighbouring strips of one
	 * pair still run close together (their 64-B rows share 128-B lines) */
	const int ns = gridDim.x, np = gridDim.y;
	if (pb > 1 && xcdmap && (ns & 7) == 0 && np % pb == 0) {
		const int id = blockIdx.x + ns * blockIdx.y, xcd = id & 7, local = id >> 3, s8 = ns >> 3;
		const int strip = xcd * s8 + (local / pb) % s8;
		pair = (local / (pb * s8)) * pb + local % pb;
		x0 = strip * CW;
	}
	const int bstride = SG_PADN(S) + 1, H = S >> 1;
	sg_c64 *base = work + (size_t)pair * S * S + x0;
	auto slot = [&](int c, int r) -> sg_c64 & { return buf[(size_t)c * bstride + sg_pad(r)]; };
	constexpr int NI = 8;
	const int items = CW * S;
	sg_c64 rk[NI], rm[NI];
	auto fetch = [&]() {
#pragma unroll
		for (int it = 0; it < NI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			rk[it] = make_double2(0.0, 0.0);
			rm[it] = make_double2(0.0, 0.0);
			if (t < items) {
				const int c = t % CW, ky = t / CW, kx = (x0 + c) & (H - 1);
				rk[it] = spec[(size_t)ky * S + kx];
				if (!kx)
					rm[it] = spec[(size_t)((S - ky) & (S - 1)) * S];
			}
		}
	};
	sg_fft_io(buf, S, CW, bstride, tw, false, [&](int c, int r) { return base[(size_t)r * S + c]; },
			[&](int c, int r, sg_c64 v) { slot(c, r) = v; });
	fetch();
	__syncthreads();
#pragma unroll
	for (int it = 0; it < NI; it++) {
		const int t = threadIdx.x + it * blockDim.x;
		if (t >= items)
			continue;
		const int c = t % CW, ky = t / CW, kx = (x0 + c) & (H - 1);
		if (kx) {
			slot(c, ky) = sg_rconj(rk[it], slot(c, ky));
			continue;
		}
		/* packed column: Z = F0 + i FN (F0, FN spectra of real columns), same for the
		 * reference; P = R0 conj F0 + i RN conj FN, written at ky and -ky */
		const int m = (S - ky) & (S - 1);
		if (m < ky)
			continue;
		const sg_c64 zk = slot(c, ky), zm = slot(c, m), r1 = rk[it], r2 = rm[it];
		const sg_c64 f0 = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
		const sg_c64 fn = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
		const sg_c64 r0 = make_double2(0.5 * (r1.x + r2.x), 0.5 * (r1.y - r2.y));
		const sg_c64 rn = make_double2(0.5 * (r1.y + r2.y), -0.5 * (r1.x - r2.x));
		const sg_c64 p0 = sg_rconj(r0, f0), pn = sg_rconj(rn, fn);
		slot(c, ky) = make_double2(p0.x - pn.y, p0.y + pn.x);
		if (m != ky)	/* P0(-k) = conj P0(k), PN(-k) = conj PN(k) */
			slot(c, m) = make_double2(p0.x + pn.y, pn.x - p0.y);
	}
	__syncthreads();
	sg_fft_io<true>(buf, S, CW, bstride, tw, true, [&](int c, int r) { return slot(c, r); },
			[&](int c, int r, sg_c64 v) { base[(size_t)r * S + c] = v; });
}

__global__ void __launch_bounds__(512)
k_reg_rows_inv_half_argmax(const sg_c64 *__restrict__ work, int S, const sg_c64 *__restrict__ tw,
		SgBest *__restrict__ best) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	sg_c64 *buf = (sg_c64 *)smem;
	__shared__ double rv[2][8];
	__shared__ int ri[2][8];
	const int row = blockIdx.x, pair = blockIdx.y, H = S >> 1;
	const sg_c64 *in = work + (size_t)pair * S * S + (size_t)row * S;
	double va = -INFINITY, vb = -INFINITY;
	int ia = 0x7fffffff, ib = 0x7fffffff;
	sg_fft_io(buf, S, 1, S, tw, true,
			[&](int, int i) {
				sg_c64 qa, qb;
				if ((i & (H - 1)) == 0) {	/* kx = 0 or S/2: the packed real pair */
					const sg_c64 a = in[0], b = in[H];
					qa = make_double2(i ? a.y : a.x, 0.0);
					qb = make_double2(i ? b.y : b.x, 0.0);
				} else if (i < H) {
					qa = in[i];
					qb = in[H + i];
				} else {
					const sg_c64 a = in[S - i], b = in[H + S - i];
					qa = make_double2(a.x, -a.y);
					qb = make_double2(b.x, -b.y);
				}
				return make_double2(qa.x - qb.y, qa.y + qb.x);
			},
			[&](int, int j, sg_c64 c) {
				const int idx = row * S + j;
				sg_argmax_merge(va, ia, c.x, idx);
				sg_argmax_merge(vb, ib, c.y, idx);
			});
	for (int o = 32; o > 0; o >>= 1) {
		const double va2 = __shfl_down(va, o, 64), vb2 = __shfl_down(vb, o, 64);
		const int ia2 = __shfl_down(ia, o, 64), ib2 = __shfl_down(ib, o, 64);
		sg_argmax_merge(va, ia, va2, ia2);
		sg_argmax_merge(vb, ib, vb2, ib2);
	}
	const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		rv[0][wave] = va;
		ri[0][wave] = ia;
		rv[1][wave] = vb;
		ri[1][wave] = ib;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < nw; w++) {
			sg_argmax_merge(va, ia, rv[0][w], ri[0][w]);
			sg_argmax_merge(vb, ib, rv[1][w], ri[1][w]);
		}
		SgBest r;
		r.va = va;
		r.ia = ia;
		r.vb = vb;
		r.ib = ib;
		best[(size_t)pair * S + row] = r;
	}
}

/* per pair: reduce the row maxima and convert to (shiftx, shifty) (:344-351) */
__global__ void __launch_bounds__(256)
k_reg_final(const SgBest *__restrict__ best, int S, int count, int *__restrict__ out /* [pair][4] */) {
	__shared__ double rv[2][4];
	__shared__ int ri[2][4];
	const int pair = blockIdx.x;
	double va = -INFINITY, vb = -INFINITY;
	int ia = 0x7fffffff, ib = 0x7fffffff;
	for (int r = threadIdx.x; r < count; r += blockDim.x) {
		const SgBest b = best[(size_t)pair * count + r];
		sg_argmax_merge(va, ia, b.va, b.ia);
		sg_argmax_merge(vb, ib, b.vb, b.ib);
	}
	for (int o = 32; o > 0; o >>= 1) {
		const double va2 = __shfl_down(va, o, 64), vb2 = __shfl_down(vb, o, 64);
		const int ia2 = __shfl_down(ia, o, 64), ib2 = __shfl_down(ib, o, 64);
		sg_argmax_merge(va, ia, va2, ia2);
		sg_argmax_merge(vb, ib, vb2, ib2);
	}
	const int wave = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		rv[0][wave] = va;
		ri[0][wave] = ia;
		rv[1][wave] = vb;
		ri[1][wave] = ib;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
			sg_argmax_merge(va, ia, rv[0][w], ri[0][w]);
			sg_argmax_merge(vb, ib, rv[1][w], ri[1][w]);
		}
		const int idx[2] = {ia, ib};
		for (int k = 0; k < 2; k++) {
			int sy = idx[k] / S, sx = idx[k] % S;
			if (sy > S / 2)
				sy -= S;
			if (sx > S / 2)
				sx -= S;
			out[pair * 4 + 2 * k] = sx;
			out[pair * 4 + 2 * k + 1] = sy;
		}
	}
}

/* ---------------------------------------------------------------------------------------
 * QualityEstimate (src/algos/quality.c).  Only subsample 3 contributes to the result:
 * dval += q * ((QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (subsample * subsample)) uses integer
 * division (:211), so the factor is 1 for subsample 3 and 0 for 4 and 5.
 * ------------------------------------------------------------------------------------- */
#define SG_Q_THRESHOLD (40 << 8)
#define SG_QROWS 4	/* subsampled rows per k_quality_sub workgroup */
#define SG_QGT 16	/* output rows per k_quality_grad tile (64 columns) */

/* SubSample (:223-234) of one 3x3 sample row, plus the running max of the middle rows
 * (the maxp[] loop :119-133 reduces to max over 0 < v < 65530) */
__global__ void __launch_bounds__(1024)
k_quality_sub(const uint16_t *__restrict__ sel, const int *__restrict__ qframes, int S, int xs, int ys,
		uint16_t *__restrict__ qbuf, unsigned int *__restrict__ qmax) {
	/* SG_QROWS output rows per workgroup; a thread forms two adjacent outputs from three
	 * 12-byte (6-pixel, dword-aligned) loads, one per input row */
	const int q = blockIdx.y;
	const uint16_t *frame = sel + (size_t)qframes[q] * S * S;
	unsigned int m = 0;
	const int j0 = blockIdx.x * SG_QROWS;
	for (int k = threadIdx.x; 2 * k < xs; k += blockDim.x) {
		/* the 3 x SG_QROWS input rows of this pair: every load issued before any is used */
		uint32_t d[SG_QROWS][3][3];
#pragma unroll
		for (int jj = 0; jj < SG_QROWS; jj++) {
			const int j = j0 + jj < ys ? j0 + jj : ys - 1;
#pragma unroll
			for (int y = 0; y < 3; y++) {
				const uint32_t *p = (const uint32_t *)(frame + (size_t)(3 * j + y) * S + 6 * k);
				d[jj][y][0] = p[0];
				d[jj][y][1] = p[1];
				d[jj][y][2] = p[2];
			}
		}
#pragma unroll
		for (int jj = 0; jj < SG_QROWS; jj++) {
			const int j = j0 + jj;
			if (j >= ys)
				break;
			const bool middle = (j >= 1 && j <= ys - 2);
			uint16_t *dst = qbuf + (size_t)q * xs * ys + (size_t)j * xs;
			int va = 0, vb = 0;
#pragma unroll
			for (int y = 0; y < 3; y++) {
				const uint32_t d0 = d[jj][y][0], d1 = d[jj][y][1], d2 = d[jj][y][2];
				va += (int)(d0 & 0xFFFFu) + (int)(d0 >> 16) + (int)(d1 & 0xFFFFu);
				vb += (int)(d1 >> 16) + (int)(d2 & 0xFFFFu) + (int)(d2 >> 16);
			}
			va /= 9;
			vb /= 9;
			dst[2 * k] = (uint16_t)va;
			if (middle && va > 0 && va < 65530 && (unsigned)va > m)
				m = (unsigned)va;
			if (2 * k + 1 < xs) {
				dst[2 * k + 1] = (uint16_t)vb;
				if (middle && vb > 0 && vb < 65530 && (unsigned)vb > m)
					m = (unsigned)vb;
			}
		}
	}
	for (int o = 32; o > 0; o >>= 1) {
		const unsigned int t = (unsigned int)__shfl_down((int)m, o, 64);
		m = t > m ? t : m;
	}
	if ((threadIdx.x & 63) == 0 && m)
		atomicMax(qmax + q, m);
}

/* stretched sample (:139-148): v * (60000 / max), truncated, clamped at 65535 */
__device__ __forceinline__ int sg_q_stretch(const uint16_t *b, int idx, double mult, bool stretch) {
	unsigned int v = b[idx];
	if (stretch) {
		v = (unsigned int)((double)v * mult);
		if (v > 65535u)
			v = 65535u;
	}
	return (int)v;
}

/* _smooth_image_16 (:324-349) + Gradient (:236-321): threshold map dilated 3x3 inside the
 * 10 % margins, gradient energy over mapped pixels; exact integer sums */
__global__ void __launch_bounds__(256)
k_quality_grad(const uint16_t *__restrict__ qbuf, int xs, int ys, const unsigned int *__restrict__ qmax,
		unsigned long long *__restrict__ acc /* [q][3]: val, pixels, thresholded */) {
	__shared__ unsigned long long sv[4], sp[4], sc[4];
	/* a 64 x SG_QGT tile of outputs: stretched samples of the 68 x (SG_QGT + 4)
	 * neighbourhood, then the smoothed values of the 66 x (SG_QGT + 2) one, each formed once
	 * in LDS; the blockDim.x / 64 waves take the output rows in turn */
	__shared__ unsigned int st[SG_QGT + 4][68];
	__shared__ int sms[SG_QGT + 2][66];
	const int q = blockIdx.z;
	const uint16_t *b = qbuf + (size_t)q * xs * ys;
	const unsigned int mx = qmax[q];
	const bool stretch = mx > 0;
	const double mult = stretch ? (double)60000 / (double)mx : 1.0;
	const int yb = (int)((double)ys * 0.1) + 1;
	const int xb = (int)((double)xs * 0.1) + 1;
	const int x0 = blockIdx.x * 64, y0 = blockIdx.y * SG_QGT;
	for (int i = threadIdx.x; i < (SG_QGT + 4) * 68; i += blockDim.x) {
		const int ly = i / 68, lx = i - ly * 68;
		const int gx = x0 - 2 + lx, gy = y0 - 2 + ly;
		st[ly][lx] = (gx >= 0 && gx < xs && gy >= 0 && gy < ys) ? (unsigned int)sg_q_stretch(b, gy * xs + gx, mult, stretch)
									     : 0u;
	}
	__syncthreads();
	for (int i = threadIdx.x; i < (SG_QGT + 2) * 66; i += blockDim.x) {
		const int ly = i / 66, lx = i - ly * 66;
		const int qx = x0 - 1 + lx, qy = y0 - 1 + ly;
		int v = 0;
		if (qx >= 1 && qx <= xs - 2 && qy >= 1 && qy <= ys - 2) {
			unsigned int sum = 0;
			for (int ey = 0; ey < 3; ey++)
				for (int ex = 0; ex < 3; ex++)
					sum += st[ly + ey][lx + ex];
			v = (int)(sum / 9);
		}
		sms[ly][lx] = v;
	}
	__syncthreads();
	const int tx = threadIdx.x & 63;
	const int x = x0 + tx;
	unsigned long long val = 0, pix = 0, cnt = 0;
	for (int ty = threadIdx.x >> 6; ty < SG_QGT; ty += (int)(blockDim.x >> 6)) {
	const int y = y0 + ty;
	if (x >= xb && x < xs - xb && y >= yb && y < ys - yb) {
		/* smoothed values on the 3x3 neighbourhood of (x, y) */
		int sm[3][3];
		for (int dy = 0; dy < 3; dy++)
			for (int dx = 0; dx < 3; dx++)
				sm[dy][dx] = sms[ty + dy][tx + dx];
		if (sm[1][1] >= SG_Q_THRESHOLD)
			cnt += 1;
		bool mapped = false;
		for (int dy = -1; dy <= 1; dy++)
			for (int dx = -1; dx <= 1; dx++) {
				const int qx = x + dx, qy = y + dy;
				if (qx >= xb && qx < xs - xb && qy >= yb && qy < ys - yb &&
						sm[dy + 1][dx + 1] >= SG_Q_THRESHOLD)
					mapped = true;
			}
		if (mapped) {
			const long long d1 = sm[1][1] - sm[1][2];
			const long long d2 = sm[1][1] - sm[2][1];
			val += (unsigned long long)(d1 * d1 + d2 * d2);
			pix += 1;
		}
	}
	}
	for (int o = 32; o > 0; o >>= 1) {
		val += __shfl_down(val, o, 64);
		pix += __shfl_down(pix, o, 64);
		cnt += __shfl_down(cnt, o, 64);
	}
	const int wave = threadIdx.x >> 6;
	if ((threadIdx.x & 63) == 0) {
		sv[wave] = val;
		sp[wave] = pix;
		sc[wave] = cnt;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		for (int w = 1; w < (int)(blockDim.x >> 6); w++) {
			val += sv[w];
			pix += sp[w];
			cnt += sc[w];
		}
		if (val)
			atomicAdd(acc + q * 3, val);
		if (pix)
			atomicAdd(acc + q * 3 + 1, pix);
		if (cnt)
			atomicAdd(acc + q * 3 + 2, cnt);
	}
}

static int reg_quality(sg_ctx *ctx, SgDevice &dv, hipStream_t s, const uint16_t *d_sel, int S,
		const std::vector<int> &frames, std::vector<double> &qual) {
	const int nq = (int)frames.size();
	qual.assign(nq, 0.0);
	if (!nq)
		return SG_OK;
	const int xs = (S - 1) / 3, ys = (S - 1) / 3;
	if (xs < 2 || ys < 2)	/* the subsample loop never runs: dval = 0 (:95-98) */
		return SG_OK;
	HIPCHK(ensure(dv.reg_qbuf, (size_t)nq * xs * ys * sizeof(uint16_t) + sizeof(int) * nq + 64));
	HIPCHK(ensure(dv.reg_qacc, (size_t)nq * (3 * sizeof(unsigned long long) + sizeof(unsigned int))));
	uint16_t *qbuf = (uint16_t *)dv.reg_qbuf.p;
	int *d_frames = (int *)((char *)dv.reg_qbuf.p + (((size_t)nq * xs * ys * sizeof(uint16_t) + 15) & ~(size_t)15));
	unsigned long long *acc = (unsigned long long *)dv.reg_qacc.p;
	unsigned int *qmax = (unsigned int *)(acc + 3 * nq);
	HIPCHK(hipMemcpyAsync(d_frames, frames.data(), sizeof(int) * nq, hipMemcpyHostToDevice, s));
	HIPCHK(hipMemsetAsync(dv.reg_qacc.p, 0, (size_t)nq * (3 * sizeof(unsigned long long) + sizeof(unsigned int)), s));
	/* one wave per workgroup, walking the row pairs: 283 us per 129 frames of 2048^2 against
	 * 332 / 348 / 403 / 618 us with 128 / 192 / 256 / 384 threads (scripts/gpu_qsub.sh) */
	const int qthr = ctx->knobs.qsub_threads;	/* A/B knob SG_QSUB_THREADS */
	hipLaunchKernelGGL(k_quality_sub, dim3((ys + SG_QROWS - 1) / SG_QROWS, nq), dim3(qthr), 0, s, d_sel, d_frames, S,
			xs, ys, qbuf, qmax);
	HIPCHK(hipGetLastError());
	/* 2 waves per 64x16 tile: 214 us per 129 frames against 238 (4 waves) and 333 (1 wave),
	 * scripts/gpu_qgrad.sh */
	const int gthr = ctx->knobs.qgrad_threads;	/* A/B knob SG_QGRAD_THREADS */
	hipLaunchKernelGGL(k_quality_grad, dim3((xs + 63) / 64, (ys + SG_QGT - 1) / SG_QGT, nq), dim3(gthr), 0, s, qbuf, xs, ys,
			qmax, acc);
	HIPCHK(hipGetLastError());
	std::vector<unsigned long long> h(3 * (size_t)nq);
	HIPCHK(hipMemcpyAsync(h.data(), acc, sizeof(unsigned long long) * 3 * nq, hipMemcpyDeviceToHost, s));
	HIPCHK(hipStreamSynchronize(s));
	for (int i = 0; i < nq; i++) {
		double q;
		if (!h[3 * i + 2]) {
			q = -1.0;
		} else {
			q = (double)h[3 * i] / (double)h[3 * i + 1];
			q = q / 10;
		}
		double dval = 0.0;
		dval += q * 1;
		qual[i] = sqrt(dval);
	}
	return SG_OK;
}

static int ilog2(int v) {
	int l = 0;
	while ((1 << l) < v)
		l++;
	return l;
}

static int reg_dft_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality, void *stream, bool normalize_q);

extern "C" int sg_register_dft_u16_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality,
		void *stream) {
	return reg_dft_device(ctx, dev_index, d_sel, nframes, S, ref_image, included, shiftx, shifty, quality, stream,
			true);
}

extern "C" int sg_register_dft_u16_device_raw(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality_raw,
		void *stream) {
	return reg_dft_device(ctx, dev_index, d_sel, nframes, S, ref_image, included, shiftx, shifty, quality_raw,
			stream, false);
}

static int reg_dft_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality, void *stream, bool normalize_q) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size() || !d_sel || !shiftx || !shifty || !quality)
		return SG_ERR_GENERIC;
	if (nframes < 1)
		return set_err(ctx, SG_ERR_GENERIC, "no frame to register%s%ld", "", nframes);
	if (S < 8 || S > 4096 || (S & (S - 1)))
		return set_err(ctx, SG_ERR_SIZE, "DFT registration needs a power-of-two selection side "
				"between 8 and 4096%s (got %ld)", "", S);
	if (ref_image < 0)
		ref_image = 0;	/* seq->reference_image == -1 -> 0 (:212-215) */
	if (ref_image >= nframes)
		return set_err(ctx, SG_ERR_GENERIC, "reference image out of range%s %ld", "", ref_image);
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	const int logS = ilog2(S);
	const size_t plane = (size_t)S * S;

	/* frames to register, in index order (the reference skips ref and excluded frames) */
	std::vector<int> todo;
	for (int f = 0; f < nframes; f++)
		if (f != ref_image && (!included || included[f]))
			todo.push_back(f);

	/* twiddles exp(-2 pi i k / S) */
	HIPCHK(ensure(dv.reg_tw, sizeof(sg_c64) * 2 * S));
	{
		/* forward full circle (k >= S/2: the negated half-circle value), then its conjugate */
		std::vector<double> tw(4 * (size_t)S);
		for (int k = 0; k < S / 2; k++) {
			const double a = -2.0 * M_PI * (double)k / (double)S;
			const double c = cos(a), sn = sin(a);
			const int kk[2] = {k, k + S / 2};
			const double sg[2] = {1.0, -1.0};
			for (int h = 0; h < 2; h++) {
				tw[2 * kk[h]] = sg[h] * c;
				tw[2 * kk[h] + 1] = sg[h] * sn;
				tw[2 * (S + kk[h])] = sg[h] * c;
				tw[2 * (S + kk[h]) + 1] = -(sg[h] * sn);
			}
		}
		HIPCHK(hipMemcpyAsync(dv.reg_tw.p, tw.data(), sizeof(double) * 4 * S, hipMemcpyHostToDevice, s));
		HIPCHK(hipStreamSynchronize(s));
	}
	const sg_c64 *tw = (const sg_c64 *)dv.reg_tw.p;

	/* quality of the reference and of every registered frame */
	std::vector<int> qframes;
	qframes.push_back(ref_image);
	qframes.insert(qframes.end(), todo.begin(), todo.end());
	std::vector<double> qual;
	int rc = reg_quality(ctx, dv, s, d_sel, S, qframes, qual);
	if (rc)
		return rc;

	/* batch of pairs per launch: up to 2 GB of pair planes (32 at S = 2048). Half-spectrum
	 * passes, configs[1]: 32 or 64 pairs 8.95-9.07 ms, 16: 9.08, 4: 9.22-9.32, 2: 9.02-9.15,
	 * 1: 9.8 ms of registration (scripts/gpu_regbatch.sh) */
	int B = (int)((size_t)(2048u << 20) / (plane * sizeof(sg_c64)));
	if (B < 1)
		B = 1;
	if (B > 64)
		B = 64;
	if (ctx->knobs.reg_batch > 0)	/* A/B knob SG_REG_BATCH: pairs per launch */
		B = ctx->knobs.reg_batch;
	const int npairs_total = (int)(todo.size() + 1) / 2;
	if (B > npairs_total && npairs_total > 0)
		B = npairs_total;
	const size_t row_lds = (size_t)SG_PADN(S) * sizeof(sg_c64);
	int CW = 8192 / S;
	if (CW < 1)
		CW = 1;
	if (CW > 8)
		CW = 8;
	if (ctx->knobs.reg_cw > 0)	/* A/B knob SG_REG_CW: columns per column-pass workgroup */
		CW = ctx->knobs.reg_cw;
	const size_t col_lds = (size_t)CW * (SG_PADN(S) + 1) * sizeof(sg_c64);
	(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)row_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_argmax, hipFuncAttributeMaxDynamicSharedMemorySize, (int)row_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_cols, hipFuncAttributeMaxDynamicSharedMemorySize, (int)col_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_cols_inv_argmax, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)col_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_xpower_rows_inv, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)(2 * row_lds));
	/* threads: 8 elements per thread in every LDS FFT (sg_stockham_pass's register budget),
	 * at least one wave */
	auto thr_for = [](int elems) { return elems / 8 < 64 ? 64 : elems / 8; };
	const int row_thr = thr_for(S), col_thr = thr_for(CW * S), xri_thr = thr_for(2 * S);
	/* pass order: 2 = half spectra (3 plane passes), 1 = full spectra with the cross-power
	 * fused into the inverse row pass (4), 0 = unfused (5) */
	const int path = ctx->knobs.reg_path;	/* A/B knob SG_REG_PATH */
	const bool fused = path == 1;
	const bool half = path == 2;
	/* half-spectrum columns: a strip stays inside one half (CW divides S/2) */
	const int CWh = CW < S / 2 ? CW : S / 2;
	const size_t colh_lds = (size_t)CWh * (SG_PADN(S) + 1) * sizeof(sg_c64);
	const int colh_thr = thr_for(CWh * S);
	(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd_half, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)row_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_half_argmax, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)row_lds);
	(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)colh_lds);
	const int xcdmap = ctx->knobs.reg_xcd;	/* A/B knob SG_REG_XCD: 0 = strips in dispatch order */

	HIPCHK(ensure(dv.reg_spec, plane * sizeof(sg_c64)));
	HIPCHK(ensure(dv.reg_work, (size_t)(B > 1 ? B : 1) * plane * sizeof(sg_c64)));
	/* row maxima of one batch, then per pair: 4 result ints, frame a, frame b (all pairs of
	 * the call, uploaded once; results read back once) */
	const int NP = npairs_total > 0 ? npairs_total : 1;
	HIPCHK(ensure(dv.reg_best, (size_t)(B > 1 ? B : 1) * S * sizeof(SgBest) + (size_t)(NP + 1) * 6 * sizeof(int) + 64));
	sg_c64 *spec = (sg_c64 *)dv.reg_spec.p, *work = (sg_c64 *)dv.reg_work.p;
	SgBest *best = (SgBest *)dv.reg_best.p;
	int *d_out = (int *)(best + (size_t)(B > 1 ? B : 1) * S);
	int *d_fa = d_out + 4 * (NP + 1);
	int *d_fb = d_fa + (NP + 1);

	/* pair k = frames todo[2k], todo[2k+1] (-1: odd count, imaginary part zero); slot NP is
	 * the reference spectrum's (ref_image, -1) */
	std::vector<int> hfa(NP + 1), hfb(NP + 1), hout(4 * (size_t)NP);
	for (int k = 0; k < npairs_total; k++) {
		hfa[k] = todo[2 * k];
		hfb[k] = (2 * (size_t)k + 1 < todo.size()) ? todo[2 * k + 1] : -1;
	}
	hfa[NP] = ref_image;
	hfb[NP] = -1;
	HIPCHK(hipMemcpyAsync(d_fa, hfa.data(), sizeof(int) * (NP + 1), hipMemcpyHostToDevice, s));
	HIPCHK(hipMemcpyAsync(d_fb, hfb.data(), sizeof(int) * (NP + 1), hipMemcpyHostToDevice, s));
	/* reference spectrum R = FFT2(ref) (half layout: the A' half only) */
	if (half) {
		hipLaunchKernelGGL(k_reg_rows_fwd_half, dim3(S, 1), dim3(row_thr), row_lds, s, d_sel, d_fa + NP, d_fb + NP,
				S, tw, spec);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_reg_cols, dim3(S / 2 / CWh, 1), dim3(colh_thr), colh_lds, s, spec, S, logS, CWh, tw, 0,
				xcdmap);
	} else {
		hipLaunchKernelGGL(k_reg_rows_fwd, dim3(S, 1), dim3(row_thr), row_lds, s, d_sel, d_fa + NP, d_fb + NP, S,
				logS, tw, spec);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_reg_cols, dim3(S / CW, 1), dim3(col_thr), col_lds, s, spec, S, logS, CW, tw, 0, xcdmap);
	}
	HIPCHK(hipGetLastError());
	shiftx[ref_image] = 0;
	shifty[ref_image] = 0;
	for (int p0 = 0; p0 < npairs_total; p0 += B) {
		const int np = npairs_total - p0 < B ? npairs_total - p0 : B;
		if (half) {
			hipLaunchKernelGGL(k_reg_rows_fwd_half, dim3(S, np), dim3(row_thr), row_lds, s, d_sel, d_fa + p0,
					d_fb + p0, S, tw, work);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_cols_xpower, dim3(S / CWh, np), dim3(colh_thr), colh_lds, s, work,
					(const sg_c64 *)spec, S, CWh, tw, xcdmap, ctx->knobs.reg_pb);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_rows_inv_half_argmax, dim3(S, np), dim3(row_thr), row_lds, s,
					(const sg_c64 *)work, S, tw, best);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_final, dim3(np), dim3(256), 0, s, (const SgBest *)best, S, S, d_out + 4 * p0);
			HIPCHK(hipGetLastError());
			continue;
		}
		hipLaunchKernelGGL(k_reg_rows_fwd, dim3(S, np), dim3(row_thr), row_lds, s, d_sel, d_fa + p0, d_fb + p0, S,
				logS, tw, work);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_reg_cols, dim3(S / CW, np), dim3(col_thr), col_lds, s, work, S, logS, CW, tw, 0,
				xcdmap);
		HIPCHK(hipGetLastError());
		if (fused) {
			/* cross-power + inverse rows (row pairs ky, -ky), then inverse columns with the
			 * arg-max: two plane round trips fewer than the unfused order */
			hipLaunchKernelGGL(k_reg_xpower_rows_inv, dim3(S / 2 + 1, np), dim3(xri_thr), 2 * row_lds, s, work,
					(const sg_c64 *)spec, S, logS, tw);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_cols_inv_argmax, dim3(S / CW, np), dim3(col_thr), col_lds, s,
					(const sg_c64 *)work, S, logS, CW, tw, best, xcdmap);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_final, dim3(np), dim3(256), 0, s, (const SgBest *)best, S, S / CW,
					d_out + 4 * p0);
		} else {
			hipLaunchKernelGGL(k_reg_xpower, dim3(1024, np), dim3(256), 0, s, work, (const sg_c64 *)spec, S);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_cols, dim3(S / CW, np), dim3(col_thr), col_lds, s, work, S, logS, CW, tw, 1,
					xcdmap);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_rows_inv_argmax, dim3(S, np), dim3(row_thr), row_lds, s, (const sg_c64 *)work,
					S, logS, tw, best);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_final, dim3(np), dim3(256), 0, s, (const SgBest *)best, S, S, d_out + 4 * p0);
		}
		HIPCHK(hipGetLastError());
	}
	if (npairs_total > 0)
		HIPCHK(hipMemcpyAsync(hout.data(), d_out, sizeof(int) * 4 * npairs_total, hipMemcpyDeviceToHost, s));
	HIPCHK(hipStreamSynchronize(s));
	for (int k = 0; k < npairs_total; k++) {
		shiftx[hfa[k]] = hout[4 * k];
		shifty[hfa[k]] = hout[4 * k + 1];
		if (hfb[k] >= 0) {
			shiftx[hfb[k]] = hout[4 * k + 2];
			shifty[hfb[k]] = hout[4 * k + 3];
		}
	}

	/* quality: q_min/q_max seeded by the reference frame, then frames in index order with
	 * the reference's min() macro (src/core/siril.h), then normalizeQualityData */
	if (!normalize_q) {	/* raw values of the processed frames (sharded registration) */
		quality[ref_image] = qual[0];
		for (size_t k = 0; k < todo.size(); k++)
			quality[todo[k]] = qual[k + 1];
		return SG_OK;
	}
	double q_min = qual[0], q_max = qual[0];
	quality[ref_image] = qual[0];
	for (size_t k = 0; k < todo.size(); k++) {
		const double qv = qual[k + 1];
		quality[todo[k]] = qv;
		if (qv > q_max)
			q_max = qv;
		q_min = (q_min < qv) ? q_min : qv;
	}
	for (int f = 0; f < nframes; f++) {
		if (included && !included[f])
			continue;
		quality[f] -= q_min;
		quality[f] /= (q_max - q_min);
	}
	return SG_OK;
}

extern "C" int sg_register_dft_u16(sg_ctx *ctx, const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality) {
	if (!ctx || ctx->dev.empty() || !sel)
		return SG_ERR_GENERIC;
	if (nframes < 1 || S < 1)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[0];
	HIPCHK(hipSetDevice(dv.id));
	const size_t bytes = (size_t)nframes * S * S * sizeof(uint16_t);
	HIPCHK(ensure(dv.reg_sel, bytes));
	HIPCHK(hipMemcpyAsync(dv.reg_sel.p, sel, bytes, hipMemcpyHostToDevice, dv.stream));
	return sg_register_dft_u16_device(ctx, 0, (const uint16_t *)dv.reg_sel.p, nframes, S, ref_image, included,
			shiftx, shifty, quality, nullptr);
}
