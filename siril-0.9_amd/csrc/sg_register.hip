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
 *   - power-of-two sides: Stockham passes of radix 8 (then 4 / 2) in LDS on half spectra
 *     (rows: one workgroup per row; columns: one workgroup per strip of CW columns), in fp32
 *     by default, fp64 for the pairs re-run below (SG_REG_FP=64: fp64 throughout), twiddles
 *     from host tables; any other side: mixed radix 8/4/2/3/5/7, or Bluestein's chirp-z for
 *     a prime factor above 7, with transposed column passes, in fp64;
 *   - the inverse row pass fuses a per-row TOP-2 arg-max (first index on ties), a tiny kernel
 *     reduces the rows in order.
 * Near ties: a maximum is decided where it beats the runner-up by more than the pass's error
 * bound, 2^-15 S^2 ||ref|| ||img|| in fp32 (the pair then re-runs in fp64) and 2^-32 in fp64
 * (far above fp64 FFT rounding: every index within it is listed and its exact integer
 * correlation computed; the largest wins, the lowest index among exact equals).  So shifts
 * equal the reference wherever FFTW's rounding does not decide between exactly equal
 * correlations (FFTW's choice there is unspecified: "parity unpinned").
 */
#include "sg_common.hpp"
#include "sg_ctx.hpp"
#include "sg_fft.hpp"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <thread>
#include <type_traits>
#include <vector>

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
template <class C, int EPT = 8>
__global__ void __launch_bounds__(1024)
k_reg_cols(C *__restrict__ work, int S, int logS, int CW, const C *__restrict__ tw, int inverse, int xcdmap) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	C *buf = (C *)smem;
	const int x0 = sg_xcd_strip(blockIdx.x, gridDim.x, xcdmap) * CW, pair = blockIdx.y;
	const int bstride = sg_col_stride<C>(S);
	C *base = work + (size_t)pair * S * S + x0;
	(void)logS;
	sg_fft_io<false, EPT>(buf, S, CW, bstride, tw, inverse != 0, [&](int c, int r) { return base[(size_t)r * S + c]; },
			[&](int c, int r, C v) { base[(size_t)r * S + c] = v; });
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
/* the frames' selections as the registration kernels read them: selection f, row r at
 * p[f fp + r rp] (elements).  Contiguous S x S selections: fp = S S, rp = S; in place in resident
 * frames (sg_register_dft_u16_device_pitched): the frames' plane / row pitches */
struct SgSel {
	const uint16_t *p;
	long long fp, rp;
	__device__ __forceinline__ const uint16_t *frame(int f) const { return p + (size_t)f * (size_t)fp; }
};

#ifndef SG_REG_FWD_WPE
#define SG_REG_FWD_WPE 4	/* forward row pass: waves per SIMD its register budget is sized for (4: 127 VGPRs, 28 B of scratch, registration 5.93 -> 5.82 ms on configs[1]; 1: 134 VGPRs; 6: 208 B of scratch, 6.97 ms) */
#endif
template <class C>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(SG_REG_FWD_WPE)))
k_reg_rows_fwd_half(SgSel sel, const int *__restrict__ fa, const int *__restrict__ fb,
		int S, const C *__restrict__ tw, C *__restrict__ work, unsigned long long *__restrict__ energy, int rpb) {
	typedef typename SgReal<C>::T T;
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	C *buf = (C *)smem;
	const int pair = blockIdx.y, H = S >> 1, per = S >> 3;
	const size_t plane = (size_t)S * S;
	const uint16_t *pa = sel.frame(fa[pair]);
	const int b = fb[pair];
	const uint16_t *pb = b >= 0 ? sel.frame(b) : nullptr;
	/* rpb rows per workgroup; the next row's samples are loaded into registers before this
	 * row's transform (the first pass's inputs: thread t takes elements t + r S / 8), so its
	 * load latency hides behind the LDS passes instead of opening every row (round 2: one row
	 * per workgroup, 1.75 ms per 64 pairs of 2048^2 at 1.8 TB/s) */
	const int t = threadIdx.x;
	const bool act = t < per;
	uint32_t ra[8], rb[8];
	auto fetch = [&](int row) {
#pragma unroll
		for (int r = 0; r < 8; r++) {
			const size_t i = (size_t)row * sel.rp + (size_t)(t + r * per);
			ra[r] = act ? (uint32_t)pa[i] : 0u;
			rb[r] = (act && pb) ? (uint32_t)pb[i] : 0u;
		}
	};
	unsigned long long ea = 0, eb = 0;
	const int row0 = blockIdx.x * rpb;
	fetch(row0);
	for (int k = 0; k < rpb; k++) {
		const int row = row0 + k;
		C v[1][8];
#pragma unroll
		for (int r = 0; r < 8; r++) {
			v[0][r] = sg_mk<C>((T)ra[r], (T)rb[r]);
			ea += (unsigned long long)(ra[r] * ra[r]);
			eb += (unsigned long long)(rb[r] * rb[r]);
		}
		if (k + 1 < rpb)
			fetch(row + 1);
		if (k > 0)
			__syncthreads();	/* the previous row's separation has read buf */
		sg_fft_io_regs<8>(buf, S, 1, S, tw, false, v, [&](int, int i, C val) { buf[sg_pad(i)] = val; });
		__syncthreads();
		C *out = work + (size_t)pair * plane + (size_t)row * S;
		for (int kx = threadIdx.x; kx < H; kx += blockDim.x) {
			const C zk = buf[sg_pad(kx)], zm = buf[sg_pad(kx ? S - kx : H)];
			C A, B;
			if (kx == 0) {
				A = sg_mk<C>(zk.x, zm.x);	/* A(0) + i A(S/2) */
				B = sg_mk<C>(zk.y, zm.y);
			} else {
				A = sg_mk<C>((T)0.5 * (zk.x + zm.x), (T)0.5 * (zk.y - zm.y));
				B = sg_mk<C>((T)0.5 * (zk.y + zm.y), (T)-0.5 * (zk.x - zm.x));
			}
			out[kx] = A;
			out[H + kx] = B;
		}
	}
	sg_energy_add(ea, eb, fa[pair], b, energy);
}

/* R conj F */
template <class C>
__device__ __forceinline__ C sg_rconj(C r, C f) {
	return sg_mk<C>(r.x * f.x + r.y * f.y, r.y * f.x - r.x * f.y);
}

/* The reference-spectrum loads of all 8 cross-power items of a thread are issued together
 * (launches are sized so that CW * S = 8 * blockDim, thr_for).  Issuing them before the
 * forward FFT instead spills (128 VGPRs at 4 waves per SIMD). */
template <class C, int EPT = 8, int WPE = 1>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE)))
k_reg_cols_xpower(C *__restrict__ work, const C *__restrict__ spec, int S, int CW,
		const C *__restrict__ tw, int xcdmap, int pb) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	C *buf = (C *)smem;
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
	typedef typename SgReal<C>::T T;
	const int bstride = sg_col_stride<C>(S), H = S >> 1;
	C *base = work + (size_t)pair * S * S + x0;
	auto slot = [&](int c, int r) -> C & { return buf[(size_t)c * bstride + sg_pad(r)]; };
	constexpr int NI = EPT;
	const int items = CW * S, lcw = sg_log2(CW);	/* CW: a power of two */
	/* the reference's packed column 0 (a strip starting at kx = 0 of either half) also needs
	 * R(-ky): read where it is used, so the other strips keep no second register array */
	C rk[NI];
	auto fetch = [&]() {
#pragma unroll
		for (int it = 0; it < NI; it++) {
			const int t = threadIdx.x + it * blockDim.x;
			rk[it] = sg_mk<C>((T)0, (T)0);
			if (t < items) {
				const int c = t & (CW - 1), ky = t >> lcw, kx = (x0 + c) & (H - 1);
				rk[it] = spec[(size_t)ky * S + kx];
			}
		}
	};
	sg_fft_io<false, EPT>(buf, S, CW, bstride, tw, false, [&](int c, int r) { return base[(size_t)r * S + c]; },
			[&](int c, int r, C v) { slot(c, r) = v; });
	fetch();
	__syncthreads();
#pragma unroll
	for (int it = 0; it < NI; it++) {
		const int t = threadIdx.x + it * blockDim.x;
		if (t >= items)
			continue;
		const int c = t & (CW - 1), ky = t >> lcw, kx = (x0 + c) & (H - 1);
		if (kx) {
			slot(c, ky) = sg_rconj(rk[it], slot(c, ky));
			continue;
		}
		/* packed column: Z = F0 + i FN (F0, FN spectra of real columns), same for the
		 * reference; P = R0 conj F0 + i RN conj FN, written at ky and -ky */
		const int m = (S - ky) & (S - 1);
		if (m < ky)
			continue;
		const C zk = slot(c, ky), zm = slot(c, m), r1 = rk[it], r2 = spec[(size_t)m * S];
		const C f0 = sg_mk<C>((T)0.5 * (zk.x + zm.x), (T)0.5 * (zk.y - zm.y));
		const C fn = sg_mk<C>((T)0.5 * (zk.y + zm.y), (T)-0.5 * (zk.x - zm.x));
		const C r0 = sg_mk<C>((T)0.5 * (r1.x + r2.x), (T)0.5 * (r1.y - r2.y));
		const C rn = sg_mk<C>((T)0.5 * (r1.y + r2.y), (T)-0.5 * (r1.x - r2.x));
		const C p0 = sg_rconj(r0, f0), pn = sg_rconj(rn, fn);
		slot(c, ky) = sg_mk<C>(p0.x - pn.y, p0.y + pn.x);
		if (m != ky)	/* P0(-k) = conj P0(k), PN(-k) = conj PN(k) */
			slot(c, m) = sg_mk<C>(p0.x + pn.y, pn.x - p0.y);
	}
	__syncthreads();
	sg_fft_io<true, EPT>(buf, S, CW, bstride, tw, true, [&](int c, int r) { return slot(c, r); },
			[&](int c, int r, C v) { base[(size_t)r * S + c] = v; });
}

/* ---------------------------------------------------------------------------------------
 * Wave-level fused column pass, fp32, S = 2048 (configs[1] / configs[4]): one WAVE per column
 * of a 4-column strip, the 2048-point transforms as 32 x 64 four-step FFTs held in registers
 * (32 complex per lane), so the block synchronises only around the coalesced strip load and
 * store.  Forward: lane l holds x[64 j + l] (j = 0..31); a 32-point DFT over j in registers,
 * twiddles w_S^(l k1), a transpose through the wave's own LDS column (rows of 66 for banks) to
 * lane m = (k1 = m / 2, h = m % 2) holding the odd / even lanes' values (i -> l = 2 i + h), a
 * 32-point DFT over i, twiddles w_64^(h k2) and one radix-2 step across the lane pair (DPP):
 * lane m, register k2 then holds X[ky], ky = m / 2 + 32 k2 + 1024 (m % 2).  The cross power is
 * elementwise at ky (the packed column 0 also reads Z(-ky), through the wave's LDS), and the
 * inverse runs the same steps mirrored, ending in natural order.  Same products and packing as
 * k_reg_cols_xpower; the FFT's rounding differs and stays within the fp32 tie tolerance
 * (sg_reg_tol).  The round-3 kernel (1024 threads, four radix-8/4 LDS passes each way) spent
 * ~15 k wave-instructions per column, mostly index arithmetic, LDS traffic and barriers.
 * ------------------------------------------------------------------------------------- */
typedef float sg_v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2 sg_cmulf(float2 a, float2 b) {
	const sg_v2f av = sg_v2f{a.x, a.y}, bv = sg_v2f{b.x, b.y};
	sg_v2f r;
	asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
	    "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
	    : "=&v"(r) : "v"(av), "v"(bv));
	return make_float2(r.x, r.y);
}
/* the same with a uniform w (a constant root: an SGPR pair, no per-use VGPR moves) */
__device__ __forceinline__ float2 sg_cmulk(float2 a, sg_v2f w) {
	const sg_v2f av = sg_v2f{a.x, a.y};
	sg_v2f r;
	asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
	    "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
	    : "=&v"(r) : "v"(av), "s"(w));
	return make_float2(r.x, r.y);
}

/* s v + o for a per-lane sign s = (+-1, +-1) (the lane pair's radix-2: v + o or o - v, exact) */
__device__ __forceinline__ float2 sg_pm_add(float2 v, float2 o, sg_v2f s2) {
	sg_v2f r;
	asm("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(r) : "v"(s2), "v"(sg_v2f{v.x, v.y}), "v"(sg_v2f{o.x, o.y}));
	return make_float2(r.x, r.y);
}
/* r conj(f) (the cross power's product) */
__device__ __forceinline__ float2 sg_rconjf(float2 r, float2 f) {
	sg_v2f d;
	asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
	    "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[0,0,1]"
	    : "=&v"(d) : "v"(sg_v2f{r.x, r.y}), "v"(sg_v2f{f.x, f.y}));
	return make_float2(d.x, d.y);
}

/* 32-point DFT of v (natural order in and out) in registers, radix-2 decimation in frequency */
/* d times -i (forward) / +i (inverse), exact: one packed multiply by (1, -1) / (-1, 1) with the
 * halves swapped */
template <bool INV>
__device__ __forceinline__ sg_v2f sg_rot_i(sg_v2f d) {
	sg_v2f r;
	asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(d), "s"(INV ? sg_v2f{-1.0f, 1.0f} : sg_v2f{1.0f, -1.0f}));
	return r;
}
__device__ __forceinline__ sg_v2f sg_cmulk2(sg_v2f a, sg_v2f w) {
	sg_v2f r;
	asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]\n\t"
	    "v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
	    : "=&v"(r) : "v"(a), "s"(w));
	return r;
}

/* 32-point DFT of v (natural order in and out) in registers, radix-2 decimation in frequency;
 * each complex value one packed register pair (v_pk_add / v_pk_mul + v_pk_fma per butterfly) */
template <bool INV>
__device__ __forceinline__ void sg_dft32_lane(float2 (&v)[32]) {
	constexpr float C[16] = {1.0f, 0.9807852506637573f, 0.9238795042037964f, 0.8314695954322815f,
		0.7071067690849304f, 0.5555702447891235f, 0.3826834261417389f, 0.19509032368659973f, 0.0f,
		-0.19509032368659973f, -0.3826834261417389f, -0.5555702447891235f, -0.7071067690849304f,
		-0.8314695954322815f, -0.9238795042037964f, -0.9807852506637573f};
	constexpr float SN[16] = {0.0f, 0.19509032368659973f, 0.3826834261417389f, 0.5555702447891235f,
		0.7071067690849304f, 0.8314695954322815f, 0.9238795042037964f, 0.9807852506637573f, 1.0f,
		0.9807852506637573f, 0.9238795042037964f, 0.8314695954322815f, 0.7071067690849304f,
		0.5555702447891235f, 0.3826834261417389f, 0.19509032368659973f};
	sg_v2f x[32];
#pragma unroll
	for (int k = 0; k < 32; k++)
		x[k] = sg_v2f{v[k].x, v[k].y};
#pragma unroll
	for (int half = 16; half >= 1; half >>= 1) {
#pragma unroll
		for (int blk = 0; blk < 32; blk += 2 * half) {
#pragma unroll
			for (int i = 0; i < half; i++) {
				const sg_v2f a = x[blk + i], b = x[blk + i + half];
				x[blk + i] = a + b;
				const sg_v2f d = a - b;
				const int m = i * (16 / half);	/* w_32^m, m < 16 */
				if (m == 0)
					x[blk + i + half] = d;
				else if (m == 8)
					x[blk + i + half] = sg_rot_i<INV>(d);
				else
					x[blk + i + half] = sg_cmulk2(d, sg_v2f{C[m], INV ? SN[m] : -SN[m]});
			}
		}
		__builtin_amdgcn_sched_barrier(0);	/* stage by stage: interleaved stages took 249 VGPRs */
	}
#pragma unroll
	for (int k = 0; k < 32; k++) {
		const sg_v2f t = x[(int)(__builtin_bitreverse32((unsigned)k) >> 27)];
		v[k] = make_float2(t.x, t.y);
	}
}

/* the lane-pair partner's value (lane ^ 1), DPP quad_perm [1, 0, 3, 2] */
__device__ __forceinline__ float2 sg_pair_swap(float2 v) {
	return make_float2(__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.x), 0xB1, 0xF, 0xF, false)),
			__int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v.y), 0xB1, 0xF, 0xF, false)));
}

/* v[k1] *= w^(lane k1) (k1 >= 1; tw: the forward or inverse table of S entries).  The table is
 * read at k1 = 1, 8, 16, 24 only (lane-scattered loads, 64 distinct lines per instruction, were
 * the pass's bottleneck: 31 of them per transform) and the powers in between are formed by
 * multiplying by w^lane: at most 7 products per twiddle, within the fp32 tie tolerance */
__device__ __forceinline__ void sg_twiddle_rows(float2 (&v)[32], const float2 *__restrict__ tw, int lane) {
	const float2 b = tw[lane];
	float2 t8[3];
#pragma unroll
	for (int q = 0; q < 3; q++)
		t8[q] = tw[lane * 8 * (q + 1)];
	float2 t = b;
#pragma unroll
	for (int k1 = 1; k1 < 32; k1++) {
		if (k1 > 1)
			t = (k1 & 7) ? sg_cmulf(t, b) : t8[(k1 >> 3) - 1];
		v[k1] = sg_cmulf(v[k1], t);
	}
}

/* 2048-point DFT of the wave's line, four-step 32 x 64: lane l holds x[64 j + l] in v[j]; on
 * return lane m holds X[m / 2 + 32 k + 1024 (m % 2)] in v[k] (INV: conjugate roots, the
 * unnormalised inverse).  col: the wave's LDS (32 rows of 66 float2).  tw: the forward table
 * (tw + 2048 is the inverse one). */
template <bool INV>
__device__ __forceinline__ void sg_fft2048_wave(float2 (&v)[32], float2 *col, const float2 *__restrict__ tw, int lane) {
	constexpr int S = 2048, P = 32, TR = 66;
	const float2 *twd = INV ? tw + S : tw;
	sg_dft32_lane<INV>(v);
	sg_twiddle_rows(v, twd, lane);
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
	for (int k1 = 0; k1 < P; k1++)
		col[k1 * TR + lane] = v[k1];
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	const int km = lane >> 1, hm = lane & 1;
#pragma unroll
	for (int i = 0; i < P; i++)
		v[i] = col[km * TR + 2 * i + hm];
	sg_dft32_lane<INV>(v);
	if (hm) {	/* odd lanes: the radix-2 stage's twiddles (uniform loads, SGPR operands) */
#pragma unroll
		for (int k = 1; k < P; k++) {
			const float2 t = twd[32 * k];
			v[k] = sg_cmulk(v[k], sg_v2f{t.x, t.y});
		}
	}
	const float sg1 = hm ? -1.0f : 1.0f;
	const sg_v2f s2 = sg_v2f{sg1, sg1};
#pragma unroll
	for (int k = 0; k < P; k++)
		v[k] = sg_pm_add(v[k], sg_pair_swap(v[k]), s2);
}

#ifndef SG_WCOL_WPE
#define SG_WCOL_WPE 2
#endif
#define SG_WCOL_CS 2120	/* LDS float2 per column: 2048 (strip) / 32 x 66 (transposes), +8 for the strip's banks */
/* physical LDS row of strip row r in column c of a CW-column strip, so that the strip's 8-byte
 * stores (32 banks, 16-lane groups) and its 8-byte reads (64 banks, 32-lane groups, CS = 8 mod 32)
 * are both conflict-free (a 2-way conflict on the stores was 20 % of the column pass's LDS
 * cycles).  CW = 4: a store group is 4 rows x 4 columns, columns 2, 3 XOR the row with 4; CW = 8:
 * 2 rows x 8 columns, column c XORs it with 2 (c / 2). */
template <int CW = 4>
__device__ __forceinline__ int sg_strip_row(int r, int c) {
	return CW == 8 ? r ^ ((c >> 1) << 1) : r ^ ((c >> 1) << 2);
}
/* specp: the reference spectrum in the column pass's lane order, specp[(kx 32 + k) 64 + 2 km + hm]
 * = spec[ky][kx] at ky = km + 32 k + 1024 hm (kx < S / 2), so that the pass reads its reference
 * column with one coalesced 512-B load per k (issued before its forward transform) instead of
 * staging a strip through LDS between two block barriers. */
/* the reference spectrum's forward column pass at S = 2048, wave-level (k_reg_cols_xpower_w's
 * strip staging and transform): columns [0, S/2) of the row-transformed reference plane, written
 * straight into specp's lane order (coalesced 512-B stores), and column 0 also back in natural
 * order (the packed column's wave reads it by ky).  Replaces k_reg_cols + k_spec_perm on the
 * wave-level path (one workgroup per CU there, 0.39 ms beside the pairs' forward rows). */
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SG_WCOL_WPE)))
k_reg_cols_fwd_perm_w(float2 *__restrict__ spec, float2 *__restrict__ specp, const float2 *__restrict__ tw) {
	constexpr int S = 2048, P = 32, CS = SG_WCOL_CS;
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	float2 *lds = (float2 *)smem;
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const int x0 = blockIdx.x * 4;
	float2 *col = lds + wave * CS;
	const int sw = sg_strip_row<4>(0, wave);	/* sg_strip_row of this wave's column: lane ^ sw */
#pragma unroll
	for (int it = 0; it < P; it++) {
		const int r = (threadIdx.x >> 2) + 64 * it, c = threadIdx.x & 3;
		lds[c * CS + sg_strip_row(r, c)] = spec[(size_t)r * S + x0 + c];
	}
	__syncthreads();
	float2 v[P];
#pragma unroll
	for (int j = 0; j < P; j++)
		v[j] = col[64 * j + (lane ^ sw)];
	sg_fft2048_wave<false>(v, col, tw, lane);
	const int kx = x0 + wave, km = lane >> 1, hm = lane & 1;
	float2 *sp = specp + (size_t)kx * S;
#pragma unroll
	for (int k = 0; k < P; k++)
		sp[64 * k + lane] = v[k];
	if (kx == 0) {
#pragma unroll
		for (int k = 0; k < P; k++)
			spec[(size_t)(km + 32 * k + 1024 * hm) * S] = v[k];
	}
}

template <bool PERM, int CW>
__global__ void __launch_bounds__(64 * CW) __attribute__((amdgpu_waves_per_eu(SG_WCOL_WPE)))
k_reg_cols_xpower_w(float2 *__restrict__ work, const float2 *__restrict__ spec, const float2 *__restrict__ specp,
		const float2 *__restrict__ tw, int xcdmap) {
	constexpr int S = 2048, H = 1024, P = 32, CS = SG_WCOL_CS, TR = 66;
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	float2 *lds = (float2 *)smem;
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const int x0 = sg_xcd_strip(blockIdx.x, gridDim.x, xcdmap) * CW, pair = blockIdx.y;
	float2 *base = work + (size_t)pair * S * S + x0;
	float2 *col = lds + wave * CS;
	const int sw = sg_strip_row<CW>(0, wave);	/* sg_strip_row of this wave's column: lane ^ sw */
	auto wsync = [] { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); };
	/* strip -> LDS: rows of 4 columns (32 B), column c at lds + c CS */
#pragma unroll
	for (int it = 0; it < P; it++) {
		const int r = threadIdx.x / CW + 64 * it, c = threadIdx.x % CW;
		lds[c * CS + sg_strip_row<CW>(r, c)] = base[(size_t)r * S + c];
	}
	__syncthreads();
	float2 v[P];
#pragma unroll
	for (int j = 0; j < P; j++)
		v[j] = col[64 * j + (lane ^ sw)];
	const int km = lane >> 1, hm = lane & 1;
	const int kx = (x0 + wave) & (H - 1);
	/* PERM: the reference column's loads issued now, in flight during the forward transform */
	float2 r[P];
	if (PERM && kx) {
		const float2 *sp = specp + (size_t)kx * S;
#pragma unroll
		for (int k = 0; k < P; k++)
			r[k] = sp[64 * k + lane];
	}
	/* ---- forward ---- */
	sg_fft2048_wave<false>(v, col, tw, lane);
	/* ---- cross power at ky = km + 32 k + 1024 hm ---- */
	/* PERM: the reference column from specp, in lane order.  Otherwise the reference spectrum's
	 * strip through LDS (coalesced 32-B rows, as the work strip; read per lane at its ky it
	 * touched 64 rows per instruction).  A packed column 0's wave keeps its LDS column for
	 * Z(-ky) and reads its reference column directly. */
	if (!PERM) {
		__syncthreads();	/* every wave is done with its transposes */
		const int kx0 = x0 & (H - 1);	/* a strip lies inside one half */
#pragma unroll
		for (int it = 0; it < P; it++) {
			const int r = threadIdx.x / CW + 64 * it, c = threadIdx.x % CW;
			if (kx0 + c)
				lds[c * CS + r] = spec[(size_t)r * S + kx0 + c];
		}
		__syncthreads();
	}
	if (kx) {
		if (PERM) {
#pragma unroll
			for (int k = 0; k < P; k++)
				v[k] = sg_rconjf(r[k], v[k]);
		} else {
#pragma unroll
			for (int k = 0; k < P; k++)
				v[k] = sg_rconjf(col[km + 32 * k + 1024 * hm], v[k]);
		}
	} else {	/* packed column: Z = F0 + i FN, the reference likewise; needs Z(-ky) */
		wsync();
#pragma unroll
		for (int k = 0; k < P; k++)
			col[km + 32 * k + 1024 * hm] = v[k];
		wsync();
#pragma unroll
		for (int k = 0; k < P; k++) {
			const int ky = km + 32 * k + 1024 * hm, m = (S - ky) & (S - 1);
			const float2 zk = v[k], zm = col[m], r1 = spec[(size_t)ky * S], r2 = spec[(size_t)m * S];
			const float2 f0 = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
			const float2 fn = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
			const float2 r0 = make_float2(0.5f * (r1.x + r2.x), 0.5f * (r1.y - r2.y));
			const float2 rn = make_float2(0.5f * (r1.y + r2.y), -0.5f * (r1.x - r2.x));
			const float2 p0 = sg_rconj(r0, f0), pn = sg_rconj(rn, fn);
			v[k] = make_float2(p0.x - pn.y, p0.y + pn.x);
		}
	}
	/* ---- inverse (unnormalised, FFTW_BACKWARD) ---- */
	{
		const float sg1 = hm ? -1.0f : 1.0f;
		const sg_v2f s2 = sg_v2f{sg1, sg1};
#pragma unroll
		for (int k = 0; k < P; k++)
			v[k] = sg_pm_add(v[k], sg_pair_swap(v[k]), s2);
	}
	if (hm) {
#pragma unroll
		for (int k = 1; k < P; k++) {
			const float2 t = tw[S + 32 * k];
			v[k] = sg_cmulk(v[k], sg_v2f{t.x, t.y});
		}
	}
	sg_dft32_lane<true>(v);
	wsync();
#pragma unroll
	for (int i = 0; i < P; i++)
		col[km * TR + 2 * i + hm] = v[i];
	wsync();
#pragma unroll
	for (int k1 = 0; k1 < P; k1++)
		v[k1] = col[k1 * TR + lane];
	sg_twiddle_rows(v, tw + S, lane);
	sg_dft32_lane<true>(v);
	wsync();
#pragma unroll
	for (int j = 0; j < P; j++)
		col[64 * j + (lane ^ sw)] = v[j];
	__syncthreads();
	{	/* every LDS read issued before the stores (one LDS latency, not eight) */
		float2 o[P];
#pragma unroll
		for (int it = 0; it < P; it++) {
			const int r = threadIdx.x / CW + 64 * it, c = threadIdx.x % CW;
			o[it] = lds[c * CS + sg_strip_row<CW>(r, c)];
		}
#pragma unroll
		for (int it = 0; it < P; it++) {
			const int r = threadIdx.x / CW + 64 * it, c = threadIdx.x % CW;
			base[(size_t)r * S + c] = o[it];
		}
	}
}

/* Wave-level fp32 forward row pass at S = 2048: one wave per row, `rpw` rows per wave (4 rows
 * per workgroup at a time, no block barrier; the wave's next row is fetched while this one is
 * transformed: one row at a time left every wave waiting out the full load latency, 2 waves per
 * SIMD being all the LDS allows), the row of a + i b through sg_fft2048_wave, then staged in
 * natural order in the wave's LDS for the separation into the half spectra A, B
 * (k_reg_rows_fwd_half's arithmetic); the frames' energies summed per wave */
/* QF (SG_REG_QFOLD, A/B): QualityEstimate's SubSample (quality.c:223-234) folded in.  A wave then
 * takes rpw consecutive rows from a multiple of 3 (rpw a multiple of 3), so each 3 x 3 block's three
 * rows pass through one wave: before a row's transform its samples (a | b << 16) go through the
 * wave's LDS, each lane adds the row's three-sample sums of outputs lane + 64 m (m < 11, xs = 682)
 * to registers, and the third row of a block writes the 9-sample means to qbuf (frame q = qbase +
 * 2 pair (+1 for b)) and keeps the middle rows' maximum for qmax (k_quality_sub's arithmetic). */
template <bool QF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SG_WCOL_WPE)))
k_reg_rows_fwd_half_w(SgSel sel, const int *__restrict__ fa, const int *__restrict__ fb,
		const float2 *__restrict__ tw, float2 *__restrict__ work, unsigned long long *__restrict__ energy, int rpw,
		uint16_t *__restrict__ qbuf, unsigned int *__restrict__ qmax, int qbase) {
	constexpr int S = 2048, H = 1024, P = 32;
	constexpr int XS = (S - 1) / 3, YS = (S - 1) / 3, QM = (XS + 63) / 64;
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const int row0 = QF ? (blockIdx.x * 4 + wave) * rpw : blockIdx.x * 4 * rpw + wave, pair = blockIdx.y;
	if (QF && row0 >= S)
		return;
	float2 *col = (float2 *)smem + wave * SG_WCOL_CS;
	const size_t plane = (size_t)S * S;
	const uint16_t *pa = sel.frame(fa[pair]);
	const int b = fb[pair];
	const uint16_t *pb = b >= 0 ? sel.frame(b) : nullptr;
	const size_t rp = (size_t)sel.rp;
	uint16_t ua[P], ub[P];
	auto fetch = [&](int row) {
#pragma unroll
		for (int j = 0; j < P; j++)
			ua[j] = pa[(size_t)row * rp + 64 * j + lane];
		if (pb) {
#pragma unroll
			for (int j = 0; j < P; j++)
				ub[j] = pb[(size_t)row * rp + 64 * j + lane];
		}
	};
	fetch(row0);
	unsigned long long ea = 0, eb = 0;
	const int km = lane >> 1, hm = lane & 1;
	uint32_t qa[QM], qb[QM], mxa = 0, mxb = 0;
	if constexpr (QF) {
#pragma unroll
		for (int m = 0; m < QM; m++)
			qa[m] = qb[m] = 0;
	}
	for (int rr = 0; rr < rpw; rr++) {
		const int row = QF ? row0 + rr : row0 + 4 * rr;
		if (QF && row >= S)
			break;
		if constexpr (QF) {	/* the row's samples through LDS, its three-sample sums added */
			uint32_t *cu = (uint32_t *)col;
			if (row < 3 * YS) {
#pragma unroll
				for (int j = 0; j < P; j++)
					cu[64 * j + lane] = (uint32_t)ua[j] | ((uint32_t)(pb ? ub[j] : 0) << 16);
				__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
				for (int m = 0; m < QM; m++) {
					const int i = 64 * m + lane;
					if (i < XS) {
						const uint32_t d0 = cu[3 * i], d1 = cu[3 * i + 1], d2 = cu[3 * i + 2];
						qa[m] += (d0 & 0xFFFFu) + (d1 & 0xFFFFu) + (d2 & 0xFFFFu);
						qb[m] += (d0 >> 16) + (d1 >> 16) + (d2 >> 16);
					}
				}
				__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");	/* the transform reuses col */
			}
		}
		float2 v[P];
#pragma unroll
		for (int j = 0; j < P; j++) {
			const uint32_t u = ua[j];
			ea += (unsigned long long)(u * u);
			v[j] = make_float2((float)u, 0.0f);
		}
		if (pb) {
#pragma unroll
			for (int j = 0; j < P; j++) {
				const uint32_t u = ub[j];
				eb += (unsigned long long)(u * u);
				v[j].y = (float)u;
			}
		}
		if (QF ? (rr + 1 < rpw && row + 1 < S) : rr + 1 < rpw)
			fetch(QF ? row + 1 : row + 4);
		if constexpr (QF) {	/* a block's third row: the 9-sample means (SubSample, :223-234) */
			if (row % 3 == 2 && row < 3 * YS) {
				const int t = row / 3;
				const bool middle = t >= 1 && t <= YS - 2;
				uint16_t *da = qbuf + (size_t)(qbase + 2 * pair) * XS * YS + (size_t)t * XS;
#pragma unroll
				for (int m = 0; m < QM; m++) {
					const int i = 64 * m + lane;
					const uint32_t va = qa[m] / 9u, vb = qb[m] / 9u;
					if (i < XS) {
						da[i] = (uint16_t)va;
						if (middle && va > 0 && va < 65530 && va > mxa)
							mxa = va;
						if (pb) {
							da[(size_t)XS * YS + i] = (uint16_t)vb;
							if (middle && vb > 0 && vb < 65530 && vb > mxb)
								mxb = vb;
						}
					}
					qa[m] = qb[m] = 0;
				}
			}
		}
		sg_fft2048_wave<false>(v, col, tw, lane);
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		/* natural order, the upper half 8 entries up: lanes km and km + 8 (hm = 0 / 1) of a
		 * 16-lane store group on different banks */
#pragma unroll
		for (int k = 0; k < P; k++)
			col[km + 32 * k + (1024 + 8) * hm] = v[k];
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
		float2 *out = work + (size_t)pair * plane + (size_t)row * S;
#pragma unroll 4
		for (int q = 0; q < H / 64; q++) {
			const int kx = 64 * q + lane;
			const float2 zk = col[kx], zm = col[(kx ? S - kx : H) + 8];
			float2 A, B;
			if (kx == 0) {
				A = make_float2(zk.x, zm.x);	/* A(0) + i A(S/2) */
				B = make_float2(zk.y, zm.y);
			} else {
				A = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
				B = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
			}
			out[kx] = A;
			out[H + kx] = B;
		}
		__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");	/* the next row's transposes reuse col */
	}
	for (int o = 32; o > 0; o >>= 1) {
		ea += __shfl_xor(ea, o, 64);
		eb += __shfl_xor(eb, o, 64);
	}
	if (lane == 0) {
		atomicAdd(energy + fa[pair], ea);
		if (b >= 0)
			atomicAdd(energy + b, eb);
	}
	if constexpr (QF) {
		for (int o = 32; o > 0; o >>= 1) {
			const uint32_t ta = (uint32_t)__shfl_xor((int)mxa, o, 64), tb = (uint32_t)__shfl_xor((int)mxb, o, 64);
			mxa = ta > mxa ? ta : mxa;
			mxb = tb > mxb ? tb : mxb;
		}
		if (lane == 0 && mxa)
			atomicMax(qmax + qbase + 2 * pair, mxa);
		if (lane == 0 && mxb)
			atomicMax(qmax + qbase + 2 * pair + 1, mxb);
	}
}

/* Wave-level fp32 inverse row pass + arg-max at S = 2048: one wave per row; the packed
 * spectrum Qa + i Qb rebuilt per element as k_reg_rows_inv_half_argmax does, the inverse
 * transform by sg_fft2048_wave<true> (its permuted output order only changes which index a
 * value carries), the row's top-2 reduced in the wave */
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SG_WCOL_WPE)))
k_reg_rows_inv_half_w(const float2 *__restrict__ work, const float2 *__restrict__ tw, SgBest *__restrict__ best) {
	constexpr int S = 2048, H = 1024, P = 32;
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const int row = blockIdx.x * 4 + wave, pair = blockIdx.y;
	float2 *col = (float2 *)smem + wave * SG_WCOL_CS;
	const float2 *in = work + (size_t)pair * S * S + (size_t)row * S;
	float2 v[P];
	/* every load unconditional (all 64 in flight; the packed-pair lane's branch had split them
	 * into dependent groups), the packing and conjugation applied after */
	float2 ra[P], rb[P];
#pragma unroll
	for (int j = 0; j < P; j++) {
		const int i = 64 * j + lane;
		const int src = (i & (H - 1)) == 0 ? 0 : (i < H ? i : S - i);
		ra[j] = in[src];
		rb[j] = in[H + src];
	}
#pragma unroll
	for (int j = 0; j < P; j++) {
		const int i = 64 * j + lane;
		float2 qa = ra[j], qb = rb[j];
		if ((i & (H - 1)) == 0) {	/* kx = 0 or S/2: the packed real pair */
			qa = make_float2(i ? qa.y : qa.x, 0.0f);
			qb = make_float2(i ? qb.y : qb.x, 0.0f);
		} else if (i >= H) {
			qa.y = -qa.y;
			qb.y = -qb.y;
		}
		v[j] = make_float2(qa.x - qb.y, qa.y + qb.x);
	}
	sg_fft2048_wave<true>(v, col, tw, lane);
	const int km = lane >> 1, hm = lane & 1;
	SgTop2T<float> ta, tb;
	sg_top2t_init(ta);
	sg_top2t_init(tb);
#pragma unroll
	for (int k = 0; k < P; k++) {
		const int idx = row * S + km + 32 * k + 1024 * hm;
		sg_top2t_add_inc(ta, v[k].x, idx);	/* idx grows with k */
		sg_top2t_add_inc(tb, v[k].y, idx);
	}
	sg_top2t_wave(ta);
	sg_top2t_wave(tb);
	const SgTop2 wa = sg_top2t_wide(ta), wb = sg_top2t_wide(tb);
	if (lane == 0) {
		best[(size_t)pair * S + row].a = wa;
		best[(size_t)pair * S + row].b = wb;
	}
}

/* per-pair result of a registration batch (frame a = the real part, frame b = the imaginary) */
struct SgRegOut {
	int sx[2], sy[2];	/* the shifts (:344-351) */
	int idx[2];		/* arg-max (row-major) */
	int amb[2];		/* near tie: the runner-up lies within `tol` of the maximum */
	double v[2], v2[2], thr[2];	/* maximum, runner-up, max - tol */
};

/* tolerance of a correlation value: 2^tol_exp S^2 ||ref|| ||img|| (the unnormalised inverse
 * scales the exact correlation sum_n ref(n+k) img(n) by S^2, and by Cauchy-Schwarz no entry
 * exceeds S^2 ||ref|| ||img||).  fp64 passes: 2^-32, many orders of magnitude above their
 * rounding; fp32 passes: 2^-15 = 3.1e-5, against a measured worst error of 2.8e-7 of that scale
 * at S = 2048 (scipy's complex64 FFT, the synthetic pair) and a log2(S^2) eps32 bound of 1.3e-6
 * per transform.  A maximum that beats every other entry by more than tol is the exact
 * maximum. */
__device__ __forceinline__ double sg_reg_tol(int S, unsigned long long eref, unsigned long long eimg, int tol_exp) {
	return ldexp((double)S * (double)S * sqrt((double)eref) * sqrt((double)eimg), tol_exp);
}

/* per pair: reduce the row / strip partials in order, convert to (shiftx, shifty) (:344-351),
 * flag near ties against the frames' energies */
__global__ void __launch_bounds__(256)
k_reg_final(const SgBest *__restrict__ best, int S, int count, const int *__restrict__ fa,
		const int *__restrict__ fb, int ref, const unsigned long long *__restrict__ energy, int tol_exp,
		SgRegOut *__restrict__ out) {
	__shared__ SgBest red[4];
	const int pair = blockIdx.x;
	SgTop2 ta, tb;
	sg_top2_init(ta);
	sg_top2_init(tb);
	for (int r = threadIdx.x; r < count; r += blockDim.x) {
		const SgBest b = best[(size_t)pair * count + r];
		sg_top2_merge(ta, b.a.v, b.a.v2, b.a.i);
		sg_top2_merge(tb, b.b.v, b.b.v2, b.b.i);
	}
	sg_best_block(ta, tb, red);
	if (threadIdx.x == 0) {
		SgRegOut o;
		const SgTop2 t[2] = {ta, tb};
		const int fr[2] = {fa[pair], fb[pair]};
		for (int k = 0; k < 2; k++) {
			int sy = t[k].i / S, sx = t[k].i % S;
			if (sy > S / 2)
				sy -= S;
			if (sx > S / 2)
				sx -= S;
			o.sx[k] = sx;
			o.sy[k] = sy;
			o.idx[k] = t[k].i;
			o.v[k] = t[k].v;
			o.v2[k] = t[k].v2;
			const double tol = fr[k] >= 0 ? sg_reg_tol(S, energy[ref], energy[fr[k]], tol_exp) : 0.0;
			o.thr[k] = t[k].v - tol;
			o.amb[k] = fr[k] >= 0 && !(t[k].v - t[k].v2 > tol);
		}
		out[pair] = o;
	}
}

/* CAND: instead of the arg-max, append every index whose correlation reaches the pair's
 * threshold (SgRegOut::thr, near ties only) to the candidate list of its frame */
template <class C, bool CAND>
__global__ void __launch_bounds__(512)
k_reg_rows_inv_half_argmax(const C *__restrict__ work, int S, const C *__restrict__ tw,
		SgBest *__restrict__ best, const SgRegOut *__restrict__ res, SgCand *__restrict__ cand) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	C *buf = (C *)smem;
	__shared__ SgBest red[8];
	const int row = blockIdx.x, pair = blockIdx.y, H = S >> 1;
	const C *in = work + (size_t)pair * S * S + (size_t)row * S;
	typedef typename SgReal<C>::T T;
	SgTop2T<T> ta, tb;
	sg_top2t_init(ta);
	sg_top2t_init(tb);
	double thr[2] = {INFINITY, INFINITY};
	if (CAND) {
		const SgRegOut r = res[pair];
		if (!r.amb[0] && !r.amb[1])
			return;
		thr[0] = r.amb[0] ? r.thr[0] : INFINITY;
		thr[1] = r.amb[1] ? r.thr[1] : INFINITY;
	}
	sg_fft_io(buf, S, 1, S, tw, true,
			[&](int, int i) {
				C qa, qb;
				if ((i & (H - 1)) == 0) {	/* kx = 0 or S/2: the packed real pair */
					const C a = in[0], b = in[H];
					qa = sg_mk<C>(i ? a.y : a.x, (T)0);
					qb = sg_mk<C>(i ? b.y : b.x, (T)0);
				} else if (i < H) {
					qa = in[i];
					qb = in[H + i];
				} else {
					const C a = in[S - i], b = in[H + S - i];
					qa = sg_mk<C>(a.x, -a.y);
					qb = sg_mk<C>(b.x, -b.y);
				}
				return sg_mk<C>(qa.x - qb.y, qa.y + qb.x);
			},
			[&](int, int j, C c) {
				const int idx = row * S + j;
				if (CAND) {
					sg_cand_push(cand + 2 * pair, c.x, thr[0], idx);
					sg_cand_push(cand + 2 * pair + 1, c.y, thr[1], idx);
					return;
				}
				sg_top2t_add(ta, c.x, idx);
				sg_top2t_add(tb, c.y, idx);
			});
	if (CAND)
		return;
	SgTop2 wa = sg_top2t_wide(ta), wb = sg_top2t_wide(tb);
	sg_best_block(wa, wb, red);
	if (threadIdx.x == 0) {
		best[(size_t)pair * S + row].a = wa;
		best[(size_t)pair * S + row].b = wb;
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
k_quality_sub(SgSel sel, int al, const int *__restrict__ qframes, int S, int xs, int ys,
		uint16_t *__restrict__ qbuf, unsigned int *__restrict__ qmax) {
	/* SG_QROWS output rows per workgroup; a thread forms two adjacent outputs from three
	 * 12-byte (6-pixel, dword-aligned) loads, one per input row */
	const int q = blockIdx.y;
	const uint16_t *frame = sel.frame(qframes[q]);
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
				const uint16_t *q16 = frame + (size_t)(3 * j + y) * sel.rp + 6 * k;
				if (al) {	/* even side, pitches and base: the 12 bytes are dword aligned */
					const uint32_t *p = (const uint32_t *)q16;
					d[jj][y][0] = p[0];
					d[jj][y][1] = p[1];
					d[jj][y][2] = p[2];
				} else {
					d[jj][y][0] = (uint32_t)q16[0] | ((uint32_t)q16[1] << 16);
					d[jj][y][1] = (uint32_t)q16[2] | ((uint32_t)q16[3] << 16);
					d[jj][y][2] = (uint32_t)q16[4] | ((uint32_t)q16[5] << 16);
				}
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

/* k_quality_grad streamed down a band: one wave per (60-column band, SG_QGS_ROWS output rows,
 * frame) of the 10 % margins' interior, lane l at column x0 - 2 + l.  Each input row is loaded
 * and stretched once (SG_QGS_PF rows in flight), its horizontal 3-sum formed with two lane
 * shuffles, and rolling three-row windows give the smoothed row, the thresholded map and the
 * gradient of output row y as rows y + 2 arrive.  Only the interior's neighbourhood is read (the
 * tiled kernel read every row and column), and no LDS or barrier: 290 -> 190 us per configs[1]
 * step (61 k tiled workgroups before), registration 3.20 -> 3.10 ms (profiles/r05x_*).  Same
 * integer sums, so the same result bit for bit. */
#define SG_QGS_ROWS 64
#define SG_QGS_PF 8
__global__ void __launch_bounds__(64)
k_quality_grad_s(const uint16_t *__restrict__ qbuf, int xs, int ys, const unsigned int *__restrict__ qmax,
		unsigned long long *__restrict__ acc) {
	const int q = blockIdx.z, lane = threadIdx.x;
	const uint16_t *b = qbuf + (size_t)q * xs * ys;
	const unsigned int mx = qmax[q];
	const bool stretch = mx > 0;
	const double mult = stretch ? (double)60000 / (double)mx : 1.0;
	const int yb = (int)((double)ys * 0.1) + 1;
	const int xb = (int)((double)xs * 0.1) + 1;
	const int x0 = xb + 60 * blockIdx.x, c = x0 - 2 + lane;
	const int y0 = yb + SG_QGS_ROWS * blockIdx.y;
	const int y1 = min(y0 + SG_QGS_ROWS, ys - yb);	/* output rows [y0, y1) */
	const bool in_x = c >= xb && c < xs - xb;	/* the map's and the output's column range */
	const bool out_lane = lane >= 2 && lane < 62 && in_x;
	const bool col_ok = c >= 0 && c < xs, sm_x = c >= 1 && c <= xs - 2;
	unsigned long long val = 0;
	unsigned int pix = 0, cnt = 0;
	/* rolling state: horizontal sums of the last three stretched rows, the last two smoothed
	 * rows (value, right neighbour's) and the last two rows' horizontally OR-ed map bits */
	unsigned int h0 = 0, h1 = 0;
	int sm_prev = 0, smr_prev = 0;
	bool th_prev2 = false, th_prev = false;
	const int ya = y0 - 2, yz = y1 + 1;	/* input rows [ya, yz] */
	for (int g = ya; g <= yz; g += SG_QGS_PF) {
		unsigned int raw[SG_QGS_PF];
#pragma unroll
		for (int k = 0; k < SG_QGS_PF; k++) {
			const int yi = g + k;
			raw[k] = (col_ok && yi >= 0 && yi < ys && yi <= yz) ? (unsigned int)b[(size_t)yi * xs + c] : 0u;
		}
#pragma unroll
		for (int k = 0; k < SG_QGS_PF; k++) {
			const int yi = g + k;
			if (yi > yz)
				break;
			unsigned int st = raw[k];
			if (stretch && col_ok && yi >= 0 && yi < ys) {
				st = (unsigned int)((double)st * mult);
				if (st > 65535u)
					st = 65535u;
			}
			const unsigned int h = st + (unsigned int)__shfl_up((int)st, 1, 64) + (unsigned int)__shfl_down((int)st, 1, 64);
			if (yi >= ya + 2) {
				/* smoothed row qy = yi - 1 from the horizontal sums of rows yi - 2 .. yi */
				const int qy = yi - 1;
				const int sm = (sm_x && qy >= 1 && qy <= ys - 2) ? (int)((h0 + h1 + h) / 9) : 0;
				const bool thr = sm >= SG_Q_THRESHOLD && in_x && qy >= yb && qy < ys - yb;
				/* both shuffles by every lane (a short-circuit || would run them under a partial
				 * exec mask) */
				const int thn = (int)thr, thl = __shfl_up(thn, 1, 64), thr1 = __shfl_down(thn, 1, 64);
				const bool th = (thn | thl | thr1) != 0;
				const int smr = __shfl_down(sm, 1, 64);
				/* output row yo = qy - 1: its row (sm_prev), the row below (sm), the map rows
				 * yo - 1 .. yo + 1 */
				const int yo = qy - 1;
				if (yo >= y0 && out_lane) {
					if (sm_prev >= SG_Q_THRESHOLD)
						cnt++;
					if (th_prev2 || th_prev || th) {
						const long long d1 = sm_prev - smr_prev;
						const long long d2 = sm_prev - sm;
						val += (unsigned long long)(d1 * d1 + d2 * d2);
						pix++;
					}
				}
				sm_prev = sm;
				smr_prev = smr;
				th_prev2 = th_prev;
				th_prev = th;
			}
			h0 = h1;
			h1 = h;
		}
	}
	unsigned long long p = pix, n = cnt;
	for (int o = 32; o > 0; o >>= 1) {
		val += __shfl_down(val, o, 64);
		p += __shfl_down(p, o, 64);
		n += __shfl_down(n, o, 64);
	}
	if (lane == 0) {
		if (val)
			atomicAdd(acc + q * 3, val);
		if (p)
			atomicAdd(acc + q * 3 + 1, p);
		if (n)
			atomicAdd(acc + q * 3 + 2, n);
	}
}

/* ---------------------------------------------------------------------------------------
 * Any selection side (FFTW plans every S, registration.c:251-257): mixed-radix Stockham
 * passes (radix 8, 4, 2, 3, 5, 7) in LDS, one line per workgroup, ping-pong between two LDS
 * buffers; a side with a prime factor above 7 goes through Bluestein's chirp-z transform
 * (X_k = c_k sum_j (x_j c_j) conj(c_{k-j}), c_j = exp(-i pi j^2 / n), as an M-point power-of-two
 * convolution, M >= 2n - 1).  Columns are transformed as rows of the transposed plane:
 *   rows(u16 -> spectrum) -> transpose -> rows -> cross power -> inverse rows -> transpose ->
 *   inverse rows + top-2 arg-max.
 * Same unnormalised FFTW_FORWARD / FFTW_BACKWARD convention and pair packing (a + i b) as the
 * power-of-two passes; the cross power works on the transposed spectra directly (the mirror of
 * (r, c) is ((S - r) % S, (S - c) % S) in either layout).
 * ------------------------------------------------------------------------------------- */
#define SG_GEN_MAXPASS 16
struct SgGenPlan {
	int n, npass;
	int radix[SG_GEN_MAXPASS];
	int bluestein, m;	/* Bluestein: convolution length m (power of two) */
};

/* cos / sin of 2 pi m / R, m < R (R = 3, 5, 7) */
template <int R>
__device__ __forceinline__ void sg_unit(int m, double &c, double &s) {
	if (m == 0) {
		c = 1.0;
		s = 0.0;
		return;
	}
	const int mm = m <= R / 2 ? m : R - m;
	const double sg = m <= R / 2 ? 1.0 : -1.0;
	if constexpr (R == 3) {
		c = -0.5;
		s = 0.86602540378443864676;
	} else if constexpr (R == 5) {
		c = mm == 1 ? 0.30901699437494742410 : -0.80901699437494742410;
		s = mm == 1 ? 0.95105651629515357212 : 0.58778525229247312917;
	} else {
		c = mm == 1 ? 0.62348980185873353053 : (mm == 2 ? -0.22252093395631440429 : -0.90096886790241912624);
		s = mm == 1 ? 0.78183148246802980871 : (mm == 2 ? 0.97492791218182360702 : 0.43388373911755812048);
	}
	s *= sg;
}

/* in-register DFT of an odd prime R: y_k = sum_j v_j w^{jk}, w = exp(-+2 pi i / R), from the
 * symmetric sums t_j = v_j + v_{R-j} and differences u_j = v_j - v_{R-j} (j <= R/2): y_k and
 * y_{R-k} share a = v_0 + sum_j t_j cos(2 pi jk / R) and b = sum_j u_j sin(2 pi jk / R),
 * y_k = a -+ i b, y_{R-k} = a +- i b (half the multiplies of the direct sum and ~half its live
 * registers: the radix-7 pass spilled at 128 VGPRs with the direct form).  Its rounding is far
 * below the fp64 tie tolerance (sg_reg_tol). */
template <int R>
__device__ __forceinline__ void sg_dft_odd(sg_c64 (&v)[R], bool inv) {
	constexpr int H = R / 2;
	sg_c64 t[H + 1], u[H + 1];
	double y0x = v[0].x, y0y = v[0].y;
#pragma unroll
	for (int j = 1; j <= H; j++) {
		t[j] = make_double2(v[j].x + v[R - j].x, v[j].y + v[R - j].y);
		u[j] = make_double2(v[j].x - v[R - j].x, v[j].y - v[R - j].y);
		y0x += t[j].x;
		y0y += t[j].y;
	}
#pragma unroll
	for (int k = 1; k <= H; k++) {
		double ax = v[0].x, ay = v[0].y, bx = 0.0, by = 0.0;
#pragma unroll
		for (int j = 1; j <= H; j++) {
			double c, sn;
			sg_unit<R>((j * k) % R, c, sn);
			ax += t[j].x * c;
			ay += t[j].y * c;
			bx += u[j].x * sn;
			by += u[j].y * sn;
		}
		/* forward: y_k = a - i b = (ax + by, ay - bx); inverse: a + i b */
		if (!inv) {
			v[k] = make_double2(ax + by, ay - bx);
			v[R - k] = make_double2(ax - by, ay + bx);
		} else {
			v[k] = make_double2(ax - by, ay + bx);
			v[R - k] = make_double2(ax + by, ay - bx);
		}
	}
	v[0] = make_double2(y0x, y0y);
}

/* Mixed-radix Stockham passes on one line, in place in ONE LDS buffer (72 KB at S = 4000, so
 * two workgroups share a CU; the round-3 ping-pong between two buffers held one workgroup of 4
 * waves per CU).  Work item j of a radix-R pass (j < n / R, k = j mod Ns) reads elements
 * j + r n / R, twiddles them by w^(r k n / (Ns R)), and writes (j - k) R + k + r Ns: every item's
 * inputs are loaded into registers before the barrier and stored after it.  The first pass reads
 * the line straight from memory (ld(i)), the last pass hands its outputs to st(i, v): two LDS
 * round trips fewer.  Items per thread: blockDim >= n / 8, and >= n / 7 when 7 divides n (host-
 * sized), so a radix-R pass has at most 4 (R = 2), 3 (3), 2 (4, 5) or 1 (7, 8) items per thread
 * (two radix-7 items per thread spilled at the 128 VGPRs of two workgroups per CU). */
template <int R> struct SgGenItems { static constexpr int v = R == 2 ? 4 : (R == 3 ? 3 : (R == 8 || R == 7 ? 1 : 2)); };

template <int R, bool IN_MEM, bool OUT_MEM, class LD, class ST>
__device__ __forceinline__ void sg_gen_pass_ip(sg_c64 *buf, int n, int Ns, const sg_c64 *__restrict__ tw, bool inv,
		LD &ld, ST &st, int tid, int nt) {
	constexpr int MAXI = SgGenItems<R>::v;
	const int per = n / R, tstep = n / (Ns * R);
	sg_c64 v[MAXI][R];
#pragma unroll
	for (int it = 0; it < MAXI; it++) {
		const int j = tid + it * nt;
		if (j < per) {
			const int k = j % Ns;
#pragma unroll
			for (int r = 0; r < R; r++)
				v[it][r] = IN_MEM ? ld(j + r * per) : buf[sg_pad(j + r * per)];
			if (Ns > 1) {
#pragma unroll
				for (int r = 1; r < R; r++)
					v[it][r] = sg_cmul(v[it][r], sg_twiddle(tw, n, r * k * tstep, inv));
			}
		}
	}
	if (!IN_MEM && !OUT_MEM)
		__syncthreads();	/* in place: every input read before any output lands */
#pragma unroll
	for (int it = 0; it < MAXI; it++) {
		const int j = tid + it * nt;
		if (j < per) {
			const int k = j % Ns;
			if constexpr (R == 2 || R == 4 || R == 8)
				sg_dft_small<R, R>(v[it], inv);
			else
				sg_dft_odd<R>(v[it], inv);
			const int base = (j - k) * R + k;
#pragma unroll
			for (int r = 0; r < R; r++) {
				if (OUT_MEM)
					st(base + r * Ns, v[it][r]);
				else
					buf[sg_pad(base + r * Ns)] = v[it][r];
			}
		}
	}
	if (!OUT_MEM)
		__syncthreads();
}

template <bool IN_MEM, bool OUT_MEM, class LD, class ST>
__device__ __forceinline__ void sg_gen_pass_r(int R, sg_c64 *buf, int n, int Ns, const sg_c64 *__restrict__ tw, bool inv,
		LD &ld, ST &st, int tid, int nt) {
	switch (R) {
	case 8: sg_gen_pass_ip<8, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	case 4: sg_gen_pass_ip<4, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	case 2: sg_gen_pass_ip<2, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	case 3: sg_gen_pass_ip<3, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	case 5: sg_gen_pass_ip<5, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	default: sg_gen_pass_ip<7, IN_MEM, OUT_MEM>(buf, n, Ns, tw, inv, ld, st, tid, nt); break;
	}
}

/* the n-point transform of the line, natural order in and out: FROM_MEM reads it through
 * ld(0..n) (else it is in buf, written and synchronised by the caller), TO_MEM hands the result
 * to st(0..n) (else it is left in buf, synchronised).  Threads tid < nt of the block take part
 * (a block may run one line per part, all parts through the same passes and barriers). */
template <bool FROM_MEM, bool TO_MEM, class LD, class ST>
__device__ __forceinline__ void sg_gen_fft_mixed(sg_c64 *buf, const SgGenPlan &pl, const sg_c64 *__restrict__ tw, bool inv, LD &ld,
		ST &st, int tid, int nt) {
	const int n = pl.n;
	if (pl.npass == 1) {
		if (FROM_MEM || TO_MEM) {
			sg_gen_pass_r<FROM_MEM, TO_MEM>(pl.radix[0], buf, n, 1, tw, inv, ld, st, tid, nt);
		} else {
			sg_gen_pass_r<false, false>(pl.radix[0], buf, n, 1, tw, inv, ld, st, tid, nt);
		}
		return;
	}
	sg_gen_pass_r<FROM_MEM, false>(pl.radix[0], buf, n, 1, tw, inv, ld, st, tid, nt);
	int Ns = pl.radix[0];
	for (int q = 1; q + 1 < pl.npass; q++) {
		sg_gen_pass_r<false, false>(pl.radix[q], buf, n, Ns, tw, inv, ld, st, tid, nt);
		Ns *= pl.radix[q];
	}
	sg_gen_pass_r<false, TO_MEM>(pl.radix[pl.npass - 1], buf, n, Ns, tw, inv, ld, st, tid, nt);
}

/* Bluestein: x (n values at buf[pad(0..n)], written and synchronised by the caller) -> X in
 * place.  The inverse is conj(forward(conj x)).  twm: twiddles of the m-point transforms,
 * chirp: c_j (j < n), bhat: FFT_m of b (b_j = conj c_|j|, wrapped). */
__device__ void sg_gen_fft_bluestein(sg_c64 *buf, const SgGenPlan &pl, const sg_c64 *__restrict__ twm,
		const sg_c64 *__restrict__ chirp, const sg_c64 *__restrict__ bhat, bool inv) {
	const int n = pl.n, m = pl.m;
	for (int j = threadIdx.x; j < m; j += blockDim.x) {
		sg_c64 a = make_double2(0.0, 0.0);
		if (j < n) {
			sg_c64 x = buf[sg_pad(j)];
			if (inv)
				x.y = -x.y;
			a = sg_cmul(x, chirp[j]);
		}
		buf[sg_pad(j)] = a;
	}
	sg_lds_fft(buf, m, 0, 1, m, twm, false);
	for (int j = threadIdx.x; j < m; j += blockDim.x)
		buf[sg_pad(j)] = sg_cmul(buf[sg_pad(j)], bhat[j]);
	sg_lds_fft(buf, m, 0, 1, m, twm, true);
	const double sc = 1.0 / (double)m;	/* exact: m is a power of two */
	for (int j = threadIdx.x; j < n; j += blockDim.x) {
		sg_c64 y = sg_cmul(buf[sg_pad(j)], chirp[j]);
		y.x *= sc;
		y.y *= sc;
		if (inv)
			y.y = -y.y;
		buf[sg_pad(j)] = y;
	}
	__syncthreads();
}

struct SgGenTables {
	const sg_c64 *tw, *twm, *chirp, *bhat;
};

enum { SG_GEN_FWD_U16 = 0, SG_GEN_C2C = 1, SG_GEN_INV_ARGMAX = 2, SG_GEN_INV_CAND = 3 };

/* one row of pair blockIdx.y: mode FWD_U16 (u16 rows of frames fa / fb packed a + i b, forward,
 * energies), C2C (in place, forward or inverse), INV_ARGMAX (inverse, top-2 arg-max over the
 * row), INV_CAND (inverse, candidates of a near tie) */
template <bool BLUE>
__global__ void __launch_bounds__(BLUE ? 1024 : 640) __attribute__((amdgpu_waves_per_eu(BLUE ? 1 : 4)))
k_gen_rows(SgSel sel, const int *__restrict__ fa, const int *__restrict__ fb,
		sg_c64 *__restrict__ data, int S, SgGenPlan pl, SgGenTables tb, int mode, int inverse,
		unsigned long long *__restrict__ energy, SgBest *__restrict__ best, const SgRegOut *__restrict__ res,
		SgCand *__restrict__ cand) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	__shared__ SgBest red[16];
	sg_c64 *b0 = (sg_c64 *)smem;
	const int row = blockIdx.x, pair = blockIdx.y;
	sg_c64 *line = data + ((size_t)pair * S + row) * S;
	const bool inv = mode >= SG_GEN_INV_ARGMAX || (mode == SG_GEN_C2C && inverse);
	double thr[2] = {INFINITY, INFINITY};
	if (mode == SG_GEN_INV_CAND) {
		const SgRegOut r = res[pair];
		if (!r.amb[0] && !r.amb[1])
			return;
		thr[0] = r.amb[0] ? r.thr[0] : INFINITY;
		thr[1] = r.amb[1] ? r.thr[1] : INFINITY;
	}
	const uint16_t *pa = nullptr, *pb = nullptr;
	const int b = mode == SG_GEN_FWD_U16 ? fb[pair] : -1;
	if (mode == SG_GEN_FWD_U16) {
		pa = sel.frame(fa[pair]) + (size_t)row * sel.rp;
		pb = b >= 0 ? sel.frame(b) + (size_t)row * sel.rp : nullptr;
	}
	if (mode == SG_GEN_FWD_U16) {	/* the frames' energies (the rows are read again by the transform, from cache) */
		unsigned long long ea = 0, eb = 0;
		for (int i = threadIdx.x; i < S; i += blockDim.x) {
			const unsigned int va = pa[i], vb = pb ? pb[i] : 0u;
			ea += (unsigned long long)(va * va);
			eb += (unsigned long long)(vb * vb);
		}
		sg_energy_add(ea, eb, fa[pair], b, energy);
	}
	SgTop2 ta, tbv;
	sg_top2_init(ta);
	sg_top2_init(tbv);
	/* element i of the input line (FWD_U16: frames a + i b) */
	auto ld = [&](int i) -> sg_c64 {
		if (mode == SG_GEN_FWD_U16)
			return make_double2((double)pa[i], pb ? (double)pb[i] : 0.0);
		return line[i];
	};
	/* element i of the transformed line */
	auto st = [&](int i, sg_c64 c) {
		if (mode <= SG_GEN_C2C) {
			line[i] = c;
		} else if (mode == SG_GEN_INV_CAND) {
			sg_cand_push(cand + 2 * pair, c.x, thr[0], row * S + i);
			sg_cand_push(cand + 2 * pair + 1, c.y, thr[1], row * S + i);
		} else {
			sg_top2_add(ta, c.x, row * S + i);
			sg_top2_add(tbv, c.y, row * S + i);
		}
	};
	if constexpr (BLUE) {
		for (int i = threadIdx.x; i < S; i += blockDim.x)
			b0[sg_pad(i)] = ld(i);
		__syncthreads();
		sg_gen_fft_bluestein(b0, pl, tb.twm, tb.chirp, tb.bhat, inv);
		for (int i = threadIdx.x; i < S; i += blockDim.x)
			st(i, b0[sg_pad(i)]);
	} else {
		sg_gen_fft_mixed<true, true>(b0, pl, tb.tw, inv, ld, st, (int)threadIdx.x, (int)blockDim.x);
	}
	if (mode <= SG_GEN_C2C || mode == SG_GEN_INV_CAND)
		return;
	sg_best_block(ta, tbv, red);
	if (threadIdx.x == 0) {
		best[(size_t)pair * S + row].a = ta;
		best[(size_t)pair * S + row].b = tbv;
	}
}

/* out[pair][x][y] = in[pair][y][x] (32 x 32 tiles in LDS) */
__global__ void __launch_bounds__(256)
k_gen_transpose(const sg_c64 *__restrict__ in, sg_c64 *__restrict__ out, int S) {
	__shared__ sg_c64 tile[32][33];
	const size_t plane = (size_t)S * S;
	const sg_c64 *src = in + (size_t)blockIdx.z * plane;
	sg_c64 *dst = out + (size_t)blockIdx.z * plane;
	const int x0 = blockIdx.x * 32, y0 = blockIdx.y * 32;
	for (int r = threadIdx.y; r < 32; r += 8) {
		const int y = y0 + r, x = x0 + threadIdx.x;
		if (y < S && x < S)
			tile[r][threadIdx.x] = src[(size_t)y * S + x];
	}
	__syncthreads();
	for (int r = threadIdx.y; r < 32; r += 8) {
		const int x = x0 + r, y = y0 + threadIdx.x;
		if (y < S && x < S)
			dst[(size_t)x * S + y] = tile[threadIdx.x][r];
	}
}

/* separate the packed spectra and form the packed cross-power spectrum, in place, for any S
 * (k_reg_xpower with modular mirrors) */
__global__ void __launch_bounds__(256)
k_gen_xpower(sg_c64 *__restrict__ work, const sg_c64 *__restrict__ spec, int S) {
	const size_t plane = (size_t)S * S;
	sg_c64 *Z = work + (size_t)blockIdx.y * plane;
	for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < plane; i += (size_t)gridDim.x * blockDim.x) {
		const int r = (int)(i / S), c = (int)(i - (size_t)r * S);
		const size_t m = (size_t)(r ? S - r : 0) * S + (c ? S - c : 0);
		if (m < i)
			continue;
		const sg_c64 zk = Z[i], zm = Z[m];
		Z[i] = sg_xpower_at(zk, zm, spec[i]);
		if (m != i)
			Z[m] = sg_xpower_at(zm, zk, spec[m]);
	}
}

/* The generic column passes fused (mixed-radix plans): rows kx and (S - kx) mod S of the
 * transposed spectrum planes (spectrum columns) in one workgroup, each half of the block one
 * row through the same passes and barriers.  Forward transform in LDS, the packed cross power
 * (the mirror of (kx, ky) is ((S - kx) mod S, (S - ky) mod S): the other row), inverse
 * transform stored back: 3 plane passes instead of the 7 of rows + k_gen_xpower + rows.  Rows
 * 0 and S/2 are their own mirror (the second half idles through the barriers).  blockDim =
 * 2 x the row kernel's thread count (<= 1024), LDS two padded rows. */
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4)))
k_gen_cols_xpower(sg_c64 *__restrict__ data, const sg_c64 *__restrict__ spec, int S, SgGenPlan pl,
		const sg_c64 *__restrict__ tw) {
	extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
	const int T = (int)blockDim.x >> 1, half = (int)threadIdx.x >= T ? 1 : 0, tid = (int)threadIdx.x - half * T;
	const int kx = blockIdx.x, pair = blockIdx.y, kxm = kx ? S - kx : 0;
	const bool single = kxm == kx, active = !(single && half);
	const int row = half ? kxm : kx;
	sg_c64 *buf = (sg_c64 *)smem + half * SG_PADN(S);
	const sg_c64 *oth = (const sg_c64 *)smem + (single ? 0 : 1 - half) * SG_PADN(S);
	sg_c64 *line = data + ((size_t)pair * S + row) * S;
	auto ld = [&](int i) -> sg_c64 { return active ? line[i] : make_double2(0.0, 0.0); };
	auto st = [&](int i, sg_c64 v) {
		if (active)
			line[i] = v;
	};
	sg_gen_fft_mixed<true, false>(buf, pl, tw, false, ld, st, tid, T);
	/* cross power: every element read (this row and the mirror row) before any is written */
	constexpr int MX = 8;	/* S <= 8 T (T >= ceil(S / 8)) */
	sg_c64 pv[MX];
#pragma unroll
	for (int it = 0; it < MX; it++) {
		const int ky = tid + it * T;
		if (ky < S && active)
			pv[it] = sg_xpower_at(buf[sg_pad(ky)], oth[sg_pad(ky ? S - ky : 0)], spec[(size_t)row * S + ky]);
	}
	__syncthreads();
#pragma unroll
	for (int it = 0; it < MX; it++) {
		const int ky = tid + it * T;
		if (ky < S && active)
			buf[sg_pad(ky)] = pv[it];
	}
	__syncthreads();
	sg_gen_fft_mixed<false, true>(buf, pl, tw, true, ld, st, tid, T);
}

/* exact sum_n ref(n + k) img(n) (circular) at every candidate k of a near tie (below 2^56) */
__global__ void __launch_bounds__(256)
k_reg_exact(SgSel sel, const int *__restrict__ fa, const int *__restrict__ fb, int ref, int S,
		SgCand *__restrict__ cand) {
	__shared__ unsigned long long part[4];
	const int c = blockIdx.x, slot = blockIdx.y;
	SgCand *cd = cand + slot;
	const unsigned int cnt = cd->count;
	if (cnt > SG_CAND_CAP || (unsigned)c >= cnt)
		return;
	const int frame = (slot & 1) ? fb[slot >> 1] : fa[slot >> 1];
	if (frame < 0)
		return;
	const int k = cd->idx[c], ky = k / S, kx = k - ky * S;
	const uint16_t *R = sel.frame(ref), *I = sel.frame(frame);
	unsigned long long acc = 0;
	for (int y = 0; y < S; y++) {
		const int yr = y + ky < S ? y + ky : y + ky - S;
		const uint16_t *rr = R + (size_t)yr * sel.rp, *ir = I + (size_t)y * sel.rp;
		for (int x = threadIdx.x; x < S; x += blockDim.x) {
			const int xr = x + kx < S ? x + kx : x + kx - S;
			acc += (unsigned long long)((unsigned int)rr[xr] * (unsigned int)ir[x]);
		}
	}
	for (int o = 32; o > 0; o >>= 1)
		acc += __shfl_down(acc, o, 64);
	if ((threadIdx.x & 63) == 0)
		part[threadIdx.x >> 6] = acc;
	__syncthreads();
	if (threadIdx.x == 0)
		cd->exact[c] = (long long)(part[0] + part[1] + part[2] + part[3]);
}

/* a near tie decided by the exact correlations: the largest, lowest index among equals
 * (amb 2 = resolved; 3 = more candidates than SG_CAND_CAP: the FFT arg-max stays) */
__global__ void __launch_bounds__(64)
k_reg_resolve(const SgCand *__restrict__ cand, int S, int np, SgRegOut *__restrict__ out) {
	const int pair = blockIdx.x * blockDim.x + threadIdx.x;
	if (pair >= np)
		return;
	SgRegOut o = out[pair];
	for (int k = 0; k < 2; k++) {
		if (o.amb[k] != 1)
			continue;
		const SgCand *cd = cand + 2 * pair + k;
		const unsigned int cnt = cd->count;
		if (cnt < 1 || cnt > SG_CAND_CAP) {
			o.amb[k] = 3;
			continue;
		}
		int bi = cd->idx[0];
		long long bv = cd->exact[0];
		for (unsigned int c = 1; c < cnt; c++)
			if (cd->exact[c] > bv || (cd->exact[c] == bv && cd->idx[c] < bi)) {
				bv = cd->exact[c];
				bi = cd->idx[c];
			}
		int sy = bi / S, sx = bi % S;
		if (sy > S / 2)
			sy -= S;
		if (sx > S / 2)
			sx -= S;
		o.idx[k] = bi;
		o.sx[k] = sx;
		o.sy[k] = sy;
		o.amb[k] = 2;
	}
	out[pair] = o;
}

/* The quality estimate of `frames`, enqueued on the device's auxiliary stream (after the work
 * already on `s`, which produced d_sel) so that it runs beside the FFT passes: its kernels are
 * short and the passes leave the chip latency-bound.  reg_quality_finish waits for the sums and
 * forms the values; *launched = false when the subsample loop never runs (dval = 0, :95-98). */
/* the estimate's buffers: qbuf (nq subsampled frames, then the frame list), acc [nq][3] + qmax [nq] */
struct SgQBufs {
	uint16_t *qbuf;
	int *frames;
	unsigned long long *acc;
	unsigned int *qmax;
};

static int reg_quality_buffers(sg_ctx *ctx, SgDevice &dv, int nq, int xs, int ys, SgQBufs &qb) {
	if (!dv.aux) {
		HIPCHK(hipStreamCreateWithFlags(&dv.aux, hipStreamNonBlocking));
		for (int k = 0; k < 2; k++)
			HIPCHK(hipEventCreateWithFlags(&dv.aux_ev[k], hipEventDisableTiming));
	}
	if (dv.qacc_h_n < 3 * (size_t)nq) {
		HIPCHK(hipStreamSynchronize(dv.aux));
		if (dv.qacc_h)
			(void)hipHostFree(dv.qacc_h);
		dv.qacc_h = nullptr;
		dv.qacc_h_n = 0;
		HIPCHK(hipHostMalloc((void **)&dv.qacc_h, sizeof(unsigned long long) * 3 * nq));
		dv.qacc_h_n = 3 * (size_t)nq;
	}
	HIPCHK(hipStreamSynchronize(dv.aux));	/* the previous call's buffers are free */
	HIPCHK(ensure(dv.reg_qbuf, (size_t)nq * xs * ys * sizeof(uint16_t) + sizeof(int) * nq + 64));
	HIPCHK(ensure(dv.reg_qacc, (size_t)nq * (3 * sizeof(unsigned long long) + sizeof(unsigned int))));
	qb.qbuf = (uint16_t *)dv.reg_qbuf.p;
	qb.frames = (int *)((char *)dv.reg_qbuf.p + (((size_t)nq * xs * ys * sizeof(uint16_t) + 15) & ~(size_t)15));
	qb.acc = (unsigned long long *)dv.reg_qacc.p;
	qb.qmax = (unsigned int *)(qb.acc + 3 * nq);
	return SG_OK;
}

/* gradient sums of the subsampled frames on the aux stream (after the work queued on it), read
 * back into the pinned block; aux_ev[0] marks them */
static int reg_quality_grad(sg_ctx *ctx, SgDevice &dv, int nq, int xs, int ys, const SgQBufs &qb) {
	/* 2 waves per 64x16 tile: 214 us per 129 frames against 238 (4 waves) and 333 (1 wave),
	 * scripts/gpu_qgrad.sh */
	const int gthr = ctx->knobs.qgrad_threads;	/* A/B knob SG_QGRAD_THREADS */
	if (ctx->knobs.qgrad_stream) {	/* A/B knob SG_QGRAD_STREAM: 0 = the tiled kernel */
		const int xb = (int)((double)xs * 0.1) + 1, yb = (int)((double)ys * 0.1) + 1;
		const int wi = xs - 2 * xb, hi = ys - 2 * yb;
		if (wi > 0 && hi > 0) {
			hipLaunchKernelGGL(k_quality_grad_s, dim3((wi + 59) / 60, (hi + SG_QGS_ROWS - 1) / SG_QGS_ROWS, nq), dim3(64),
					0, dv.aux, qb.qbuf, xs, ys, qb.qmax, qb.acc);
			HIPCHK(hipGetLastError());
		}
	} else {
		hipLaunchKernelGGL(k_quality_grad, dim3((xs + 63) / 64, (ys + SG_QGT - 1) / SG_QGT, nq), dim3(gthr), 0, dv.aux, qb.qbuf,
				xs, ys, qb.qmax, qb.acc);
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipMemcpyAsync(dv.qacc_h, qb.acc, sizeof(unsigned long long) * 3 * nq, hipMemcpyDeviceToHost, dv.aux));
	HIPCHK(hipEventRecord(dv.aux_ev[0], dv.aux));
	return SG_OK;
}

/* The quality estimate of `frames`, enqueued on the device's auxiliary stream (after the work
 * already on `s`, which produced d_sel) so that it runs beside the FFT passes: its kernels are
 * short and the passes leave the chip latency-bound.  reg_quality_finish waits for the sums and
 * forms the values; *launched = false when the subsample loop never runs (dval = 0, :95-98). */
static int reg_quality_launch(sg_ctx *ctx, SgDevice &dv, hipStream_t s, SgSel d_sel, int S,
		const std::vector<int> &frames, bool *launched) {
	*launched = false;
	const int nq = (int)frames.size();
	const int xs = (S - 1) / 3, ys = (S - 1) / 3;
	if (!nq || xs < 2 || ys < 2)
		return SG_OK;
	SgQBufs qb;
	if (int r = reg_quality_buffers(ctx, dv, nq, xs, ys, qb))
		return r;
	HIPCHK(hipEventRecord(dv.aux_ev[1], s));
	HIPCHK(hipStreamWaitEvent(dv.aux, dv.aux_ev[1], 0));
	HIPCHK(hipMemcpyAsync(qb.frames, frames.data(), sizeof(int) * nq, hipMemcpyHostToDevice, dv.aux));
	HIPCHK(hipMemsetAsync(qb.acc, 0, (size_t)nq * (3 * sizeof(unsigned long long) + sizeof(unsigned int)), dv.aux));
	/* one wave per workgroup, walking the row pairs: 283 us per 129 frames of 2048^2 against
	 * 332 / 348 / 403 / 618 us with 128 / 192 / 256 / 384 threads (scripts/gpu_qsub.sh) */
	const int qthr = ctx->knobs.qsub_threads;	/* A/B knob SG_QSUB_THREADS */
	/* the dword loads of k_quality_sub need an even side, even pitches and a dword-aligned base */
	const int al = !(S & 1) && !(d_sel.rp & 1) && !(d_sel.fp & 1) && !((uintptr_t)d_sel.p & 3);
	hipLaunchKernelGGL(k_quality_sub, dim3((ys + SG_QROWS - 1) / SG_QROWS, nq), dim3(qthr), 0, dv.aux, d_sel, al, qb.frames,
			S, xs, ys, qb.qbuf, qb.qmax);
	HIPCHK(hipGetLastError());
	if (int r = reg_quality_grad(ctx, dv, nq, xs, ys, qb))
		return r;
	*launched = true;
	return SG_OK;
}

static int reg_quality_finish(sg_ctx *ctx, SgDevice &dv, int nq, bool launched, std::vector<double> &qual) {
	qual.assign(nq, 0.0);
	if (!launched)
		return SG_OK;
	HIPCHK(hipEventSynchronize(dv.aux_ev[0]));
	const unsigned long long *h = dv.qacc_h;
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

/* forward full circle exp(-2 pi i k / n), k < n, then its conjugate (the inverse), as the
 * device transforms read them (sg_twiddle).  Power of two: the half circle, negated exactly
 * for k >= n/2; otherwise every k directly. */
static void make_twiddles(int n, std::vector<double> &tw) {
	tw.assign(4 * (size_t)n, 0.0);
	const bool pow2 = (n & (n - 1)) == 0;
	for (int k = 0; k < (pow2 ? n / 2 : n); k++) {
		const double a = -2.0 * M_PI * (double)k / (double)n;
		const double c = cos(a), sn = sin(a);
		const int nk = pow2 ? 2 : 1;
		const int kk[2] = {k, k + n / 2};
		const double sg[2] = {1.0, -1.0};
		for (int h = 0; h < nk; h++) {
			tw[2 * kk[h]] = sg[h] * c;
			tw[2 * kk[h] + 1] = sg[h] * sn;
			tw[2 * (n + kk[h])] = sg[h] * c;
			tw[2 * (n + kk[h]) + 1] = -(sg[h] * sn);
		}
	}
}

/* radices of an n-point mixed-radix plan (8, 4, 2, 3, 5, 7); false: a prime factor > 7 */
static bool make_plan(int n, SgGenPlan &pl) {
	memset(&pl, 0, sizeof pl);
	pl.n = n;
	int r = n;
	const int rad[6] = {8, 4, 2, 3, 5, 7};
	for (int q = 0; q < 6; q++)
		while (r % rad[q] == 0 && pl.npass < SG_GEN_MAXPASS) {
			pl.radix[pl.npass++] = rad[q];
			r /= rad[q];
		}
	return r == 1;
}

/* in-place radix-2 complex DFT on the host (Bluestein's chirp spectrum, computed once per call) */
static void host_fft_pow2(std::vector<double> &re, std::vector<double> &im, int n) {
	for (int i = 1, j = 0; i < n; i++) {
		int bit = n >> 1;
		for (; j & bit; bit >>= 1)
			j ^= bit;
		j ^= bit;
		if (i < j) {
			std::swap(re[i], re[j]);
			std::swap(im[i], im[j]);
		}
	}
	for (int len = 2; len <= n; len <<= 1) {
		for (int i = 0; i < n; i += len)
			for (int k = 0; k < len / 2; k++) {
				const double a = -2.0 * M_PI * (double)k / (double)len;
				const double wr = cos(a), wi = sin(a);
				const double xr = re[i + k + len / 2], xi = im[i + k + len / 2];
				const double vr = xr * wr - xi * wi, vi = xr * wi + xi * wr;
				re[i + k + len / 2] = re[i + k] - vr;
				im[i + k + len / 2] = im[i + k] - vi;
				re[i + k] += vr;
				im[i + k] += vi;
			}
	}
}

static int reg_dft_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel_p, int64_t fpitch, int64_t rpitch,
		int nframes, int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality, void *stream,
		bool normalize_q);

extern "C" int sg_register_dft_u16_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality,
		void *stream) {
	return reg_dft_device(ctx, dev_index, d_sel, (int64_t)S * S, S, nframes, S, ref_image, included, shiftx, shifty,
			quality, stream, true);
}

extern "C" int sg_register_dft_u16_device_raw(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int nframes,
		int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality_raw,
		void *stream) {
	return reg_dft_device(ctx, dev_index, d_sel, (int64_t)S * S, S, nframes, S, ref_image, included, shiftx, shifty,
			quality_raw, stream, false);
}

/* selections read in place from resident frames: selection f row r at d_sel[f frame_pitch + r row_pitch] */
extern "C" int sg_register_dft_u16_device_pitched(sg_ctx *ctx, int dev_index, const uint16_t *d_sel, int64_t frame_pitch,
		int64_t row_pitch, int nframes, int S, int ref_image, const int *included, int *shiftx, int *shifty,
		double *quality, int raw_quality, void *stream) {
	if (ctx && (row_pitch < S || frame_pitch < 0))
		return set_err(ctx, SG_ERR_SIZE, "selection pitches: a row pitch below the side S%s (%ld)", "", (long)row_pitch);
	return reg_dft_device(ctx, dev_index, d_sel, frame_pitch, row_pitch, nframes, S, ref_image, included, shiftx, shifty,
			quality, stream, !raw_quality);
}

static int reg_dft_device(sg_ctx *ctx, int dev_index, const uint16_t *d_sel_p, int64_t fpitch, int64_t rpitch,
		int nframes, int S, int ref_image, const int *included, int *shiftx, int *shifty, double *quality, void *stream,
		bool normalize_q) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size() || !d_sel_p || !shiftx || !shifty || !quality)
		return SG_ERR_GENERIC;
	const SgSel d_sel{d_sel_p, (long long)fpitch, (long long)rpitch};
	if (nframes < 1)
		return set_err(ctx, SG_ERR_GENERIC, "no frame to register%s%ld", "", nframes);
	if (S < 4 || S > 4096)
		return set_err(ctx, SG_ERR_SIZE, "DFT registration takes selection sides 4 to 4096%s (got %ld)", "", S);
	if (ref_image < 0)
		ref_image = 0;	/* seq->reference_image == -1 -> 0 (:212-215) */
	if (ref_image >= nframes)
		return set_err(ctx, SG_ERR_GENERIC, "reference image out of range%s %ld", "", ref_image);
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	const int logS = ilog2(S);
	const size_t plane = (size_t)S * S;
	/* power-of-two sides take the half-spectrum passes; any other side the generic mixed-radix /
	 * Bluestein passes (SG_REG_PATH=3 forces those for a power of two, A/B; the round-1/2 full-
	 * spectrum pass orders 0 / 1 were removed in round 4) */
	const int path = ctx->knobs.reg_path;	/* A/B knob SG_REG_PATH */
	const bool generic = (S & (S - 1)) != 0 || S < 8 || path == 3;
	const bool half = !generic;	/* power of two: the half-spectrum passes */
	/* the call's tie statistics: the device's record (one host thread per device), published to
	 * the context when the call returns */
	dv.stats.reg_ties_resolved = dv.stats.reg_ties_unresolved = dv.stats.reg_fp64_reruns = 0;
	dv.stats.reg_ms = 0.0;
	struct Publish {
		sg_ctx *c;
		const sg_stack_stats &s;
		~Publish() {
			std::lock_guard<std::mutex> lk(c->mu);
			c->stats.reg_ties_resolved = s.reg_ties_resolved;
			c->stats.reg_ties_unresolved = s.reg_ties_unresolved;
			c->stats.reg_fp64_reruns = s.reg_fp64_reruns;
			c->stats.reg_ms = s.reg_ms;
		}
	} publish{ctx, dv.stats};

	/* frames to register, in index order (the reference skips ref and excluded frames) */
	std::vector<int> todo;
	for (int f = 0; f < nframes; f++)
		if (f != ref_image && (!included || included[f]))
			todo.push_back(f);

	/* tables: twiddles exp(-2 pi i k / S); generic path: its plan, and for Bluestein the
	 * m-point twiddles, the chirp c_j = exp(-i pi j^2 / S) and FFT_m(b) */
	SgGenPlan pl;
	memset(&pl, 0, sizeof pl);
	SgGenTables tbl;
	memset(&tbl, 0, sizeof tbl);
	{
		const bool blue = generic && !make_plan(S, pl);
		size_t m = 1;
		if (blue) {
			pl.bluestein = 1;
			pl.m = 1;
			while (pl.m < 2 * S - 1)
				pl.m <<= 1;
			m = pl.m;
		}
		/* table layout: tw (4 S), then for Bluestein twm (4 m), the chirp (2 S), bhat (2 m) */
		const size_t n_tw = 4 * (size_t)S, n_twm = blue ? 4 * m : 0, n_ch = blue ? 2 * (size_t)S : 0;
		const size_t total = n_tw + n_twm + n_ch + (blue ? 2 * m : 0);
		/* the tables depend on S (and the path) only: uploaded when either changes */
		if (dv.reg_tab_S != S || dv.reg_tab_generic != (int)generic) {
			std::vector<double> tw, twm, ch, bh;
			make_twiddles(S, tw);
			if (blue) {
				make_twiddles((int)m, twm);
				ch.assign(2 * (size_t)S, 0.0);
				std::vector<double> br(m, 0.0), bi(m, 0.0);
				for (int j = 0; j < S; j++) {
					const long long q = ((long long)j * j) % (2ll * S);	/* j^2 mod 2S keeps the angle exact */
					const double a = -M_PI * (double)q / (double)S;
					ch[2 * j] = cos(a);
					ch[2 * j + 1] = sin(a);
					br[j] = ch[2 * j];
					bi[j] = -ch[2 * j + 1];	/* b_j = conj c_j */
					if (j) {
						br[m - j] = br[j];
						bi[m - j] = bi[j];
					}
				}
				host_fft_pow2(br, bi, (int)m);
				bh.assign(2 * m, 0.0);
				for (size_t k = 0; k < m; k++) {
					bh[2 * k] = br[k];
					bh[2 * k + 1] = bi[k];
				}
			}
			dv.reg_tab_S = 0;
			HIPCHK(ensure(dv.reg_tw, sizeof(double) * total));
			double *d = (double *)dv.reg_tw.p;
			HIPCHK(hipMemcpyAsync(d, tw.data(), sizeof(double) * n_tw, hipMemcpyHostToDevice, s));
			if (blue) {
				HIPCHK(hipMemcpyAsync(d + n_tw, twm.data(), sizeof(double) * n_twm, hipMemcpyHostToDevice, s));
				HIPCHK(hipMemcpyAsync(d + n_tw + n_twm, ch.data(), sizeof(double) * n_ch, hipMemcpyHostToDevice, s));
				HIPCHK(hipMemcpyAsync(d + n_tw + n_twm + n_ch, bh.data(), sizeof(double) * 2 * m, hipMemcpyHostToDevice, s));
			}
			HIPCHK(hipStreamSynchronize(s));	/* the host vectors die here */
			dv.reg_tab_S = S;
			dv.reg_tab_generic = (int)generic;
		}
		double *d = (double *)dv.reg_tw.p;
		tbl.tw = (const sg_c64 *)d;
		if (blue) {
			tbl.twm = (const sg_c64 *)(d + n_tw);
			tbl.chirp = (const sg_c64 *)(d + n_tw + n_twm);
			tbl.bhat = (const sg_c64 *)(d + n_tw + n_twm + n_ch);
		}
	}
	const sg_c64 *tw = tbl.tw;

	HIPCHK(hipEventRecord(dv.ev[0], s));	/* the call's device span (sg_stack_stats.reg_ms) */
	/* quality of the reference and of every registered frame */
	std::vector<int> qframes;
	qframes.push_back(ref_image);
	qframes.insert(qframes.end(), todo.begin(), todo.end());
	std::vector<double> qual;
	bool q_launched = false;
	int rc = SG_OK;

	/* precision of the main passes: the power-of-two half-spectrum passes run in fp32
	 * (SG_REG_FP=32, default: half the plane bytes and LDS), and a pair whose correlation
	 * maximum is a near tie at fp32 tolerance is re-run in fp64 (the arg-max is then exactly
	 * the fp64 one wherever fp64 is not itself near a tie; those go to the exact integer
	 * correlations).  The other pass orders and the generic path are fp64. */
	const bool fp32 = half && ctx->knobs.reg_fp == 32;
	const size_t esz = fp32 ? sizeof(float2) : sizeof(sg_c64);
	/* pairs per launch: up to 2 GB of pair planes (32 at S = 2048 on the fp64 half path).
	 * Half-spectrum passes, configs[1]: 32 or 64 pairs 8.95-9.07 ms, 16: 9.08, 4: 9.22-9.32,
	 * 2: 9.02-9.15, 1: 9.8 ms of registration (round-2 gpu_regbatch.sh) */
	const size_t pair_bytes = plane * esz * (generic ? 2 : 1);	/* generic: + transposed plane */
	int B = (int)((size_t)(2048u << 20) / pair_bytes);
	if (B < 1)
		B = 1;
	if (B > 64)
		B = 64;
	if (ctx->knobs.reg_batch > 0)	/* A/B knob SG_REG_BATCH: pairs per launch */
		B = ctx->knobs.reg_batch;
	const int npairs_total = (int)(todo.size() + 1) / 2;
	if (B > npairs_total && npairs_total > 0)
		B = npairs_total;
	const int Bc = B > 1 ? B : 1;
	/* fp64 re-runs of near ties in the same work buffer */
	const int B64 = fp32 ? (int)std::max<size_t>(1, (size_t)Bc * pair_bytes / (plane * sizeof(sg_c64))) : Bc;
	const size_t row_lds = (size_t)SG_PADN(S) * sizeof(sg_c64), row_lds32 = (size_t)SG_PADN(S) * sizeof(float2);
	int CW = 8192 / S;
	if (CW < 1)
		CW = 1;
	if (CW > 8)
		CW = 8;
	if (ctx->knobs.reg_cw > 0)	/* A/B knob SG_REG_CW: columns per column-pass workgroup */
		CW = ctx->knobs.reg_cw;
	/* threads: 8 elements per thread in every fp64 LDS FFT (sg_stockham_pass's register
	 * budget), 16 in the fp32 column pass; at least one wave, at most 1024 */
	auto thr_for = [](int elems) { return elems / 8 < 64 ? 64 : elems / 8; };
	const int row_thr = thr_for(S);
	/* half-spectrum columns: a strip stays inside one half (CW divides S/2) */
	const int CWh = CW < S / 2 ? CW : S / 2;
	const size_t colh_lds = (size_t)CWh * sg_col_stride<sg_c64>(S) * sizeof(sg_c64);
	const int colh_thr = thr_for(CWh * S);
	/* fp32 columns: CW32 columns per strip (8: 64-B row segments), 16 elements per thread */
	int CW32 = ctx->knobs.reg_cw32;
	while (CW32 > 1 && (CW32 > S / 2 || CW32 * S > 16 * 1024))
		CW32 >>= 1;
	const int ept32 = CW32 * S / 1024 > 8 ? 16 : 8;
	const int colh_thr32 = std::max(64, CW32 * S / ept32);
	const size_t colh_lds32 = (size_t)CW32 * sg_col_stride<float2>(S) * sizeof(float2);
	const int colocc = ctx->knobs.reg_colocc;
	/* the wave-level fp32 column pass: S = 2048 only (32 x 64 four-step transforms) */
	const bool wcol = S == 2048 && ctx->knobs.reg_wcol;
	int rpw = ctx->knobs.reg_rpw;	/* A/B knob SG_REG_RPW: rows per wave of the wave-level forward rows */
	while (rpw > 1 && (S / 4) % rpw)
		rpw >>= 1;
	const size_t wcol_lds = (size_t)4 * SG_WCOL_CS * sizeof(float2);
	/* rows per forward-row workgroup (the next row prefetched during this one's transform) */
	int rpb = ctx->knobs.reg_rpb;
	while (rpb > 1 && S % rpb != 0)
		rpb >>= 1;
	const int xcdmap = ctx->knobs.reg_xcd;	/* A/B knob SG_REG_XCD: 0 = strips in dispatch order */
	/* generic rows: Bluestein needs m/8 threads (sg_lds_fft), the mixed passes ceil(S / 8) (ceil(S / 7)
	 * with a radix-7 pass) rounded to whole waves (sg_gen_pass_ip's items per thread) */
	bool has7 = false;
	for (int q = 0; q < pl.npass; q++)
		has7 |= pl.radix[q] == 7;
	const int gen_thr = pl.bluestein ? (pl.m / 8 < 64 ? 64 : pl.m / 8)
					 : std::max(64, ((has7 ? (S + 6) / 7 : (S + 7) / 8) + 63) / 64 * 64);
	const size_t gen_lds = pl.bluestein ? (size_t)SG_PADN(pl.m) * sizeof(sg_c64) : row_lds;
	/* one instantiation per transform kind (register allocation is per kernel) */
	const void *k_rows = pl.bluestein ? (const void *)k_gen_rows<true> : (const void *)k_gen_rows<false>;
	/* the fused generic column pass: mixed-radix plans whose two rows fit a block and the LDS
	 * (SG_REG_GENFUSE=0: the three-kernel sequence, A/B) */
	const bool gen_fuse = generic && !pl.bluestein && 2 * gen_thr <= 1024 && 2 * gen_lds <= 160 * 1024 &&
			ctx->knobs.reg_genfuse;
	if (gen_fuse)
		(void)hipFuncSetAttribute((const void *)k_gen_cols_xpower, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)(2 * gen_lds));
	auto gen_rows = [&](dim3 grid, auto... a) {
		if (pl.bluestein)
			hipLaunchKernelGGL(k_gen_rows<true>, grid, dim3(gen_thr), gen_lds, s, a...);
		else
			hipLaunchKernelGGL(k_gen_rows<false>, grid, dim3(gen_thr), gen_lds, s, a...);
	};
	if (!generic) {
		(void)hipFuncSetAttribute((const void *)k_reg_cols<sg_c64, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd_half<sg_c64>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)row_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_half_argmax<sg_c64, false>,
				hipFuncAttributeMaxDynamicSharedMemorySize, (int)row_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_half_argmax<sg_c64, true>,
				hipFuncAttributeMaxDynamicSharedMemorySize, (int)row_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower<sg_c64, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd_half<float2>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)row_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_half_argmax<float2, false>,
				hipFuncAttributeMaxDynamicSharedMemorySize, (int)row_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols<float2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols<float2, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower<float2, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower<float2, 8, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower<float2, 16>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)colh_lds32);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower_w<true, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower_w<true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)(2 * wcol_lds));
		(void)hipFuncSetAttribute((const void *)k_reg_cols_xpower_w<false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_cols_fwd_perm_w, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd_half_w<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_fwd_half_w<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
		(void)hipFuncSetAttribute((const void *)k_reg_rows_inv_half_w, hipFuncAttributeMaxDynamicSharedMemorySize,
				(int)wcol_lds);
	} else {
		(void)hipFuncSetAttribute(k_rows, hipFuncAttributeMaxDynamicSharedMemorySize, (int)gen_lds);
	}

	/* device workspace: reference spectrum (fp64, and fp32 behind it), pair planes, per-row
	 * partials, then (all pairs of the call, uploaded once / read back once) the pair table,
	 * the per-pair results, the frames' energies (two sets: the main passes and the near-tie
	 * re-runs) and the near-tie candidates of one batch */
	const int NP = npairs_total > 0 ? npairs_total : 1;
	/* wave-level column pass: the fp32 reference spectrum also in its lane order (k_spec_perm,
	 * SG_REG_SPECP=0: staged through LDS, A/B) */
	const bool specp_on = fp32 && wcol && ctx->knobs.reg_specp;
	HIPCHK(ensure(dv.reg_spec, plane * sizeof(sg_c64) + (fp32 ? plane * sizeof(float2) : 0) +
			(specp_on ? plane / 2 * sizeof(float2) : 0)));
	/* the fp64 near-tie re-runs use the same buffer: at least one fp64 plane (B64 >= 1 even
	 * when the fp32 batch is a single pair, whose plane is half that size) */
	HIPCHK(ensure(dv.reg_work, std::max((size_t)Bc * pair_bytes, (size_t)B64 * plane * sizeof(sg_c64))));
	const size_t o_out = ((size_t)std::max(Bc, B64) * S * sizeof(SgBest) + 255) & ~(size_t)255;
	const size_t o_fab = o_out + (((size_t)(NP + 1) * sizeof(SgRegOut) + 255) & ~(size_t)255);
	const size_t o_en = o_fab + (((size_t)(NP + 1) * 4 * sizeof(int) + 255) & ~(size_t)255);
	const size_t o_cand = o_en + (((size_t)nframes * 2 * sizeof(unsigned long long) + 255) & ~(size_t)255);
	const size_t o_res2 = o_cand + (((size_t)std::max(Bc, B64) * 2 * sizeof(SgCand) + 255) & ~(size_t)255);
	const size_t ws = o_res2 + (size_t)(NP + 1) * sizeof(SgRegOut);
	HIPCHK(ensure(dv.reg_best, ws));
	char *wsp = (char *)dv.reg_best.p;
	sg_c64 *spec = (sg_c64 *)dv.reg_spec.p, *work = (sg_c64 *)dv.reg_work.p;
	float2 *spec32 = (float2 *)((char *)dv.reg_spec.p + plane * sizeof(sg_c64)), *work32 = (float2 *)dv.reg_work.p;
	float2 *specp32 = specp_on ? spec32 + plane : nullptr;
	sg_c64 *work2 = work + (size_t)Bc * plane;	/* generic path: transposed planes */
	SgBest *best = (SgBest *)wsp;
	SgRegOut *d_out = (SgRegOut *)(wsp + o_out), *d_res2 = (SgRegOut *)(wsp + o_res2);
	int *d_fa = (int *)(wsp + o_fab), *d_fb = d_fa + (NP + 1), *d_fa2 = d_fb + (NP + 1), *d_fb2 = d_fa2 + (NP + 1);
	unsigned long long *energy = (unsigned long long *)(wsp + o_en), *energy2 = energy + nframes;
	SgCand *cand = (SgCand *)(wsp + o_cand);
	HIPCHK(hipMemsetAsync(energy, 0, sizeof(unsigned long long) * 2 * nframes, s));
	/* fp32 twiddles, rounded from the fp64 table (behind the fp64 tables in reg_tw) */
	const float2 *tw32 = nullptr;
	if (fp32) {
		if (dv.reg_tw32_S != S) {
			dv.reg_tw32_S = 0;
			HIPCHK(ensure(dv.reg_tw32, 2 * (size_t)S * sizeof(float2)));
			std::vector<double> t64;
			make_twiddles(S, t64);
			std::vector<float> t32(t64.size());
			for (size_t i = 0; i < t64.size(); i++)
				t32[i] = (float)t64[i];
			HIPCHK(hipMemcpyAsync(dv.reg_tw32.p, t32.data(), sizeof(float) * t32.size(), hipMemcpyHostToDevice, s));
			HIPCHK(hipStreamSynchronize(s));
			dv.reg_tw32_S = S;
		}
		tw32 = (const float2 *)dv.reg_tw32.p;
	}

	const bool ref_conc = fp32 && ctx->knobs.reg_refconc;	/* A/B knob SG_REG_REFCONC */
	/* SG_REG_QFOLD (A/B): the quality estimate's subsample from the wave-level forward rows (every
	 * frame of qframes passes through them: the reference and each pair), then only the gradient
	 * kernel on the aux stream behind the last batch's forward rows */
	const int qfold = (specp32 && npairs_total > 0 && S == 2048) ? ctx->knobs.reg_qfold : 0;
	SgQBufs qfb{};
	int q_qbase = 0;
	bool q_fold_last = false;
	auto fwd_w_launch = [&](hipStream_t st, const int *fa, const int *fb, int np, float2 *out, unsigned long long *en,
			int rows, int qbase) {
		if (qfold) {
			const int waves = (S + qfold - 1) / qfold;
			hipLaunchKernelGGL(k_reg_rows_fwd_half_w<true>, dim3((waves + 3) / 4, np), dim3(256), wcol_lds, st, d_sel, fa,
					fb, tw32, out, en, qfold, qfb.qbuf, qfb.qmax, qbase);
		} else {
			hipLaunchKernelGGL(k_reg_rows_fwd_half_w<false>, dim3(S / 4 / rows, np), dim3(256), wcol_lds, st, d_sel, fa,
					fb, tw32, out, en, rows, (uint16_t *)nullptr, (unsigned int *)nullptr, 0);
		}
	};
	bool ref_pending = false, q_deferred = false;
	if (ref_conc && !dv.aux2) {
		HIPCHK(hipStreamCreateWithFlags(&dv.aux2, hipStreamNonBlocking));
		for (int k = 0; k < 2; k++)
			HIPCHK(hipEventCreateWithFlags(&dv.aux2_ev[k], hipEventDisableTiming));
	}

	/* pair k = frames todo[2k], todo[2k+1] (-1: odd count, imaginary part zero); slot NP is
	 * the reference spectrum's (ref_image, -1) */
	std::vector<int> hfa(NP + 1), hfb(NP + 1);
	std::vector<SgRegOut> hout((size_t)NP);
	for (int k = 0; k < npairs_total; k++) {
		hfa[k] = todo[2 * k];
		hfb[k] = (2 * (size_t)k + 1 < todo.size()) ? todo[2 * k + 1] : -1;
	}
	hfa[NP] = ref_image;
	hfb[NP] = -1;
	/* the pair table goes up, and the results come back, through a pinned block (the previous
	 * call's copies are done: every call ends on a stream synchronize) */
	const size_t pin_res = ((size_t)2 * (NP + 1) * sizeof(int) + 63) & ~(size_t)63;
	const size_t pin_bytes = pin_res + (size_t)NP * sizeof(SgRegOut);
	if (dv.reg_pin_n < pin_bytes) {
		if (dv.reg_pin)
			(void)hipHostFree(dv.reg_pin);
		dv.reg_pin = nullptr;
		dv.reg_pin_n = 0;
		HIPCHK(hipHostMalloc(&dv.reg_pin, pin_bytes));
		dv.reg_pin_n = pin_bytes;
	}
	int *pfab = (int *)dv.reg_pin;
	SgRegOut *pout = (SgRegOut *)((char *)dv.reg_pin + pin_res);
	memcpy(pfab, hfa.data(), sizeof(int) * (NP + 1));
	memcpy(pfab + (NP + 1), hfb.data(), sizeof(int) * (NP + 1));
	HIPCHK(hipMemcpyAsync(d_fa, pfab, sizeof(int) * 2 * (NP + 1), hipMemcpyHostToDevice, s));	/* d_fb = d_fa + NP + 1 */

	const dim3 tgrid((S + 31) / 32, (S + 31) / 32);
	/* generic passes up to the cross power's inverse: transposed spectrum of the rows of `fa`
	 * / `fb` pairs -> `work` holds the pairs' inverse column transforms in row layout */
	auto gen_forward = [&](const int *fa, const int *fb, int np, unsigned long long *en) -> int {
		gen_rows(dim3(S, np), d_sel, fa, fb, work, S, pl, tbl,
				(int)SG_GEN_FWD_U16, 0, en, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_gen_transpose, dim3(tgrid.x, tgrid.y, np), dim3(32, 8), 0, s, (const sg_c64 *)work, work2, S);
		HIPCHK(hipGetLastError());
		if (gen_fuse) {	/* forward columns + cross power + inverse columns in one pass */
			hipLaunchKernelGGL(k_gen_cols_xpower, dim3(S / 2 + 1, np), dim3(2 * gen_thr), 2 * gen_lds, s, work2,
					(const sg_c64 *)spec, S, pl, tw);
			HIPCHK(hipGetLastError());
		} else {
			gen_rows(dim3(S, np), d_sel, fa, fb, work2, S, pl, tbl,
					(int)SG_GEN_C2C, 0, en, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_gen_xpower, dim3(1024, np), dim3(256), 0, s, work2, (const sg_c64 *)spec, S);
			HIPCHK(hipGetLastError());
			gen_rows(dim3(S, np), d_sel, fa, fb, work2, S, pl, tbl,
					(int)SG_GEN_C2C, 1, en, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
			HIPCHK(hipGetLastError());
		}
		hipLaunchKernelGGL(k_gen_transpose, dim3(tgrid.x, tgrid.y, np), dim3(32, 8), 0, s, (const sg_c64 *)work2, work, S);
		HIPCHK(hipGetLastError());
		return SG_OK;
	};
	/* half-spectrum passes of the pairs (fa, fb)[0, np): the reference spectrum (spec) of the
	 * precision (fp64 or fp32), `mode` 0 = top-2 arg-max into best, 1 = near-tie candidates */
	auto half_spec64 = [&]() -> int {
		hipLaunchKernelGGL(k_reg_rows_fwd_half<sg_c64>, dim3(S / rpb, 1), dim3(row_thr), row_lds, s, d_sel, d_fa + NP,
				d_fb + NP, S, tw, spec, energy2, rpb);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL((k_reg_cols<sg_c64, 8>), dim3(S / 2 / CWh, 1), dim3(colh_thr), colh_lds, s, spec, S, logS,
				CWh, tw, 0, xcdmap);
		HIPCHK(hipGetLastError());
		return SG_OK;
	};
	auto half64 = [&](const int *fa, const int *fb, int np, unsigned long long *en, int mode, const SgRegOut *res)
			-> int {
		hipLaunchKernelGGL(k_reg_rows_fwd_half<sg_c64>, dim3(S / rpb, np), dim3(row_thr), row_lds, s, d_sel, fa, fb, S, tw,
				work, en, rpb);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL((k_reg_cols_xpower<sg_c64, 8>), dim3(S / CWh, np), dim3(colh_thr), colh_lds, s, work,
				(const sg_c64 *)spec, S, CWh, tw, xcdmap, ctx->knobs.reg_pb);
		HIPCHK(hipGetLastError());
		if (mode)
			hipLaunchKernelGGL((k_reg_rows_inv_half_argmax<sg_c64, true>), dim3(S, np), dim3(row_thr), row_lds, s,
					(const sg_c64 *)work, S, tw, best, res, cand);
		else
			hipLaunchKernelGGL((k_reg_rows_inv_half_argmax<sg_c64, false>), dim3(S, np), dim3(row_thr), row_lds, s,
					(const sg_c64 *)work, S, tw, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
		HIPCHK(hipGetLastError());
		return SG_OK;
	};
	auto half32 = [&](const int *fa, const int *fb, int np, unsigned long long *en) -> int {
		if (wcol)
			fwd_w_launch(s, fa, fb, np, work32, en, rpw, q_qbase);
		else
			hipLaunchKernelGGL(k_reg_rows_fwd_half<float2>, dim3(S / rpb, np), dim3(row_thr), row_lds32, s, d_sel, fa,
					fb, S, tw32, work32, en, rpb);
		HIPCHK(hipGetLastError());
		if (q_deferred) {	/* SG_REG_QAFTER: the quality estimate beside the column pass instead */
			q_deferred = false;
			if (int r = reg_quality_launch(ctx, dv, s, d_sel, S, qframes, &q_launched))
				return r;
		}
		if (ref_pending) {	/* the reference spectrum, from its stream */
			HIPCHK(hipStreamWaitEvent(s, dv.aux2_ev[1], 0));
			ref_pending = false;
		}
		if (qfold && q_fold_last) {	/* every frame subsampled (the reference's rows waited for above) */
			const int nq = (int)qframes.size(), xs = (S - 1) / 3;
			HIPCHK(hipEventRecord(dv.aux_ev[1], s));
			HIPCHK(hipStreamWaitEvent(dv.aux, dv.aux_ev[1], 0));
			if (int r = reg_quality_grad(ctx, dv, nq, xs, xs, qfb))
				return r;
			q_launched = true;
		}
		if (wcol && specp32 && ctx->knobs.reg_wcolw == 8)	/* 8-column strips: 64-B row segments, one workgroup per CU */
			hipLaunchKernelGGL((k_reg_cols_xpower_w<true, 8>), dim3(S / 8, np), dim3(512), 2 * wcol_lds, s, work32,
					(const float2 *)spec32, (const float2 *)specp32, tw32, xcdmap);
		else if (wcol && specp32)	/* S = 2048: the wave-level column pass (SG_REG_WCOL=0: the block-level one, A/B) */
			hipLaunchKernelGGL((k_reg_cols_xpower_w<true, 4>), dim3(S / 4, np), dim3(256), wcol_lds, s, work32,
					(const float2 *)spec32, (const float2 *)specp32, tw32, xcdmap);
		else if (wcol)
			hipLaunchKernelGGL((k_reg_cols_xpower_w<false, 4>), dim3(S / 4, np), dim3(256), wcol_lds, s, work32,
					(const float2 *)spec32, (const float2 *)nullptr, tw32, xcdmap);
		else if (ept32 == 16)
			hipLaunchKernelGGL((k_reg_cols_xpower<float2, 16>), dim3(S / CW32, np), dim3(colh_thr32), colh_lds32, s,
					work32, (const float2 *)spec32, S, CW32, tw32, xcdmap, 1);
		else if (colocc)	/* default (SG_REG_COLOCC=1): 64 VGPRs (8 waves / SIMD, two 1024-thread workgroups per CU) */
			hipLaunchKernelGGL((k_reg_cols_xpower<float2, 8, 8>), dim3(S / CW32, np), dim3(colh_thr32), colh_lds32, s,
					work32, (const float2 *)spec32, S, CW32, tw32, xcdmap, 1);
		else
			hipLaunchKernelGGL((k_reg_cols_xpower<float2, 8>), dim3(S / CW32, np), dim3(colh_thr32), colh_lds32, s,
					work32, (const float2 *)spec32, S, CW32, tw32, xcdmap, 1);
		HIPCHK(hipGetLastError());
		if (wcol)
			hipLaunchKernelGGL(k_reg_rows_inv_half_w, dim3(S / 4, np), dim3(256), wcol_lds, s, (const float2 *)work32,
					tw32, best);
		else
			hipLaunchKernelGGL((k_reg_rows_inv_half_argmax<float2, false>), dim3(S, np), dim3(row_thr), row_lds32, s,
					(const float2 *)work32, S, tw32, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
		HIPCHK(hipGetLastError());
		return SG_OK;
	};

	/* the quality estimate on the aux stream, queued behind the main stream's table uploads and
	 * fills (queued ahead of them, its long-running workgroups held the fills' single workgroup
	 * back 0.2 ms, profiles/r05m_*) */
	if (qfold) {	/* the sums zeroed on the call's stream, ahead of every forward row launch */
		const int nq = (int)qframes.size(), xs = (S - 1) / 3;
		if (int r = reg_quality_buffers(ctx, dv, nq, xs, xs, qfb))
			return r;
		HIPCHK(hipMemsetAsync(qfb.acc, 0, (size_t)nq * (3 * sizeof(unsigned long long) + sizeof(unsigned int)), s));
	} else if (fp32 && npairs_total > 0 && ctx->knobs.reg_qafter) {
		q_deferred = true;
	} else {
		rc = reg_quality_launch(ctx, dv, s, d_sel, S, qframes, &q_launched);
		if (rc)
			return rc;
	}

	/* reference spectrum R = FFT2(ref) (half layout: the A' half only; generic: transposed) */
	if (generic) {
		gen_rows(dim3(S, 1), d_sel, d_fa + NP, d_fb + NP, work, S, pl,
				tbl, (int)SG_GEN_FWD_U16, 0, energy, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_gen_transpose, dim3(tgrid.x, tgrid.y, 1), dim3(32, 8), 0, s, (const sg_c64 *)work, spec, S);
		HIPCHK(hipGetLastError());
		gen_rows(dim3(S, 1), d_sel, d_fa + NP, d_fb + NP, spec, S, pl,
				tbl, (int)SG_GEN_C2C, 0, energy, best, (const SgRegOut *)nullptr, (SgCand *)nullptr);
	} else if (fp32) {
		/* the reference spectrum on its own stream beside the first batch's forward rows (which do
		 * not read it; the batch's column pass waits for it).  One workgroup per CU at most: run
		 * alone it is 0.27 ms of latency-bound passes ahead of every pair (profiles/r05l_*) */
		hipStream_t rs = s;
		if (ref_conc) {
			HIPCHK(hipEventRecord(dv.aux2_ev[0], s));
			HIPCHK(hipStreamWaitEvent(dv.aux2, dv.aux2_ev[0], 0));
			rs = dv.aux2;
		}
		if (specp32) {	/* wave-level passes: one row per wave, the columns straight into lane order */
			fwd_w_launch(rs, d_fa + NP, d_fb + NP, 1, spec32, energy, 1, 0);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_cols_fwd_perm_w, dim3(S / 2 / 4), dim3(256), wcol_lds, rs, spec32, specp32, tw32);
		} else {
			hipLaunchKernelGGL(k_reg_rows_fwd_half<float2>, dim3(S / rpb, 1), dim3(row_thr), row_lds32, rs, d_sel,
					d_fa + NP, d_fb + NP, S, tw32, spec32, energy, rpb);
			HIPCHK(hipGetLastError());
			if (ept32 == 16)
				hipLaunchKernelGGL((k_reg_cols<float2, 16>), dim3(S / 2 / CW32, 1), dim3(colh_thr32), colh_lds32, rs,
						spec32, S, logS, CW32, tw32, 0, xcdmap);
			else
				hipLaunchKernelGGL((k_reg_cols<float2, 8>), dim3(S / 2 / CW32, 1), dim3(colh_thr32), colh_lds32, rs,
						spec32, S, logS, CW32, tw32, 0, xcdmap);
		}
		if (ref_conc) {
			HIPCHK(hipGetLastError());
			HIPCHK(hipEventRecord(dv.aux2_ev[1], dv.aux2));
			ref_pending = true;
		}
	} else {
		hipLaunchKernelGGL(k_reg_rows_fwd_half<sg_c64>, dim3(S / rpb, 1), dim3(row_thr), row_lds, s, d_sel, d_fa + NP,
				d_fb + NP, S, tw, spec, energy, rpb);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL((k_reg_cols<sg_c64, 8>), dim3(S / 2 / CWh, 1), dim3(colh_thr), colh_lds, s, spec, S, logS,
				CWh, tw, 0, xcdmap);
	}
	HIPCHK(hipGetLastError());
	shiftx[ref_image] = 0;
	shifty[ref_image] = 0;
	const int tol_main = fp32 ? -15 : -32;
	for (int p0 = 0; p0 < npairs_total; p0 += B) {
		const int np = npairs_total - p0 < B ? npairs_total - p0 : B;
		int count = S;	/* row partials per pair */
		if (generic) {
			if (int r = gen_forward(d_fa + p0, d_fb + p0, np, energy))
				return r;
			gen_rows(dim3(S, np), d_sel, d_fa + p0, d_fb + p0, work, S,
					pl, tbl, (int)SG_GEN_INV_ARGMAX, 1, energy, best, (const SgRegOut *)nullptr,
					(SgCand *)nullptr);
		} else if (fp32) {
			q_qbase = 1 + 2 * p0;	/* qframes = ref, todo...: pair k's frames are entries 1 + 2k, 2 + 2k */
			q_fold_last = p0 + np >= npairs_total;
			if (int r = half32(d_fa + p0, d_fb + p0, np, energy))
				return r;
		} else {
			if (int r = half64(d_fa + p0, d_fb + p0, np, energy, 0, nullptr))
				return r;
		}
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_reg_final, dim3(np), dim3(256), 0, s, (const SgBest *)best, S, count,
				(const int *)d_fa + p0, (const int *)d_fb + p0, ref_image, (const unsigned long long *)energy, tol_main,
				d_out + p0);
		HIPCHK(hipGetLastError());
	}
	if (ref_pending) {
		HIPCHK(hipStreamWaitEvent(s, dv.aux2_ev[1], 0));
		ref_pending = false;
	}
	if (npairs_total > 0)
		HIPCHK(hipMemcpyAsync(pout, d_out, sizeof(SgRegOut) * npairs_total, hipMemcpyDeviceToHost, s));
	HIPCHK(hipStreamSynchronize(s));
	if (npairs_total > 0)
		memcpy(hout.data(), pout, sizeof(SgRegOut) * npairs_total);

	/* near ties (the runner-up within the tolerance of the maximum): re-run those pairs.  After
	 * fp32 passes, first in fp64 (a fresh arg-max at the fp64 tolerance); what is still a near
	 * tie then lists every index within the tolerance, computes their exact integer
	 * correlations and takes the largest (lowest index among exact equals) */
	auto ambiguous = [&](std::vector<int> &amb) {
		amb.clear();
		for (int k = 0; k < npairs_total; k++)
			if (hout[k].amb[0] == 1 || hout[k].amb[1] == 1)
				amb.push_back(k);
	};
	auto upload_subset = [&](const std::vector<int> &amb, std::vector<SgRegOut> &ares) -> int {
		const int na = (int)amb.size();
		std::vector<int> afa(na), afb(na);
		ares.resize(na);
		for (int i = 0; i < na; i++) {
			afa[i] = hfa[amb[i]];
			afb[i] = hfb[amb[i]];
			ares[i] = hout[amb[i]];
		}
		HIPCHK(hipMemcpyAsync(d_fa2, afa.data(), sizeof(int) * na, hipMemcpyHostToDevice, s));
		HIPCHK(hipMemcpyAsync(d_fb2, afb.data(), sizeof(int) * na, hipMemcpyHostToDevice, s));
		HIPCHK(hipMemcpyAsync(d_res2, ares.data(), sizeof(SgRegOut) * na, hipMemcpyHostToDevice, s));
		HIPCHK(hipStreamSynchronize(s));	/* the host vectors die here */
		return SG_OK;
	};
	std::vector<int> amb;
	std::vector<SgRegOut> ares;
	ambiguous(amb);
	if (!amb.empty() && fp32) {
		/* fp64 re-run: the fp64 reference spectrum, then the pairs' fp64 passes and arg-max */
		if (int r = upload_subset(amb, ares))
			return r;
		if (int r = half_spec64())
			return r;
		const int na = (int)amb.size();
		for (int p0 = 0; p0 < na; p0 += B64) {
			const int np = na - p0 < B64 ? na - p0 : B64;
			if (int r = half64(d_fa2 + p0, d_fb2 + p0, np, energy2, 0, nullptr))
				return r;
			hipLaunchKernelGGL(k_reg_final, dim3(np), dim3(256), 0, s, (const SgBest *)best, S, S,
					(const int *)d_fa2 + p0, (const int *)d_fb2 + p0, ref_image, (const unsigned long long *)energy,
					-32, d_res2 + p0);
			HIPCHK(hipGetLastError());
		}
		HIPCHK(hipMemcpyAsync(ares.data(), d_res2, sizeof(SgRegOut) * na, hipMemcpyDeviceToHost, s));
		HIPCHK(hipStreamSynchronize(s));
		for (int i = 0; i < na; i++)
			hout[amb[i]] = ares[i];
		dv.stats.reg_fp64_reruns += (uint64_t)na;
		ambiguous(amb);
	}
	if (!amb.empty()) {
		if (int r = upload_subset(amb, ares))
			return r;
		const int na = (int)amb.size();
		for (int p0 = 0; p0 < na; p0 += B64) {
			const int np = na - p0 < B64 ? na - p0 : B64;
			HIPCHK(hipMemsetAsync(cand, 0, sizeof(SgCand) * 2 * np, s));
			if (generic) {
				if (int r = gen_forward(d_fa2 + p0, d_fb2 + p0, np, energy2))
					return r;
				gen_rows(dim3(S, np), d_sel, d_fa2 + p0, d_fb2 + p0,
						work, S, pl, tbl, (int)SG_GEN_INV_CAND, 1, energy2, best, (const SgRegOut *)(d_res2 + p0),
						cand);
			} else {
				/* the fp64 spectrum exists on the fp64 half path, and after the fp64 re-run */
				if (int r = half64(d_fa2 + p0, d_fb2 + p0, np, energy2, 1, (const SgRegOut *)(d_res2 + p0)))
					return r;
			}
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_exact, dim3(SG_CAND_CAP, 2 * np), dim3(256), 0, s, d_sel, (const int *)d_fa2 + p0,
					(const int *)d_fb2 + p0, ref_image, S, cand);
			HIPCHK(hipGetLastError());
			hipLaunchKernelGGL(k_reg_resolve, dim3((np + 63) / 64), dim3(64), 0, s, (const SgCand *)cand, S, np,
					d_res2 + p0);
			HIPCHK(hipGetLastError());
		}
		HIPCHK(hipMemcpyAsync(ares.data(), d_res2, sizeof(SgRegOut) * na, hipMemcpyDeviceToHost, s));
		HIPCHK(hipStreamSynchronize(s));
		for (int i = 0; i < na; i++)
			hout[amb[i]] = ares[i];
	}
	for (int k = 0; k < npairs_total; k++) {
		const int fr[2] = {hfa[k], hfb[k]};
		for (int h = 0; h < 2; h++) {
			if (fr[h] < 0)
				continue;
			shiftx[fr[h]] = hout[k].sx[h];
			shifty[fr[h]] = hout[k].sy[h];
			if (hout[k].amb[h] == 2)
				dv.stats.reg_ties_resolved++;
			else if (hout[k].amb[h])
				dv.stats.reg_ties_unresolved++;
		}
	}

	if (q_launched)	/* the span ends with the quality estimate's stream */
		HIPCHK(hipStreamWaitEvent(s, dv.aux_ev[0], 0));
	HIPCHK(hipEventRecord(dv.ev[1], s));
	if (int qrc = reg_quality_finish(ctx, dv, (int)qframes.size(), q_launched, qual))
		return qrc;
	{
		float ms = 0.f;
		HIPCHK(hipEventSynchronize(dv.ev[1]));
		HIPCHK(hipEventElapsedTime(&ms, dv.ev[0], dv.ev[1]));
		dv.stats.reg_ms = ms;
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

/*
 * host selections: one device registers everything; several devices split the frames to
 * register into contiguous shards (frames are independent), each device driven by
 * its own host thread with the reference selection and its shard uploaded, the reference
 * spectrum and quality computed on every device.  The raw shard results are reassembled and
 * the quality bookkeeping of the reference (q_min / q_max seeded by the reference frame, the
 * frames in index order, the min() macro, normalizeQualityData :163-176) replayed over all of
 * them, so the result is the one-device result (test_register_raw_shards_reassemble).
 */
static int reg_host(sg_ctx *ctx, const uint16_t *sel, int nframes, int S, int ref_image, const int *included,
		int *shiftx, int *shifty, double *quality, bool normalize_q) {
	if (!ctx || ctx->dev.empty() || !sel || !shiftx || !shifty || !quality)
		return SG_ERR_GENERIC;
	if (nframes < 1 || S < 1)
		return SG_ERR_GENERIC;
	if (ref_image < 0)
		ref_image = 0;
	if (ref_image >= nframes)
		return set_err(ctx, SG_ERR_GENERIC, "reference image out of range%s %ld", "", ref_image);
	const size_t plane = (size_t)S * S;
	std::vector<int> todo;
	for (int f = 0; f < nframes; f++)
		if (f != ref_image && (!included || included[f]))
			todo.push_back(f);
	const int G = (int)std::max<size_t>(1, std::min(ctx->dev.size(), todo.size()));
	if (G == 1) {
		SgDevice &dv = ctx->dev[0];
		HIPCHK(hipSetDevice(dv.id));
		const size_t bytes = (size_t)nframes * plane * sizeof(uint16_t);
		HIPCHK(ensure(dv.reg_sel, bytes));
		HIPCHK(hipMemcpyAsync(dv.reg_sel.p, sel, bytes, hipMemcpyHostToDevice, dv.stream));
		return reg_dft_device(ctx, 0, (const uint16_t *)dv.reg_sel.p, (int64_t)S * S, S, nframes, S, ref_image, included,
				shiftx, shifty,
				quality, nullptr, normalize_q);
	}
	/* shard g: local frame 0 = the reference, 1..k = todo[t0 .. t1) */
	std::vector<int> rcs((size_t)G, SG_OK);
	std::vector<double> qraw((size_t)nframes, 0.0);
	std::vector<double> qref((size_t)G, 0.0);
	auto run = [&](int g) {
		const size_t t0 = todo.size() * (size_t)g / (size_t)G, t1 = todo.size() * (size_t)(g + 1) / (size_t)G;
		const int k = (int)(t1 - t0);
		SgDevice &dv = ctx->dev[(size_t)g];
		int &rc = rcs[(size_t)g];
		if (hipSetDevice(dv.id) != hipSuccess) {
			rc = set_err(ctx, SG_ERR_DEVICE, "hipSetDevice failed%s %ld", "", dv.id);
			return;
		}
		const size_t bytes = (size_t)(k + 1) * plane * sizeof(uint16_t);
		if (ensure(dv.reg_sel, bytes) != hipSuccess) {
			rc = set_err(ctx, SG_ERR_DEVICE, "no device memory for the selections%s (%ld frames)", "", k + 1);
			return;
		}
		uint16_t *d = (uint16_t *)dv.reg_sel.p;
		hipError_t e = hipMemcpyAsync(d, sel + (size_t)ref_image * plane, plane * sizeof(uint16_t),
				hipMemcpyHostToDevice, dv.stream);
		for (int j = 0; j < k && e == hipSuccess; j++)
			e = hipMemcpyAsync(d + (size_t)(j + 1) * plane, sel + (size_t)todo[t0 + (size_t)j] * plane,
					plane * sizeof(uint16_t), hipMemcpyHostToDevice, dv.stream);
		if (e != hipSuccess) {
			rc = set_err(ctx, SG_ERR_DEVICE, "selection upload failed%s %ld", "", g);
			return;
		}
		std::vector<int> lx((size_t)k + 1), ly((size_t)k + 1);
		std::vector<double> lq((size_t)k + 1);
		rc = reg_dft_device(ctx, g, d, (int64_t)S * S, S, k + 1, S, 0, nullptr, lx.data(), ly.data(), lq.data(), nullptr,
				false);
		if (rc)
			return;
		qref[(size_t)g] = lq[0];
		for (int j = 0; j < k; j++) {
			const int f = todo[t0 + (size_t)j];
			shiftx[f] = lx[(size_t)j + 1];
			shifty[f] = ly[(size_t)j + 1];
			qraw[(size_t)f] = lq[(size_t)j + 1];
		}
	};
	{
		/* a thread that cannot start fails its slot (and the call) instead of escaping the C ABI;
		 * the threads that did start are always joined */
		std::vector<std::thread> th;
		bool started = true;
		for (int g = 1; g < G; g++) {
			try {
				th.emplace_back(run, g);
			} catch (...) {
				for (int h = g; h < G; h++)
					rcs[(size_t)h] = set_err(ctx, SG_ERR_GENERIC, "could not start the thread of device slot%s %ld", "", h);
				started = false;
				break;
			}
		}
		if (started)
			run(0);
		else
			rcs[0] = SG_ERR_GENERIC;
		for (std::thread &t : th)
			t.join();
	}
	sg_stack_stats agg;
	memset(&agg, 0, sizeof agg);
	for (int g = 0; g < G; g++) {
		const sg_stack_stats &st = ctx->dev[(size_t)g].stats;
		agg.reg_ties_resolved += st.reg_ties_resolved;
		agg.reg_ties_unresolved += st.reg_ties_unresolved;
		agg.reg_fp64_reruns += st.reg_fp64_reruns;
		agg.reg_ms = std::max(agg.reg_ms, st.reg_ms);
	}
	{
		std::lock_guard<std::mutex> lk(ctx->mu);
		ctx->stats.reg_ties_resolved = agg.reg_ties_resolved;
		ctx->stats.reg_ties_unresolved = agg.reg_ties_unresolved;
		ctx->stats.reg_fp64_reruns = agg.reg_fp64_reruns;
		ctx->stats.reg_ms = agg.reg_ms;
	}
	for (int g = 0; g < G; g++)
		if (rcs[(size_t)g])
			return rcs[(size_t)g];
	shiftx[ref_image] = shifty[ref_image] = 0;
	quality[ref_image] = qref[0];
	for (int f : todo)
		quality[f] = qraw[(size_t)f];
	if (!normalize_q)
		return SG_OK;
	double q_min = qref[0], q_max = qref[0];
	for (int f : todo) {
		const double qv = qraw[(size_t)f];
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
	return reg_host(ctx, sel, nframes, S, ref_image, included, shiftx, shifty, quality, true);
}

extern "C" int sg_register_dft_u16_raw(sg_ctx *ctx, const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality_raw) {
	return reg_host(ctx, sel, nframes, S, ref_image, included, shiftx, shifty, quality_raw, false);
}
