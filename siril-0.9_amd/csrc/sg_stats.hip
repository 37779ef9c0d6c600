/*
 * sg_stats.hip - per-frame location / scale for stacking normalisation:
 * what statistics(fit, 0, NULL, STATS_IKSS, STATS_ZERO_NULLCHECK) stores in imstats
 * (src/algos/statistics.c:152-326) and _compute_normalization_for_image reads
 * (src/stacking/stacking.c:79-123, through seq_get_imstats src/io/sequence.c:1107-1118).
 *
 * The reference sorts the frame's non-zero samples as doubles (x / norm, norm = 255 or
 * 65535 by the frame maximum, src/core/utils.c:454-459) and iterates IKSS: median, MAD (a
 * second sort), the biweight midvariance (sequential double sums over the sorted data),
 * 4-sigma clipping.  Every one of these is a function of the frame's 65536-bin histogram:
 *   - k_ikss_hist: layer-0 histogram of the non-zero samples (u16 counter pairs in LDS per
 *     65535-sample chunk, flushed with global atomics) and the maximum over all layers;
 *   - k_ikss_prefix: exclusive prefix counts P[x] = #samples < x;
 *   - k_ikss_solve: one lane per frame runs the IKSS loop on the prefix table: medians are
 *     rank lookups, the MAD is a merge of the two monotone delta sequences on either side
 *     of the median, and the BWMV sums add each distinct value's term count(x) times with
 *     sg_add_repeat (sg_repadd.h), which reproduces the sequential double sum exactly.
 * All double expressions are written as the reference writes them (no contraction), so
 * location / scale equal the reference's bit for bit (tests/test_gpu_stats.py against the
 * CPU restatement in tests/).
 */
#include "sg_common.hpp"
#include "sg_ctx.hpp"
#include "sg_repadd.h"
#include <math.h>
#include <vector>

#define SG_ST_BINS 65536
#define SG_ST_CHUNK 65535	/* samples per histogram workgroup: the u16 LDS counters cannot wrap */

/* layer-0 histogram of frame blockIdx.y's non-zero samples into hist[x * nf + f] (frame-minor:
 * the solver's 64 lanes read one bin of 64 frames as one coalesced row), max over all layers */
__global__ void __launch_bounds__(1024)
k_ikss_hist(const uint16_t *__restrict__ frames, int64_t fstride, int C, int64_t npix, int nf, int f0,
		uint32_t *__restrict__ hist, uint32_t *__restrict__ maxi) {
	extern __shared__ uint32_t lh[];	/* 32768 dwords: bin pairs */
	const int f = blockIdx.y;
	const int64_t p0 = (int64_t)blockIdx.x * SG_ST_CHUNK;
	const int64_t p1 = p0 + SG_ST_CHUNK < npix ? p0 + SG_ST_CHUNK : npix;
	for (int i = threadIdx.x; i < SG_ST_BINS / 2; i += blockDim.x)
		lh[i] = 0;
	__syncthreads();
	const uint16_t *fr = frames + (int64_t)(f0 + f) * fstride;
	uint32_t mx = 0;
	for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
		const uint32_t v = fr[p];
		mx = v > mx ? v : mx;
		if (v)
			atomicAdd(&lh[v >> 1], 1u << ((v & 1u) * 16u));
	}
	for (int c = 1; c < C; c++)
		for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
			const uint32_t v = fr[(int64_t)c * npix + p];
			mx = v > mx ? v : mx;
		}
	for (int o = 32; o > 0; o >>= 1) {
		const uint32_t t = (uint32_t)__shfl_xor((int)mx, o, 64);
		mx = t > mx ? t : mx;
	}
	if ((threadIdx.x & 63) == 0 && mx)
		atomicMax(&maxi[f], mx);
	__syncthreads();
	for (int i = threadIdx.x; i < SG_ST_BINS / 2; i += blockDim.x) {
		const uint32_t w = lh[i];
		if (w & 0xFFFFu)
			atomicAdd(&hist[(size_t)(2 * i) * nf + f], w & 0xFFFFu);
		if (w >> 16)
			atomicAdd(&hist[(size_t)(2 * i + 1) * nf + f], w >> 16);
	}
}

/* in place: hist[x][f] -> P[x][f] = #samples < x, row SG_ST_BINS = total */
__global__ void __launch_bounds__(64) k_ikss_prefix(uint32_t *__restrict__ hist, int nf) {
	const int f = blockIdx.x * 64 + threadIdx.x;
	if (f >= nf)
		return;
	uint32_t run = 0;
	for (int x = 0; x < SG_ST_BINS; x++) {
		const uint32_t c = hist[(size_t)x * nf + f];
		hist[(size_t)x * nf + f] = run;
		run += c;
	}
	hist[(size_t)SG_ST_BINS * nf + f] = run;
}

struct SgIk {
	const uint32_t *P;
	int nf, f;
	double norm;
};

__device__ __forceinline__ uint32_t ik_P(const SgIk &k, int x) {
	return k.P[(size_t)x * k.nf + k.f];
}
__device__ __forceinline__ double ik_val(const SgIk &k, int x) {
	return (double)x / k.norm;	/* newdata[i] = (double) data[i] / ((double) hist_size - 1) (:281) */
}
/* value of the sample at rank r (0-based, sorted non-zero samples) */
__device__ int ik_x_at(const SgIk &k, uint32_t r) {
	int lo = 1, hi = SG_ST_BINS - 1;
	while (lo < hi) {
		const int mid = (lo + hi) >> 1;
		if (ik_P(k, mid + 1) > r)
			hi = mid;
		else
			lo = mid + 1;
	}
	return lo;
}
/* samples of value x among ranks [i, j) */
__device__ __forceinline__ uint32_t ik_cnt(const SgIk &k, int x, uint32_t i, uint32_t j) {
	uint32_t a = ik_P(k, x), b = ik_P(k, x + 1);
	a = a > i ? a : i;
	b = b < j ? b : j;
	return b > a ? b - a : 0u;
}
/* gsl_stats_median_from_sorted_data(data + i, 1, j - i) */
__device__ double ik_median(const SgIk &k, uint32_t i, uint32_t j) {
	const uint32_t n = j - i, lhs = i + (n - 1) / 2, rhs = i + n / 2;
	const double a = ik_val(k, ik_x_at(k, lhs));
	if (lhs == rhs)
		return a;
	return (a + ik_val(k, ik_x_at(k, rhs))) / 2.0;
}
/* siril_stats_double_mad (:82-100): median of |data - m| over ranks [i, j) */
__device__ double ik_mad(const SgIk &k, uint32_t i, uint32_t j, double m) {
	const uint32_t n = j - i, rl = (n - 1) / 2, rr = n / 2;
	const int xi = ik_x_at(k, i), xj = ik_x_at(k, j - 1);
	int lo_b = xi, hi_b = xj + 1;	/* first x with val(x) >= m */
	while (lo_b < hi_b) {
		const int mid = (lo_b + hi_b) >> 1;
		if (ik_val(k, mid) >= m)
			hi_b = mid;
		else
			lo_b = mid + 1;
	}
	int hi = lo_b, lo = lo_b - 1;
	uint32_t seen = 0;
	double vl = 0.0, vr = 0.0;
	bool have_l = false;
	for (;;) {
		while (lo >= xi && ik_cnt(k, lo, i, j) == 0)
			lo--;
		while (hi <= xj && ik_cnt(k, hi, i, j) == 0)
			hi++;
		bool take_hi;
		if (lo < xi)
			take_hi = true;
		else if (hi > xj)
			take_hi = false;
		else
			take_hi = fabs(ik_val(k, hi) - m) <= fabs(ik_val(k, lo) - m);
		const int x = take_hi ? hi : lo;
		const double d = fabs(ik_val(k, x) - m);
		const uint32_t c = ik_cnt(k, x, i, j);
		if (!have_l && rl < seen + c) {
			vl = d;
			have_l = true;
		}
		if (rr < seen + c) {
			vr = d;
			break;
		}
		seen += c;
		if (take_hi)
			hi++;
		else
			lo--;
	}
	return rl == rr ? vl : (vl + vr) / 2.0;
}
/* siril_stats_double_bwmv (:128-150) over the sorted ranks [i, j) */
__device__ double ik_bwmv(const SgIk &k, uint32_t i, uint32_t j, double mad, double median) {
	double bwmv = 0.0, up = 0.0, down = 0.0;
	if (mad > 0.0) {
		const int xi = ik_x_at(k, i), xj = ik_x_at(k, j - 1);
		for (int x = xi; x <= xj; x++) {
			const uint32_t c = ik_cnt(k, x, i, j);
			if (!c)
				continue;
			const double d = ik_val(k, x);
			const double yi = (d - median) / (9 * mad);
			const double yi2 = yi * yi;
			const double ai = (fabs(yi) < 1.0) ? 1.0 : 0.0;
			const double tu = ai * ((d - median) * (d - median)) * (((1 - yi2) * (1 - yi2)) * ((1 - yi2) * (1 - yi2)));
			const double td = (ai * (1 - yi2) * (1 - 5 * yi2));
			up = sg_add_repeat(up, tu, c);
			down = sg_add_repeat(down, td, c);
		}
		bwmv = (double)(j - i) * (up / (down * down));
	}
	return bwmv;
}

/* IKSS (:152-187), one lane per frame; rc[f] = -1 when the frame has no non-zero sample */
__global__ void __launch_bounds__(64)
k_ikss_solve(const uint32_t *__restrict__ P, const uint32_t *__restrict__ maxi, int nf, double *__restrict__ out,
		int *__restrict__ rc) {
	const int f = blockIdx.x * 64 + threadIdx.x;
	if (f >= nf)
		return;
	SgIk k;
	k.P = P;
	k.nf = nf;
	k.f = f;
	k.norm = maxi[f] <= 255u ? 255.0 : 65535.0;	/* get_normalized_value, src/core/utils.c:454-459 */
	const uint32_t n = ik_P(k, SG_ST_BINS);
	double location = 0.0, scale = 0.0;
	int r = 0;
	if (!n) {
		r = -1;	/* ngoodpix == 0: statistics() returns NULL (:249-252) */
	} else {
		uint32_t i = 0, j = n;
		double s0 = 1;
		for (int guard = 0;; guard++) {
			if (guard > 10000) {
				r = -2;	/* no convergence (the reference would loop) */
				break;
			}
			if (j - i < 1) {
				location = scale = 0;
				break;
			}
			const double m = ik_median(k, i, j);
			const double mad = ik_mad(k, i, j, m);
			const double s = sqrt(ik_bwmv(k, i, j, mad, m));
			if (s < 2E-23) {
				location = m;
				scale = 0;
				break;
			}
			if (((s0 - s) / s) < 10E-6) {
				location = m;
				scale = 0.991 * s;
				break;
			}
			s0 = s;
			const double xlow = m - 4 * s, xhigh = m + 4 * s;
			/* while (data[i] < xlow) i++: first x with val(x) >= xlow */
			int lo = 1, hi = SG_ST_BINS;
			while (lo < hi) {
				const int mid = (lo + hi) >> 1;
				if (ik_val(k, mid) >= xlow)
					hi = mid;
				else
					lo = mid + 1;
			}
			const uint32_t ni = ik_P(k, lo);
			i = ni > i ? ni : i;
			/* while (data[j - 1] > xhigh) j--: last x with val(x) <= xhigh */
			lo = 0;
			hi = SG_ST_BINS - 1;
			while (lo < hi) {
				const int mid = (lo + hi + 1) >> 1;
				if (ik_val(k, mid) <= xhigh)
					lo = mid;
				else
					hi = mid - 1;
			}
			const uint32_t nj = ik_P(k, lo + 1);
			j = nj < j ? nj : j;
		}
	}
	out[2 * f] = location * k.norm;	/* back to the original range (:286-288) */
	out[2 * f + 1] = scale * k.norm;
	rc[f] = r;
}

extern "C" int sg_frame_stats_ikss_device(sg_ctx *ctx, int dev_index, const uint16_t *d_frames, int nframes, int C,
		int H, int W, int64_t frame_stride, double *location, double *scale, void *stream) {
	if (!ctx || dev_index < 0 || dev_index >= (int)ctx->dev.size() || !d_frames || nframes < 1 || C < 1 || C > 3 ||
			H < 1 || W < 1 || !location || !scale)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	const int64_t npix = (int64_t)H * W;
	if (frame_stride == 0)
		frame_stride = npix * C;
	if (npix >= (1ll << 32))
		return set_err(ctx, SG_ERR_SIZE, "frame too large for the statistics path%s (%ld pixels)", "", (long)npix);
	const int chunk = nframes < 256 ? nframes : 256;	/* frames per pass: 65537 x 256 x 4 B = 64 MiB */
	const size_t hist_bytes = (size_t)(SG_ST_BINS + 1) * chunk * sizeof(uint32_t);
	HIPCHK(ensure(dv.stats_buf, hist_bytes + (size_t)chunk * (sizeof(uint32_t) + 2 * sizeof(double) + sizeof(int)) + 64));
	uint32_t *hist = (uint32_t *)dv.stats_buf.p;
	uint32_t *maxi = hist + (size_t)(SG_ST_BINS + 1) * chunk;
	double *res = (double *)(((uintptr_t)(maxi + chunk) + 15) & ~(uintptr_t)15);
	int *rcs = (int *)(res + 2 * chunk);
	(void)hipFuncSetAttribute((const void *)k_ikss_hist, hipFuncAttributeMaxDynamicSharedMemorySize,
			(int)(SG_ST_BINS / 2 * sizeof(uint32_t)));
	std::vector<double> hres(2 * (size_t)chunk);
	std::vector<int> hrc(chunk);
	int ret = SG_OK;
	for (int f0 = 0; f0 < nframes; f0 += chunk) {
		const int nf = nframes - f0 < chunk ? nframes - f0 : chunk;
		HIPCHK(hipMemsetAsync(hist, 0, (size_t)(SG_ST_BINS + 1) * nf * sizeof(uint32_t), s));
		HIPCHK(hipMemsetAsync(maxi, 0, (size_t)nf * sizeof(uint32_t), s));
		const unsigned gx = (unsigned)((npix + SG_ST_CHUNK - 1) / SG_ST_CHUNK);
		hipLaunchKernelGGL(k_ikss_hist, dim3(gx, (unsigned)nf), dim3(1024), SG_ST_BINS / 2 * sizeof(uint32_t), s,
				d_frames, frame_stride, C, npix, nf, f0, hist, maxi);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_ikss_prefix, dim3((unsigned)((nf + 63) / 64)), dim3(64), 0, s, hist, nf);
		HIPCHK(hipGetLastError());
		hipLaunchKernelGGL(k_ikss_solve, dim3((unsigned)((nf + 63) / 64)), dim3(64), 0, s, (const uint32_t *)hist,
				(const uint32_t *)maxi, nf, res, rcs);
		HIPCHK(hipGetLastError());
		HIPCHK(hipMemcpyAsync(hres.data(), res, sizeof(double) * 2 * nf, hipMemcpyDeviceToHost, s));
		HIPCHK(hipMemcpyAsync(hrc.data(), rcs, sizeof(int) * nf, hipMemcpyDeviceToHost, s));
		HIPCHK(hipStreamSynchronize(s));
		for (int k = 0; k < nf; k++) {
			location[f0 + k] = hres[2 * k];
			scale[f0 + k] = hres[2 * k + 1];
			if (hrc[k] && ret == SG_OK)
				ret = set_err(ctx, SG_ERR_GENERIC, "frame %s%ld: no statistics (no non-zero pixel, or IKSS "
						"did not converge)", "", (long)(f0 + k));
		}
	}
	return ret;
}

/* compute_normalization (src/stacking/stacking.c:125-190 + :79-123) from per-frame
 * location / scale: host arithmetic, the reference frame first (it fixes the *0 values),
 * ref_image indexing the stacked frames as the reference does */
extern "C" int sg_compute_normalization(int mode, int nframes, int ref_image, const double *location,
		const double *scale_in, double *offset, double *mul, double *scale) {
	if (nframes < 1 || !offset || !mul || !scale || (mode != SG_NO_NORM && (!location || !scale_in)))
		return SG_ERR_GENERIC;
	if (ref_image < 0)
		ref_image = 0;
	if (ref_image >= nframes)
		return SG_ERR_GENERIC;
	for (int i = 0; i < nframes; i++) {
		offset[i] = 0.0;
		mul[i] = 1.0;
		scale[i] = 1.0;
	}
	if (mode == SG_NO_NORM)
		return SG_OK;
	double scale0 = 0.0, mul0 = 0.0, offset0 = 0.0;
	for (int pass = 0; pass < 2; pass++)
		for (int i = 0; i < nframes; i++) {
			if ((pass == 0) != (i == ref_image))
				continue;
			switch (mode) {
			default:
			case SG_ADDITIVE_SCALING:
				scale[i] = scale_in[i];
				if (i == ref_image)
					scale0 = scale[ref_image];
				scale[i] = scale0 / scale[i];
				/* fall through */
			case SG_ADDITIVE:
				offset[i] = location[i];
				if (i == ref_image)
					offset0 = offset[ref_image];
				offset[i] = scale[i] * offset[i] - offset0;
				break;
			case SG_MULTIPLICATIVE_SCALING:
				scale[i] = scale_in[i];
				if (i == ref_image)
					scale0 = scale[ref_image];
				scale[i] = scale0 / scale[i];
				/* fall through */
			case SG_MULTIPLICATIVE:
				mul[i] = location[i];
				if (i == ref_image)
					mul0 = mul[ref_image];
				mul[i] = mul0 / mul[i];
				break;
			}
		}
	return SG_OK;
}

/* host frames: one frame at a time through the context's frame buffer (the reference computes
 * the statistics of one loaded frame at a time too, seq_get_imstats) */
extern "C" int sg_frame_stats_ikss(sg_ctx *ctx, const uint16_t *frames, int nframes, int C, int H, int W,
		double *location, double *scale) {
	if (!ctx || ctx->dev.empty() || !frames || nframes < 1 || C < 1 || C > 3 || H < 1 || W < 1 || !location ||
			!scale)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[0];
	HIPCHK(hipSetDevice(dv.id));
	const size_t fbytes = (size_t)C * H * W * sizeof(uint16_t);
	HIPCHK(ensure(dv.reg_sel, fbytes));
	int ret = SG_OK;
	for (int f = 0; f < nframes; f++) {
		HIPCHK(hipMemcpyAsync(dv.reg_sel.p, frames + (size_t)f * C * H * W, fbytes, hipMemcpyHostToDevice, dv.stream));
		const int rc = sg_frame_stats_ikss_device(ctx, 0, (const uint16_t *)dv.reg_sel.p, 1, C, H, W, 0, location + f,
				scale + f, nullptr);
		if (rc == SG_ERR_GENERIC)
			ret = SG_ERR_GENERIC;	/* a frame without non-zero pixel: keep going, report */
		else if (rc)
			return rc;
	}
	return ret;
}
