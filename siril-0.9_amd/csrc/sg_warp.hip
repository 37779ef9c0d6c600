/*
 * sg_warp.hip - perspective warp of a frame, replacing cvTransformImage
 * (src/opencv/opencv.cpp:242-309) as called by the star-alignment registration
 * (src/registration/registration.c:719-723: the image is flipped top-to-bottom, warped,
 * flipped back, so the warp works in display (top-down) coordinates).
 *
 * cvTransformImage runs OpenCV's warpPerspective(in, out, H, Size(ref), interpolation) on a
 * CV_16UC3 image (each channel independently; mono images go through as three equal
 * channels) with the default BORDER_CONSTANT 0 and without WARP_INVERSE_MAP.  OpenCV is
 * not in this container and its version is unpinned (configure.ac:129-135), so its
 * published algorithm (imgwarp.cpp, OpenCV 2.4-4.x) is restated here - parity unpinned:
 *   - M = H^-1 (cv::invert, DECOMP_LU: closed form for 3x3 with 1/det), host, double;
 *   - per destination pixel (x, y): X0 = M0 x + M1 y + M2, Y0 = M3 x + M4 y + M5,
 *     W = M6 x + M7 y + M8 (double);
 *     NEAREST: W = W ? 1/W : 0, X = cvRound(X0 W), Y = cvRound(Y0 W), the source pixel or
 *     0 outside;
 *     LINEAR / CUBIC / LANCZOS4: W = W ? 32/W : 0, X = cvRound(X0 W) (INTER_BITS = 5),
 *     integer part X >> 5, sub-pixel index (Y & 31) * 32 + (X & 31) into the 2-D float
 *     coefficient table of initInterTab2D (outer products of the 1-D coefficients:
 *     linear 1-x, x; cubic A = -0.75; Lanczos-4 with its sin table and 1/sum
 *     normalisation), the weighted sum accumulated in float in OpenCV's order, then
 *     saturate_cast<ushort> (round half to even, clamp);
 *   - BORDER_CONSTANT: a pixel whose taps are all outside gets 0, taps outside the image
 *     read 0 (remapBilinear / remapBicubic / remapLanczos4 border branches);
 *   - INTER_AREA is INTER_LINEAR in warpPerspective.
 * cvRound is lrint (round half to even) on the x86 builds of Siril; __double2int_rn /
 * rintf here.  One thread per destination pixel and channel; the source plane is read
 * through the L2 (the gathers of neighbouring threads hit the same lines).
 */
#include "sg_common.hpp"
#include "sg_ctx.hpp"
#include <math.h>
#include <vector>

#define SG_INTER_BITS 5
#define SG_INTER_TAB 32

enum { SG_WARP_NEAREST = 0, SG_WARP_LINEAR = 1, SG_WARP_AREA = 2, SG_WARP_CUBIC = 3, SG_WARP_LANCZOS4 = 4 };

struct SgWarp {
	const uint16_t *in;
	uint16_t *out;
	int W, H, C, oW, oH;
	int64_t in_plane, out_plane;
	double M[9];
	int bw;			/* OpenCV's block width (x association of the coordinate sums) */
	const float *tab;	/* [1024][k*k] */
};

__device__ __forceinline__ uint16_t sg_sat_u16(float v) {
	const float r = rintf(v);
	return r <= 0.f ? 0 : (r >= 65535.f ? 65535 : (uint16_t)r);
}

__device__ __forceinline__ int sg_sat_short(int v) {
	return v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
}

/* sample of source display row y, column x (0 outside) */
__device__ __forceinline__ float sg_src(const SgWarp &w, const uint16_t *plane, int x, int y) {
	if ((unsigned)x >= (unsigned)w.W || (unsigned)y >= (unsigned)w.H)
		return 0.f;
	return (float)plane[(int64_t)(w.H - 1 - y) * w.W + x];
}

template <int K>	/* taps per axis: 1 nearest, 2 linear, 4 cubic, 8 lanczos4 */
__global__ void __launch_bounds__(256) k_warp(SgWarp w) {
	const int x = blockIdx.x * 64 + (threadIdx.x & 63);
	const int yd = blockIdx.y * 4 + (threadIdx.x >> 6);	/* destination display row */
	const int c = blockIdx.z;
	if (x >= w.oW || yd >= w.oH)
		return;
	const uint16_t *plane = w.in + (int64_t)c * w.in_plane;
	/* WarpPerspectiveInvoker: per block row X0 = M0 xb + M1 y + M2, then X0 + M0 (x - xb) */
	const int xb = (x / w.bw) * w.bw, x1 = x - xb;
	const double X0 = w.M[0] * xb + w.M[1] * yd + w.M[2];
	const double Y0 = w.M[3] * xb + w.M[4] * yd + w.M[5];
	const double W0 = w.M[6] * xb + w.M[7] * yd + w.M[8];
	double W = W0 + w.M[6] * x1;
	uint16_t v;
	if (K == 1) {
		W = W != 0.0 ? 1.0 / W : 0.0;
		const double fX = fmax((double)INT_MIN, fmin((double)INT_MAX, (X0 + w.M[0] * x1) * W));
		const double fY = fmax((double)INT_MIN, fmin((double)INT_MAX, (Y0 + w.M[3] * x1) * W));
		const int X = sg_sat_short(__double2int_rn(fX)), Y = sg_sat_short(__double2int_rn(fY));
		v = (uint16_t)sg_src(w, plane, X, Y);
	} else {
		W = W != 0.0 ? (double)SG_INTER_TAB / W : 0.0;
		const double fX = fmax((double)INT_MIN, fmin((double)INT_MAX, (X0 + w.M[0] * x1) * W));
		const double fY = fmax((double)INT_MIN, fmin((double)INT_MAX, (Y0 + w.M[3] * x1) * W));
		const int X = __double2int_rn(fX), Y = __double2int_rn(fY);
		const int sx = sg_sat_short(X >> SG_INTER_BITS) - (K / 2 - 1), sy = sg_sat_short(Y >> SG_INTER_BITS) - (K / 2 - 1);
		const float *wt = w.tab + ((Y & (SG_INTER_TAB - 1)) * SG_INTER_TAB + (X & (SG_INTER_TAB - 1))) * K * K;
		if (sx >= w.W || sx + K - 1 < 0 || sy >= w.H || sy + K - 1 < 0) {
			v = 0;	/* every tap outside: the border value */
		} else if (K == 2) {
			/* remapBilinear, both branches: v0*w[0] + v1*w[1] + v2*w[2] + v3*w[3] (taps
			 * outside read the border value 0) */
			const float sum = sg_src(w, plane, sx, sy) * wt[0] + sg_src(w, plane, sx + 1, sy) * wt[1] +
				sg_src(w, plane, sx, sy + 1) * wt[2] + sg_src(w, plane, sx + 1, sy + 1) * wt[3];
			v = sg_sat_u16(sum);
		} else if (sx >= 0 && sx + K <= w.W && sy >= 0 && sy + K <= w.H) {
			/* remapBicubic / remapLanczos4 interior: sum += (row r, taps left to right) */
			float sum = 0.f;
#pragma unroll
			for (int r = 0; r < K; r++) {
				float row = sg_src(w, plane, sx, sy + r) * wt[r * K];
#pragma unroll
				for (int t = 1; t < K; t++)
					row = row + sg_src(w, plane, sx + t, sy + r) * wt[r * K + t];
				sum = r ? sum + row : row;
			}
			v = sg_sat_u16(sum);
		} else {
			/* border branch: sum = cval; sum += (S - cval) * w for every tap inside */
			float sum = 0.f;
			for (int r = 0; r < K; r++) {
				if ((unsigned)(sy + r) >= (unsigned)w.H)
					continue;
				for (int t = 0; t < K; t++)
					if ((unsigned)(sx + t) < (unsigned)w.W)
						sum = sum + sg_src(w, plane, sx + t, sy + r) * wt[r * K + t];
			}
			v = sg_sat_u16(sum);
		}
	}
	w.out[(int64_t)c * w.out_plane + (int64_t)(w.oH - 1 - yd) * w.oW + x] = v;
}

/* initInterTab1D / initInterTab2D (float) */
static void sg_coeffs(int interp, float x, float *k) {
	if (interp == SG_WARP_LINEAR) {
		k[0] = 1.f - x;
		k[1] = x;
	} else if (interp == SG_WARP_CUBIC) {
		const float A = -0.75f;
		k[0] = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A;
		k[1] = ((A + 2) * x - (A + 3)) * x * x + 1;
		k[2] = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1;
		k[3] = 1.f - k[0] - k[1] - k[2];
	} else {	/* Lanczos-4 */
		static const double s45 = 0.70710678118654752440084436210485;
		static const double cs[][2] = {{1, 0}, {-s45, -s45}, {0, 1}, {s45, -s45}, {-1, 0}, {s45, s45}, {0, -1}, {-s45, s45}};
		if (x < 1.192092896e-07f) {	/* FLT_EPSILON */
			for (int i = 0; i < 8; i++)
				k[i] = 0;
			k[3] = 1;
			return;
		}
		float sum = 0;
		const double y0 = -(x + 3) * M_PI * 0.25, s0 = sin(y0), c0 = cos(y0);
		for (int i = 0; i < 8; i++) {
			const double y = -(x + 3 - i) * M_PI * 0.25;
			k[i] = (float)((cs[i][0] * s0 + cs[i][1] * c0) / (y * y));
			sum += k[i];
		}
		sum = 1.f / sum;
		for (int i = 0; i < 8; i++)
			k[i] *= sum;
	}
}

static int sg_ksize(int interp) {
	return interp == SG_WARP_NEAREST ? 1 : interp == SG_WARP_CUBIC ? 4 : interp == SG_WARP_LANCZOS4 ? 8 : 2;
}

static void sg_tab2d(int interp, std::vector<float> &tab) {
	const int K = sg_ksize(interp);
	std::vector<float> t1((size_t)SG_INTER_TAB * K);
	for (int i = 0; i < SG_INTER_TAB; i++)
		sg_coeffs(interp, i * (1.f / SG_INTER_TAB), &t1[(size_t)i * K]);
	tab.assign((size_t)SG_INTER_TAB * SG_INTER_TAB * K * K, 0.f);
	for (int i = 0; i < SG_INTER_TAB; i++)
		for (int j = 0; j < SG_INTER_TAB; j++)
			for (int k1 = 0; k1 < K; k1++)
				for (int k2 = 0; k2 < K; k2++)
					tab[((size_t)(i * SG_INTER_TAB + j) * K + k1) * K + k2] = t1[(size_t)i * K + k1] * t1[(size_t)j * K + k2];
}

/* cv::invert(DECOMP_LU) of a 3x3: closed form with 1/det; 0 if singular */
static int sg_invert3(const double *a, double *o) {
	const double d = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) +
		a[2] * (a[3] * a[7] - a[4] * a[6]);
	if (d == 0.0)
		return 0;
	const double t = 1.0 / d;
	o[0] = (a[4] * a[8] - a[5] * a[7]) * t;
	o[1] = (a[2] * a[7] - a[1] * a[8]) * t;
	o[2] = (a[1] * a[5] - a[2] * a[4]) * t;
	o[3] = (a[5] * a[6] - a[3] * a[8]) * t;
	o[4] = (a[0] * a[8] - a[2] * a[6]) * t;
	o[5] = (a[2] * a[3] - a[0] * a[5]) * t;
	o[6] = (a[3] * a[7] - a[4] * a[6]) * t;
	o[7] = (a[1] * a[6] - a[0] * a[7]) * t;
	o[8] = (a[0] * a[4] - a[1] * a[3]) * t;
	return 1;
}

extern "C" int sg_warp_u16_device(sg_ctx *ctx, int dev_index, const uint16_t *d_in, int width, int height,
		int nb_layers, uint16_t *d_out, int out_width, int out_height, const double *hom, int interpolation,
		void *stream) {
	if (!ctx || !d_in || !d_out || !hom || dev_index < 0 || dev_index >= (int)ctx->dev.size() || width <= 0 ||
			height <= 0 || out_width <= 0 || out_height <= 0 || nb_layers < 1 || nb_layers > 3 ||
			interpolation < 0 || interpolation > SG_WARP_LANCZOS4)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t s = stream ? (hipStream_t)stream : dv.stream;
	const int interp = interpolation == SG_WARP_AREA ? SG_WARP_LINEAR : interpolation;
	SgWarp w;
	if (!sg_invert3(hom, w.M)) {
		for (int i = 0; i < 9; i++)
			w.M[i] = 0.0;	/* cv::invert leaves a zero matrix for a singular one */
	}
	w.in = d_in;
	w.out = d_out;
	w.W = width;
	w.H = height;
	w.C = nb_layers;
	w.oW = out_width;
	w.oH = out_height;
	w.in_plane = (int64_t)width * height;
	w.out_plane = (int64_t)out_width * out_height;
	w.tab = nullptr;
	{	/* WarpPerspectiveInvoker block size: BLOCK_SZ = 32 */
		int bh0 = out_height < 16 ? out_height : 16;
		int bw0 = 1024 / bh0 < out_width ? 1024 / bh0 : out_width;
		w.bw = bw0 > 0 ? bw0 : 1;
	}
	if (interp != SG_WARP_NEAREST) {
		if (dv.warp_tab_interp != interp) {
			std::vector<float> tab;
			sg_tab2d(interp, tab);
			HIPCHK(ensure(dv.warp_tab, tab.size() * sizeof(float)));
			HIPCHK(hipMemcpyAsync(dv.warp_tab.p, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice, s));
			HIPCHK(hipStreamSynchronize(s));
			dv.warp_tab_interp = interp;
		}
		w.tab = (const float *)dv.warp_tab.p;
	}
	const dim3 grid((unsigned)((out_width + 63) / 64), (unsigned)((out_height + 3) / 4), (unsigned)nb_layers);
	switch (sg_ksize(interp)) {
	case 1:
		hipLaunchKernelGGL(k_warp<1>, grid, dim3(256), 0, s, w);
		break;
	case 2:
		hipLaunchKernelGGL(k_warp<2>, grid, dim3(256), 0, s, w);
		break;
	case 4:
		hipLaunchKernelGGL(k_warp<4>, grid, dim3(256), 0, s, w);
		break;
	default:
		hipLaunchKernelGGL(k_warp<8>, grid, dim3(256), 0, s, w);
	}
	HIPCHK(hipGetLastError());
	if (!stream)
		HIPCHK(hipStreamSynchronize(s));
	return SG_OK;
}

extern "C" int sg_warp_u16(sg_ctx *ctx, const uint16_t *in, int width, int height, int nb_layers, uint16_t *out,
		int out_width, int out_height, const double *hom, int interpolation) {
	if (!ctx || ctx->dev.empty() || !in || !out)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[0];
	HIPCHK(hipSetDevice(dv.id));
	const size_t nin = (size_t)width * height * nb_layers, nout = (size_t)out_width * out_height * nb_layers;
	HIPCHK(ensure(dv.frames, nin * sizeof(uint16_t)));
	HIPCHK(ensure(dv.out, nout * sizeof(uint16_t)));
	HIPCHK(hipMemcpyAsync(dv.frames.p, in, nin * sizeof(uint16_t), hipMemcpyHostToDevice, dv.stream));
	const int rc = sg_warp_u16_device(ctx, 0, (const uint16_t *)dv.frames.p, width, height, nb_layers,
			(uint16_t *)dv.out.p, out_width, out_height, hom, interpolation, nullptr);
	if (rc)
		return rc;
	HIPCHK(hipMemcpyAsync(out, dv.out.p, nout * sizeof(uint16_t), hipMemcpyDeviceToHost, dv.stream));
	HIPCHK(hipStreamSynchronize(dv.stream));
	return SG_OK;
}
