/*
 * or_registration.c - CPU restatement of Siril 0.9 DFT registration and the planetary
 * quality estimate (TEST INFRASTRUCTURE ONLY; parity unpinned, see oracle.h).
 *
 *   register_shift_dft      src/registration/registration.c:182-400
 *   normalizeQualityData    src/registration/registration.c:163-176
 *   QualityEstimate         src/algos/quality.c:46-218
 *   SubSample / Gradient / _smooth_image_16   src/algos/quality.c:223-349
 *
 * FFTW3 (third-party, version unpinned, configure.ac:65) is replaced by a plain
 * double-precision DFT with FFTW's conventions: unnormalised, FFTW_FORWARD = e^{-i},
 * FFTW_BACKWARD = e^{+i}, row-major 2-D.  Only the arg-max of the correlation survives
 * into the result, so any accurate DFT gives the same shifts except at near ties.
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <stdint.h>
#include "oracle.h"

/* out-of-place 1-D complex DFT of length n (input stride `is`): recursive mixed radix by
 * decimation in time over the smallest prime factor p of n (n = p m: p sub-transforms of the
 * decimated sequences, combined with twiddles exp(sign 2 pi i k / n)); a prime n is summed
 * directly in O(n^2).  Plain double, FFTW's sign convention. */
static void dft_rec(const double *xr, const double *xi, int is, double *yr, double *yi, int n, int sign) {
	if (n == 1) {
		yr[0] = xr[0];
		yi[0] = xi[0];
		return;
	}
	int p = 2;
	while (p * p <= n && n % p)
		p++;
	if (n % p)
		p = n;	/* prime */
	if (p == n) {
		for (int k = 0; k < n; k++) {
			double sr = 0, si = 0;
			for (int t = 0; t < n; t++) {
				const double a = sign * 2.0 * M_PI * (double)(((long)k * t) % n) / n;
				const double c = cos(a), s = sin(a);
				sr += xr[(size_t)t * is] * c - xi[(size_t)t * is] * s;
				si += xr[(size_t)t * is] * s + xi[(size_t)t * is] * c;
			}
			yr[k] = sr;
			yi[k] = si;
		}
		return;
	}
	const int m = n / p;
	/* sub-transform q (inputs x[q], x[q+p], ...) into y[q m .. q m + m) */
	for (int q = 0; q < p; q++)
		dft_rec(xr + (size_t)q * is, xi + (size_t)q * is, is * p, yr + (size_t)q * m, yi + (size_t)q * m, m, sign);
	double *tr = malloc((size_t)n * sizeof(double)), *ti = malloc((size_t)n * sizeof(double));
	for (int k = 0; k < m; k++)
		for (int s = 0; s < p; s++) {
			/* X[k + s m] = sum_q W_n^{q (k + s m)} Y_q[k] */
			const int kk = k + s * m;
			double sr = 0, si = 0;
			for (int q = 0; q < p; q++) {
				const double a = sign * 2.0 * M_PI * (double)(((long)q * kk) % n) / n;
				const double c = cos(a), sn = sin(a);
				const double ur = yr[(size_t)q * m + k], ui = yi[(size_t)q * m + k];
				sr += ur * c - ui * sn;
				si += ur * sn + ui * c;
			}
			tr[kk] = sr;
			ti[kk] = si;
		}
	memcpy(yr, tr, (size_t)n * sizeof(double));
	memcpy(yi, ti, (size_t)n * sizeof(double));
	free(tr);
	free(ti);
}

/* in-place 1-D complex DFT of length n with stride 1 (radix-2 if n is a power of two,
 * otherwise the recursive mixed radix above).  tw: the radix-2 stages' twiddles, stage len at
 * tw + 2 (len / 2 - 1) as (cos, sin)(sign 2 pi k / len), k < len / 2 - the values the plain
 * loop computes per stage, tabulated once per 2-D transform */
static void dft1d(double *re, double *im, int n, int sign, const double *tw) {
	if ((n & (n - 1)) == 0) {
		/* bit reversal */
		for (int i = 1, j = 0; i < n; i++) {
			int bit = n >> 1;
			for (; j & bit; bit >>= 1)
				j ^= bit;
			j ^= bit;
			if (i < j) {
				double t = re[i]; re[i] = re[j]; re[j] = t;
				t = im[i]; im[i] = im[j]; im[j] = t;
			}
		}
		for (int len = 2; len <= n; len <<= 1) {
			const double *w = tw + 2 * (len / 2 - 1);
			for (int i = 0; i < n; i += len) {
				for (int k = 0; k < len / 2; k++) {
					double ur = re[i + k], ui = im[i + k];
					double xr = re[i + k + len / 2], xi = im[i + k + len / 2];
					double vr = xr * w[2 * k] - xi * w[2 * k + 1];
					double vi = xr * w[2 * k + 1] + xi * w[2 * k];
					re[i + k] = ur + vr;
					im[i + k] = ui + vi;
					re[i + k + len / 2] = ur - vr;
					im[i + k + len / 2] = ui - vi;
				}
			}
		}
	} else {
		double *tr = malloc(n * sizeof(double)), *ti = malloc(n * sizeof(double));
		dft_rec(re, im, 1, tr, ti, n, sign);
		memcpy(re, tr, n * sizeof(double));
		memcpy(im, ti, n * sizeof(double));
		free(tr);
		free(ti);
	}
}

void or_dft2d(double *re, double *im, int S, int sign) {
	/* stage tables: sum over stages of len / 2 = S - 1 (cos, sin) pairs */
	double *tw = malloc(2 * (size_t)(S > 1 ? S : 2) * sizeof(double));
	if ((S & (S - 1)) == 0)
		for (int len = 2; len <= S; len <<= 1) {
			const double ang = sign * 2.0 * M_PI / len;
			double *w = tw + 2 * (len / 2 - 1);
			for (int k = 0; k < len / 2; k++) {
				w[2 * k] = cos(ang * k);
				w[2 * k + 1] = sin(ang * k);
			}
		}
	double *cr = malloc(S * sizeof(double)), *ci = malloc(S * sizeof(double));
	for (int y = 0; y < S; y++)
		dft1d(re + (size_t)y * S, im + (size_t)y * S, S, sign, tw);
	for (int x = 0; x < S; x++) {
		for (int y = 0; y < S; y++) {
			cr[y] = re[(size_t)y * S + x];
			ci[y] = im[(size_t)y * S + x];
		}
		dft1d(cr, ci, S, sign, tw);
		for (int y = 0; y < S; y++) {
			re[(size_t)y * S + x] = cr[y];
			im[(size_t)y * S + x] = ci[y];
		}
	}
	free(tw); free(cr); free(ci);
}

/* quality.h constants */
#define MAXP 6
#define QMARGIN 0.1
#define QSUBSAMPLE_INC 1
#define QSUBSAMPLE_MAX 5
#define QSUBSAMPLE_MIN 3
#define THRESHOLD 40

static int32_t SubSample(const uint16_t *ptr, int img_wid, int x_size, int y_size) {
	int x, y, val = 0;
	for (y = 0; y < y_size; ++y) {
		for (x = 0; x < x_size; x++)
			val += ptr[x];
		ptr += img_wid;
	}
	return val / (x_size * y_size);
}

static uint16_t *smooth_image_16(const uint16_t *buf, int width, int height) {
	uint16_t *new_buff = calloc((size_t)width * height * 2, sizeof(uint16_t));
	for (int y = 1; y < height - 1; ++y) {
		int o = y * width + 1;
		for (int x = 1; x < width - 1; ++x, ++o) {
			unsigned int v = buf[o];
			v += buf[o - width - 1];
			v += buf[o - width];
			v += buf[o - width + 1];
			v += buf[o - 1];
			v += buf[o + 1];
			v += buf[o + width - 1];
			v += buf[o + width];
			v += buf[o + width + 1];
			new_buff[o] = v / 9;
		}
	}
	return new_buff;
}

static double Gradient(const uint16_t *buf, int width, int height) {
	int pixels, x, y;
	int yborder = (int)((double)height * QMARGIN) + 1;
	int xborder = (int)((double)width * QMARGIN) + 1;
	double d1, d2, val, avg = 0;
	int threshhold = (THRESHOLD) << 8;
	unsigned char *map = calloc((size_t)width * height, 1);
	pixels = 0;
	for (y = yborder; y < height - yborder; ++y) {
		int o = y * width + xborder;
		for (x = xborder; x < width - xborder; ++x, ++o) {
			if (buf[o] >= threshhold) {
				map[o - width - 1] = map[o - width] = map[o - width + 1] = 1;
				map[o - 1] = map[o] = map[o + 1] = 1;
				map[o + width - 1] = map[o + width] = map[o + width + 1] = 1;
				++pixels;
				avg += buf[o];
			}
		}
	}
	if (!pixels) {
		val = -1.0;
		goto end;
	}
	val = 0;
	pixels = 0;
	for (y = yborder; y < height - yborder; ++y) {
		int o = y * width + xborder;
		for (x = xborder; x < width - xborder; ++x, ++o)
			if (map[o]) {
				d1 = buf[o];
				d2 = buf[o];
				d1 = d1 - (int)(buf[o + 1]);
				d2 = d2 - (int)(buf[o + width]);
				val += (d1 * d1 + d2 * d2);
				pixels++;
			}
	}
	val = val / (double)pixels;
	val = val / 10;
end:
	free(map);
	return val;
}

double or_quality_estimate(const uint16_t *buffer, int width, int height) {
	int region_w = width - 1, region_h = height - 1;
	int x1 = 0, y1 = 0;
	int subsample, i, j, n, x, y, max, maxp[MAXP], x_inc, x_samples, y_samples, y_last;
	double mult, q, dval = 0.0;
	uint16_t *buf = calloc((size_t)region_w * region_h + 1, sizeof(uint16_t));
	subsample = QSUBSAMPLE_MIN;
	while (subsample <= QSUBSAMPLE_MAX) {
		const uint16_t *ptr;
		x_samples = region_w / subsample;
		y_samples = region_h / subsample;
		if (x_samples < 2 || y_samples < 2)
			break;
		y_last = y1 + (y_samples - 1) * subsample;
		x_inc = subsample;
		for (i = 0; i < MAXP; ++i)
			maxp[i] = 0;
		y = y1;
		n = 0;
		ptr = buffer + (y * width + x1);
		for (x = 0; x < x_samples; ++x, ptr += x_inc)
			buf[n++] = SubSample(ptr, width, subsample, subsample);
		for (y += subsample; y < y_last; y += subsample) {
			ptr = buffer + (y * width + x1);
			for (x = 0; x < x_samples; ++x, ptr += x_inc) {
				int v = SubSample(ptr, width, subsample, subsample);
				if (v > maxp[2] && v < 65530) {
					int slot;
					if (v > maxp[0])
						slot = 0;
					else if (v > maxp[1])
						slot = 1;
					else
						slot = 2;
					for (j = MAXP - 1; j > slot; --j) {
						maxp[j] = maxp[j - 1];
						maxp[j] = v;
					}
				}
				buf[n++] = v;
			}
		}
		ptr = buffer + (y * width + x1);
		for (x = 0; x < x_samples; ++x, ptr += x_inc)
			buf[n++] = SubSample(ptr, width, subsample, subsample);
		j = MAXP / 2;
		for (i = j, max = 0; i < MAXP; ++i)
			max += maxp[i];
		max /= (MAXP - j);
		if (max > 0) {
			mult = (double)60000 / (double)max;
			for (i = 0; i < n; ++i) {
				unsigned int v = buf[i];
				v = (unsigned int)((double)v * mult);
				if (v > 65535)
					v = 65535;
				buf[i] = v;
			}
		}
		uint16_t *new_image = smooth_image_16(buf, x_samples, y_samples);
		q = Gradient(new_image, x_samples, y_samples);
		free(new_image);
		dval += (q * ((QSUBSAMPLE_MIN * QSUBSAMPLE_MIN) / (subsample * subsample)));
		do {
			subsample += QSUBSAMPLE_INC;
		} while (width / subsample == x_samples && height / subsample == y_samples);
	}
	dval = sqrt(dval);
	free(buf);
	return dval;
}

int or_register_shift_dft(const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality) {
	size_t sq = (size_t)S * S;
	double *inr = malloc(sq * sizeof(double)), *ini = malloc(sq * sizeof(double));
	double q_max, q_min;
	if (ref_image < 0)
		ref_image = 0;
	const uint16_t *refsel = sel + (size_t)ref_image * sq;
	for (size_t j = 0; j < sq; j++) {
		inr[j] = (double)refsel[j];
		ini[j] = 0.0;
	}
	quality[ref_image] = or_quality_estimate(refsel, S, S);
	or_dft2d(inr, ini, S, -1);
	shiftx[ref_image] = 0;
	shifty[ref_image] = 0;
	/* the frames in an OpenMP loop with per-thread buffers, as the reference's
	 * `omp parallel for ... firstprivate(fit) schedule(static)` (:276-279); q_min / q_max are
	 * formed afterwards in index order (the reference's omp critical takes them in completion
	 * order, which only matters for NaN qualities through the min() macro) */
#pragma omp parallel
	{
		double *ar = malloc(sq * sizeof(double)), *ai = malloc(sq * sizeof(double));
#pragma omp for schedule(static)
		for (int frame = 0; frame < nframes; ++frame) {
			if (frame == ref_image)
				continue;
			if (included && !included[frame])
				continue;
			const uint16_t *img = sel + (size_t)frame * sq;
			for (size_t x = 0; x < sq; x++) {
				ar[x] = (double)img[x];
				ai[x] = 0.0;
			}
			quality[frame] = or_quality_estimate(img, S, S);
			or_dft2d(ar, ai, S, -1);
			/* convol2 = in * conj(out2) */
			for (size_t x = 0; x < sq; x++) {
				double br = ar[x], bi = -ai[x];
				double cr = inr[x] * br - ini[x] * bi;
				double ci = inr[x] * bi + ini[x] * br;
				ar[x] = cr;
				ai[x] = ci;
			}
			or_dft2d(ar, ai, S, +1);
			size_t shift = 0;
			for (size_t x = 1; x < sq; ++x)
				if (ar[x] > ar[shift])
					shift = x;
			int sy = (int)(shift / S), sx = (int)(shift % S);
			if (sy > S / 2)
				sy -= S;
			if (sx > S / 2)
				sx -= S;
			shiftx[frame] = sx;
			shifty[frame] = sy;
		}
		free(ar);
		free(ai);
	}
	q_min = q_max = quality[ref_image];
	for (int frame = 0; frame < nframes; ++frame) {
		if (frame == ref_image || (included && !included[frame]))
			continue;
		const double qual = quality[frame];
		if (qual > q_max)
			q_max = qual;
		q_min = (q_min < qual) ? q_min : qual;	/* siril.h:30-33 min() */
	}
	/* normalizeQualityData */
	for (int frame = 0; frame < nframes; ++frame) {
		if (included && !included[frame])
			continue;
		quality[frame] -= q_min;
		quality[frame] /= (q_max - q_min);
	}
	free(inr); free(ini);
	return 0;
}

/* The exact value behind one entry of the reference's correlation plane: FFTW_BACKWARD of
 * FFT(ref) conj(FFT(img)) (registration.c:326-334) is S^2 sum_n ref(n + k) img(n) (circular,
 * row-major k = ky S + kx); the sum is an integer below 2^56 for S <= 4096. */
long long or_xcorr_at(const uint16_t *ref, const uint16_t *img, int S, int ky, int kx) {
	long long acc = 0;
	for (int y = 0; y < S; y++) {
		const uint16_t *rr = ref + (size_t)((y + ky) % S) * S, *ir = img + (size_t)y * S;
		for (int x = 0; x < S; x++)
			acc += (long long)rr[(x + kx) % S] * ir[x];
	}
	return acc;
}
