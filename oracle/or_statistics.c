/*
 * or_statistics.c - TEST INFRASTRUCTURE ONLY (see oracle.h): the location / scale that
 * stacking normalisation reads from a frame's imstats (_compute_normalization_for_image,
 * src/stacking/stacking.c:79-123 -> seq_get_imstats src/io/sequence.c:1107-1118 ->
 * statistics(fit, 0, NULL, STATS_EXTRA, STATS_ZERO_NULLCHECK), src/algos/statistics.c:221-326).
 * Only the IKSS part feeds normalisation (stat->location, stat->scale).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static int cmp_d(const void *a, const void *b) {
	const double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : (x > y ? 1 : 0);
}

/* gsl_stats_median_from_sorted_data (GSL statistics/median_source.c) */
static double median_sorted_d(const double *a, size_t n) {
	const size_t lhs = (n - 1) / 2, rhs = n / 2;
	if (n == 0)
		return 0.0;
	if (lhs == rhs)
		return a[lhs];
	return (a[lhs] + a[rhs]) / 2.0;
}

/* siril_stats_double_mad, statistics.c:82-100 */
static double stats_double_mad(const double *data, size_t n, double m) {
	double *tmp = (double *)calloc(n ? n : 1, sizeof(double));
	for (size_t i = 0; i < n; i++)
		tmp[i] = fabs(data[i] - m);
	qsort(tmp, n, sizeof(double), cmp_d);	/* quicksort_d: any sort gives the same order */
	const double med = median_sorted_d(tmp, n);
	free(tmp);
	return med;
}

#define OR_SQR(x) ((x) * (x))	/* src/core/siril.h:34 */

/* siril_stats_double_bwmv, statistics.c:128-150 (sequential sums in data order) */
static double stats_double_bwmv(const double *data, size_t n, double mad, double median) {
	double bwmv = 0.0, up = 0.0, down = 0.0;
	if (mad > 0.0) {
		for (size_t i = 0; i < n; i++) {
			const double yi = (data[i] - median) / (9 * mad);
			const double yi2 = yi * yi;
			const double ai = (fabs(yi) < 1.0) ? 1.0 : 0.0;
			up += ai * OR_SQR(data[i] - median) * OR_SQR(OR_SQR(1 - yi2));
			down += (ai * (1 - yi2) * (1 - 5 * yi2));
		}
		bwmv = n * (up / (down * down));
	}
	return bwmv;
}

/* IKSS, statistics.c:152-187, on sorted data */
static void ikss(double *data, size_t n, double *location, double *scale) {
	size_t i = 0, j = n;
	double s0 = 1;
	qsort(data, n, sizeof(double), cmp_d);
	for (;;) {
		if (j - i < 1) {
			*location = *scale = 0;
			break;
		}
		const double m = median_sorted_d(data + i, j - i);
		const double mad = stats_double_mad(data + i, j - i, m);
		const double s = sqrt(stats_double_bwmv(data + i, j - i, mad, m));
		if (s < 2E-23) {
			*location = m;
			*scale = 0;
			break;
		}
		if (((s0 - s) / s) < 10E-6) {
			*location = m;
			*scale = 0.991 * s;
			break;
		}
		s0 = s;
		const double xlow = m - 4 * s, xhigh = m + 4 * s;
		while (data[i] < xlow)
			i++;
		while (data[j - 1] > xhigh)
			j--;
	}
}

/* statistics(fit, 0, NULL, STATS_IKSS, STATS_ZERO_NULLCHECK) location / scale of layer 0 of
 * a frame [C][H][W]: zeros are null pixels (reassign_data :189-200), the data are divided by
 * hist_size - 1 where hist_size = get_normalized_value(fit) + 1 (src/core/utils.c:454-459:
 * 255 when the frame's maximum over all layers is <= 255, else 65535) and the result is
 * scaled back (:283-292).  Returns -1 when no pixel is non-zero (statistics() returns NULL). */
int or_statistics_ikss(const uint16_t *frame, int C, int H, int W, double *location, double *scale) {
	const size_t npix = (size_t)H * W;
	unsigned maxi = 0;
	for (size_t k = 0; k < npix * (size_t)C; k++)
		maxi = frame[k] > maxi ? frame[k] : maxi;
	const double norm = maxi <= 255 ? 255.0 : 65535.0;	/* (double) hist_size - 1 */
	size_t ngood = 0;
	for (size_t k = 0; k < npix; k++)
		ngood += frame[k] > 0;
	if (!ngood)
		return -1;
	double *d = (double *)malloc(ngood * sizeof(double));
	size_t t = 0;
	for (size_t k = 0; k < npix; k++)
		if (frame[k] > 0)
			d[t++] = (double)frame[k] / norm;
	ikss(d, ngood, location, scale);
	*location *= norm;
	*scale *= norm;
	free(d);
	return 0;
}
