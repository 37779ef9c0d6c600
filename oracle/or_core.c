/*
 * or_core.c - restated helpers (TEST INFRASTRUCTURE ONLY, see oracle.h; parity unpinned).
 *
 * round_to_WORD  : src/core/utils.c:68-74
 * quicksort_s    : src/core/utils.c:512-533
 * GSL statistics : third-party, not in /root/reference.  GSL (version unpinned by
 *                  configure.ac:68-71) statistics/mean_source.c, variance_source.c,
 *                  median_source.c and fit/linear.c, restated from their published
 *                  algorithms.  Call sites: src/stacking/stacking.c:767,1662,1676-1678,
 *                  1698-1700,1713-1727,1760.  The long double recurrences are x87 80-bit
 *                  on x86-64, which is what this file compiles to (gcc, -O2, no FMA).
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include "oracle.h"

uint16_t or_round_to_WORD(double x) {
	if (x <= 0.0)
		return (uint16_t)0;
	if (x > 65535.0)
		return 65535;
	return (uint16_t)(x + 0.5);
}

void or_quicksort_s(uint16_t *a, int n) {
	if (n < 2)
		return;
	uint16_t p = a[n / 2];
	uint16_t *l = a;
	uint16_t *r = a + n - 1;
	while (l <= r) {
		if (*l < p) {
			l++;
			continue;
		}
		if (*r > p) {
			r--;
			continue;
		}
		uint16_t t = *l;
		*l++ = *r;
		*r-- = t;
	}
	or_quicksort_s(a, (int)(r - a + 1));
	or_quicksort_s(l, (int)(a + n - l));
}

/* gsl_stats_ushort_mean: long double running mean */
double or_gsl_mean_u16(const uint16_t *data, size_t n) {
	long double mean = 0;
	size_t i;
	for (i = 0; i < n; i++)
		mean += (data[i] - mean) / (i + 1);
	return mean;
}

/* compute_variance: delta is formed in double (ushort - double), accumulated in long double */
static double or_gsl_compute_variance(const uint16_t *data, size_t n, double mean) {
	long double variance = 0;
	size_t i;
	for (i = 0; i < n; i++) {
		const long double delta = (data[i] - mean);
		variance += (delta * delta - variance) / (i + 1);
	}
	return variance;
}

/* gsl_stats_ushort_sd = sd_m(data, mean(data)) */
double or_gsl_sd_u16(const uint16_t *data, size_t n) {
	const double mean = or_gsl_mean_u16(data, n);
	const double variance = or_gsl_compute_variance(data, n, mean);
	return sqrt(variance * ((double)n / (double)(n - 1)));
}

double or_gsl_median_from_sorted_u16(const uint16_t *sorted, size_t n) {
	double median;
	const size_t lhs = (n - 1) / 2;
	const size_t rhs = n / 2;
	if (n == 0)
		return 0.0;
	if (lhs == rhs)
		median = sorted[lhs];
	else
		median = (sorted[lhs] + sorted[rhs]) / 2.0;
	return median;
}

/* gsl_fit_linear (y = c0 + c1 x), all double */
void or_gsl_fit_linear(const double *x, const double *y, size_t n, double *c0, double *c1) {
	double m_x = 0, m_y = 0, m_dx2 = 0, m_dxdy = 0;
	size_t i;
	for (i = 0; i < n; i++) {
		m_x += (x[i] - m_x) / (i + 1.0);
		m_y += (y[i] - m_y) / (i + 1.0);
	}
	for (i = 0; i < n; i++) {
		const double dx = x[i] - m_x;
		const double dy = y[i] - m_y;
		m_dx2 += (dx * dx - m_dx2) / (i + 1.0);
		m_dxdy += (dx * dy - m_dxdy) / (i + 1.0);
	}
	{
		double b = m_dxdy / m_dx2;
		double a = m_y - m_x * b;
		*c0 = a;
		*c1 = b;
	}
}
