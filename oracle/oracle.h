/*
 * oracle.h - CPU restatement of Siril 0.9 registration + stacking (TEST INFRASTRUCTURE ONLY).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker or as the CPU baseline: the product path
 * (siril-0.9_amd/) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned".  The reference has no tests, no golden vectors and
 * cannot be built in this image (GTK3/GSL/FFTW/libconfig headers absent),
 * so this restatement is pinned only by (1) line-by-line citation of the reference
 * (file:line in each function), (2) an independent numpy restatement
 * (tests/oracle_numpy.py, x87 long double via numpy.longdouble) and (3) the committed
 * golden fixtures in tests/golden/ generated from both.  The third-party arithmetic
 * boundaries (GSL sd/median/fit_linear, FFTW) are restated from their published
 * algorithms (GSL 1.x/2.x statistics/mean_source.c, variance_source.c,
 * median_source.c, fit/linear.c; FFTW = unnormalised DFT).
 *
 * Data layout: frames[N][C][H][W] u16 in Siril memory order (bottom-up rows,
 * planar channels, src/core/siril.h:391-442).  Outputs are [C][H][W] bottom-up.
 */
#ifndef SG_ORACLE_H
#define SG_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
void or_synth_window(uint16_t *out, int nframes, int c, int y0, int x0, int h, int w, uint64_t seed,
		int maxshift);
#endif

/* src/stacking/stacking.h:14-21 */
enum { OR_NO_REJEC, OR_PERCENTILE, OR_SIGMA, OR_SIGMEDIAN, OR_WINSORIZED, OR_LINEARFIT };
/* src/stacking/stacking.h:24-30 */
enum { OR_NO_NORM, OR_ADDITIVE, OR_MULTIPLICATIVE, OR_ADDITIVE_SCALING, OR_MULTIPLICATIVE_SCALING };

typedef struct {
	int N, W, H, C;
	const uint16_t *frames;	/* [N][C][H][W] */
} or_seq;

typedef struct {
	long channel, start_row, end_row, height;
} or_block;

/* --- core helpers (src/core/utils.c) --- */
uint16_t or_round_to_WORD(double x);
void or_quicksort_s(uint16_t *a, int n);

/* --- GSL restatements --- */
double or_gsl_mean_u16(const uint16_t *data, size_t n);
double or_gsl_sd_u16(const uint16_t *data, size_t n);
double or_gsl_median_from_sorted_u16(const uint16_t *sorted, size_t n);
void or_gsl_fit_linear(const double *x, const double *y, size_t n, double *c0, double *c1);

/* --- stacking (src/stacking/stacking.c) --- */
/* block partition, stacking.c:1397-1476; returns number of blocks or <0 if the
 * reference would index uninitialised blocks (UB) */
int or_make_blocks(long H, int nb_channels, int max_number_of_rows, int nb_threads,
		or_block *blocks, int max_blocks);
/* libgomp schedule(static) chunk of thread t among nthr for n iterations */
void or_omp_static_chunk(long n, int nthr, int t, long *begin, long *end);

int or_stack_mean_with_rejection(const or_seq *seq, int rejection, int normalize,
		const double sig[2], const int *shiftx, const int *shifty,
		const double *offset, const double *mul, const double *scale,
		int max_thread, int max_number_of_rows, uint16_t *out, uint64_t rej[3][2]);
int or_stack_mean_with_rejection_rows(const or_seq *seq, int rejection, int normalize,
		const double sig[2], const int *shiftx, const int *shifty,
		const double *offset, const double *mul, const double *scale,
		int max_thread, int max_number_of_rows, uint16_t *out, uint64_t rej[3][2], uint64_t *row_rej);
int or_stack_median(const or_seq *seq, int normalize, const double *offset,
		const double *mul, const double *scale, int max_thread,
		int max_number_of_rows, uint16_t *out);
int or_stack_summing(const or_seq *seq, const int *shiftx, const int *shifty,
		uint16_t *out, uint64_t *maxim);
int or_stack_addmax(const or_seq *seq, const int *shiftx, const int *shifty, uint16_t *out);
int or_stack_addmin(const or_seq *seq, const int *shiftx, const int *shifty, uint16_t *out);

/* normalisation coefficients from per-frame (location, scale), stacking.c:79-190 */
/* statistics(fit, 0, NULL, STATS_IKSS, STATS_ZERO_NULLCHECK) -> location / scale
 * (src/algos/statistics.c:152-326), or_statistics.c */
int or_statistics_ikss(const uint16_t *frame, int C, int H, int W, double *location, double *scale);
int or_compute_normalization(int nb, int ref_image, int mode, const double *location,
		const double *scalev, double *offset, double *mul, double *scale);

/* --- registration (src/registration/registration.c:182-400) --- */
/* sel: [nframes][S][S] u16 selections (bottom-up, already extracted); quality in/out */
int or_register_shift_dft(const uint16_t *sel, int nframes, int S, int ref_image,
		const int *included, int *shiftx, int *shifty, double *quality);
/* src/algos/quality.c:46-218 on a W x H u16 plane */
double or_quality_estimate(const uint16_t *buffer, int width, int height);
/* 2-D unnormalised complex DFT in double, sign -1 forward (FFTW_FORWARD) / +1 backward */
void or_dft2d(double *re, double *im, int S, int sign);
/* exact circular cross-correlation sum_n ref(n + k) img(n) at shift k = (ky, kx) (int64) */
long long or_xcorr_at(const uint16_t *ref, const uint16_t *img, int S, int ky, int kx);

void or_synth_window(uint16_t *out, int nframes, int c, int y0, int x0, int h, int w, uint64_t seed,
		int maxshift);

#ifdef __cplusplus
}
#endif
#endif
