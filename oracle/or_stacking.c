/*
 * or_stacking.c - CPU restatement of Siril 0.9's stackers (TEST INFRASTRUCTURE ONLY;
 * see oracle.h: parity unpinned, checked against tests/oracle_numpy.py + tests/golden/).
 *
 * Follows src/stacking/stacking.c line for line:
 *   stack_summing              :196-355
 *   stack_median               :362-816
 *   stack_addmax / addmin      :824-1128
 *   rejection helpers          :1130-1187
 *   stack_mean_with_rejection  :1189-1858
 *   block partition            :1397-1476 (identical in median :570-646)
 *   normalisation              :79-190
 * The OpenMP region `omp parallel for num_threads(com.max_thread) schedule(static)`
 * (:1513-1516) is emulated explicitly: emulated thread t owns the libgomp static chunk
 * of blocks and its own _data_block (stack, rejected[] calloc'ed at :1497), so the
 * reference's cross-pixel stale-rejected[] state (SURVEY.md §8a a3 quirk iii) is
 * reproduced deterministically.  Emulated threads run in parallel with real OpenMP.
 *
 * Frame regions are read through or_read_region(), the restatement of
 * seq_opened_read_region (src/io/sequence.c:690-700) for SER/FITS: a top-down band.
 */
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle.h"

/* seq_opened_read_region: band rows y..y+h-1 counted top-down; memory is bottom-up
 * (read_opened_fits_partial :581-635 reads rows ry-y-h+1..ry-y then reverses them;
 * ser_read_opened_partial reads the top-down file rows directly, src/io/ser.c:772-818) */
static int or_read_region(const or_seq *seq, int layer, int index, uint16_t *buffer,
		int ax, int ay, int aw, int ah) {
	if (ax < 0 || ay < 0 || ax >= seq->W || ay >= seq->H || aw <= 0 || ah <= 0 ||
			ax + aw > seq->W || ay + ah > seq->H)
		return 1;	/* FITS reader returns 1, callers ignore it (stacking.c:1583) */
	const uint16_t *plane = seq->frames + ((size_t)index * seq->C + layer) * (size_t)seq->W * seq->H;
	for (int t = 0; t < ah; t++) {
		long memrow = seq->H - 1 - (ay + t);
		memcpy(buffer + (size_t)t * aw, plane + (size_t)memrow * seq->W + ax, aw * sizeof(uint16_t));
	}
	return 0;
}

void or_omp_static_chunk(long n, int nthr, int t, long *begin, long *end) {
	long q = n / nthr, r = n % nthr;
	if (t < r) {
		q++;
		*begin = q * t;
	} else {
		*begin = q * t + r;
	}
	*end = *begin + q;
}

int or_make_blocks(long H, int nb_channels, int max_number_of_rows, int nb_threads,
		or_block *blocks, int max_blocks) {
	long naxes1 = H;
	int size_of_stacks = max_number_of_rows / nb_threads;
	if (size_of_stacks == 0)
		size_of_stacks = 1;
	long nb_parallel_stacks;
	int remainder;
	if (naxes1 / size_of_stacks < 4) {
		nb_parallel_stacks = 4 * nb_channels;
		size_of_stacks = naxes1 / 4;
		remainder = naxes1 % 4;
	} else {
		nb_parallel_stacks = naxes1 * nb_channels / size_of_stacks;
		if (nb_parallel_stacks % nb_channels != 0
				|| (naxes1 * nb_channels) % size_of_stacks != 0) {
			nb_parallel_stacks += nb_channels - (nb_parallel_stacks % nb_channels);
			size_of_stacks = naxes1 * nb_channels / nb_parallel_stacks;
		}
		remainder = naxes1 - (nb_parallel_stacks / nb_channels * size_of_stacks);
	}
	if (size_of_stacks <= 0 || nb_parallel_stacks > max_blocks)
		return -1;
	long channel = 0, row = 0, end, j = 0;
	do {
		if (j >= nb_parallel_stacks)
			return -1;
		blocks[j].channel = channel;
		blocks[j].start_row = row;
		end = row + size_of_stacks - 1;
		if (remainder > 0) {
			end++;
			remainder--;
		}
		if (end >= naxes1 - 1 || (naxes1 - end < size_of_stacks / 10)) {
			end = naxes1 - 1;
			row = 0;
			channel++;
			remainder = naxes1 - (nb_parallel_stacks / nb_channels * size_of_stacks);
		} else {
			row = end + 1;
		}
		blocks[j].end_row = end;
		blocks[j].height = blocks[j].end_row - blocks[j].start_row + 1;
		j++;
	} while (channel < nb_channels);
	/* the OpenMP loop runs over nb_parallel_stacks entries (:1516): fewer initialised
	 * blocks would make the reference read uninitialised memory */
	if (j != nb_parallel_stacks)
		return -1;
	return (int)j;
}

static int percentile_clipping(uint16_t pixel, const double sig[], double median, uint64_t rej[]) {
	double plow = sig[0];
	double phigh = sig[1];
	if ((median - (double)pixel) / median > plow) {
		rej[0]++;
		return -1;
	} else if (((double)pixel - median) / median > phigh) {
		rej[1]++;
		return 1;
	} else
		return 0;
}

static int sigma_clipping(uint16_t pixel, const double sig[], double sigma, double median, uint64_t rej[]) {
	double sigmalow = sig[0];
	double sigmahigh = sig[1];
	if (median - (double)pixel > sigmalow * sigma) {
		rej[0]++;
		return -1;
	} else if ((double)pixel - median > sigmahigh * sigma) {
		rej[1]++;
		return 1;
	} else
		return 0;
}

static int or_is_sorted_u16(const uint16_t *a, int n) {
	for (int i = 1; i < n; i++)
		if (a[i] < a[i - 1])
			return 0;
	return 1;
}

/* quicksort_s (src/core/utils.c:512-533) where the reference calls it inside a rejection loop:
 * from the second pass on the stack is already sorted (removal keeps the order, clamping keeps it
 * sorted), and sorting a sorted array is the identity, so the sort runs only when an element is
 * out of order: the same array either way, a test-time saving only */
static void or_sort_stack(uint16_t *a, int n) {
	if (!or_is_sorted_u16(a, n))
		or_quicksort_s(a, n);
}

static void winsorize(uint16_t *pixel, double m0, double m1) {
	if (*pixel < m0)
		*pixel = or_round_to_WORD(m0);
	else if (*pixel > m1)
		*pixel = or_round_to_WORD(m1);
}

static int line_clipping(uint16_t pixel, const double sig[], double sigma, int i, double a,
		double b, uint64_t rej[]) {
	double sigmalow = sig[0];
	double sigmahigh = sig[1];
	if (((a * (double)i + b - (double)pixel) / sigma) > sigmalow) {
		rej[0]++;
		return -1;
	} else if ((((double)pixel - a * (double)i - b) / sigma) > sigmahigh) {
		rej[1]++;
		return 1;
	} else
		return 0;
}

static void remove_pixel(uint16_t *arr, int i, int N) {
	memmove(&arr[i], &arr[i + 1], (N - i - 1) * sizeof(*arr));
}

/* the per-pixel rejection + mean of stacking.c:1656-1794, on data->stack / data->rejected */
static uint16_t reject_and_mean(uint16_t *stack, int *rejected, int nb_frames, int type,
		const double sig[2], uint64_t crej[2]) {
	int N = nb_frames;
	double median, sigma = -1.0;
	int n, j, r = 0, frame;
	switch (type) {
	case OR_PERCENTILE:
		or_sort_stack(stack, N);
		median = or_gsl_median_from_sorted_u16(stack, N);
		for (frame = 0; frame < N; frame++)
			rejected[frame] = percentile_clipping(stack[frame], sig, median, crej);
		for (frame = 0, j = 0; frame < N; frame++, j++) {
			if (rejected[j] != 0 && N > 1) {
				remove_pixel(stack, frame, N);
				frame--;
				N--;
			}
		}
		break;
	case OR_SIGMA:
		do {
			sigma = or_gsl_sd_u16(stack, N);
			or_sort_stack(stack, N);
			median = or_gsl_median_from_sorted_u16(stack, N);
			n = 0;
			for (frame = 0; frame < N; frame++) {
				rejected[frame] = sigma_clipping(stack[frame], sig, sigma, median, crej);
				if (rejected[frame])
					r++;
				if (N - r <= 4)
					break;
			}
			for (frame = 0, j = 0; frame < N - n; frame++, j++) {
				if (rejected[j] != 0) {
					remove_pixel(stack, frame, N - n);
					n++;
					frame--;
				}
			}
			N = N - n;
		} while (n > 0 && N > 3);
		break;
	case OR_SIGMEDIAN:
		do {
			sigma = or_gsl_sd_u16(stack, N);
			or_sort_stack(stack, N);
			median = or_gsl_median_from_sorted_u16(stack, N);
			n = 0;
			for (frame = 0; frame < N; frame++) {
				if (sigma_clipping(stack[frame], sig, sigma, median, crej)) {
					stack[frame] = or_round_to_WORD(median);
					n++;
				}
			}
		} while (n > 0 && N > 3);
		break;
	case OR_WINSORIZED:
		do {
			double sigma0;
			sigma = or_gsl_sd_u16(stack, N);
			or_sort_stack(stack, N);
			median = or_gsl_median_from_sorted_u16(stack, N);
			uint16_t *w_stack = malloc(N * sizeof(uint16_t));
			memcpy(w_stack, stack, N * sizeof(uint16_t));
			do {
				int jj;
				double m0 = median - 1.5 * sigma;
				double m1 = median + 1.5 * sigma;
				for (jj = 0; jj < N; jj++)
					winsorize(&w_stack[jj], m0, m1);
				or_sort_stack(w_stack, N);	/* :1722 */
				median = or_gsl_median_from_sorted_u16(w_stack, N);
				sigma0 = sigma;
				sigma = 1.134 * or_gsl_sd_u16(w_stack, N);
			} while ((fabs(sigma - sigma0) / sigma0) > 0.0005);
			free(w_stack);
			n = 0;
			for (frame = 0; frame < N; frame++) {
				rejected[frame] = sigma_clipping(stack[frame], sig, sigma, median, crej);
				if (rejected[frame] != 0)
					r++;
				if (N - r <= 4)
					break;
			}
			for (frame = 0, j = 0; frame < N - n; frame++, j++) {
				if (rejected[j] != 0) {
					remove_pixel(stack, frame, N - n);
					frame--;
					n++;
				}
			}
			N = N - n;
		} while (n > 0 && N > 3);
		break;
	case OR_LINEARFIT:
		do {
			double *xf = malloc(N * sizeof(double));
			double *yf = malloc(N * sizeof(double));
			double a, b;
			or_sort_stack(stack, N);
			for (frame = 0; frame < N; frame++) {
				xf[frame] = (double)frame;
				yf[frame] = (double)stack[frame];
			}
			/* gsl_fit_linear(xf, 1, yf, 1, N, &b, &a, ...): b = intercept, a = slope */
			or_gsl_fit_linear(xf, yf, N, &b, &a);
			sigma = 0.0;
			for (frame = 0; frame < N; frame++)
				sigma += (fabs((double)stack[frame] - (a * (double)frame + b)));
			sigma /= (double)N;
			n = 0;
			for (frame = 0; frame < N; frame++) {
				rejected[frame] = line_clipping(stack[frame], sig, sigma, frame, a, b, crej);
				if (rejected[frame] != 0)
					r++;
				if (N - r <= 4)
					break;
			}
			for (frame = 0, j = 0; frame < N - n; frame++, j++) {
				if (rejected[j] != 0) {
					remove_pixel(stack, frame, N - n);
					frame--;
					n++;
				}
			}
			N = N - n;
			free(xf);
			free(yf);
		} while (n > 0 && N > 3);
		break;
	default:
	case OR_NO_REJEC:
		;
	}
	double sum = 0.0;
	for (frame = 0; frame < N; ++frame)
		sum += stack[frame];
	return or_round_to_WORD(sum / (double)N);
}

static uint16_t normalize_value(uint16_t pix, int normalize, double offset, double mul, double scale) {
	double tmp;
	switch (normalize) {
	default:
	case OR_NO_NORM:
		return pix;
	case OR_ADDITIVE:
	case OR_ADDITIVE_SCALING:
		tmp = (double)pix * scale;
		return or_round_to_WORD(tmp - offset);
	case OR_MULTIPLICATIVE:
	case OR_MULTIPLICATIVE_SCALING:
		tmp = (double)pix * scale;
		return or_round_to_WORD(tmp * mul);
	}
}

int or_stack_mean_with_rejection(const or_seq *seq, int rejection, int normalize,
		const double sig[2], const int *shiftx, const int *shifty,
		const double *offset, const double *mul, const double *scale,
		int max_thread, int max_number_of_rows, uint16_t *out, uint64_t rej[3][2]) {
	return or_stack_mean_with_rejection_rows(seq, rejection, normalize, sig, shiftx, shifty, offset, mul, scale,
			max_thread, max_number_of_rows, out, rej, NULL);
}

/* the same, also returning each memory row's low / high rejection counts (row_rej[(c H + r) 2 + k],
 * test infrastructure: a row band's counters are the sum over its rows) */
int or_stack_mean_with_rejection_rows(const or_seq *seq, int rejection, int normalize,
		const double sig[2], const int *shiftx, const int *shifty,
		const double *offset, const double *mul, const double *scale,
		int max_thread, int max_number_of_rows, uint16_t *out, uint64_t rej[3][2], uint64_t *row_rej) {
	const int nb_frames = seq->N;
	const long W = seq->W, H = seq->H;
	const int nb_channels = seq->C;
	if (nb_frames < 2)
		return -1;	/* :1217-1220 */
	if (max_thread < 1)
		max_thread = 1;
	or_block *blocks = malloc(sizeof(or_block) * (4 * 3 + H * 3 + 16));
	int nblocks = or_make_blocks(H, nb_channels, max_number_of_rows, max_thread, blocks,
			(int)(4 * 3 + H * 3 + 16));
	if (nblocks < 0) {
		free(blocks);
		return -1;
	}
	long largest_block_height = 0;
	for (int i = 0; i < nblocks; i++)
		if (largest_block_height < blocks[i].height)
			largest_block_height = blocks[i].height;
	const long npixels_in_block = largest_block_height * W;
	for (int c = 0; c < 3; c++)
		rej[c][0] = rej[c][1] = 0;
	int retval = 0;
	uint64_t (*trej)[3][2] = calloc(max_thread, sizeof(*trej));

#pragma omp parallel for schedule(static, 1)
	for (int t = 0; t < max_thread; t++) {
		long b0, b1;
		or_omp_static_chunk(nblocks, max_thread, t, &b0, &b1);
		if (b0 >= b1)
			continue;
		/* per-thread _data_block, :1491-1507 */
		uint16_t *tmp = malloc((size_t)nb_frames * npixels_in_block * sizeof(uint16_t));
		uint16_t *stack = malloc(nb_frames * sizeof(uint16_t));
		int *rejected = calloc(nb_frames, sizeof(int));
		for (long i = b0; i < b1; i++) {
			or_block *my_block = blocks + i;
			for (int frame = 0; frame < nb_frames; ++frame) {
				int sy = 0, clear = 0, readdata = 1;
				long off = 0;
				int ax = 0, ay = (int)my_block->start_row, aw = (int)W, ah = (int)my_block->height;
				uint16_t *pixf = tmp + (size_t)frame * npixels_in_block;
				if (shifty) {	/* :1550-1570 */
					sy = shifty[frame];
					if (ay + ah - 1 + sy < 0 || ay + sy >= H) {
						clear = 1;
						readdata = 0;
					} else if (ay + sy < 0) {
						clear = 1;
						ah += ay + sy;
						off = W * (ay - sy);
						ay = 0;
						/* reference heap overflow when start_row > 0 */
						if (off + (long)ah * W > npixels_in_block) {
							retval = -4;
							readdata = 0;
						}
					} else if (ay + ah - 1 + sy >= H) {
						clear = 1;
						ay += sy;
						ah += (int)(H - (ay + ah));
					} else {
						ay += sy;
					}
				}
				if (clear)
					memset(pixf, 0, npixels_in_block * sizeof(uint16_t));
				if (readdata)
					or_read_region(seq, (int)my_block->channel, frame, pixf + off, ax, ay, aw, ah);
			}
			for (long y = 0; y < my_block->height; y++) {
				long pdata_idx = (H - (my_block->start_row + y) - 1) * W;
				long pix_idx = y * W;
				uint64_t crej[2] = {0, 0};
				uint16_t *outp = out + (size_t)my_block->channel * W * H;
				for (long x = 0; x < W; ++x) {
					for (int frame = 0; frame < nb_frames; ++frame) {
						int sx = shiftx ? shiftx[frame] : 0;
						if (sx && (x - sx >= W || x - sx < 0)) {
							stack[frame] = 0;
						} else {
							uint16_t pix = tmp[(size_t)frame * npixels_in_block + pix_idx + x - sx];
							stack[frame] = normalize_value(pix, normalize,
									offset ? offset[frame] : 0.0,
									mul ? mul[frame] : 1.0,
									scale ? scale[frame] : 1.0);
						}
					}
					outp[pdata_idx++] = reject_and_mean(stack, rejected, nb_frames,
							rejection, sig, crej);
				}
				trej[t][my_block->channel][0] += crej[0];
				trej[t][my_block->channel][1] += crej[1];
				if (row_rej) {
					uint64_t *rr = row_rej + ((size_t)my_block->channel * H + (H - (my_block->start_row + y) - 1)) * 2;
					rr[0] = crej[0];
					rr[1] = crej[1];
				}
			}
		}
		free(tmp);
		free(stack);
		free(rejected);
	}
	for (int t = 0; t < max_thread; t++)
		for (int c = 0; c < 3; c++) {
			rej[c][0] += trej[t][c][0];
			rej[c][1] += trej[t][c][1];
		}
	free(trej);
	free(blocks);
	return retval;
}

int or_stack_median(const or_seq *seq, int normalize, const double *offset,
		const double *mul, const double *scale, int max_thread,
		int max_number_of_rows, uint16_t *out) {
	const int nb_frames = seq->N;
	const long W = seq->W, H = seq->H;
	if (nb_frames < 2)
		return -1;	/* :390-393 */
	if (max_thread < 1)
		max_thread = 1;
	or_block *blocks = malloc(sizeof(or_block) * (4 * 3 + H * 3 + 16));
	int nblocks = or_make_blocks(H, seq->C, max_number_of_rows, max_thread, blocks,
			(int)(4 * 3 + H * 3 + 16));
	if (nblocks < 0) {
		free(blocks);
		return -1;
	}
	long largest = 0;
	for (int i = 0; i < nblocks; i++)
		if (largest < blocks[i].height)
			largest = blocks[i].height;
	const long npix = largest * W;
#pragma omp parallel for schedule(static, 1)
	for (int t = 0; t < max_thread; t++) {
		long b0, b1;
		or_omp_static_chunk(nblocks, max_thread, t, &b0, &b1);
		if (b0 >= b1)
			continue;
		uint16_t *tmp = calloc((size_t)nb_frames * npix, sizeof(uint16_t));
		uint16_t *stack = calloc(nb_frames, sizeof(uint16_t));
		for (long i = b0; i < b1; i++) {
			or_block *b = blocks + i;
			/* :703-722: no registration shifts in the median stacker */
			for (int frame = 0; frame < nb_frames; ++frame)
				or_read_region(seq, (int)b->channel, frame, tmp + (size_t)frame * npix, 0,
						(int)b->start_row, (int)W, (int)b->height);
			for (long y = 0; y < b->height; y++) {
				long pixel_idx = (H - (b->start_row + y) - 1) * W;
				uint16_t *outp = out + (size_t)b->channel * W * H;
				for (long x = 0; x < W; ++x) {
					for (int ii = 0; ii < nb_frames; ++ii) {
						double sc = scale ? scale[ii] : 1.0;
						double tmpv = (double)tmp[(size_t)ii * npix + y * W + x] * sc;
						switch (normalize) {
						default:
						case OR_NO_NORM:
						case OR_ADDITIVE:
						case OR_ADDITIVE_SCALING:
							stack[ii] = or_round_to_WORD(tmpv - (offset ? offset[ii] : 0.0));
							break;
						case OR_MULTIPLICATIVE:
						case OR_MULTIPLICATIVE_SCALING:
							stack[ii] = or_round_to_WORD(tmpv * (mul ? mul[ii] : 1.0));
							break;
						}
					}
					or_quicksort_s(stack, nb_frames);
					/* implicit double -> WORD truncation, :766-767 */
					outp[pixel_idx] = (uint16_t)or_gsl_median_from_sorted_u16(stack, nb_frames);
					pixel_idx++;
				}
			}
		}
		free(tmp);
		free(stack);
	}
	free(blocks);
	return 0;
}

/* stack_summing :196-355 (single-threaded in the reference) */
int or_stack_summing(const or_seq *seq, const int *shiftx, const int *shifty,
		uint16_t *out, uint64_t *maxim_out) {
	const int nb = seq->N, C = seq->C;
	const long rx = seq->W, ry = seq->H, nbdata = rx * ry;
	if (nb <= 1)
		return -1;
	unsigned long *somme = calloc((size_t)nbdata * C, sizeof(unsigned long));
	unsigned long maxim = 0;
	for (int j = 0; j < nb; ++j) {
		int sx = shiftx ? shiftx[j] : 0, sy = shifty ? shifty[j] : 0;
		const uint16_t *frame = seq->frames + (size_t)j * C * nbdata;
		long i = 0;
		for (long y = 0; y < ry; ++y) {
			for (long x = 0; x < rx; ++x) {
				long nx = x - sx, ny = y - sy;
				if (nx >= 0 && nx < rx && ny >= 0 && ny < ry) {
					long ii = ny * rx + nx;
					if (ii > 0 && ii < rx * ry) {	/* pixel 0 never summed */
						for (int layer = 0; layer < C; ++layer) {
							uint16_t cur = frame[(size_t)layer * nbdata + ii];
							somme[(size_t)layer * nbdata + i] += cur;
							if (somme[(size_t)layer * nbdata + i] > maxim)
								maxim = somme[(size_t)layer * nbdata + i];
						}
					}
				}
				++i;
			}
		}
	}
	double ratio = (maxim > 65535) ? 65535.0 / (double)maxim : 1.0;
	for (long k = 0; k < nbdata * C; k++) {
		if (ratio == 1.0)
			out[k] = or_round_to_WORD((double)somme[k]);
		else
			out[k] = or_round_to_WORD((double)somme[k] * ratio);
	}
	if (maxim_out)
		*maxim_out = maxim;
	free(somme);
	return 0;
}

static int or_stack_addmaxmin(const or_seq *seq, const int *shiftx, const int *shifty,
		uint16_t *out, int is_max) {
	const int nb = seq->N, C = seq->C;
	const long rx = seq->W, ry = seq->H, nbdata = rx * ry;
	if (nb <= 1)
		return -1;
	for (long k = 0; k < nbdata * C; k++)
		out[k] = is_max ? 0 : 65535;	/* calloc :882 / memset(USHRT_MAX) :1038 */
	for (int j = 0; j < nb; ++j) {
		int sx = shiftx ? shiftx[j] : 0, sy = shifty ? shifty[j] : 0;
		const uint16_t *frame = seq->frames + (size_t)j * C * nbdata;
		long i = 0;
		for (long y = 0; y < ry; ++y) {
			for (long x = 0; x < rx; ++x) {
				long nx = x - sx, ny = y - sy;
				if (nx >= 0 && nx < rx && ny >= 0 && ny < ry) {
					long ii = ny * rx + nx;
					if (ii > 0 && ii < rx * ry) {
						for (int layer = 0; layer < C; ++layer) {
							uint16_t cur = frame[(size_t)layer * nbdata + ii];
							uint16_t *fp = &out[(size_t)layer * nbdata + i];
							if (is_max ? (cur > *fp) : (cur < *fp))
								*fp = cur;
						}
					}
				}
				++i;
			}
		}
	}
	return 0;
}

int or_stack_addmax(const or_seq *seq, const int *shiftx, const int *shifty, uint16_t *out) {
	return or_stack_addmaxmin(seq, shiftx, shifty, out, 1);
}

int or_stack_addmin(const or_seq *seq, const int *shiftx, const int *shifty, uint16_t *out) {
	return or_stack_addmaxmin(seq, shiftx, shifty, out, 0);
}

/* compute_normalization + _compute_normalization_for_image, :79-190, from cached
 * stats (location, scale) of layer 0 of every frame */
int or_compute_normalization(int nb, int ref_image, int mode, const double *location,
		const double *scalev, double *offset, double *mul, double *scale) {
	double scale0 = 0.0, mul0 = 0.0, offset0 = 0.0;
	for (int i = 0; i < nb; i++) {
		offset[i] = 0.0;
		mul[i] = 1.0;
		scale[i] = 1.0;
	}
	if (mode == OR_NO_NORM)
		return 0;
	/* reference frame first, then the others (the order only matters for *0) */
	for (int pass = 0; pass < 2; pass++) {
		for (int i = 0; i < nb; i++) {
			if ((pass == 0) != (i == ref_image))
				continue;
			switch (mode) {
			default:
			case OR_ADDITIVE_SCALING:
				scale[i] = scalev[i];
				if (i == ref_image)
					scale0 = scale[ref_image];
				scale[i] = scale0 / scale[i];
				/* fall through */
			case OR_ADDITIVE:
				offset[i] = location[i];
				if (i == ref_image)
					offset0 = offset[ref_image];
				offset[i] = scale[i] * offset[i] - offset0;
				break;
			case OR_MULTIPLICATIVE_SCALING:
				scale[i] = scalev[i];
				if (i == ref_image)
					scale0 = scale[ref_image];
				scale[i] = scale0 / scale[i];
				/* fall through */
			case OR_MULTIPLICATIVE:
				mul[i] = location[i];
				if (i == ref_image)
					mul0 = mul[ref_image];
				mul[i] = mul0 / mul[i];
				break;
			}
		}
	}
	return 0;
}
