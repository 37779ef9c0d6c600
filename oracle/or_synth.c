/*
 * or_synth.c - CPU fill of the synthetic sequence of include/sg_synth.h (TEST
 * INFRASTRUCTURE ONLY): lets tests and bench.py's cpu_baseline build the exact
 * frames the GPU generator writes into HBM.
 */
#include <stdint.h>
#include <stddef.h>
#include "../include/sg_synth.h"

void or_synth_fill(uint16_t *frames, int nframes, int C, int H, int W, int row_begin,
		int row_end, uint64_t seed, int maxshift) {
#pragma omp parallel for schedule(static)
	for (int f = 0; f < nframes; f++)
		for (int c = 0; c < C; c++)
			for (int R = row_begin; R < row_end; R++)
				for (int x = 0; x < W; x++)
					frames[(((size_t)f * C + c) * H + R) * W + x] =
						sg_synth_pixel(seed, f, c, R, x, maxshift);
}

void or_synth_shift(uint64_t seed, int f, int maxshift, int *dx, int *dy) {
	sg_synth_shift(seed, f, maxshift, dx, dy);
}

/* one channel's window [y0, y0+h) x [x0, x0+w) of every frame: out[f][r][x] (the registration
 * selection of a sequence too large to generate whole, e.g. configs[4]'s 256 x 3 x 4000 x 6000) */
void or_synth_window(uint16_t *out, int nframes, int c, int y0, int x0, int h, int w, uint64_t seed,
		int maxshift) {
#pragma omp parallel for schedule(static)
	for (int f = 0; f < nframes; f++)
		for (int r = 0; r < h; r++)
			for (int x = 0; x < w; x++)
				out[((size_t)f * h + r) * w + x] = sg_synth_pixel(seed, f, c, y0 + r, x0 + x, maxshift);
}
