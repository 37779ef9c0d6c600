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
