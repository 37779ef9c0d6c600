/*
 * sg_synth.h - deterministic synthetic frame generator (SURVEY.md §8d "Synthetic inputs").
 *
 * Integer-only so the host C build and the gfx950 HIP build produce bit-identical
 * frames: tests generate the same sequence on the CPU (for the oracle) and on the
 * GPU (for the product path and bench.py, so 16 GiB never crosses PCIe).
 *
 * Scene (memory order = Siril's bottom-up FITS order, src/core/siril.h:391-442):
 *   background 1000 + 400*c, Irwin-Hall(4) noise scaled to sigma ~= 30 ADU,
 *   one Gaussian star (sigma 1.5 px, peak 5000..40000) in ~78 % of 256x256 cells,
 *   outliers: 0.05 % pixels = 65535 (cosmics), 0.01 % = 0 (dead).
 * Frame f shows the scene translated by (dx_f, dy_f) in [-maxshift, maxshift]^2,
 * frame 0 untranslated; so frame_f[y][x] = scene[y - dy_f][x - dx_f] and the
 * registration shifts that re-align it are (shiftx, shifty) = (-dx_f, -dy_f)
 * (stacking reads frame_f[y - shifty][x - shiftx], src/stacking/stacking.c:299-305).
 */
#ifndef SG_SYNTH_H
#define SG_SYNTH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SG_HD __host__ __device__ static inline
#else
#define SG_HD static inline
#endif

#define SG_SYNTH_CELL 256
#define SG_SYNTH_BG 1000
#define SG_SYNTH_BG_CH 400

SG_HD uint64_t sg_mix64(uint64_t z) {
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

/* per-frame translation; frame 0 is the reference and never moves */
SG_HD void sg_synth_shift(uint64_t seed, int f, int maxshift, int *dx, int *dy) {
	if (f == 0 || maxshift <= 0) {
		*dx = 0;
		*dy = 0;
		return;
	}
	uint64_t h = sg_mix64(seed ^ 0x51B1ull ^ ((uint64_t)(uint32_t)f << 32));
	uint32_t span = (uint32_t)(2 * maxshift + 1);
	*dx = (int)((uint32_t)h % span) - maxshift;
	*dy = (int)((uint32_t)(h >> 32) % span) - maxshift;
}

SG_HD int sg_floordiv(int a, int b) {
	int q = a / b;
	if ((a % b != 0) && ((a < 0) != (b < 0)))
		q--;
	return q;
}

/* star contribution at scene coordinates (xs, ys), integer Gaussian profile */
SG_HD uint32_t sg_synth_star(uint64_t seed, int xs, int ys) {
	/* round(65536*exp(-d^2/4.5)), d = 0..7 (sigma = 1.5 px) */
	const uint32_t prof[8] = {65536u, 52477u, 26943u, 8869u, 1872u, 253u, 22u, 1u};
	int cx = sg_floordiv(xs, SG_SYNTH_CELL);
	int cy = sg_floordiv(ys, SG_SYNTH_CELL);
	uint64_t h = sg_mix64(seed ^ 0xC0FFEEull ^ ((uint64_t)(uint32_t)cx << 20) ^ ((uint64_t)(uint32_t)cy << 42));
	if ((h & 127u) >= 100u)	/* ~78 % of cells hold a star */
		return 0;
	int sx = cx * SG_SYNTH_CELL + 32 + (int)((h >> 8) % 192u);
	int sy = cy * SG_SYNTH_CELL + 32 + (int)((h >> 24) % 192u);
	uint32_t peak = 5000u + (uint32_t)((h >> 40) % 35000u);
	int ddx = xs - sx, ddy = ys - sy;
	if (ddx < 0) ddx = -ddx;
	if (ddy < 0) ddy = -ddy;
	if (ddx > 7 || ddy > 7)
		return 0;
	uint64_t v = (uint64_t)peak * prof[ddx];
	v = (v * prof[ddy]) >> 32;
	return (uint32_t)v;
}

/* value of pixel (x, y) of channel c of frame f (memory coordinates) */
SG_HD uint16_t sg_synth_pixel(uint64_t seed, int f, int c, int y, int x, int maxshift) {
	int dx, dy;
	sg_synth_shift(seed, f, maxshift, &dx, &dy);
	uint64_t key = ((uint64_t)(uint32_t)f << 40) ^ ((uint64_t)(uint32_t)c << 36) ^
		((uint64_t)(uint32_t)y << 18) ^ (uint64_t)(uint32_t)x;
	uint64_t h = sg_mix64(sg_mix64(seed) ^ key);
	uint32_t u = (uint32_t)(h & 0xFFFFFu);
	if (u < 524u)
		return 65535;	/* cosmic */
	if (u < 629u)
		return 0;	/* dead pixel */
	uint64_t h2 = sg_mix64(h);
	int64_t sum = (int64_t)(h2 & 0xFFFF) + (int64_t)((h2 >> 16) & 0xFFFF) +
		(int64_t)((h2 >> 32) & 0xFFFF) + (int64_t)(h2 >> 48);
	int64_t noise = ((sum - 131070) * 30) / 37838;
	int64_t v = SG_SYNTH_BG + SG_SYNTH_BG_CH * c + noise +
		(int64_t)sg_synth_star(seed, x - dx, y - dy);
	if (v < 0) v = 0;
	if (v > 65535) v = 65535;
	return (uint16_t)v;
}

#endif /* SG_SYNTH_H */
