/*
 * sg_repadd.h - acc + t + t + ... (k additions, each rounded to nearest-even in double),
 * exactly as the sequential loop computes it, in O(number of binades crossed) steps.
 *
 * Why: the reference sums per-sample terms sequentially over SORTED data
 * (siril_stats_double_bwmv, src/algos/statistics.c:128-150, called by IKSS :152-187), so a
 * run of c equal samples adds the same term c times.  Within one binade of the running sum
 * (all values multiples of the same ulp u) the rounded increment is constant: round(t/u)
 * u when t/u is not a half-integer; for a half-integer the first step lands on an even
 * multiple of u and every later step adds the even neighbour of t/u.  So two equal
 * consecutive increments are followed by the same increment until a sum would leave the
 * binade (kept one ulp away from the boundary, where the unit changes); there one step is
 * done literally.  Checked against the literal loop by the CPU test suite (tests/).
 */
#ifndef SG_REPADD_H
#define SG_REPADD_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define SG_RA_HD __host__ __device__ static inline
#else
#define SG_RA_HD static inline
#endif

SG_RA_HD int sg_ra_exp(double x) {	/* binade exponent e: 2^e <= |x| < 2^(e+1), normal x */
	uint64_t b;
	__builtin_memcpy(&b, &x, 8);
	return (int)((b >> 52) & 0x7FF) - 1023;
}

SG_RA_HD double sg_add_repeat(double acc, double t, uint64_t k) {
	while (k > 0) {
		if (t == 0.0)
			return acc + t;	/* adding +-0 again changes nothing after the first time */
		const double a1 = acc + t;
		k--;
		if (a1 == acc)
			return acc;	/* |t| below half an ulp of acc: the sum never moves again */
		if (k == 0)
			return a1;
		const double a2 = a1 + t;
		k--;
		if (k == 0)
			return a2;
		/* steady increment d within the binade of a1 / a2 (same sign, both normal) */
		const uint64_t min_normal = 0x0010000000000000ull;
		uint64_t b1, b2;
		__builtin_memcpy(&b1, &a1, 8);
		__builtin_memcpy(&b2, &a2, 8);
		const int ok = a1 != 0.0 && a2 != 0.0 && ((b1 ^ b2) >> 52) == 0 &&	/* same sign and exponent */
				(b2 & 0x7FFFFFFFFFFFFFFFull) >= min_normal;
		const double d1 = a1 - acc, d2 = a2 - a1;
		if (!ok || d1 != d2) {
			acc = a2;
			continue;
		}
		/* integer units of u = ulp(a2): A = |a2| / u in [2^52, 2^53), D = |d2| / u */
		const int e = sg_ra_exp(a2);
		const double u = ldexp(1.0, e - 52);
		const uint64_t A = (uint64_t)(fabs(a2) / u);
		const double dd = fabs(d2) / u;
		if (!(dd >= 1.0) || dd > 9007199254740992.0) {
			acc = a2;
			continue;
		}
		const uint64_t D = (uint64_t)dd;
		const int away = (a2 > 0.0) == (d2 > 0.0);	/* |sum| grows */
		uint64_t s;
		if (away)	/* stay <= 2^53 - 2 units: the exact sum then stays below 2^(e+1) */
			s = (((1ull << 53) - 2) >= A) ? (((1ull << 53) - 2) - A) / D : 0;
		else		/* stay >= 2^52 + 1 units */
			s = (A >= (1ull << 52) + 1) ? (A - ((1ull << 52) + 1)) / D : 0;
		if (s > k)
			s = k;
		acc = a2 + (double)s * d2;
		k -= s;
	}
	return acc;
}

#endif /* SG_REPADD_H */
