/*
 * sg_f80.h - software x87 80-bit extended arithmetic (64-bit mantissa, round to nearest
 * even), host + gfx950 device.
 *
 * Why: Siril's rejection stackers call gsl_stats_ushort_sd (src/stacking/stacking.c:1676,
 * 1698,1713,1727), whose running mean/variance recurrences are long double, i.e. x87
 * extended on x86-64.  The GPU fast path decides with exact integer moments and hands
 * every pixel whose decision lies within a rounding band of a threshold to the literal
 * slow path, which replays GSL's recurrences through this type so its sigma is
 * bit-identical to the reference's.  Only normal numbers and zero are needed (inputs
 * are u16 samples, counts and their squares).  Checked against native long double by
 * tests/test_f80.py.
 */
#ifndef SG_F80_H
#define SG_F80_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define F80_HD __host__ __device__ static inline
#else
#define F80_HD static inline
#endif

typedef struct {
	uint64_t m;	/* normalised mantissa (bit 63 set) or 0 for zero */
	int32_t e;	/* value = (-1)^s * m * 2^(e - 63) */
	int32_t s;
} sg_f80;

F80_HD int f80_clz64(uint64_t x) {
#if defined(__HIPCC__) || defined(__GNUC__)
	return x ? __builtin_clzll(x) : 64;
#else
	int n = 0;
	if (!x) return 64;
	while (!(x & (1ull << 63))) { x <<= 1; n++; }
	return n;
#endif
}

F80_HD void f80_mul64(uint64_t a, uint64_t b, uint64_t *hi, uint64_t *lo) {
	uint64_t a0 = a & 0xFFFFFFFFull, a1 = a >> 32, b0 = b & 0xFFFFFFFFull, b1 = b >> 32;
	uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
	uint64_t mid = (p00 >> 32) + (p01 & 0xFFFFFFFFull) + (p10 & 0xFFFFFFFFull);
	*lo = (p00 & 0xFFFFFFFFull) | (mid << 32);
	*hi = p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}

F80_HD sg_f80 f80_zero(void) {
	sg_f80 r = {0, 0, 0};
	return r;
}

/* (hi:lo) normalised (hi bit 63 set), value = (hi:lo) * 2^(E - 127); round to 64 bits */
F80_HD sg_f80 f80_round128(uint64_t hi, uint64_t lo, int sticky, int32_t E, int32_t s) {
	uint64_t m = hi;
	int rb = (int)(lo >> 63);
	int st = ((lo << 1) != 0) || sticky;
	if (rb && (st || (m & 1))) {
		m++;
		if (m == 0) {
			m = 1ull << 63;
			E++;
		}
	}
	sg_f80 r = {m, E, s};
	return r;
}

F80_HD sg_f80 f80_from_u64(uint64_t x) {
	if (!x) return f80_zero();
	int sh = f80_clz64(x);
	sg_f80 r = {x << sh, 63 - sh, 0};
	return r;
}

F80_HD sg_f80 f80_from_double(double d) {
	uint64_t bits;
	memcpy(&bits, &d, 8);
	int s = (int)(bits >> 63);
	int ex = (int)((bits >> 52) & 0x7FF);
	uint64_t fr = bits & 0xFFFFFFFFFFFFFull;
	if (ex == 0 && fr == 0) {
		sg_f80 z = {0, 0, s};
		return z;
	}
	if (ex == 0) {	/* subnormal double: normalise */
		int sh = f80_clz64(fr);
		sg_f80 r = {fr << sh, -1074 + 63 - sh, s};
		return r;
	}
	sg_f80 r = {(fr | (1ull << 52)) << 11, ex - 1023, s};
	return r;
}

F80_HD double f80_to_double(sg_f80 a) {
	if (!a.m) return a.s ? -0.0 : 0.0;
	uint64_t keep = a.m >> 11, rem = a.m & 0x7FF;
	int32_t e = a.e;
	if (rem > 0x400 || (rem == 0x400 && (keep & 1))) {
		keep++;
		if (keep == (1ull << 53)) {
			keep >>= 1;
			e++;
		}
	}
	/* normal range only (|e| < 1023 for every value this library sees) */
	uint64_t bits = ((uint64_t)a.s << 63) | ((uint64_t)(e + 1023) << 52) | (keep & 0xFFFFFFFFFFFFFull);
	double d;
	memcpy(&d, &bits, 8);
	return d;
}

F80_HD sg_f80 f80_neg(sg_f80 a) {
	a.s ^= 1;
	return a;
}

F80_HD sg_f80 f80_add(sg_f80 a, sg_f80 b) {
	if (!a.m) return b.m ? b : (a.s && b.s ? a : f80_zero());
	if (!b.m) return a;
	if (b.e > a.e || (b.e == a.e && b.m > a.m)) {
		sg_f80 t = a;
		a = b;
		b = t;
	}
	int32_t d = a.e - b.e;
	uint64_t Ah = a.m, Al = 0, Bh, Bl;
	int sticky = 0;
	if (d == 0) {
		Bh = b.m;
		Bl = 0;
	} else if (d < 64) {
		Bh = b.m >> d;
		Bl = b.m << (64 - d);
	} else if (d < 128) {
		Bh = 0;
		Bl = (d == 64) ? b.m : (b.m >> (d - 64));
		sticky = (d > 64) && ((b.m << (128 - d)) != 0);
	} else {
		Bh = 0;
		Bl = 0;
		sticky = 1;
	}
	if (a.s == b.s) {
		uint64_t lo = Al + Bl;
		uint64_t c = lo < Al;
		uint64_t t = Ah + Bh;
		uint64_t c1 = t < Ah;
		uint64_t hi = t + c;
		uint64_t c2 = hi < t;
		int carry = (int)(c1 | c2);
		if (carry) {
			sticky |= (int)(lo & 1);
			lo = (lo >> 1) | (hi << 63);
			hi = (hi >> 1) | (1ull << 63);
			return f80_round128(hi, lo, sticky, a.e + 1, a.s);
		}
		return f80_round128(hi, lo, sticky, a.e, a.s);
	} else {
		/* |A| >= |B|; a dropped sticky tail of B means the true B is a bit larger */
		uint64_t lo = Al - Bl;
		uint64_t bw = Al < Bl;
		uint64_t hi = Ah - Bh - bw;
		if (sticky) {
			uint64_t b2 = (lo == 0);
			lo -= 1;
			hi -= b2;
		}
		if (!hi && !lo) return f80_zero();
		int32_t E = a.e;
		int sh = hi ? f80_clz64(hi) : 64 + f80_clz64(lo);
		if (sh >= 64) {
			hi = lo << (sh - 64);
			lo = 0;
		} else if (sh > 0) {
			hi = (hi << sh) | (lo >> (64 - sh));
			lo <<= sh;
		}
		return f80_round128(hi, lo, sticky, E - sh, a.s);
	}
}

F80_HD sg_f80 f80_sub(sg_f80 a, sg_f80 b) {
	return f80_add(a, f80_neg(b));
}

F80_HD sg_f80 f80_mul(sg_f80 a, sg_f80 b) {
	if (!a.m || !b.m) return f80_zero();
	uint64_t hi, lo;
	f80_mul64(a.m, b.m, &hi, &lo);
	int32_t E = a.e + b.e + 1;
	if (!(hi >> 63)) {
		hi = (hi << 1) | (lo >> 63);
		lo <<= 1;
		E--;
	}
	return f80_round128(hi, lo, 0, E, a.s ^ b.s);
}

F80_HD sg_f80 f80_div(sg_f80 a, sg_f80 b) {
	if (!a.m) return f80_zero();
	/* Q' = floor(a.m * 2^65 / b.m), 65 or 66 bits, by restoring division */
	uint64_t rem = a.m, q_top = 0, q_lo = 0;
	if (rem >= b.m) {
		rem -= b.m;
		q_lo = 1;
	}
	for (int i = 0; i < 65; i++) {
		uint64_t carry = rem >> 63;
		rem <<= 1;
		uint64_t bit = 0;
		if (carry || rem >= b.m) {
			rem -= b.m;
			bit = 1;
		}
		/* shift (q_top:q_lo) left by one and insert bit */
		q_top = (q_top << 1) | (q_lo >> 63);
		q_lo = (q_lo << 1) | bit;
	}
	int st = rem != 0;
	uint64_t m;
	int rb;
	int32_t E;
	if (q_top & 2) {	/* 66-bit quotient */
		m = (q_top << 62) | (q_lo >> 2);
		rb = (int)((q_lo >> 1) & 1);
		st |= (int)(q_lo & 1);
		E = a.e - b.e;
	} else {		/* 65-bit quotient */
		m = (q_top << 63) | (q_lo >> 1);
		rb = (int)(q_lo & 1);
		E = a.e - b.e - 1;
	}
	if (rb && (st || (m & 1))) {
		m++;
		if (m == 0) {
			m = 1ull << 63;
			E++;
		}
	}
	sg_f80 r = {m, E, a.s ^ b.s};
	return r;
}

/* a / d for an integer 1 <= d < 2^20, rounded exactly as f80_div(a, f80_from_u64(d)).
 * Long division of the 128-bit a.m * 2^64 by d in 32-bit digits: the remainder stays
 * below d, so every partial dividend rem * 2^32 + digit is below 2^52 and exact in a
 * double; the double quotient digit is off by at most one and is corrected from the
 * integer remainder.  Four steps instead of f80_div's 65-step restoring loop. */
F80_HD sg_f80 f80_div_u32(sg_f80 a, uint32_t d) {
	if (!a.m) return f80_zero();
	const uint64_t dg[4] = {a.m >> 32, a.m & 0xFFFFFFFFull, 0, 0};
	uint64_t q[4], rem = 0;
	for (int k = 0; k < 4; k++) {
		const uint64_t x = (rem << 32) | dg[k];
		int64_t qk = (int64_t)((double)x / (double)d);
		int64_t r = (int64_t)x - qk * (int64_t)d;
		if (r < 0) {
			qk--;
			r += d;
		} else if (r >= (int64_t)d) {
			qk++;
			r -= d;
		}
		q[k] = (uint64_t)qk;
		rem = (uint64_t)r;
	}
	uint64_t hi = (q[0] << 32) | q[1], lo = (q[2] << 32) | q[3];
	const int sh = f80_clz64(hi);	/* hi = floor(a.m / d) >= 2^43 */
	if (sh > 0) {
		hi = (hi << sh) | (lo >> (64 - sh));
		lo <<= sh;
	}
	return f80_round128(hi, lo, rem != 0, a.e - sh, a.s);
}

F80_HD sg_f80 f80_div_count(sg_f80 a, uint64_t d) {
	return d < (1u << 20) ? f80_div_u32(a, (uint32_t)d) : f80_div(a, f80_from_u64(d));
}

/* gsl_stats_ushort_mean / sd restated on sg_f80 (see or_core.c for the algorithm) */
F80_HD double f80_gsl_mean_u16(const uint16_t *data, int n) {
	sg_f80 mean = f80_zero();
	for (int i = 0; i < n; i++) {
		sg_f80 t = f80_sub(f80_from_u64(data[i]), mean);
		t = f80_div_count(t, (uint64_t)i + 1);
		mean = f80_add(mean, t);
	}
	return f80_to_double(mean);
}

F80_HD double f80_gsl_variance_m_u16(const uint16_t *data, int n, double mean) {
	sg_f80 var = f80_zero();
	for (int i = 0; i < n; i++) {
		double dd = (double)data[i] - mean;	/* formed in double, as in GSL */
		sg_f80 delta = f80_from_double(dd);
		sg_f80 t = f80_sub(f80_mul(delta, delta), var);
		t = f80_div_count(t, (uint64_t)i + 1);
		var = f80_add(var, t);
	}
	return f80_to_double(var);
}

/* ---------------------------------------------------------------------------------------
 * The same recurrences on hardware fp64: an x87 value (64-bit mantissa) is held exactly as a
 * double-double hi + lo.  Each operation is evaluated in double-double (TwoSum / TwoProd /
 * Fast2Sum; the accurate double-double sum and the double-double-by-double quotient of Joldes,
 * Muller and Popescu, relative error below 2^-104) and rounded to 64 bits with round-to-nearest-
 * even on lo / ulp.  Where the double-double value lies within 2^-30 ulp of a rounding
 * midpoint (or on a binade edge), the operation is redone in the soft sg_f80 above, so every
 * result is the x87 one; such steps are rare (the error bound is 2^-40 ulp).  About ten times
 * fewer instructions than the integer emulation (one 512-sample sd took ~3 M cycles on one
 * lane of k_stack_replay).
 * ------------------------------------------------------------------------------------- */
typedef struct {
	double hi, lo;
} sg_dd;

F80_HD uint64_t f80_dbits(double d) {
	uint64_t b;
	memcpy(&b, &d, 8);
	return b;
}
F80_HD double f80_bitsd(uint64_t b) {
	double d;
	memcpy(&d, &b, 8);
	return d;
}
/* 2^k for a normal-range k */
F80_HD double f80_pow2(int k) {
	return f80_bitsd((uint64_t)(k + 1023) << 52);
}

F80_HD sg_dd dd_two_sum(double a, double b) {
	sg_dd r;
	r.hi = a + b;
	const double bb = r.hi - a;
	r.lo = (a - (r.hi - bb)) + (b - bb);
	return r;
}
F80_HD sg_dd dd_fast_two_sum(double a, double b) {	/* |a| >= |b| or a == 0 */
	sg_dd r;
	r.hi = a + b;
	r.lo = b - (r.hi - a);
	return r;
}
F80_HD sg_dd dd_two_prod(double a, double b) {
	sg_dd r;
	r.hi = a * b;
	r.lo = fma(a, b, -r.hi);
	return r;
}

/* exact conversions between sg_f80 and the double-double form (fallback steps) */
F80_HD sg_dd f80_to_dd(sg_f80 a) {
	sg_dd r = {0.0, 0.0};
	if (!a.m)
		return r;
	const double sg = a.s ? -1.0 : 1.0;
	/* top 53 and low 11 mantissa bits (exact), then normalised (|lo| <= ulp(hi) / 2) */
	return dd_fast_two_sum(sg * (double)(a.m >> 11) * f80_pow2(a.e - 52), sg * (double)(a.m & 0x7FFull) * f80_pow2(a.e - 63));
}
F80_HD sg_f80 dd_to_f80(sg_dd v) {	/* v: a value with a 64-bit mantissa */
	if (v.hi == 0.0 && v.lo == 0.0)
		return f80_zero();
	const int s = v.hi < 0.0 || (v.hi == 0.0 && v.lo < 0.0);
	double hi = s ? -v.hi : v.hi, lo = s ? -v.lo : v.lo;
	if (hi == 0.0) {
		hi = lo;
		lo = 0.0;
	}
	int e = (int)((f80_dbits(hi) >> 52) & 0x7FF) - 1023;
	const double u = f80_pow2(e - 63);
	int64_t M = (int64_t)(uint64_t)(hi / u) + (int64_t)(lo / u);	/* both exact integers */
	uint64_t m = (uint64_t)M;
	while (!(m >> 63)) {	/* the value lay below 2^e (hi a power of two, lo < 0) */
		m <<= 1;
		e--;
	}
	sg_f80 r = {m, e, s};
	return r;
}

/* v ~ hi + lo (normalised) rounded to a 64-bit mantissa (round to nearest even); *amb set when
 * v is not exact and lies within 2^-30 ulp of a midpoint.  With hi a power of two, lo's sign
 * picks the binade: a value within the error bound (2^-103 |v|) of hi rounds to hi in either */
F80_HD sg_dd dd_round64(double hi, double lo, int exact, int *amb) {
	if (hi == 0.0) {
		sg_dd z = {lo, 0.0};	/* |lo| < 2^53 ulp: in our sums lo == 0 whenever hi == 0 */
		if (lo != 0.0)
			*amb = 1;
		return z;
	}
	const uint64_t hb = f80_dbits(hi);
	int e = (int)((hb >> 52) & 0x7FF) - 1023;
	if ((hb & 0xFFFFFFFFFFFFFull) == 0 && lo != 0.0 && ((lo < 0.0) != (hi < 0.0)))
		e--;	/* hi a power of two, the value in the binade below */
	const double u = f80_pow2(e - 63);
	/* exact: a power-of-two scale (a multiply; a division here cost a full fp64 divide sequence
	 * per rounding, three per recurrence step) */
	const double x = e > -900 ? lo * f80_pow2(63 - e) : lo / u;
	const double rx = rint(x);	/* ties to even: hi / u is a multiple of 2^10 */
	if (!exact && fabs(fabs(x - rx) - 0.5) < 9.3e-10)
		*amb = 1;
	return dd_fast_two_sum(hi, rx * u);
}

/* x87 a + b (a, b 64-bit values as double-doubles) */
F80_HD sg_dd dd80_add(sg_dd a, sg_dd b) {
	const sg_dd s = dd_two_sum(a.hi, b.hi), t = dd_two_sum(a.lo, b.lo);
	const sg_dd v = dd_fast_two_sum(s.hi, s.lo + t.hi);
	const sg_dd z = dd_fast_two_sum(v.hi, t.lo + v.lo);
	int amb = 0;
	const sg_dd r = dd_round64(z.hi, z.lo, 0, &amb);
	if (!amb)
		return r;
	return f80_to_dd(f80_add(dd_to_f80(a), dd_to_f80(b)));
}
/* x87 a / d for an integer count 1 <= d < 2^21 */
F80_HD sg_dd dd80_div_count(sg_dd a, uint32_t d) {
	const double y = (double)d;
	/* one division per step: th only needs to lie within a few ulps of a.hi / y (the exact
	 * remainder a - th y corrects it) and tl's relative error 2^-52 on a remainder of a few
	 * ulp(th) stays far below the 2^-93 |v| the midpoint test allows */
	const double ry = 1.0 / y;
	const double th = a.hi * ry;
	const sg_dd p = dd_two_prod(th, y);
	const double dh = a.hi - p.hi, dl = a.lo - p.lo;
	const double tl = (dh + dl) * ry;
	const sg_dd z = dd_fast_two_sum(th, tl);
	int amb = 0;
	const sg_dd r = dd_round64(z.hi, z.lo, 0, &amb);
	if (!amb)
		return r;
	return f80_to_dd(f80_div_count(dd_to_f80(a), d));
}

/* gsl_stats_ushort_mean / variance_m as f80_gsl_mean_u16 / f80_gsl_variance_m_u16 */
F80_HD double f80dd_gsl_mean_u16(const uint16_t *data, int n) {
	sg_dd mean = {0.0, 0.0};
	for (int i = 0; i < n; i++) {
		const sg_dd x = {(double)data[i], 0.0};
		const sg_dd nm = {-mean.hi, -mean.lo};
		const sg_dd t = dd80_add(x, nm);
		mean = dd80_add(mean, dd80_div_count(t, (uint32_t)i + 1));
	}
	return mean.hi + mean.lo;	/* x87 -> double: the correctly rounded sum */
}
F80_HD double f80dd_gsl_variance_m_u16(const uint16_t *data, int n, double mean) {
	sg_dd var = {0.0, 0.0};
	for (int i = 0; i < n; i++) {
		const double dd = (double)data[i] - mean;	/* formed in double, as in GSL */
		const sg_dd pr = dd_two_prod(dd, dd);
		int amb = 0;
		const sg_dd sq = dd_round64(pr.hi, pr.lo, 1, &amb);	/* exact product: never ambiguous */
		const sg_dd nv = {-var.hi, -var.lo};
		const sg_dd t = dd80_add(sq, nv);
		var = dd80_add(var, dd80_div_count(t, (uint32_t)i + 1));
	}
	return var.hi + var.lo;
}

#endif /* SG_F80_H */
