/*
 * tbf_sin.h -- the device's double sin with wave-uniform fast paths.
 *
 * The render kernels take sin from the ROCm device library (OCML __ocml_sin_f64): the
 * small-argument reduction __ocmlpriv_trigredsmall_f64 (n = rint (|x| 2/pi), a three-part
 * Cody-Waite subtraction of n pi/2) and __ocmlpriv_sincosred2_f64, which evaluates BOTH the
 * sine and the cosine polynomial of the reduced argument and selects one by n & 1.  The
 * preamp's density waveshaper (src/overdrive.cpp:111-136) takes sin of |x| pi/2 clamped to
 * [0, 1.57079633] four times per sample at character 0.5, and the reverb input stage
 * (src/reverb.cpp:371) sin of a small value: there n is 0 or 1, and the samples of a wave
 * mostly share it (at the bench's registration 99.9 / 94 / 71 / 56 % of 32-sample tiles for
 * the four density sines).  So when every active lane of the wave has n == 0, only the sine
 * polynomial of r = |x| (no reduction: trigredsmall gives hi = |x|, lo = +0 for n = 0) is
 * evaluated; when every lane has n == 1, the reduction with n = 1 and only the cosine
 * polynomial; otherwise OCML's sin itself.  Each path is OCML's sequence of operations for
 * the lanes it serves (explicit fma where OCML has llvm.fma, plain operations elsewhere,
 * compiled with -ffp-contract=off), so the result is OCML's bits on every path -- the same
 * values the kernels produced with sin () (bit-identical to the oracle's glibc sin on every
 * parity test; DESIGN.md section 2, licensed differences).  Constants are OCML's, given by
 * their bit patterns.
 */
#ifndef TBF_SIN_H
#define TBF_SIN_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TBF_D(bits) __builtin_bit_cast (double, (uint64_t)(bits##ull))

/* __ocmlpriv_trigredsmall_f64 for a given n: |x| - n pi/2 as hi + lo */
__device__ __forceinline__ void tbf_trigred_small (double a, double n, double& hi, double& lo)
{
	const double r4  = __builtin_fma (n, TBF_D (0xBFF921FB54442D18), a);
	const double r5  = __builtin_fma (n, TBF_D (0xBC91A62633145C00), r4);
	const double m6  = n * TBF_D (0x3C91A62633145C00);
	const double e8  = __builtin_fma (n, TBF_D (0x3C91A62633145C00), -m6);
	const double r9  = r4 - m6;
	const double r10 = r4 - r9;
	const double r11 = r10 - m6;
	const double r12 = r9 - r5;
	const double r13 = r12 + r11;
	const double r14 = r13 - e8;
	const double r15 = __builtin_fma (n, TBF_D (0xB97B839A252049C0), r14);
	hi               = r5 + r15;
	const double r17 = hi - r5;
	lo               = r15 - r17;
}

/* the sine half of __ocmlpriv_sincosred2_f64 (x = hi, y = lo) */
__device__ __forceinline__ double tbf_sinred (double x, double y)
{
	const double x2  = x * x;
	const double s18 = __builtin_fma (x2, TBF_D (0x3DE5E0B2F9A43BB8), TBF_D (0xBE5AE600B42FDFA7));
	const double s19 = __builtin_fma (x2, s18, TBF_D (0x3EC71DE3796CDE01));
	const double s20 = __builtin_fma (x2, s19, TBF_D (0xBF2A01A019E83E5C));
	const double s21 = __builtin_fma (x2, s20, TBF_D (0x3F81111111110BB3));
	const double x23 = x * (-x2);
	const double s24 = y * 0.5;
	const double s25 = __builtin_fma (x23, s21, s24);
	const double s26 = __builtin_fma (x2, s25, -y);
	const double s27 = __builtin_fma (x23, TBF_D (0xBFC5555555555555), s26);
	return x - s27;
}

/* the cosine half of __ocmlpriv_sincosred2_f64 */
__device__ __forceinline__ double tbf_cosred (double x, double y)
{
	const double x2  = x * x;
	const double h   = x2 * 0.5;
	const double c5  = 1.0 - h;
	const double c6  = 1.0 - c5;
	const double c7  = c6 - h;
	const double x4  = x2 * x2;
	const double p9  = __builtin_fma (x2, TBF_D (0xBDA907DB46CC5E42), TBF_D (0x3E21EEB69037AB78));
	const double p10 = __builtin_fma (x2, p9, TBF_D (0xBE927E4FA17F65F6));
	const double p11 = __builtin_fma (x2, p10, TBF_D (0x3EFA01A019F4EC90));
	const double p12 = __builtin_fma (x2, p11, TBF_D (0xBF56C16C16C16967));
	const double p13 = __builtin_fma (x2, p12, TBF_D (0x3FA5555555555555));
	const double c15 = __builtin_fma (x, -y, c7);
	const double c16 = __builtin_fma (x4, p13, c15);
	return c5 + c16;
}

/* OCML's sign rule: the selected value's sign flipped when x is negative (n & 2 is 0 here) */
__device__ __forceinline__ double tbf_sign_of (double r, double x)
{
	const uint64_t s = __builtin_bit_cast (uint64_t, x) & 0x8000000000000000ull;
	return __builtin_bit_cast (double, __builtin_bit_cast (uint64_t, r) ^ s);
}

/* __ocml_sin_f64 for |x| < 2^30 (the trigredsmall branch): both polynomials, the one n & 1
 * selects, the sign flipped for n & 2 and for negative x */
__device__ __forceinline__ double tbf_sin_small (double x, double a, double n)
{
	double hi, lo;
	tbf_trigred_small (a, n, hi, lo);
	const double   s = tbf_sinred (hi, lo), c = tbf_cosred (hi, lo);
	const int      q = (int)n & 3;
	const uint64_t r = __builtin_bit_cast (uint64_t, (q & 1) ? c : s);
	const uint64_t f = (q > 1 ? 0x8000000000000000ull : 0ull) ^ (__builtin_bit_cast (uint64_t, x) & 0x8000000000000000ull);
	return __builtin_bit_cast (double, r ^ f);
}

#ifndef SIN_EXPECT
#define SIN_EXPECT 1 /* the first fast path (every lane's quadrant 0) likely, the library call for huge
                      * arguments unlikely: the compiler lays the common path out as the fall-through */
#endif
#if SIN_EXPECT
#define TBF_LIKELY(x) __builtin_expect (!!(x), 1)
#define TBF_UNLIKELY(x) __builtin_expect (!!(x), 0)
#else
#define TBF_LIKELY(x) (x)
#define TBF_UNLIKELY(x) (x)
#endif
#define TBF_N(a) __builtin_rint ((a) * TBF_D (0x3FE45F306DC9C883))
#define TBF_SMALL(a) ((a) < TBF_D (0x41D0000000000000)) /* 2^30; false for NaN (OCML's test) */

/* sin (x), OCML's bits, with the wave-uniform fast paths above */
__device__ __forceinline__ double tbf_sin (double x)
{
	const double a = fabs (x);
	const double n = TBF_N (a);
	if (TBF_LIKELY (__all (n == 0.0)))
		return tbf_sign_of (tbf_sinred (a, 0.0), x);
	if (__all (n == 1.0)) {
		double hi, lo;
		tbf_trigred_small (a, 1.0, hi, lo);
		return tbf_sign_of (tbf_cosred (hi, lo), x);
	}
	if (!TBF_UNLIKELY (!__all (TBF_SMALL (a))))
		return tbf_sin_small (x, a, n);
	return sin (x);
}

/* two independent sines at once: one wave vote for both, and straight-line code on every
 * path, so the compiler interleaves the two dependency chains (a lone sine is a chain of
 * ~20 dependent FP64 operations, latency-bound at two waves per SIMD) */
__device__ __forceinline__ void tbf_sin2 (double x0, double x1, double& r0, double& r1)
{
	const double a0 = fabs (x0), a1 = fabs (x1);
	const double n0 = TBF_N (a0), n1 = TBF_N (a1);
	if (TBF_LIKELY (__all (n0 == 0.0 && n1 == 0.0))) {
		r0 = tbf_sign_of (tbf_sinred (a0, 0.0), x0);
		r1 = tbf_sign_of (tbf_sinred (a1, 0.0), x1);
	} else if (__all (n0 == 1.0 && n1 == 1.0)) {
		double h0, l0, h1, l1;
		tbf_trigred_small (a0, 1.0, h0, l0);
		tbf_trigred_small (a1, 1.0, h1, l1);
		r0 = tbf_sign_of (tbf_cosred (h0, l0), x0);
		r1 = tbf_sign_of (tbf_cosred (h1, l1), x1);
	} else if (!TBF_UNLIKELY (!__all (TBF_SMALL (a0) && TBF_SMALL (a1)))) {
		r0 = tbf_sin_small (x0, a0, n0);
		r1 = tbf_sin_small (x1, a1, n1);
	} else {
		r0 = sin (x0);
		r1 = sin (x1);
	}
}

/* N independent sines in place, one wave vote for all of them (tbf_sin2 for N values) */
template <int N>
__device__ __forceinline__ void tbf_sin_n (double (&x)[N])
{
	double a[N], n[N];
	bool   z = true, o = true, sm = true;
#pragma unroll
	for (int i = 0; i < N; i++) {
		a[i] = fabs (x[i]);
		n[i] = TBF_N (a[i]);
		z    = z && n[i] == 0.0;
		o    = o && n[i] == 1.0;
		sm   = sm && TBF_SMALL (a[i]);
	}
	if (TBF_LIKELY (__all (z))) {
#pragma unroll
		for (int i = 0; i < N; i++)
			x[i] = tbf_sign_of (tbf_sinred (a[i], 0.0), x[i]);
	} else if (__all (o)) {
#pragma unroll
		for (int i = 0; i < N; i++) {
			double hi, lo;
			tbf_trigred_small (a[i], 1.0, hi, lo);
			x[i] = tbf_sign_of (tbf_cosred (hi, lo), x[i]);
		}
	} else if (!TBF_UNLIKELY (!__all (sm))) {
#pragma unroll
		for (int i = 0; i < N; i++)
			x[i] = tbf_sin_small (x[i], a[i], n[i]);
	} else {
#pragma unroll
		for (int i = 0; i < N; i++)
			x[i] = sin (x[i]);
	}
}

/* __ocml_asin_f64's |x| < 0.5 branch: the polynomial in x^2 */
__device__ __forceinline__ double tbf_asin_poly (double x)
{
	const double a  = fabs (x);
	const double t  = x * x;
	double       p  = __builtin_fma (t, TBF_D (0x3FA059859FEA6A70), TBF_D (0xBF90A5A378A05EAF));
	p               = __builtin_fma (t, p, TBF_D (0x3F94052137024D6A));
	p               = __builtin_fma (t, p, TBF_D (0x3F7AB3A098A70509));
	p               = __builtin_fma (t, p, TBF_D (0x3F88ED60A300C8D2));
	p               = __builtin_fma (t, p, TBF_D (0x3F8C6FA84B77012B));
	p               = __builtin_fma (t, p, TBF_D (0x3F91C6C111DCCB70));
	p               = __builtin_fma (t, p, TBF_D (0x3F96E89F0A0ADACF));
	p               = __builtin_fma (t, p, TBF_D (0x3F9F1C72C668963F));
	p               = __builtin_fma (t, p, TBF_D (0x3FA6DB6DB41CE4BD));
	p               = __builtin_fma (t, p, TBF_D (0x3FB333333336FD5B));
	p               = __builtin_fma (t, p, TBF_D (0x3FC5555555555380));
	const double s  = t * p;
	const double r  = __builtin_fma (a, s, a);
	return __builtin_copysign (r, x);
}

#undef TBF_SMALL
#undef TBF_N
#undef TBF_D

#endif
