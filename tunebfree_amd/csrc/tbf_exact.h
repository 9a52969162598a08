/*
 * tbf_exact.h -- exact shortcuts for serial recurrences of the reference, shared by the
 * kernel and a host test hook (tbf_debug_exact) so CPU tests can check them against
 * the literal recurrences.
 */
#ifndef TBF_EXACT_H
#define TBF_EXACT_H

#include <hip/hip_runtime.h>
#include <math.h>

#define TBF_HD __host__ __device__ __forceinline__

/* count after n increments of `count++; if (count < 0 || count > d) count = 0` */
TBF_HD int cnt_adv (int c0, int d, int n)
{
	if (c0 >= 0 && c0 <= d && n <= d + 1) { /* steady state: one wrap at most */
		const int v = c0 + n;
		return v > d ? v - d - 1 : v;
	}
	if (n == 0)
		return c0;
	if (c0 > d || c0 < 0)
		return (n - 1) % (d + 1);
	return (c0 + n) % (d + 1);
}

/* Exact closed form of `v += d` repeated (src/reverb.cpp:479-496 vibrato phases).
 * Inside one binade [2^(e-1), 2^e) of |v| every sum lands on the grid u = 2^(e-53), so
 * fl(v + d) = v + D with D = rint(d/u)*u, unless d/u is a tie.  Valid for a run of m
 * steps when the first and last values stay at least one grid step inside the binade
 * (the exact sums then never reach a binade edge).  Returns false otherwise. */
TBF_HD bool phase_run (double v0, double d, int m, double& D)
{
	if (!(d >= 0.0) || !(fabs (v0) > 0.0) || !isfinite (v0))
		return false;
	int e;
	frexp (v0, &e);
	const double u  = ldexp (1.0, e - 53);
	const double lo = ldexp (1.0, e - 1) + u, hi = ldexp (1.0, e) - u;
	const double k  = ldexp (d, 53 - e); /* d / u: u is a power of two, so the same correctly rounded value without a division */
	const double r  = rint (k);
	if (fabs (k - r) == 0.5)
		return false;
	D              = r * u;
	const double w = v0 + (double)m * D;
	const double a0 = fabs (v0), a1 = fabs (w);
	return a0 >= lo && a0 <= hi && a1 >= lo && a1 <= hi && ((v0 < 0) == (w < 0));
}

/* phase_run with a per-line cache: the step D and the binade it belongs to only change
 * when the phase crosses a binade, so the frexp/ldexp/rint analysis runs only then.
 * Same result as phase_run (v0, d, m, D). */
TBF_HD bool phase_run_cached (double v0, double d, int m, double& D, double& cD, double& cLo, double& cHi)
{
	if (cD > 0.0) {
		const double w = v0 + (double)m * cD, a0 = fabs (v0), a1 = fabs (w);
		if (a0 >= cLo && a0 <= cHi && a1 >= cLo && a1 <= cHi && ((v0 < 0) == (w < 0))) {
			D = cD;
			return true;
		}
	}
	if (!phase_run (v0, d, m, D))
		return false;
	if (D > 0.0) {
		int e;
		frexp (v0, &e);
		const double u = ldexp (1.0, e - 53);
		cD             = D;
		cLo            = ldexp (1.0, e - 1) + u;
		cHi            = ldexp (1.0, e) - u;
	}
	return true;
}

/* fmod (x, 1.0) for the rotor angle update (src/whirl.cpp:1428-1429): for x in [0, 2)
 * fmod is x or x - 1, the latter exact by Sterbenz; anything else takes libm. */
TBF_HD double wrap1 (double x)
{
	if (x >= 0.0 && x < 2.0)
		return x >= 1.0 ? x - 1.0 : x;
	return fmod (x, 1.0);
}

/* xorshift32 of the Airwindows dither (src/overdrive.cpp:158-160, src/reverb.cpp:775-783) */
TBF_HD uint32_t xs_step (uint32_t x)
{
	x ^= x << 13;
	x ^= x >> 17;
	x ^= x << 5;
	return x;
}

/* xorshift32 is linear over GF(2): the state after k steps from x0 is the XOR, over the
 * set bits j of x0, of the k-step image of (1 << j).  J[j * cols + k] holds that image. */
static inline void xs_jump_table (uint32_t* J, int cols)
{
	for (int j = 0; j < 32; j++) {
		uint32_t x = 1u << j;
		for (int k = 0; k < cols; k++) {
			J[j * cols + k] = x;
			x               = xs_step (x);
		}
	}
}

/* nibble-sliced form of J: N[(i * 16 + v) * cols + k] = XOR over the set bits b of v of
 * J[(4 i + b) * cols + k], so the k-step state is the XOR of 8 entries, one per nibble */
static inline void xs_nib_table (uint32_t* N, const uint32_t* J, int cols)
{
	for (int i = 0; i < 8; i++)
		for (int v = 0; v < 16; v++)
			for (int k = 0; k < cols; k++) {
				uint32_t r = 0;
				for (int b = 0; b < 4; b++)
					if ((v >> b) & 1)
						r ^= J[(4 * i + b) * cols + k];
				N[(i * 16 + v) * cols + k] = r;
			}
}

TBF_HD uint32_t xs_jump_ref (const uint32_t* J, int cols, uint32_t x0, int k)
{
	uint32_t r = 0;
	for (int j = 0; j < 32; j++)
		if ((x0 >> j) & 1u)
			r ^= J[j * cols + k];
	return r;
}

#endif
