/*
 * oracle/orc_base.c -- TEST INFRASTRUCTURE ONLY (see orc.h).
 * glibc rand() restatement and the MTS-ESP frequency table logic.
 */
#include "orc.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* glibc srandom_r/random_r with TYPE_3 (degree 31, separation 3), the generator
 * behind rand() on the reference's Linux hosts.  The reference seeds with
 * srand(time(NULL)) (b_synth/lv2.cpp:949, src/main.cpp:805); the oracle takes the
 * seed explicitly.  Pinned against libc rand() in tests/test_oracle_cpu.py. */
void orc_srand (orc_rand* s, unsigned int seed)
{
	int     i;
	int32_t word;
	if (seed == 0)
		seed = 1;
	s->state[0] = (int32_t)seed;
	word        = (int32_t)seed;
	for (i = 1; i < 31; ++i) {
		int64_t hi = word / 127773;
		int64_t lo = word % 127773;
		word       = 16807 * lo - 2836 * hi;
		if (word < 0)
			word += 2147483647;
		s->state[i] = (int32_t)word;
	}
	s->f = 3;
	s->r = 0;
	for (i = 0; i < 310; ++i)
		(void)orc_rand_next (s);
}

int32_t orc_rand_next (orc_rand* s)
{
	uint32_t val       = (uint32_t)s->state[s->f] + (uint32_t)s->state[s->r];
	s->state[s->f]     = (int32_t)val;
	int32_t result     = (int32_t)(val >> 1);
	if (++s->f >= 31) {
		s->f = 0;
		++s->r;
	} else {
		if (++s->r >= 31)
			s->r = 0;
	}
	return result;
}

/* src/tuning.cpp:48-106 inferScaleSize */
void orc_infer_scale_size (const double* frequency, int* scaleSizeRet, float* periodRet)
{
	int   scaleSize, i, mismatch;
	float period;
	for (period = 2.0f; period < 10.0f; period++) {
		for (scaleSize = 1; scaleSize < 128; scaleSize++) {
			mismatch = 0;
			for (i = 0; i < 128 - scaleSize; i++) {
				if (fabs (frequency[i + scaleSize] / frequency[i] - period) > 1e-6) {
					mismatch = 1;
					break;
				}
			}
			if (!mismatch) {
				*scaleSizeRet = scaleSize;
				*periodRet    = period;
				return;
			}
		}
	}
	for (scaleSize = 1; scaleSize < 128; scaleSize++) {
		period   = (float)(frequency[scaleSize] / frequency[0]);
		mismatch = 0;
		for (i = 0; i < 128 - scaleSize; i++) {
			if (fabs (frequency[i + scaleSize] / frequency[i] - period) > 1e-6) {
				mismatch = 1;
				break;
			}
		}
		if (!mismatch) {
			*scaleSizeRet = scaleSize;
			*periodRet    = period;
			return;
		}
	}
	*scaleSizeRet = -1;
	*periodRet    = -1.0f;
}

/* src/tuning.cpp:142-147 getFrequencies = MTS pull (tuning.cpp:25-34) + extendFrequencies
 * (tuning.cpp:115-135).  With no MTS-ESP master connected, the un-vendored ODDSound
 * MTS-ESP client (libs/MTS-ESP, pinned commit not recoverable) answers 12-TET with
 * A4 = 440 Hz: 440 * 2^((n-69)/12), pinned by the doctest values at tuning.cpp:183-206. */
void orc_get_frequencies (double* frequency, const double* mts128)
{
	int   i, scaleSize;
	float period;
	for (i = 0; i < 128; i++)
		frequency[i] = mts128 ? mts128[i] : 440. * pow (2., (i - 69.) / 12.);
	orc_infer_scale_size (frequency, &scaleSize, &period);
	if (scaleSize > 0) {
		for (i = 128; i < ORC_NOF_FREQS; i++)
			frequency[i] = period * frequency[i - scaleSize];
	} else {
		for (i = 128; i < ORC_NOF_FREQS; i++)
			frequency[i] = frequency[127];
	}
}

/* src/tuning.cpp:153-174 wheelPairs / getPairedWheel */
static const short wheelPairs[92] = {
	0,
	49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60,
	61, 62, 63, 64, 65, 66, 67, 68, 69, 70, 71, 72,
	73, 74, 75, 76, 77, 78, 79, 80, 81, 82, 83, 84,
	0, 0, 0, 0, 0, 85, 86, 87, 88, 89, 90, 91,
	1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12,
	13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24,
	25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36,
	42, 43, 44, 45, 46, 47, 48
};

short orc_paired_wheel (short n)
{
	int q = n / 92, r = n % 92;
	return (short)(q * 92 + wheelPairs[r]);
}
