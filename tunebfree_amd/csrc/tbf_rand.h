/*
 * tbf_rand.h -- jump-ahead for glibc's rand() (random_r TYPE_3: degree 31, separation 3),
 * shared by the host (GlibcRand::discard) and the device template builder
 * (k_tpl_rand).
 *
 * The generator's words form the sequence y[i] = y[i-31] + y[i-3] (mod 2^32); rand()
 * returns y[i] >> 1.  With the shift operator S, P(S) y = 0 for
 * P(x) = x^31 - x^28 - 1, so for c(x) = x^k mod P(x) = sum_m c_m x^m,
 * y[i + k + j] = sum_m c_m y[i + m + j] for every j: a window of 31 words k steps
 * ahead is a Z/2^32-linear combination of the current window extended by 30 words.
 * tonegen's initOscillators draws one rand() per wave sample in wheel order
 * (src/tonegen.cpp:1402-1457), so the draw of sample n of wheel w is rand number
 * off[w] + n of the template's stream: each device thread jumps to its chunk.
 */
#ifndef TBF_RAND_H
#define TBF_RAND_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TBF_RHD __host__ __device__ inline

/* out = a * b mod P (31 coefficients each, mod 2^32); out must not alias a or b */
TBF_RHD void gr_mulmod (const uint32_t* a, const uint32_t* b, uint32_t* out)
{
	uint32_t t[61];
	for (int i = 0; i < 61; i++)
		t[i] = 0;
	for (int i = 0; i < 31; i++)
		for (int j = 0; j < 31; j++)
			t[i + j] += a[i] * b[j];
	for (int k = 60; k >= 31; k--) { /* x^k = x^(k-3) + x^(k-31) */
		t[k - 3] += t[k];
		t[k - 31] += t[k];
	}
	for (int i = 0; i < 31; i++)
		out[i] = t[i];
}

/* c = x^k mod P */
TBF_RHD void gr_xpow (uint64_t k, uint32_t* c)
{
	uint32_t tmp[31];
	for (int i = 0; i < 31; i++)
		c[i] = 0;
	c[0] = 1;
	int top = 63;
	while (top >= 0 && !((k >> top) & 1))
		top--;
	for (int b = top; b >= 0; b--) {
		gr_mulmod (c, c, tmp);
		if ((k >> b) & 1) { /* times x */
			const uint32_t hi = tmp[30];
			for (int i = 30; i > 0; i--)
				c[i] = tmp[i - 1];
			c[0] = hi;
			c[28] += hi;
		} else {
			for (int i = 0; i < 31; i++)
				c[i] = tmp[i];
		}
	}
}

/* E[0..60]: a window of 31 words extended by the recurrence; W[j] = E[k + j] */
TBF_RHD void gr_jump_window (const uint32_t* E, uint64_t k, uint32_t* W)
{
	uint32_t c[31];
	gr_xpow (k, c);
	for (int j = 0; j < 31; j++) {
		uint32_t v = 0;
		for (int m = 0; m < 31; m++)
			v += c[m] * E[m + j];
		W[j] = v;
	}
}

/* extend a 31-word window to 61 words */
TBF_RHD void gr_extend (const uint32_t* W, uint32_t* E)
{
	for (int j = 0; j < 31; j++)
		E[j] = W[j];
	for (int j = 31; j < 61; j++)
		E[j] = E[j - 31] + E[j - 3];
}

#endif
