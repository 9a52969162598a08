/*
 * tbf_tpl.hip -- tone-generator templates built on the device:
 * the wave bank of initOscillators/writeSamples (src/tonegen.cpp:1402-1457, 1470-1630)
 * for a batch of templates (tunings x seeds) in two launches.
 *
 *   k_tpl_rand: the per-sample rand() LSB draws.  One thread per 512-draw chunk of a
 *               template's stream jumps to its chunk (tbf_rand.h: x^k mod P over
 *               Z/2^32, k = the chunk's first draw) and runs the TYPE_3 recurrence.
 *   k_tpl_wave: one thread per sample: the nonzero partials' sines plus the LSB,
 *               the reference's expression and evaluation order.
 *
 * The host keeps the cheap, rand()-free steps (frequencies, play matrix, wheel lengths
 * and spectra: TgTemplate::prepare) and the draws after the bank (envelopes:
 * TgTemplate::finish after GlibcRand::discard).
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tbf_rand.h"
#include "tbf_tpl.h"

#define TPL_CHUNK 512

__global__ void __launch_bounds__ (64) k_tpl_rand (const uint32_t* __restrict__ E61, const uint64_t* __restrict__ total,
                                                   const uint64_t* __restrict__ base, uint8_t* __restrict__ lsb)
{
	const uint32_t t  = blockIdx.y;
	const uint64_t q0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * TPL_CHUNK;
	if (q0 >= total[t])
		return;
	uint32_t W[31];
	gr_jump_window (E61 + 61 * (size_t)t, q0, W);
	const uint64_t m = total[t] - q0 < TPL_CHUNK ? total[t] - q0 : TPL_CHUNK;
	uint8_t*       o = lsb + base[t] + q0;
	int            f = 0; /* W[f] = y[i-31]; the next draw is y[i] = y[i-31] + y[i-3] */
	for (uint64_t j = 0; j < m; j++) {
		const int      r = f + 28 >= 31 ? f - 3 : f + 28;
		const uint32_t y = W[f] + W[r];
		W[f]             = y;
		f                = f == 30 ? 0 : f + 1;
		o[j]             = (int32_t)(y >> 1) < (2147483647 >> 1) ? 1 : 0; /* src/tonegen.cpp:1449 */
	}
}

__global__ void __launch_bounds__ (256) k_tpl_wave (const tbf_tpl_wheel* __restrict__ wh, const uint64_t* __restrict__ base,
                                                    const uint8_t* __restrict__ lsb, float* __restrict__ bank, double sr)
{
	const uint32_t       t = blockIdx.z;
	const tbf_tpl_wheel& w = wh[(size_t)t * TBF_NW + blockIdx.y];
	const uint32_t       n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= w.len)
		return;
	const double fullCircle = 2.0 * M_PI;
	double       s          = 0.0;
	for (int q = 0; q < w.np; q++)
		s += w.amp[q] * sin (remainder ((w.hz[q] * fullCircle * (double)n) / sr, fullCircle));
	const size_t i = base[t] + w.off + n;
	const float  v = lsb[i] ? (float)(1.0 / 32767.0) : 0.0f;
	bank[i]        = (float)((double)v + (w.U * s));
}

extern "C" int tbf_tpl_launch (uint32_t ntpl, uint32_t maxChunks, uint32_t maxLen, const uint32_t* E61,
                               const uint64_t* total, const uint64_t* base, const tbf_tpl_wheel* wh, uint8_t* lsb,
                               float* bank, double sr, hipStream_t s)
{
	if (ntpl == 0)
		return 0;
	for (uint32_t t0 = 0; t0 < ntpl; t0 += 65535) {
		const uint32_t nt = ntpl - t0 < 65535 ? ntpl - t0 : 65535;
		k_tpl_rand<<<dim3 ((maxChunks + 63) / 64, nt), 64, 0, s>>> (E61 + 61 * (size_t)t0, total + t0, base + t0, lsb);
		if (hipGetLastError () != hipSuccess)
			return -5;
		k_tpl_wave<<<dim3 ((maxLen + 255) / 256, TBF_NW, nt), 256, 0, s>>> (wh + (size_t)t0 * TBF_NW, base + t0, lsb, bank, sr);
		if (hipGetLastError () != hipSuccess)
			return -5;
	}
	return 0;
}
