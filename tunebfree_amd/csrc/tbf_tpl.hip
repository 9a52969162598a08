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
 *   k_tpl_matrix: the play matrix (applyManualDefaults / applyPedalDefaults /
 *               applyDefaultCrosstalk / compilePlayMatrix, src/tonegen.cpp:707-879,
 *               1061-1213), one wave per (template, key); k_tpl_offsets + k_tpl_gather
 *               pack the key lists for one download.
 *
 * The host keeps the cheap, rand()-free steps (frequencies, wheel lengths and spectra:
 * TgTemplate::prepare; the cfg-only list inputs: MatrixInputs) and the draws after the
 * bank (envelopes: TgTemplate::finish after GlibcRand::discard).
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

/* one key's play matrix (row t of freq / ratio, key k = blockIdx.x, 64 lanes; lane l
 * stands for wheels l + 1 + 64 r, r < MX_R):
 *   keyTaper     the cfg's list, else for a manual key (k < 256) per bus b the wheel whose
 *                ratio to the key is nearest the bus ratio in cents (applyManualDefaults
 *                707-802: a strict < over wheels 1..TBF_NW, so the first of equals; the
 *                first and last wheel dropped) -- a wave argmin over the lanes' wheels;
 *                for a pedal key (256..287) the fixed offsets (810-841);
 *   keyCrosstalk the cfg's list, else for a manual key every taper element on each other
 *                bus of its manual at wiringXT x level / bus distance (849-879), generated
 *                in order as the events are walked;
 *   compile      cpmInsert (1061-1120): each element times its terminal's mix, a nonzero
 *                product added to the (wheel, bus) cell in event order -- the lane of a
 *                wheel owns its cells, so every cell sums in the reference's order; then
 *                the cells at or above the floor (1183-1201; raised to the minimum) by
 *                wheel, then bus: the reference's insertion-sorted list. */
#define MX_W 64
#define MX_R (TBF_NW / MX_W)
static_assert (TBF_NW % MX_W == 0, "wheels spread evenly over the lanes");
__device__ static inline uint32_t mx_incl (uint32_t v) /* inclusive prefix over the wave */
{
	const int lane = (int)threadIdx.x;
	for (int d = 1; d < MX_W; d <<= 1) {
		const uint32_t o = __shfl_up (v, d, MX_W);
		if (lane >= d)
			v += o;
	}
	return v;
}

__global__ void __launch_bounds__ (MX_W) k_tpl_matrix (tbf_tpl_mx mx, const double* __restrict__ freq,
                                                       const double* __restrict__ ratio, tbf_contrib* __restrict__ stage,
                                                       uint32_t* __restrict__ cnt)
{
	const int      K = (int)blockIdx.x, lane = (int)threadIdx.x;
	const size_t   q = (size_t)blockIdx.y * 384 + K;
	const double*  fq = freq + TBF_NW * (size_t)blockIdx.y;
	const double*  tr = ratio + 9 * (size_t)blockIdx.y;
	__shared__ tbf_le dflt[9];
	__shared__ float    g[MX_R][27][MX_W]; /* cell (wheel lane + 1 + 64 r, bus) in g[r][bus][lane] */
	__shared__ uint32_t ex[MX_R][MX_W];    /* the cells of the wheel that exist, a bit per bus */
	const tbf_le*     tp  = mx.tp + mx.tpOff[K];
	int               ntp = (int)(mx.tpOff[K + 1] - mx.tpOff[K]);
	if (ntp == 0 && K < 288) {
		int n = 0;
		if (K < 256) {
			const int    k = K & 127, busOffset = (K >> 7) * 9;
			const double fk = fq[k];
			float        rt[MX_R];
			for (int r = 0; r < MX_R; r++)
				rt[r] = (float)(fmin (fmax (fq[lane + MX_W * r], 12.0), 2.5e10) / fk);
			for (int b = 0; b < 9; b++) {
				float bv = __builtin_inff ();
				int   bi = 0;
				for (int r = 0; r < MX_R; r++) {
					const float c = (float)(1200 * fabs (log2 (tr[b] / (double)rt[r])));
					if (c < bv)
						bv = c, bi = lane + 1 + MX_W * r;
				}
				for (int d = 1; d < MX_W; d <<= 1) { /* the smallest, the lowest wheel of equals */
					const float ov = __shfl_xor (bv, d, MX_W);
					const int   oi = __shfl_xor (bi, d, MX_W);
					if (ov < bv || (ov == bv && oi < bi))
						bv = ov, bi = oi;
				}
				if (bi != 1 && bi != TBF_NW) {
					if (lane == 0)
						dflt[n] = {(int16_t)bi, (int16_t)(b + busOffset), mx.taper[k * 9 + b]};
					n++;
				}
			}
		} else {
			const int PDoffset[9] = {-12, 7, 0, 12, 19, 24, 28, 31, 36};
			for (int b = 0; b < 9; b++) {
				const int tn = (K - 256 + 1) + PDoffset[b];
				if (tn < 1 || TBF_NW < tn)
					continue;
				if (lane == 0)
					dflt[n] = {(int16_t)tn, (int16_t)(b + 18), 1.0f}; /* dBToGain (0.0) */
				n++;
			}
		}
		__syncthreads ();
		tp  = dflt;
		ntp = n;
	}
	const tbf_le* xt  = mx.xt + mx.xtOff[K];
	const int     nxt = (int)(mx.xtOff[K + 1] - mx.xtOff[K]);
	for (int r = 0; r < MX_R; r++)
		ex[r][lane] = 0;
	auto ins = [&] (const tbf_le lep) {
		const uint32_t bus = (uint8_t)lep.sb;
		for (uint32_t j = mx.tmOff[lep.sa]; j < mx.tmOff[lep.sa + 1]; j++) {
			const tbf_le tl   = mx.tm[j];
			const float  gain = tl.fc * lep.fc;
			if (gain == 0.0f)
				continue;
			const int wl = tl.sa - 1 - lane; /* wheel - 1 - lane: 64 r when it is this lane's */
			if (wl < 0 || (wl & (MX_W - 1)))
				continue;
			const int r = wl / MX_W;
			const uint32_t e = ex[r][lane];
			g[r][bus][lane]  = (e >> bus & 1u) ? g[r][bus][lane] + gain : gain;
			ex[r][lane]      = e | 1u << bus;
		}
	};
	for (int i = 0; i < ntp; i++)
		ins (tp[i]);
	if (nxt > 0)
		for (int i = 0; i < nxt; i++)
			ins (xt[i]);
	else if (K < 256)
		for (int b = 0; b < 9; b++) {
			const int busNumber = (K >> 7) * 9 + b;
			for (int i = 0; i < ntp; i++) {
				const tbf_le e = tp[i];
				if (e.sb == busNumber)
					continue;
				ins ({e.sa, (int16_t)busNumber, (float)((mx.wiringXT * (double)e.fc) / abs (busNumber - e.sb))});
			}
		}
	/* the kept cells, by wheel (row r: wheels 64 r + 1 .. 64 r + 64), then bus */
	uint32_t pos = 0, total = 0;
	for (int r = 0; r < MX_R; r++) {
		uint32_t kept = 0;
		for (int b = 0; b < 27; b++)
			if ((ex[r][lane] >> b & 1u) && !((double)g[r][b][lane] < mx.floor))
				kept |= 1u << b;
		const uint32_t c = (uint32_t)__builtin_popcount (kept), incl = mx_incl (c);
		pos              = total + incl - c;
		total += __shfl (incl, MX_W - 1, MX_W);
		tbf_contrib* out = stage + q * mx.cap;
		for (; kept; kept &= kept - 1) {
			const int b   = __builtin_ctz (kept);
			float     lvl = g[r][b][lane];
			if ((double)lvl < mx.minLevel)
				lvl = (float)mx.minLevel;
			if (pos < mx.cap)
				out[pos] = {(uint16_t)(lane + 1 + MX_W * r), (uint16_t)b, lvl};
			pos++;
		}
	}
	if (lane == 0)
		cnt[q] = total;
}

/* exclusive prefix of the key list lengths (capped) over all templates: off[0..n] */
__global__ void __launch_bounds__ (1024) k_tpl_offsets (const uint32_t* __restrict__ cnt, uint32_t n, uint32_t cap,
                                                       uint32_t* __restrict__ off)
{
	__shared__ uint32_t sh[1024];
	const uint32_t      tid   = threadIdx.x;
	uint32_t            carry = 0;
	if (tid == 0)
		off[0] = 0;
	for (uint32_t base = 0; base < n; base += 1024) {
		sh[tid] = base + tid < n ? min (cnt[base + tid], cap) : 0u;
		__syncthreads ();
		for (uint32_t d = 1; d < 1024; d <<= 1) {
			const uint32_t o = tid >= d ? sh[tid - d] : 0u;
			__syncthreads ();
			sh[tid] += o;
			__syncthreads ();
		}
		if (base + tid < n)
			off[base + tid + 1] = carry + sh[tid];
		carry += sh[1023];
		__syncthreads ();
	}
}

__global__ void __launch_bounds__ (MX_W) k_tpl_gather (const tbf_contrib* __restrict__ stage, const uint32_t* __restrict__ off,
                                                       uint32_t cap, tbf_contrib* __restrict__ out)
{
	const size_t   q = blockIdx.x;
	const uint32_t o = off[q], m = off[q + 1] - o;
	for (uint32_t i = threadIdx.x; i < m; i += MX_W)
		out[o + i] = stage[q * cap + i];
}

extern "C" int tbf_tpl_matrix_launch (uint32_t ntpl, const tbf_tpl_mx* mx, const double* freq, const double* ratio,
                                      tbf_contrib* stage, uint32_t* cnt, uint32_t* off, tbf_contrib* out, hipStream_t s)
{
	if (ntpl == 0)
		return 0;
	for (uint32_t t0 = 0; t0 < ntpl; t0 += 65535) {
		const uint32_t nt = ntpl - t0 < 65535 ? ntpl - t0 : 65535;
		k_tpl_matrix<<<dim3 (384, nt), MX_W, 0, s>>> (*mx, freq + TBF_NW * (size_t)t0, ratio + 9 * (size_t)t0,
		                                               stage + (size_t)t0 * 384 * mx->cap, cnt + (size_t)t0 * 384);
		if (hipGetLastError () != hipSuccess)
			return -5;
	}
	const uint32_t n = ntpl * 384u;
	k_tpl_offsets<<<1, 1024, 0, s>>> (cnt, n, mx->cap, off);
	if (hipGetLastError () != hipSuccess)
		return -5;
	k_tpl_gather<<<n, MX_W, 0, s>>> (stage, off, mx->cap, out);
	return hipGetLastError () != hipSuccess ? -5 : 0;
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
