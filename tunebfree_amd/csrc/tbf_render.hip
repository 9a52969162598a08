/*
 * tbf_render.hip -- gfx950 render kernel for the tuneBfree block quartet
 *   oscGenerateFragment -> preamp -> b_reverb::reverb -> whirlProc3
 * (src/tonegen.cpp:3218, src/overdrive.cpp:329, src/reverb.cpp:274, src/whirl.cpp:1653).
 *
 * Mapping: one workgroup = one wave64 = one organ instance; the kernel loops over the
 * segment's 128-sample blocks with the instance's DSP state resident in LDS.
 *   - tonegen:   lane = sample (2 samples/lane), wheel loop in active-list order
 *   - vibrato:   lane-parallel scatter recast as an ordered per-slot gather
 *   - overdrive, reverb, whirl: sub-blocks of 64 samples, lane = sample; every ring
 *     read of a sub-block happens before its ring writes (write-after-read), which is
 *     exact because every ring delay exceeds the sub-block (reverb >= 560, whirl >= 79
 *     samples ahead); per-sample IIR/phase recurrences run on single lanes in the
 *     reference's literal operation order.
 * Float discipline: compiled with -ffp-contract=off, no fast-math, denormals kept;
 * every expression follows the reference's evaluation order so results are
 * bit-identical to the strict-IEEE oracle except for FP64 libm (sin/asin) ulps.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "tbf_types.h"
#include "tbf_exact.h"

#define NL 64

struct TgScratch {
	float swl[TBF_BLK];
	float vin[TBF_BLK];
	float prc[TBF_BLK];
	union {
		struct { /* core-program entries resolved by the interpreter prologue */
			uint32_t base[TBF_NW + 8]; /* bank index of the wheel's current sample */
			uint32_t lim[TBF_NW + 8];  /* samples before the wheel's wrap */
			uint32_t len[TBF_NW + 8];  /* wheel length */
		} ent;
		struct {
			float    vout[TBF_BLK];
			float    va[TBF_BLK];
			float    vg[TBF_BLK];
			int32_t  vh[TBF_BLK];
			float    pe[TBF_BLK];
			float    kc[TBF_BLK];
			double   odx[TBF_BLK];
			double   odh[TBF_BLK];
			uint32_t fpd[TBF_BLK + 1];
		};
	};
};

struct RvScratch {
	double   a[2][TBF_SUB]; /* predelay output -> biquadA output */
	double   b[2][TBF_SUB]; /* tap mix -> biquadB -> asin -> biquadC output */
	double   t[8][TBF_SUB]; /* one channel's vibrato offsets */
	double   vn[2][8];      /* vibrato phases after the sub-block */
	double   fbn[2][8];     /* feedback of the sub-block's last sample */
	uint32_t fpd[2][TBF_SUB + 1];
};

struct WhScratch {
	double   ang[2][TBF_SUB];
	float    xx[TBF_SUB + 1];
	float    xf[TBF_SUB + 4];
	float    x1[TBF_SUB + 4];
	float    x2[TBF_SUB + 4];
	float    xd1[TBF_SUB + 1];
	float    xd2[TBF_SUB];
	float    rd[2][TBF_SUB];
	float    y[2][TBF_SUB];
	float    ma[3][TBF_SUB];
	float    mb[3][TBF_SUB];
	int32_t  mu[3][TBF_SUB]; /* unwrapped write slot (outpos wrap folded in) */
};

template <int W>
struct Lds {
	tbf_inst_state st;
	float          wring[4][W];
	float          bufA[TBF_BLK];
	float          bufB[TBF_BLK];
	float          bufC[TBF_BLK];
	union {
		TgScratch tg;
		RvScratch rv;
		WhScratch wh;
	} u;
	int brake;
	unsigned long long prof[TBF_PROF_SLOTS];
	unsigned long long plast;
};

/* optional stage timing (tbf_debug_profile): wave-clock cycles accumulated per mark */
#define TBF_MARK(k)                                                                      \
	do {                                                                                 \
		if (P.prof) {                                                                    \
			__syncthreads ();                                                            \
			if (threadIdx.x == 0) {                                                      \
				const unsigned long long _t = __builtin_amdgcn_s_memtime ();              \
				sm.prof[k] += _t - sm.plast;                                             \
				sm.plast = _t;                                                           \
			}                                                                            \
			__syncthreads ();                                                            \
		}                                                                                \
	} while (0)

__device__ __forceinline__ uint32_t xorshift (uint32_t s)
{
	s ^= s << 13;
	s ^= s >> 17;
	s ^= s << 5;
	return s;
}

__device__ __forceinline__ int wave_min (int v)
{
	for (int o = 32; o > 0; o >>= 1)
		v = min (v, __shfl_xor (v, o));
	return v;
}

__device__ __forceinline__ int wave_max (int v)
{
	for (int o = 32; o > 0; o >>= 1)
		v = max (v, __shfl_xor (v, o));
	return v;
}


/* Airwindows 32-bit dither term, src/overdrive.cpp:153-159 / src/reverb.cpp:775-783.
 * The reference multiplies by a long double literal; FP64 here (the
 * difference reaches the float output with probability ~1e-17 per sample). */
__device__ __forceinline__ double dither_add (double v, uint32_t fpd)
{
	int expon;
	frexpf ((float)v, &expon);
	double t = ((double)fpd - 2147483647.0) * 5.5e-36;
	t        = t * ldexp (1.0, expon + 62);
	return v + t;
}

/* fmodf (x, 1.f) (src/whirl.cpp:1436, 1458): for finite x >= 0 it is x - floorf (x),
 * which is exact (the fractional bits of x); anything else takes libm */
__device__ __forceinline__ float frac1 (float x)
{
	if (x >= 0.f && x < 16777216.f)
		return x - floorf (x);
	return fmodf (x, 1.f);
}

/* RBJ biquad, Direct Form II in float (EQ_IIR, src/whirl.cpp:1479-1485) */
__device__ __forceinline__ float eq_iir (const float* c, float& z0, float& z1, float x)
{
	float temp = x - (c[0] * z0) - (c[1] * z1);
	float y    = (temp * c[2]) + (c[3] * z0) + (c[4] * z1);
	z1         = z0;
	z0         = temp;
	return y;
}

/* ------------------------------------------------------------------ tonegen */
template <int W>
__device__ void stage_tonegen (const tbf_launch& P, Lds<W>& sm, const tbf_seg_ctl& G, const tbf_tpl_desc* T)
{
	const int        lane = threadIdx.x;
	TgScratch&       s    = sm.u.tg;
	tbf_inst_state&  st   = sm.st;
	const tbf_prog_entry* __restrict__ prog = P.prog + G.prog_off;
	const int        np   = (int)G.prog_len;
	float            sw0 = 0.f, sw1 = 0.f, vb0 = 0.f, vb1 = 0.f, pc0 = 0.f, pc1 = 0.f;

	/* core interpreter, src/tonegen.cpp:3607-3687 (wrap split folded into the index).
	 * Prologue, lane per entry: resolve the wheel's bank position and advance st.pos
	 * (each wheel appears once per program). */
	for (int e = lane; e < np; e += NL) {
		const uint32_t w   = prog[e].wheel;
		const uint32_t pos = st.pos[w];
		const uint32_t len = T->len[w];
		s.ent.base[e]      = T->off[w] + pos;
		s.ent.lim[e]       = len - pos;
		s.ent.len[e]       = len;
		st.pos[w]          = (len < pos + TBF_BLK) ? pos + TBF_BLK - len : pos + TBF_BLK;
	}
	__syncthreads ();
	/* main loop in program order (the adds keep the reference's order); unrolled so
	 * several entries' wave loads are in flight together */
#pragma unroll 4
	for (int e = 0; e < np; e++) {
		const tbf_prog_entry E    = prog[e];
		const uint32_t       base = s.ent.base[e];
		const uint32_t       lim  = s.ent.lim[e];
		const uint32_t       len  = s.ent.len[e];
		const uint32_t       i0   = (uint32_t)lane < lim ? base + lane : base + lane - len;
		const uint32_t       i1   = (uint32_t)(lane + NL) < lim ? base + lane + NL : base + lane + NL - len;
		const float          x0   = P.bank[i0];
		const float          x1   = P.bank[i1];
		float       a0, a1, b0, b1, c0, c1;
		if (E.env) {
			const float* ep = (E.env == 1 ? T->attackEnv[E.row] : T->releaseEnv[E.row]);
			const float  e0 = ep[lane], e1 = ep[lane + NL];
			const float  ds = E.nsg - E.sg, dv = E.nvg - E.vg, dp = E.npg - E.pg;
			a0 = x0 * (E.sg + (e0 * ds));
			a1 = x1 * (E.sg + (e1 * ds));
			b0 = x0 * (E.vg + (e0 * dv));
			b1 = x1 * (E.vg + (e1 * dv));
			c0 = x0 * (E.pg + (e0 * dp));
			c1 = x1 * (E.pg + (e1 * dp));
		} else {
			a0 = x0 * E.sg;
			a1 = x1 * E.sg;
			b0 = x0 * E.vg;
			b1 = x1 * E.vg;
			c0 = x0 * E.pg;
			c1 = x1 * E.pg;
		}
		if (e == 0) {
			sw0 = a0; sw1 = a1; vb0 = b0; vb1 = b1; pc0 = c0; pc1 = c1;
		} else {
			sw0 = sw0 + a0; sw1 = sw1 + a1; vb0 = vb0 + b0; vb1 = vb1 + b1; pc0 = pc0 + c0; pc1 = pc1 + c1;
		}
	}
	__syncthreads (); /* the entry table is overwritten below */
	s.swl[lane] = sw0; s.swl[lane + NL] = sw1;
	s.vin[lane] = vb0; s.vin[lane + NL] = vb1;
	s.prc[lane] = pc0; s.prc[lane + NL] = pc1;
	__syncthreads ();

	const uint32_t routing = G.routing;
	TBF_MARK (0);
	/* vibrato scanner, src/vibrato.cpp:365-411 */
	if (routing & 0x03) {
		const uint32_t* otab   = P.vibTab + 2048u * G.vibTable;
		const uint32_t  out0   = st.outPos;
		const uint32_t  stat0  = st.stator;
		const float     fnorm  = (float)(1.0 / 65536.0);
		for (int k = 0; k < 2; k++) {
			const int      n   = lane + k * NL;
			const uint32_t op  = (out0 + n) & 0x3FFu;
			const uint32_t sn  = (stat0 + (uint32_t)n * P.statorInc) & 0x07ffffffu;
			const uint32_t j   = ((op << 16) + otab[sn >> 16]) & 0x03FFFFFFu;
			const int      h   = (int)(j >> 16);
			const float    f   = fnorm * ((float)(j & 0xFFFF));
			const float    x   = s.vin[n];
			const float    g   = f * x;
			s.va[n] = x - g;
			s.vg[n] = g;
			s.vh[n] = n + (int)(((uint32_t)h - op) & 0x3FFu); /* slot offset from out0 */
		}
		__syncthreads ();
		/* ordered gather: slot W_o collects, in sample order, x-g from samples with
		 * H==W_o and g from samples with H+1==W_o; valid while H is non-decreasing and
		 * within 32 ahead (checked; lane 0 replays serially otherwise) */
		int bad = 0, dmn = 1 << 20, dmx = -(1 << 20);
		for (int k = 0; k < 2; k++) {
			const int n  = lane + k * NL;
			const int d  = s.vh[n] - n;
			if (d < 1 || d > 31) bad = 1;
			if (n > 0 && s.vh[n] < s.vh[n - 1]) bad = 1;
			dmn = min (dmn, d);
			dmx = max (dmx, d);
		}
		bad = __any (bad);
		dmn = wave_min (dmn);
		dmx = wave_max (dmx);
		if (!bad) {
			/* sample m reaches slot wo iff m + d_m is wo or wo - 1: m in [wo-1-dmax, wo-dmin] */
			for (int wo = lane; wo < TBF_BLK + 32; wo += NL) {
				const uint32_t slot = (out0 + wo) & (TBF_VRING - 1);
				float          v    = st.vring[slot];
				const int      m0   = wo - 1 - dmx < 0 ? 0 : wo - 1 - dmx;
				const int      m1   = wo - dmn > TBF_BLK - 1 ? TBF_BLK - 1 : wo - dmn;
				for (int m = m0; m <= m1; m++) {
					const int hm = s.vh[m];
					if (hm == wo)
						v += s.va[m];
					else if (hm + 1 == wo)
						v += s.vg[m];
				}
				if (wo < TBF_BLK) {
					const float x = s.vin[wo];
					s.vout[wo]    = G.vibMixed ? (x + v) * (float)0.7071067811865475 : v;
					st.vring[slot] = 0.f;
				} else {
					st.vring[slot] = v;
				}
			}
		} else {
			if (lane == 0) {
				atomicOr (P.errFlags, 1u);
				for (int n = 0; n < TBF_BLK; n++) {
					const uint32_t op = (out0 + n) & 0x3FFu;
					const int      h  = (int)((op + (uint32_t)(s.vh[n] - n)) & 0x3FFu);
					const int      k2 = (h + 1) & 0x3FF;
					st.vring[h & (TBF_VRING - 1)] += s.va[n];
					st.vring[k2 & (TBF_VRING - 1)] += s.vg[n];
					const float x = s.vin[n];
					const float v = st.vring[op & (TBF_VRING - 1)];
					s.vout[n]     = G.vibMixed ? (x + v) * (float)0.7071067811865475 : v;
					st.vring[op & (TBF_VRING - 1)] = 0.f;
				}
			}
		}
		__syncthreads ();
		if (lane == 0) {
			st.outPos = (out0 + TBF_BLK) & 0x3FFu;
			st.stator = (stat0 + (uint32_t)TBF_BLK * P.statorInc) & 0x07ffffffu;
		}
	}

	TBF_MARK (1);
	/* mixdown, src/tonegen.cpp:3712-3777: the two per-sample gain chases run as
	 * independent chains, lane 0 keyCompLevel += delta, lane 1 percEnvGain *= decay */
	if (lane < 2) {
		const float keyCompDelta = (G.keyCompTarget - st.keyCompLevel) / (float)TBF_BLK;
		const bool  perc         = (routing & 0x0C) != 0;
		const float dec          = G.percEnvGainDecay;
		float       v            = lane == 0 ? st.keyCompLevel : st.percEnvGain;
		float*      out          = lane == 0 ? s.kc : s.pe;
		for (int i0 = 0; i0 < TBF_BLK; i0 += 8) {
			float o[8];
#pragma unroll
			for (int k = 0; k < 8; k++) {
				o[k]           = v;
				const float va = v + keyCompDelta;
				const float vm = perc ? v * dec : v;
				v              = lane == 0 ? va : vm;
			}
#pragma unroll
			for (int k = 0; k < 8; k++)
				out[i0 + k] = o[k];
		}
		if (lane == 0)
			st.keyCompLevel = v;
		else
			st.percEnvGain = G.resetPercAtEnd ? G.percEnvGainReset : v;
	}
	__syncthreads ();
	for (int k = 0; k < 2; k++) {
		const int   n = lane + k * NL;
		const float x = s.swl[n];
		float       y;
		if (routing & 0x0C) {
			/* HIPASS_PERCUSSION first difference, tonegen.cpp:3719-3731 */
			const float p = (n == 0 ? st.pz : s.prc[n - 1]) - s.prc[n];
			if (routing & 0x03)
				y = (G.outputGain * s.kc[n] * ((x + s.vout[n]) + (p * s.pe[n])));
			else
				y = (G.outputGain * s.kc[n] * (x + (p * s.pe[n])));
		} else if (routing & 0x03) {
			y = (G.swellPedalGain * s.kc[n] * (x + s.vout[n]));
		} else {
			y = (G.swellPedalGain * s.kc[n] * x);
		}
		sm.bufA[n] = y;
	}
	__syncthreads ();
	if (lane == 0 && (routing & 0x0C))
		st.pz = s.prc[TBF_BLK - 1];
	__syncthreads ();
	TBF_MARK (2);
}

/* ------------------------------------------------------------------ overdrive */
template <int W>
__device__ void stage_overdrive (const tbf_launch& P, Lds<W>& sm, const tbf_seg_ctl& G)
{
	const int       lane = threadIdx.x;
	TgScratch&      s    = sm.u.tg;
	tbf_inst_state& st   = sm.st;
	if (G.odClean) {
		sm.bufB[lane]      = sm.bufA[lane];
		sm.bufB[lane + NL] = sm.bufA[lane + NL];
		__syncthreads ();
		return;
	}
	/* src/overdrive.cpp:89-168; serial: xorshift sequence + alternating one-pole HPF */
	{
		/* xorshift dither sequence F[0..128] on the scalar unit, written into lanes */
		uint32_t f  = __builtin_amdgcn_readfirstlane (st.odFpd);
		const uint32_t f0 = f;
		uint32_t lo = 0, hi = 0;
		for (int i = 0; i < NL; i++) {
			f  = xorshift (f);
			lo = (lane == i) ? f : lo;
		}
		for (int i = 0; i < NL; i++) {
			f  = xorshift (f);
			hi = (lane == i) ? f : hi;
		}
		s.fpd[lane + 1]      = lo;
		s.fpd[lane + 1 + NL] = hi;
		if (lane == 0) {
			s.fpd[0] = f0;
			st.odFpd = f;
		}
	}
	__syncthreads ();
	for (int k = 0; k < 2; k++) { /* denormal guard, dry copy */
		const int n = lane + k * NL;
		double    x = (double)sm.bufA[n];
		if (fabs (x) < 1.18e-23)
			x = s.fpd[n] * 1.18e-17;
		s.odx[n] = x;
	}
	__syncthreads ();
	if (lane < 2) {
		/* alternating one-pole HPF (fpFlip): lane 0 carries iirSampleA over the samples it
		 * owns, lane 1 iirSampleB over the others; 128 samples keep fpFlip unchanged */
		const int    start = ((lane == 0) == (st.fpFlip != 0)) ? 0 : 1;
		const double a     = G.odIir;
		double       iir   = lane == 0 ? st.iirA : st.iirB;
		for (int i0 = 0; i0 < TBF_BLK / 2; i0 += 8) {
			double xv[8];
#pragma unroll
			for (int k = 0; k < 8; k++)
				xv[k] = s.odx[start + 2 * (i0 + k)];
#pragma unroll
			for (int k = 0; k < 8; k++) {
				iir                           = (iir * (1.0 - a)) + (xv[k] * a);
				s.odh[start + 2 * (i0 + k)] = xv[k] - iir;
			}
		}
		if (lane == 0)
			st.iirA = iir;
		else
			st.iirB = iir;
	}
	__syncthreads ();
	TBF_MARK (3);
	for (int k = 0; k < 2; k++) {
		const int n   = lane + k * NL;
		double    x   = s.odh[n];
		double    dry = s.odx[n];
		double    br;
		for (int c = 0; c < G.odIter; c++) {
			br = fabs (x) * 1.57079633;
			if (br > 1.57079633)
				br = 1.57079633;
			br = sin (br);
			x  = (x > 0.0) ? br : -br;
		}
		br = fabs (x) * 1.57079633;
		if (br > 1.57079633)
			br = 1.57079633;
		br = G.odDensityPos ? sin (br) : 1 - cos (br);
		if (x > 0)
			x = (x * (1 - G.odOut)) + (br * G.odOut);
		else
			x = (x * (1 - G.odOut)) - (br * G.odOut);
		if (G.odOutput < 1.0)
			x *= G.odOutput;
		if (G.odWet < 1.0)
			x = (dry * G.odDry) + (x * G.odWet);
		x = dither_add (x, s.fpd[n + 1]);
		sm.bufB[n] = (float)x;
	}
	__syncthreads ();
	TBF_MARK (4);
}

/* ------------------------------------------------------------------ reverb */

/* Serial IIR chains of one sub-block on lanes 0..nch-1: lane j runs the biquad
 * coefficient set q[j] with state (s7, s8) over 64 samples of its LDS row, in place. */
__device__ __forceinline__ void rv_chains (const tbf_inst_const& K, tbf_inst_state& st, double* row, int q, int c)
{
	const double* cf = K.bq[q];
	const double  c0 = cf[0], c1 = cf[1], c2 = cf[2], c3 = cf[3], c4 = cf[4];
	double        s7 = st.bq[q][2 * c], s8 = st.bq[q][2 * c + 1];
	for (int i0 = 0; i0 < TBF_SUB; i0 += 8) {
		double xv[8];
#pragma unroll
		for (int k = 0; k < 8; k++)
			xv[k] = row[i0 + k];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const double x = xv[k];
			const double t = (x * c0) + s7;
			s7             = (x * c1) - (t * c3) + s8;
			s8             = (x * c2) - (t * c4);
			row[i0 + k]    = t;
		}
	}
	st.bq[q][2 * c]     = s7;
	st.bq[q][2 * c + 1] = s8;
}

/* b_reverb::reverb (src/reverb.cpp:274-794), 64-sample sub-blocks, lane = sample.
 * All 13 rings are >= 560 samples long (the reference's fixed A..F settings), so every
 * ring read of a sub-block precedes the ring writes of that sub-block.  Serial parts:
 * the two dither sequences (lanes 0,1); biquadA (predelay output) and biquadB (tap mix)
 * of both channels together on lanes 0..3 -- their inputs are known once the reads are
 * done; biquadC on lanes 0,1. */
template <int W>
__device__ void stage_reverb (const tbf_launch& P, Lds<W>& sm, const tbf_seg_ctl& G, const tbf_inst_const& K,
                              double* __restrict__ slab)
{
	const int       lane = threadIdx.x;
	RvScratch&      s    = sm.u.rv;
	tbf_inst_state& st   = sm.st;
	const double    wet  = G.rvWet;

#pragma unroll 1
	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const int n = lane; /* sample within the sub-block */
		/* dither sequences (src/reverb.cpp:775-783) on the scalar unit, into lanes */
		{
			uint32_t fL = __builtin_amdgcn_readfirstlane (st.fpdL);
			uint32_t fR = __builtin_amdgcn_readfirstlane (st.fpdR);
			const uint32_t gL = fL, gR = fR;
			uint32_t nL = 0, nR = 0;
			for (int i = 0; i < TBF_SUB; i++) {
				fL = xorshift (fL);
				fR = xorshift (fR);
				nL = (lane == i) ? fL : nL;
				nR = (lane == i) ? fR : nR;
			}
			s.fpd[0][lane + 1] = nL;
			s.fpd[1][lane + 1] = nR;
			__syncthreads (); /* all lanes have read st.fpdL/R */
			if (lane == 0) {
				s.fpd[0][0] = gL;
				s.fpd[1][0] = gR;
				st.fpdL     = fL;
				st.fpdR     = fR;
			}
		}
		TBF_MARK (5);
		const double inS = (double)sm.bufB[sb * TBF_SUB + n];
		/* ---- predelay M (line 12) ---- */
		const int dM  = K.delay[12];
		const int cMn = cnt_adv (st.count[12], dM, n);     /* write slot */
		const int cMr = cnt_adv (st.count[12], dM, n + 1); /* read slot  */
		double*   mL  = slab + K.ringOff[12];
		double*   mR  = slab + K.ringOff[13 + 12];
		s.a[0][n]     = mL[cMr];
		s.a[1][n]     = mR[cMr];
		/* ---- allpass reads (lines 8..11) ---- */
		double apOld[2][4];
		int    apW[4];
		for (int l = 8; l < 12; l++) {
			const int d  = K.delay[l];
			const int cr = cnt_adv (st.count[l], d, n + 1);
			apW[l - 8]   = cnt_adv (st.count[l], d, n);
			apOld[0][l - 8] = slab[K.ringOff[l] + cr];
			apOld[1][l - 8] = slab[K.ringOff[13 + l] + cr];
		}
		/* ---- delay-line taps (lines 0..7) with the vibrato offsets; Householder
		 * feedback and tap mix (src/reverb.cpp:479-560, 686-724) ---- */
		double fb[2][8];
		for (int c = 0; c < 2; c++) {
			/* pass 1: vibrato phases and offsets (one sin per line) -> LDS */
#pragma unroll 1
			for (int l = 0; l < 8; l++) {
				const double v0 = st.vib[c][l], dl = K.vibDelta[l];
				double       D, v;
				if (phase_run (v0, dl, TBF_SUB, D)) {
					v = v0 + (double)(n + 1) * D;
				} else {
					v = v0;
					for (int i = 0; i <= n; i++)
						v += dl;
				}
				s.t[l][n] = (sin (v) + 1.0) * K.vibDepth;
				if (n == TBF_SUB - 1)
					s.vn[c][l] = v;
			}
			/* pass 2: all 16 tap loads of the channel in flight together */
			double r0[8], r1[8], fr[8];
#pragma unroll
			for (int l = 0; l < 8; l++) {
				const int     d   = K.delay[l];
				const int     cn  = cnt_adv (st.count[l], d, n + 1);
				const double  off = s.t[l][n];
				const int     wk  = (int)(cn + off);
				const int     w0  = wk - ((wk > d) ? d + 1 : 0);
				const int     w1  = wk + 1 - ((wk + 1 > d) ? d + 1 : 0);
				const double* a   = slab + K.ringOff[c * 13 + l];
				fr[l]             = off - floor (off);
				r0[l]             = a[w0];
				r1[l]             = a[w1];
			}
			double I[8];
#pragma unroll
			for (int l = 0; l < 8; l++) {
				double x = (r0[l] * (1 - fr[l]));
				x += (r1[l] * fr[l]);
				I[l] = ((1.0 - K.blend) * x) + (r0[l] * K.blend);
			}
			I[0]     = (I[0] * K.oneMinusAbsCm) + (I[4] * K.crossmod);
			I[4]     = (I[4] * K.oneMinusAbsCm) + (I[0] * K.crossmod);
			fb[c][0] = (I[0] - (I[1] + I[2] + I[3])) * K.regen;
			fb[c][1] = (I[1] - (I[0] + I[2] + I[3])) * K.regen;
			fb[c][2] = (I[2] - (I[0] + I[1] + I[3])) * K.regen;
			fb[c][3] = (I[3] - (I[0] + I[1] + I[2])) * K.regen;
			fb[c][4] = (I[4] - (I[5] + I[6] + I[7])) * K.regen;
			fb[c][5] = (I[5] - (I[4] + I[6] + I[7])) * K.regen;
			fb[c][6] = (I[6] - (I[4] + I[5] + I[7])) * K.regen;
			fb[c][7] = (I[7] - (I[4] + I[5] + I[6])) * K.regen;
			s.b[c][n] = (I[0] + I[1] + I[2] + I[3] + I[4] + I[5] + I[6] + I[7]) / 8.0;
		}
		TBF_MARK (6);
		__syncthreads (); /* all ring reads of the sub-block are complete */
		if (lane < 16)
			st.vib[lane >> 3][lane & 7] = s.vn[lane >> 3][lane & 7];
		for (int c = 0; c < 2; c++) {
			double x = inS;
			if (fabs (x) < 1.18e-23)
				x = s.fpd[c][n] * 1.18e-17;
			(c ? mR : mL)[cMn] = x;
		}
		/* ---- biquadA (predelay out) and biquadB (tap mix), both channels, lanes 0..3 ---- */
		if (lane < 4)
			rv_chains (K, st, lane < 2 ? s.a[lane] : s.b[lane - 2], lane >> 1, lane & 1);
		__syncthreads ();
		TBF_MARK (7);
		/* ---- allpasses and delay-line writes; clamp + asin of the biquadB output ---- */
		static const int srcAp[8] = {3, 2, 1, 0, 0, 1, 2, 3};
		for (int c = 0; c < 2; c++) {
			const double a0 = sin (s.a[c][n] * wet);
			double       ap[4];
			for (int l = 0; l < 4; l++) {
				double a = a0;
				a -= apOld[c][l] * 0.5;
				slab[K.ringOff[c * 13 + 8 + l] + apW[l]] = a;
				a *= 0.5;
				a += apOld[c][l];
				ap[l] = a;
			}
			for (int l = 0; l < 8; l++) {
				double prev = __shfl_up (fb[c][l], 1);
				if (lane == 0)
					prev = st.fb[c][l];
				slab[K.ringOff[c * 13 + l] + cnt_adv (st.count[l], K.delay[l], n)] = ap[srcAp[l]] + prev;
				if (lane == NL - 1)
					s.fbn[c][l] = fb[c][l];
			}
			double y = s.b[c][n];
			if (y > 1.0) y = 1.0;
			if (y < -1.0) y = -1.0;
			s.b[c][n] = asin (y);
		}
		__syncthreads ();
		if (lane < 16)
			st.fb[lane >> 3][lane & 7] = s.fbn[lane >> 3][lane & 7];
		TBF_MARK (8);
		/* ---- biquadC, lanes 0,1 ---- */
		if (lane < 2)
			rv_chains (K, st, s.b[lane], 2, lane);
		__syncthreads ();
		TBF_MARK (9);
		double o[2];
		for (int c = 0; c < 2; c++) {
			double x = s.b[c][n];
			if (wet != 1.0) {
				double dry = inS;
				if (fabs (dry) < 1.18e-23)
					dry = s.fpd[c][n] * 1.18e-17;
				x += (dry * (1.0 - wet));
			}
			o[c] = dither_add (x, s.fpd[c][n + 1]);
		}
		sm.bufC[sb * TBF_SUB + n] = (float)(0.7071067811865476 * (o[0] + o[1]));
		__syncthreads ();
		if (lane < 13)
			st.count[lane] = cnt_adv (st.count[lane], K.delay[lane], TBF_SUB);
		__syncthreads ();
		TBF_MARK (10);
	}
}

/* ------------------------------------------------------------------ whirl */
__device__ void whirl_speed (tbf_inst_state& st, const tbf_inst_const& K, int revOpt, int& brake)
{
	/* useRevOption (src/whirl.cpp:174-196) for an event landing before this block */
	if (revOpt >= 0) {
		const int i   = revOpt % 9;
		st.hornTarget = K.revHorn[i];
		st.drumTarget = K.revDrum[i];
		if (st.hornIncr < st.hornTarget)
			st.hornAcDc = 1;
		else if (st.hornTarget < st.hornIncr)
			st.hornAcDc = -1;
		if (st.drumIncr < st.drumTarget)
			st.drumAcDc = 1;
		else if (st.drumTarget < st.drumIncr)
			st.drumAcDc = -1;
	}
	/* src/whirl.cpp:1219-1374 */
	if (st.hornAcDc) {
		int flywheel = 0;
		if (K.hnBrakePos > 0 && st.hornTarget == 0 && st.hornIncr > 0 && st.hornIncr < K.hnHardstop) {
			const double targetPos = fmod (1.25 - K.hnBrakePos, 1.0);
			if (fabs (st.hornAngle - targetPos) < (2.0 / 16384)) {
				st.hornAngle = targetPos;
				st.hornIncr  = 0;
			} else {
				const float diffinc = (float)(fmod (1. + targetPos - st.hornAngle, 1.0) / (float)TBF_BLK);
				if (st.hornIncr > diffinc)
					st.hornIncr = diffinc;
				else if (st.hornIncr < K.minspeed)
					st.hornIncr = K.minspeed;
				flywheel = 1;
			}
		}
		if (!flywheel) {
			const double l = st.hornAcDc > 0 ? K.lAcc[0] : K.lAcc[1];
			st.hornIncr += (1 - l) * (st.hornTarget - st.hornIncr);
		}
		if (fabs (st.hornTarget - st.hornIncr) < K.deadzone) {
			st.hornAcDc = 0;
			st.hornIncr = st.hornTarget;
		}
	}
	if (st.drumAcDc) {
		int flywheel = 0;
		if (K.drBrakePos > 0 && st.drumTarget == 0 && st.drumIncr > 0 && st.drumIncr < K.drHardstop) {
			const double targetPos = fmod (K.drBrakePos + .75, 1.0);
			if (fabs (st.drumAngle - targetPos) < (2.0 / 16384)) {
				st.drumAngle = targetPos;
				st.drumIncr  = 0;
			} else {
				const float diffinc = (float)(fmod (1. + targetPos - st.drumAngle, 1.0) / (float)TBF_BLK);
				if (st.drumIncr > diffinc)
					st.drumIncr = diffinc;
				else if (st.drumIncr < K.minspeed)
					st.drumIncr = K.minspeed;
				flywheel = 1;
			}
		}
		if (!flywheel) {
			const double l = st.drumAcDc > 0 ? K.lAcc[2] : K.lAcc[3];
			st.drumIncr += (1 - l) * (st.drumTarget - st.drumIncr);
		}
		if (fabs (st.drumTarget - st.drumIncr) < K.deadzone) {
			st.drumAcDc = 0;
			st.drumIncr = st.drumTarget;
		}
	}
	brake = 0;
	if (K.hnBrakePos > 0) {
		const double targetPos = fmod (1.25 - K.hnBrakePos, 1.0);
		if (!st.hornAcDc && st.hornIncr == 0 && st.hornAngle != targetPos) {
			brake |= 1;
			if (fabs (st.hornAngle - targetPos) < (2.0 / 16384)) {
				st.hornAngle = targetPos;
			} else {
				st.hornIncr = fmod (1. + targetPos - st.hornAngle, 1.0) / (float)TBF_BLK;
				if (st.hornIncr > K.hnLimit)
					st.hornIncr = K.hnLimit;
			}
		}
	}
	if (K.drBrakePos > 0) {
		const double targetPos = fmod (K.drBrakePos + .75, 1.0);
		if (!st.drumAcDc && st.drumIncr == 0 && st.drumAngle != targetPos) {
			brake |= 2;
			if (fabs (st.drumAngle - targetPos) < (2.0 / 16384)) {
				st.drumAngle = targetPos;
			} else {
				st.drumIncr = fmod (1. + targetPos - st.drumAngle, 1.0) / (float)TBF_BLK;
				if (st.drumIncr > K.drLimit)
					st.drumIncr = K.drLimit;
			}
		}
	}
}


/* Ordered ring accumulation of one 64-sample sub-block (HN_MOTION / DR_MOTION adds,
 * src/whirl.cpp:1432-1469).  The reference adds, sample by sample and motion by motion
 * in source order, a into slot U and b into slot U+1.  Per slot this is a sequence of
 * float adds whose order must be kept; it is rebuilt lane-parallel:
 *   - a motion's slot U_n is non-decreasing in n with steps 0..2 and stays within 2 of
 *     U_0 + n, so slot t receives its a/b terms from samples n in [t-U_0-4, t-U_0+3],
 *     in sample order;
 *   - inside one ring the motion with the larger spacing is >= 2 slots ahead of the
 *     next at every sample, so every slot it shares with that motion got that motion's
 *     terms from earlier samples: running the motions as passes, farthest first,
 *     reproduces the per-slot order.
 * Both properties are checked per ring and sub-block (wave vote); when either fails the
 * serial replay runs instead, so the result is bit-identical in all cases.  s.mu/ma/mb
 * hold the ring's three motions in source order (q = 0, 1, 2 -> motion (r&1) + 2q). */
template <int W>
__device__ void ring_accumulate (float* ring, WhScratch& s, int lane)
{
	const uint32_t WM = (uint32_t)W - 1u;
	int ok = 1;
	for (int q = 0; q < 3; q++) {
		const int u  = s.mu[q][lane];
		const int u0 = s.mu[q][0];
		const int up = lane ? s.mu[q][lane - 1] : u;
		const int dv = u - u0 - lane;
		if (u - up < 0 || u - up > 2 || dv < -2 || dv > 2)
			ok = 0;
		if (q < 2 && u + 2 > s.mu[q + 1][lane])
			ok = 0;
	}
	if (__all (ok)) {
		for (int q = 2; q >= 0; q--) { /* farthest motion first */
			const int u0 = s.mu[q][0];
			const int ns = s.mu[q][TBF_SUB - 1] + 2 - u0; /* slots u0 .. U_63+1 (<= 67) */
			for (int o = lane; o < ns; o += NL) {
				/* slot t = u0 + o takes terms from samples o-3 .. o+2 (|U_m - u0 - m| <= 2) */
				const int t = u0 + o;
				int       um[6];
				float     ta[6], tb[6];
#pragma unroll
				for (int j = 0; j < 6; j++) {
					const int m  = o - 3 + j;
					const int mc = m < 0 ? 0 : (m > TBF_SUB - 1 ? TBF_SUB - 1 : m);
					um[j]        = (m == mc) ? s.mu[q][mc] : INT32_MIN;
					ta[j]        = s.ma[q][mc];
					tb[j]        = s.mb[q][mc];
				}
				float v = ring[(uint32_t)t & WM];
#pragma unroll
				for (int j = 0; j < 6; j++) {
					if (um[j] == t - 1)
						v += tb[j];
					else if (um[j] == t)
						v += ta[j];
				}
				ring[(uint32_t)t & WM] = v;
			}
			__syncthreads ();
		}
	} else {
		/* serial replay in the reference order: sample-major, motions in source order */
		if (lane == 0) {
			for (int i = 0; i < TBF_SUB; i++) {
				for (int q = 0; q < 3; q++) {
					const uint32_t sl = (uint32_t)s.mu[q][i] & WM;
					ring[sl] += s.ma[q][i];
					ring[(sl + 1) & WM] += s.mb[q][i];
				}
			}
		}
		__syncthreads ();
	}
}

template <int W>
__device__ void stage_whirl (const tbf_launch& P, Lds<W>& sm, const tbf_seg_ctl& G, const tbf_inst_const& K,
                             int firstBlock, float* __restrict__ oL, float* __restrict__ oR)
{
	const int       lane = threadIdx.x;
	WhScratch&      s    = sm.u.wh;
	tbf_inst_state& st   = sm.st;
	const float*    hnFwd = P.whTab;
	const float*    hnBwd = P.whTab + 16384;
	const float*    drFwd = P.whTab + 2 * 16384;
	const float*    drBwd = P.whTab + 3 * 16384;
	const float*    bfw   = P.whBw;
	const float*    bbw   = P.whBw + 16384 * 5;

	if (G.whBypass) {
		/* whirlProc2 bypass (src/whirl.cpp:1197-1215) + whirlProc3 mix */
		for (int k = 0; k < 2; k++) {
			const int   n = lane + k * NL;
			const float x = sm.bufC[n];
			oL[n] = x * K.mic[0] + x * K.mic[1] + 0.f * K.mic[2] + 0.f * K.mic[3];
			oR[n] = x * K.mic[4] + x * K.mic[5] + 0.f * K.mic[6] + 0.f * K.mic[7];
		}
		return;
	}
	if (lane == 0) {
		int brake;
		whirl_speed (st, K, firstBlock ? G.whRevOption : -1, brake);
		sm.brake = brake;
	}
	__syncthreads ();
	TBF_MARK (11);
	const double hornIncr = st.hornIncr, drumIncr = st.drumIncr;
	const uint32_t WM     = (uint32_t)W - 1u;

#pragma unroll 1
	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const int      n      = lane;
		const uint32_t outpos = (st.outpos + (uint32_t)n) & 2047u;
		const int32_t  unwrap = (int32_t)(st.outpos + (uint32_t)n - outpos); /* 0 or 2048 */
		const float    xin    = (float)((double)sm.bufC[sb * TBF_SUB + n] + 1e-14);
		s.xx[n + 1]           = xin;
		if (lane == 0)
			s.xx[0] = st.z[2];
		__syncthreads ();
		/* ring reads + clear at outpos: before this sub-block's writes, which land >= 79
		 * slots ahead (src/whirl.cpp:1585-1600) */
		const uint32_t o   = outpos & WM;
		const float    hlv = sm.wring[0][o], hrv = sm.wring[1][o];
		s.rd[0][n]         = sm.wring[2][o];
		s.rd[1][n]         = sm.wring[3][o];
		sm.wring[0][o]     = 0.f;
		sm.wring[1][o]     = 0.f;
		sm.wring[2][o]     = 0.f;
		sm.wring[3][o]     = 0.f;
		if (lane < 4) {
			const int i = lane;
			s.xf[i] = st.adx[0][(st.adi[0] + 3 - i) & 7];
			s.x1[i] = st.adx[1][(st.adi[1] + 3 - i) & 7];
			s.x2[i] = st.adx[2][(st.adi[2] + 3 - i) & 7];
		}
		__syncthreads ();
		/* independent serial biquads as lane chains: lane 0 horn filter A (hafw), lanes
		 * 1, 2 drum shelves (drfL, drfR); then lane 0 horn filter B (hbfw) while lanes 1, 2
		 * step the rotor angles */
		if (lane < 3) {
			const float* c  = lane == 0 ? K.hafw : K.drf;
			const int    fi = lane == 0 ? 0 : lane + 1;
			const float* in = lane == 0 ? s.xx + 1 : s.rd[lane - 1];
			float*       ou = lane == 0 ? s.xf + 4 : s.y[lane - 1];
			float        z0 = st.fz[fi][0], z1 = st.fz[fi][1];
			for (int i0 = 0; i0 < TBF_SUB; i0 += 8) {
				float xv[8];
#pragma unroll
				for (int k = 0; k < 8; k++)
					xv[k] = in[i0 + k];
#pragma unroll
				for (int k = 0; k < 8; k++)
					ou[i0 + k] = eq_iir (c, z0, z1, xv[k]);
			}
			st.fz[fi][0] = z0;
			st.fz[fi][1] = z1;
		}
		if (lane == 0) {
			float  z0 = st.fz[1][0], z1 = st.fz[1][1];
			float* io = s.xf + 4;
			for (int i0 = 0; i0 < TBF_SUB; i0 += 8) {
				float xv[8];
#pragma unroll
				for (int k = 0; k < 8; k++)
					xv[k] = io[i0 + k];
#pragma unroll
				for (int k = 0; k < 8; k++)
					io[i0 + k] = eq_iir (K.hbfw, z0, z1, xv[k]);
			}
			st.fz[1][0] = z0;
			st.fz[1][1] = z1;
		} else if (lane < 3) {
			double       a   = lane == 1 ? st.hornAngle : st.drumAngle;
			const double inc = lane == 1 ? hornIncr : drumIncr;
			for (int i0 = 0; i0 < TBF_SUB; i0 += 8) {
				double av[8];
#pragma unroll
				for (int k = 0; k < 8; k++) {
					av[k] = a;
					a     = wrap1 (a + inc);
				}
#pragma unroll
				for (int k = 0; k < 8; k++)
					s.ang[lane - 1][i0 + k] = av[k];
			}
			if (lane == 1) st.hornAngle = a; else st.drumAngle = a;
		}
		__syncthreads ();
		TBF_MARK (12);
		/* reflection filters FILTER_C (src/whirl.cpp:1472-1477), lane-parallel */
		const float xf   = s.xf[n + 4];
		const float xfp  = n == 0 ? st.z[0] : s.xf[n + 3];
		const float x1v  = (float)((0.4 * xf) + (0.4 * xfp));
		s.x1[n + 4]      = x1v;
		const float xdp  = s.xx[n];
		const float xd1v = (float)((0.4 * xin) + (0.4 * xdp));
		s.xd1[n + 1]     = xd1v;
		if (lane == 0)
			s.xd1[0] = st.z[3];
		__syncthreads ();
		const float x1p  = n == 0 ? st.z[1] : s.x1[n + 3];
		const float x2v  = (float)((0.4 * x1v) + (0.4 * x1p));
		s.x2[n + 4]      = x2v;
		const float xd2v = (float)((0.4 * xd1v) + (0.4 * s.xd1[n]));
		__syncthreads ();

		TBF_MARK (13);
		TBF_MARK (14);
		/* ---- per ring (HL, HR, DL, DR): its three motions, then the ordered adds ---- */
		const double ha = s.ang[0][n];
		const double da = s.ang[1][n];
#pragma unroll 1
		for (int r = 0; r < 4; r++) {
			for (int q = 0; q < 3; q++) {
				const int p = (r & 1) + 2 * q;
				const bool fwd = (p == 0 || p == 3 || p == 4);
				float xa, t;
				if (r < 2) {
					/* HN_MOTION, src/whirl.cpp:1432-1453 */
					const float*  hist = p < 2 ? s.xf : (p < 4 ? s.x1 : s.x2);
					const float*  dsp  = fwd ? hnFwd : hnBwd;
					const float*  bw   = fwd ? bbw : bfw;
					const double  ang  = ha + ((p & 1) ? K.bwAng : K.fwAng);
					const float   h1   = (float)(ang * (unsigned int)16384 + K.hornPhase[p]);
					const float   hd   = frac1 (h1);
					const unsigned hl  = ((unsigned int)floorf (h1)) & 16383u;
					const unsigned hh  = (hl + 1) & 16383u;
					const float   intp = dsp[hl] * (1.f - hd) + hd * dsp[hh];
					const unsigned kk  = ((unsigned int)roundf (h1)) & 16383u;
					t                  = K.hornSpacing[p] + intp + (float)outpos;
					const float*  b    = bw + 5 * kk;
					xa                 = b[0] * hist[n + 4];
					xa += b[1] * hist[n + 3];
					xa += b[2] * hist[n + 2];
					xa += b[3] * hist[n + 1];
					xa += b[4] * hist[n + 0];
				} else {
					/* DR_MOTION, src/whirl.cpp:1455-1469 */
					xa                = p < 2 ? xin : (p < 4 ? xd1v : xd2v);
					const float* dsp  = fwd ? drFwd : drBwd;
					const float  d1   = (float)(da * (unsigned int)16384 + K.hornPhase[p]);
					const float  dd   = frac1 (d1);
					const unsigned dl = ((unsigned int)floorf (d1)) & 16383u;
					const unsigned dh = (dl + 1) & 16383u;
					const float  intp = dsp[dl] * (1.f - dd) + dd * dsp[dh];
					t                 = K.drumSpacing[p] + intp + (float)outpos;
				}
				const float rr = floorf (t);
				const float qq = xa * (t - rr);
				s.mu[q][n]     = (int32_t)((unsigned int)rr) + unwrap;
				s.ma[q][n]     = xa - qq;
				s.mb[q][n]     = qq;
			}
			__syncthreads ();
			TBF_MARK (15);
			ring_accumulate<W> (sm.wring[r], s, lane);
			TBF_MARK (16);
		}
		/* ---- outputs (whirlProc2 outHL/outHR/outDL/outDR + whirlProc3 mix) ---- */
		{
			const float leak = xf * K.leakage;
			const float hL   = K.hornLevel * hlv + leak;
			const float hR   = K.hornLevel * hrv + leak;
			const float dL   = s.y[0][n];
			const float dR   = s.y[1][n];
			oL[sb * TBF_SUB + n] = hL * K.mic[0] + hR * K.mic[1] + dL * K.mic[2] + dR * K.mic[3];
			oR[sb * TBF_SUB + n] = hL * K.mic[4] + hR * K.mic[5] + dL * K.mic[6] + dR * K.mic[7];
		}
		/* ---- carry filter taps and histories ---- */
		if (lane == NL - 1) {
			st.z[0] = xf;
			st.z[1] = x1v;
			st.z[2] = xin;
			st.z[3] = xd1v;
		}
		__syncthreads ();
		if (lane == 0) {
			for (int j = 0; j < 8; j++) {
				st.adx[0][(st.adi[0] + j) & 7] = s.xf[4 + TBF_SUB - 1 - j];
				st.adx[1][(st.adi[1] + j) & 7] = s.x1[4 + TBF_SUB - 1 - j];
				st.adx[2][(st.adi[2] + j) & 7] = s.x2[4 + TBF_SUB - 1 - j];
			}
			st.outpos = (st.outpos + TBF_SUB) & 2047u;
		}
		__syncthreads ();
		TBF_MARK (17);
	}
	if (lane == 0) {
		/* NaN scrub, src/whirl.cpp:1622-1630 */
		for (int f = 0; f < 4; f++)
			for (int j = 0; j < 2; j++)
				if (isnan (st.fz[f][j]))
					st.fz[f][j] = 0.f;
		for (int j = 0; j < 4; j++)
			if (isnan (st.z[j]))
				st.z[j] = 0.f;
		if (sm.brake & 1) st.hornIncr = 0;
		if (sm.brake & 2) st.drumIncr = 0;
	}
	__syncthreads ();
}

/* ------------------------------------------------------------------ kernel */
template <int W>
__global__ void __launch_bounds__ (NL, (W <= 1024 ? 2 : 1))
tbf_render_kernel (const tbf_launch P, const tbf_inst_const* __restrict__ cst, const tbf_seg_ctl* __restrict__ ctl,
                   const tbf_tpl_desc* __restrict__ tpls)
{
	__shared__ Lds<W> sm;
	const int      lane = threadIdx.x;
	const uint32_t inst = blockIdx.x + P.instBase;
	if (inst >= P.nInst)
		return;
	/* read-only per-instance records come in as restrict kernel arguments so their
	 * uniform fields are fetched with scalar loads */
	const tbf_inst_const& K = cst[inst];
	const tbf_seg_ctl&    G = ctl[inst];
	const tbf_tpl_desc*   T = tpls + K.tpl;
	tbf_inst_state*       S = P.st + inst;
	float*                wr = P.wring + (size_t)inst * 4 * W;
	double*               slab = P.rslab + (size_t)inst * P.slabLen;

	if (P.prof) {
		if (lane < TBF_PROF_SLOTS)
			sm.prof[lane] = 0;
		if (lane == 0)
			sm.plast = __builtin_amdgcn_s_memtime ();
	}
	/* state -> LDS */
	{
		const uint32_t* src = (const uint32_t*)S;
		uint32_t*       dst = (uint32_t*)&sm.st;
		for (uint32_t i = lane; i < sizeof (tbf_inst_state) / 4; i += NL)
			dst[i] = src[i];
		for (uint32_t i = lane; i < 4u * W; i += NL)
			(&sm.wring[0][0])[i] = wr[i];
	}
	__syncthreads ();
	TBF_MARK (18);

	for (uint32_t blk = 0; blk < P.nBlocks; blk++) {
		stage_tonegen<W> (P, sm, G, T);
		float* oL = P.outL + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		float* oR = P.outR + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		if (P.chain == 1) {
			oL[lane]      = sm.bufA[lane];
			oL[lane + NL] = sm.bufA[lane + NL];
			oR[lane]      = sm.bufA[lane];
			oR[lane + NL] = sm.bufA[lane + NL];
			continue;
		}
		stage_overdrive<W> (P, sm, G);
		if (P.chain == 2) { /* stage tap: preamp output */
			oL[lane] = oR[lane] = sm.bufB[lane];
			oL[lane + NL] = oR[lane + NL] = sm.bufB[lane + NL];
			continue;
		}
		stage_reverb<W> (P, sm, G, K, slab);
		if (P.chain == 3) { /* stage tap: reverb output */
			oL[lane] = oR[lane] = sm.bufC[lane];
			oL[lane + NL] = oR[lane + NL] = sm.bufC[lane + NL];
			continue;
		}
		stage_whirl<W> (P, sm, G, K, blk == 0, oL, oR);
	}

	__syncthreads ();
	{
		uint32_t*       dst = (uint32_t*)S;
		const uint32_t* src = (const uint32_t*)&sm.st;
		for (uint32_t i = lane; i < sizeof (tbf_inst_state) / 4; i += NL)
			dst[i] = src[i];
		for (uint32_t i = lane; i < 4u * W; i += NL)
			wr[i] = (&sm.wring[0][0])[i];
	}
	TBF_MARK (19);
	if (P.prof && lane < TBF_PROF_SLOTS)
		P.prof[(size_t)inst * TBF_PROF_SLOTS + lane] += sm.prof[lane];
}

extern "C" int tbf_launch_render (const tbf_launch* P, hipStream_t stream)
{
	if (P->nInst == 0 || P->nBlocks == 0)
		return 0;
	dim3 grid (P->nInst), block (NL);
	switch (P->wringLen) {
		case 512: hipLaunchKernelGGL (tbf_render_kernel<512>, grid, block, 0, stream, *P, P->cst, P->ctl, P->tpls); break;
		case 1024: hipLaunchKernelGGL (tbf_render_kernel<1024>, grid, block, 0, stream, *P, P->cst, P->ctl, P->tpls); break;
		case 2048: hipLaunchKernelGGL (tbf_render_kernel<2048>, grid, block, 0, stream, *P, P->cst, P->ctl, P->tpls); break;
		default: return -22;
	}
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
