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

#define NL 64

struct TgScratch {
	float    swl[TBF_BLK];
	float    vin[TBF_BLK];
	float    prc[TBF_BLK];
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

struct RvScratch {
	double   x[2][TBF_SUB];
	double   y[2][TBF_SUB];
	double   vph[16][TBF_SUB];
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
	float    rd[4][TBF_SUB];
	float    y[2][TBF_SUB];
	float    ma[12][TBF_SUB];
	float    mb[12][TBF_SUB];
	uint16_t ms[12][TBF_SUB];
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
};

__device__ __forceinline__ uint32_t xorshift (uint32_t s)
{
	s ^= s << 13;
	s ^= s >> 17;
	s ^= s << 5;
	return s;
}

/* count after n increments of `count++; if (count < 0 || count > d) count = 0` */
__device__ __forceinline__ int cnt_adv (int c0, int d, int n)
{
	if (n == 0)
		return c0;
	if (c0 > d || c0 < 0)
		return (n - 1) % (d + 1);
	return (c0 + n) % (d + 1);
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
	const tbf_prog_entry* prog = P.prog + G.prog_off;
	const int        np   = (int)G.prog_len;
	float            sw0 = 0.f, sw1 = 0.f, vb0 = 0.f, vb1 = 0.f, pc0 = 0.f, pc1 = 0.f;

	/* core interpreter, src/tonegen.cpp:3607-3687 (wrap split folded into the index) */
	for (int e = 0; e < np; e++) {
		const tbf_prog_entry E   = prog[e];
		const uint32_t       pos = st.pos[E.wheel];
		const uint32_t       len = T->len[E.wheel];
		const float*         wv  = P.bank + T->off[E.wheel];
		uint32_t             i0  = pos + lane;
		uint32_t             i1  = pos + lane + NL;
		if (i0 >= len) i0 -= len;
		if (i1 >= len) i1 -= len;
		const float x0 = wv[i0];
		const float x1 = wv[i1];
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
		if (lane == 0)
			st.pos[E.wheel] = (len < pos + TBF_BLK) ? pos + TBF_BLK - len : pos + TBF_BLK;
	}
	s.swl[lane] = sw0; s.swl[lane + NL] = sw1;
	s.vin[lane] = vb0; s.vin[lane + NL] = vb1;
	s.prc[lane] = pc0; s.prc[lane + NL] = pc1;
	__syncthreads ();

	const uint32_t routing = G.routing;
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
		int bad = 0;
		for (int k = 0; k < 2; k++) {
			const int n  = lane + k * NL;
			const int d  = s.vh[n] - n;
			if (d < 1 || d > 31) bad = 1;
			if (n > 0 && s.vh[n] < s.vh[n - 1]) bad = 1;
		}
		bad = __any (bad);
		if (!bad) {
			for (int wo = lane; wo < TBF_BLK + 32; wo += NL) {
				const uint32_t slot = (out0 + wo) & (TBF_VRING - 1);
				float          v    = st.vring[slot];
				const int      m0   = wo - 32 < 0 ? 0 : wo - 32;
				const int      m1   = wo - 1 > TBF_BLK - 1 ? TBF_BLK - 1 : wo - 1;
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

	/* mixdown, src/tonegen.cpp:3712-3777: serial gain chases on lane 0 */
	if (lane == 0) {
		const float keyCompDelta = (G.keyCompTarget - st.keyCompLevel) / (float)TBF_BLK;
		float       kcl          = st.keyCompLevel;
		float       peg          = st.percEnvGain;
		const bool  perc         = (routing & 0x0C) != 0;
		for (int n = 0; n < TBF_BLK; n++) {
			s.kc[n] = kcl;
			s.pe[n] = peg;
			if (perc)
				peg *= G.percEnvGainDecay;
			kcl += keyCompDelta;
		}
		st.keyCompLevel = kcl;
		st.percEnvGain  = G.resetPercAtEnd ? G.percEnvGainReset : peg;
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
}

/* ------------------------------------------------------------------ overdrive */
template <int W>
__device__ void stage_overdrive (Lds<W>& sm, const tbf_seg_ctl& G)
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
	if (lane == 0) {
		uint32_t f = st.odFpd;
		s.fpd[0]   = f;
		for (int n = 0; n < TBF_BLK; n++) {
			f           = xorshift (f);
			s.fpd[n + 1] = f;
		}
		st.odFpd       = f;
		double   iirA  = st.iirA, iirB = st.iirB;
		uint32_t flip  = st.fpFlip;
		const double a = G.odIir;
		for (int n = 0; n < TBF_BLK; n++) {
			double x = (double)sm.bufA[n];
			if (fabs (x) < 1.18e-23)
				x = s.fpd[n] * 1.18e-17;
			s.odx[n] = x; /* dry sample */
			if (flip) {
				iirA = (iirA * (1.0 - a)) + (x * a);
				x -= iirA;
			} else {
				iirB = (iirB * (1.0 - a)) + (x * a);
				x -= iirB;
			}
			flip     = !flip;
			s.odh[n] = x;
		}
		st.iirA   = iirA;
		st.iirB   = iirB;
		st.fpFlip = flip;
	}
	__syncthreads ();
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
}

/* ------------------------------------------------------------------ reverb */
__device__ __forceinline__ double rv_biquad (const double* c, double& s7, double& s8, double x)
{
	/* src/reverb.cpp:361-369 with c = biquad[2..6] */
	double t = (x * c[0]) + s7;
	s7       = (x * c[1]) - (t * c[3]) + s8;
	s8       = (x * c[2]) - (t * c[4]);
	return t;
}

template <int W>
__device__ void stage_reverb (const tbf_launch& P, Lds<W>& sm, const tbf_seg_ctl& G, const tbf_inst_const& K,
                              double* __restrict__ slab)
{
	const int       lane = threadIdx.x;
	RvScratch&      s    = sm.u.rv;
	tbf_inst_state& st   = sm.st;
	const double    wet  = G.rvWet;

	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const int n = lane; /* sample within the sub-block */
		/* serial sequences: dither states (lanes 0,1) and the 16 vibrato phases
		 * (lanes 0..15, exact repeated addition, src/reverb.cpp:479-496) */
		if (lane < 2) {
			uint32_t f = lane == 0 ? st.fpdL : st.fpdR;
			s.fpd[lane][0] = f;
			for (int i = 0; i < TBF_SUB; i++) {
				f                  = xorshift (f);
				s.fpd[lane][i + 1] = f;
			}
			if (lane == 0) st.fpdL = f; else st.fpdR = f;
		}
		if (lane < 16) {
			const int    c = lane >> 3, l = lane & 7;
			double       v = st.vib[c][l];
			const double d = K.vibDelta[l];
			for (int i = 0; i < TBF_SUB; i++) {
				v += d;
				s.vph[lane][i] = v;
			}
			st.vib[c][l] = v;
		}
		__syncthreads ();

		const double inS = (double)sm.bufB[sb * TBF_SUB + n];
		double       in2[2], dry[2];
		for (int c = 0; c < 2; c++) {
			double x = inS;
			if (fabs (x) < 1.18e-23)
				x = s.fpd[c][n] * 1.18e-17;
			in2[c] = x;
			dry[c] = x;
		}
		/* ---- predelay M (line 12): read new count slot, then write ---- */
		const int dM  = K.delay[12];
		const int cMn = cnt_adv (st.count[12], dM, n);     /* write slot */
		const int cMr = cnt_adv (st.count[12], dM, n + 1); /* read slot  */
		double*   mL  = slab + K.ringOff[12];
		double*   mR  = slab + K.ringOff[13 + 12];
		const double pdL = mL[cMr], pdR = mR[cMr];
		/* ---- allpass reads (lines 8..11) ---- */
		double apOld[2][4];
		int    apW[4];
		for (int l = 8; l < 12; l++) {
			const int d  = K.delay[l];
			const int cw = cnt_adv (st.count[l], d, n);
			const int cr = cnt_adv (st.count[l], d, n + 1);
			apW[l - 8]   = cw;
			apOld[0][l - 8] = slab[K.ringOff[l] + cr];
			apOld[1][l - 8] = slab[K.ringOff[13 + l] + cr];
		}
		/* ---- delay-line reads (lines 0..7) at the incremented count + offset ---- */
		double interp[2][8];
		int    dlW[8];
		for (int l = 0; l < 8; l++) {
			const int d  = K.delay[l];
			dlW[l]       = cnt_adv (st.count[l], d, n);
			const int cn = cnt_adv (st.count[l], d, n + 1);
			for (int c = 0; c < 2; c++) {
				const double  off = (sin (s.vph[c * 8 + l][n]) + 1.0) * K.vibDepth;
				const int     wk  = (int)(cn + off);
				const int     w0  = wk - ((wk > d) ? d + 1 : 0);
				const int     w1  = wk + 1 - ((wk + 1 > d) ? d + 1 : 0);
				const double* a   = slab + K.ringOff[c * 13 + l];
				const double  fr  = off - floor (off);
				const double  r0  = a[w0];
				double        v   = (r0 * (1 - fr));
				v += (a[w1] * fr);
				interp[c][l] = ((1.0 - K.blend) * v) + (r0 * K.blend);
			}
		}
		s.x[0][n] = pdL;
		s.x[1][n] = pdR;
		__syncthreads (); /* all ring reads of the sub-block are complete */
		mL[cMn] = in2[0];
		mR[cMn] = in2[1];

		/* ---- biquadA, serial per channel ---- */
		if (lane < 2) {
			const int c  = lane;
			double    s7 = st.bq[0][2 * c], s8 = st.bq[0][2 * c + 1];
			for (int i = 0; i < TBF_SUB; i++)
				s.y[c][i] = rv_biquad (K.bq[0], s7, s8, s.x[c][i]);
			st.bq[0][2 * c]     = s7;
			st.bq[0][2 * c + 1] = s8;
		}
		__syncthreads ();
		double xs[2];
		for (int c = 0; c < 2; c++) {
			double x = s.y[c][n];
			x *= wet;
			xs[c] = sin (x);
		}
		/* ---- allpasses: compute and write ---- */
		double ap[2][4];
		for (int l = 0; l < 4; l++) {
			for (int c = 0; c < 2; c++) {
				double a = xs[c];
				a -= apOld[c][l] * 0.5;
				slab[K.ringOff[c * 13 + 8 + l] + apW[l]] = a;
				a *= 0.5;
				a += apOld[c][l];
				ap[c][l] = a;
			}
		}
		/* ---- crossmod + Householder feedback + mix (src/reverb.cpp:686-724) ---- */
		double fb[2][8], mix[2];
		for (int c = 0; c < 2; c++) {
			double* I = interp[c];
			I[0]      = (I[0] * K.oneMinusAbsCm) + (I[4] * K.crossmod);
			I[4]      = (I[4] * K.oneMinusAbsCm) + (I[0] * K.crossmod);
			fb[c][0]  = (I[0] - (I[1] + I[2] + I[3])) * K.regen;
			fb[c][1]  = (I[1] - (I[0] + I[2] + I[3])) * K.regen;
			fb[c][2]  = (I[2] - (I[0] + I[1] + I[3])) * K.regen;
			fb[c][3]  = (I[3] - (I[0] + I[1] + I[2])) * K.regen;
			fb[c][4]  = (I[4] - (I[5] + I[6] + I[7])) * K.regen;
			fb[c][5]  = (I[5] - (I[4] + I[6] + I[7])) * K.regen;
			fb[c][6]  = (I[6] - (I[4] + I[5] + I[7])) * K.regen;
			fb[c][7]  = (I[7] - (I[4] + I[5] + I[6])) * K.regen;
			mix[c]    = (I[0] + I[1] + I[2] + I[3] + I[4] + I[5] + I[6] + I[7]) / 8.0;
		}
		/* ---- delay-line writes: ap + feedback of the previous sample ---- */
		{
			static const int srcAp[8] = {3, 2, 1, 0, 0, 1, 2, 3};
			for (int c = 0; c < 2; c++)
				for (int l = 0; l < 8; l++) {
					double prev = __shfl_up (fb[c][l], 1);
					if (lane == 0)
						prev = st.fb[c][l];
					slab[K.ringOff[c * 13 + l] + dlW[l]] = ap[c][srcAp[l]] + prev;
				}
		}
		__syncthreads ();
		if (lane == NL - 1) {
			for (int c = 0; c < 2; c++)
				for (int l = 0; l < 8; l++)
					st.fb[c][l] = fb[c][l];
		}
		s.x[0][n] = mix[0];
		s.x[1][n] = mix[1];
		__syncthreads ();
		/* ---- biquadB (serial), clamp, asin, biquadC (serial) ---- */
		if (lane < 2) {
			const int c  = lane;
			double    s7 = st.bq[1][2 * c], s8 = st.bq[1][2 * c + 1];
			for (int i = 0; i < TBF_SUB; i++)
				s.y[c][i] = rv_biquad (K.bq[1], s7, s8, s.x[c][i]);
			st.bq[1][2 * c]     = s7;
			st.bq[1][2 * c + 1] = s8;
		}
		__syncthreads ();
		for (int c = 0; c < 2; c++) {
			double x = s.y[c][n];
			if (x > 1.0) x = 1.0;
			if (x < -1.0) x = -1.0;
			s.x[c][n] = asin (x);
		}
		__syncthreads ();
		if (lane < 2) {
			const int c  = lane;
			double    s7 = st.bq[2][2 * c], s8 = st.bq[2][2 * c + 1];
			for (int i = 0; i < TBF_SUB; i++)
				s.y[c][i] = rv_biquad (K.bq[2], s7, s8, s.x[c][i]);
			st.bq[2][2 * c]     = s7;
			st.bq[2][2 * c + 1] = s8;
		}
		__syncthreads ();
		double o[2];
		for (int c = 0; c < 2; c++) {
			double x = s.y[c][n];
			if (wet != 1.0)
				x += (dry[c] * (1.0 - wet));
			o[c] = dither_add (x, s.fpd[c][n + 1]);
		}
		sm.bufC[sb * TBF_SUB + n] = (float)(0.7071067811865476 * (o[0] + o[1]));
		__syncthreads ();
		if (lane == 0) {
			for (int l = 0; l < 13; l++)
				st.count[l] = cnt_adv (st.count[l], K.delay[l], TBF_SUB);
		}
		__syncthreads ();
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
	const double hornIncr = st.hornIncr, drumIncr = st.drumIncr;
	const uint32_t WM     = (uint32_t)W - 1u;

	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const int      n      = lane;
		const uint32_t outpos = (st.outpos + (uint32_t)n) & 2047u;
		const float    xin    = (float)((double)sm.bufC[sb * TBF_SUB + n] + 1e-14);
		s.xx[n + 1]           = xin;
		if (lane == 0)
			s.xx[0] = st.z[2];
		__syncthreads ();
		/* serial lanes: horn filters A,B (lane 0); rotor angles (lanes 1, 2) */
		if (lane == 0) {
			float a0 = st.fz[0][0], a1 = st.fz[0][1], b0 = st.fz[1][0], b1 = st.fz[1][1];
			for (int i = 0; i < 4; i++) {
				s.xf[i] = st.adx[0][(st.adi[0] + 3 - i) & 7];
				s.x1[i] = st.adx[1][(st.adi[1] + 3 - i) & 7];
				s.x2[i] = st.adx[2][(st.adi[2] + 3 - i) & 7];
			}
			for (int i = 0; i < TBF_SUB; i++) {
				float x = s.xx[i + 1];
				x       = eq_iir (K.hafw, a0, a1, x);
				x       = eq_iir (K.hbfw, b0, b1, x);
				s.xf[i + 4] = x;
			}
			st.fz[0][0] = a0; st.fz[0][1] = a1; st.fz[1][0] = b0; st.fz[1][1] = b1;
		} else if (lane == 1 || lane == 2) {
			double       a   = lane == 1 ? st.hornAngle : st.drumAngle;
			const double inc = lane == 1 ? hornIncr : drumIncr;
			for (int i = 0; i < TBF_SUB; i++) {
				s.ang[lane - 1][i] = a;
				a                  = fmod (a + inc, 1.0);
			}
			if (lane == 1) st.hornAngle = a; else st.drumAngle = a;
		}
		__syncthreads ();
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

		/* ---- horn motions (HN_MOTION, src/whirl.cpp:1432-1453) ---- */
		const double ha = s.ang[0][n];
		const double da = s.ang[1][n];
		for (int p = 0; p < 6; p++) {
			const float*  hist = p < 2 ? s.xf : (p < 4 ? s.x1 : s.x2);
			const float   x    = hist[n + 4];
			const bool    fwd  = (p == 0 || p == 3 || p == 4);
			const float*  dsp  = fwd ? hnFwd : hnBwd;
			const float*  bw   = fwd ? bbw : bfw;
			const double  ang  = ha + ((p & 1) ? K.bwAng : K.fwAng);
			const float   h1   = (float)(ang * (unsigned int)16384 + K.hornPhase[p]);
			const float   hd   = fmodf (h1, 1.f);
			const unsigned hl  = ((unsigned int)floorf (h1)) & 16383u;
			const unsigned hh  = (hl + 1) & 16383u;
			const float   intp = dsp[hl] * (1.f - hd) + hd * dsp[hh];
			const unsigned kk  = ((unsigned int)roundf (h1)) & 16383u;
			const float   t    = K.hornSpacing[p] + intp + (float)outpos;
			const float   r    = floorf (t);
			const float*  b    = bw + 5 * kk;
			float         xa   = b[0] * x;
			xa += b[1] * hist[n + 3];
			xa += b[2] * hist[n + 2];
			xa += b[3] * hist[n + 1];
			xa += b[4] * hist[n + 0];
			const float q = xa * (t - r);
			s.ms[p][n]    = (uint16_t)(((unsigned int)r) & WM);
			s.ma[p][n]    = xa - q;
			s.mb[p][n]    = q;
		}
		/* ---- drum motions (DR_MOTION, src/whirl.cpp:1455-1469) ---- */
		for (int p = 0; p < 6; p++) {
			const float  x    = p < 2 ? xin : (p < 4 ? xd1v : xd2v);
			const bool   fwd  = (p == 0 || p == 3 || p == 4);
			const float* dsp  = fwd ? drFwd : drBwd;
			const float  d1   = (float)(da * (unsigned int)16384 + K.hornPhase[p]);
			const float  dd   = fmodf (d1, 1.f);
			const unsigned dl = ((unsigned int)floorf (d1)) & 16383u;
			const unsigned dh = (dl + 1) & 16383u;
			const float  intp = dsp[dl] * (1.f - dd) + dd * dsp[dh];
			const float  t    = K.drumSpacing[p] + intp + (float)outpos;
			const float  r    = floorf (t);
			const float  q    = x * (t - r);
			s.ms[6 + p][n]    = (uint16_t)(((unsigned int)r) & WM);
			s.ma[6 + p][n]    = x - q;
			s.mb[6 + p][n]    = q;
		}
		/* ---- ring reads + clear at outpos (before this sub-block's writes) ---- */
		const uint32_t o = outpos & WM;
		const float    hlv = sm.wring[0][o], hrv = sm.wring[1][o];
		s.rd[2][n]         = sm.wring[2][o];
		s.rd[3][n]         = sm.wring[3][o];
		sm.wring[0][o] = 0.f;
		sm.wring[1][o] = 0.f;
		sm.wring[2][o] = 0.f;
		sm.wring[3][o] = 0.f;
		__syncthreads ();
		/* ---- serial lanes: drum shelves (0,1) and ordered ring accumulation (0..3) ---- */
		if (lane < 2) {
			float z0 = st.fz[2 + lane][0], z1 = st.fz[2 + lane][1];
			for (int i = 0; i < TBF_SUB; i++)
				s.y[lane][i] = eq_iir (K.drf, z0, z1, s.rd[2 + lane][i]);
			st.fz[2 + lane][0] = z0;
			st.fz[2 + lane][1] = z1;
		}
		if (lane < 4) {
			/* ring 0 = HL (horn 0,2,4), 1 = HR (horn 1,3,5), 2 = DL (drum 0,2,4), 3 = DR */
			float*    ring = sm.wring[lane];
			const int base = (lane < 2 ? 0 : 6) + (lane & 1);
			for (int i = 0; i < TBF_SUB; i++) {
				for (int p = base; p < base + 6; p += 2) {
					const uint32_t sl = s.ms[p][i];
					ring[sl] += s.ma[p][i];
					ring[(sl + 1) & WM] += s.mb[p][i];
				}
			}
		}
		__syncthreads ();
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
__global__ void __launch_bounds__ (NL) tbf_render_kernel (const tbf_launch P)
{
	__shared__ Lds<W> sm;
	const int      lane = threadIdx.x;
	const uint32_t inst = blockIdx.x + P.instBase;
	if (inst >= P.nInst)
		return;
	const tbf_inst_const& K = P.cst[inst];
	const tbf_seg_ctl&    G = P.ctl[inst];
	const tbf_tpl_desc*   T = P.tpls + K.tpl;
	tbf_inst_state*       S = P.st + inst;
	float*                wr = P.wring + (size_t)inst * 4 * W;
	double*               slab = P.rslab + (size_t)inst * P.slabLen;

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
		stage_overdrive<W> (sm, G);
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
}

extern "C" int tbf_launch_render (const tbf_launch* P, hipStream_t stream)
{
	if (P->nInst == 0 || P->nBlocks == 0)
		return 0;
	dim3 grid (P->nInst), block (NL);
	switch (P->wringLen) {
		case 512: hipLaunchKernelGGL (tbf_render_kernel<512>, grid, block, 0, stream, *P); break;
		case 1024: hipLaunchKernelGGL (tbf_render_kernel<1024>, grid, block, 0, stream, *P); break;
		case 2048: hipLaunchKernelGGL (tbf_render_kernel<2048>, grid, block, 0, stream, *P); break;
		default: return -22;
	}
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
