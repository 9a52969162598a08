/*
 * oracle/orc_fx.c -- TEST INFRASTRUCTURE ONLY (see orc.h).
 * Restatement of the effect stages: Airwindows Density overdrive
 * (src/overdrive.cpp), Airwindows MatrixVerb (src/reverb.cpp), the whirl
 * Leslie model (src/whirl.cpp) and the RBJ biquad designer (src/eqcomp.cpp).
 */
#include "orc_internal.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------ overdrive */

/* src/overdrive.cpp:344-378 allocPreamp (Density part) + initPreamp (583-600) */
void orc_preamp_init (struct orc_preamp* pp, orc_rand* rnd, double sr)
{
	uint32_t fpdL = 1;
	memset (pp, 0, sizeof (*pp));
	pp->A           = 0.0f;
	pp->B           = 0.0f;
	pp->C           = 1.0f;
	pp->D           = 0.5f;
	pp->fpFlip      = 1;
	while (fpdL < 16386)
		fpdL = (uint32_t)orc_rand_next (rnd) * 0xFFFFFFFFu;
	pp->fpdL        = fpdL;
	pp->isClean     = 1;
	pp->SampleRateD = sr;
}

/* src/overdrive.cpp:547-574 linseg + fsetCharacter */
void orc_preamp_set_character (struct orc_preamp* pp, float A)
{
	static const double Aval[5] = {0.0, 0.25, 0.50, 0.75, 1.00};
	static const double Cval[5] = {1.0, 0.70, 0.25, 0.15, 0.13};
	int                 i;
	pp->A = A;
	for (i = 0; i < 4; i++) {
		if (A <= Aval[i + 1]) {
			float a = (float)Aval[i], b = (float)Aval[i + 1], p = (float)Cval[i], q = (float)Cval[i + 1];
			pp->C   = p + (A - a) * (q - p) / (b - a);
			return;
		}
	}
}

/* src/overdrive.cpp:60-170 airwindows_density; 329-342 preamp */
void orc_preamp_run (struct orc_preamp* pp, const float* in1, float* out1, int sampleFrames)
{
	if (pp->isClean) {
		memcpy (out1, in1, sizeof (float) * sampleFrames);
		return;
	}
	{
		float  A = pp->A, B = pp->B, C = pp->C, D = pp->D;
		double overallscale = 1.0;
		double density, iirAmount, output, wet, dry, bridgerectifier, out, count;
		double inputSampleL, drySampleL;
		overallscale /= 44100.0;
		overallscale *= pp->SampleRateD;
		density   = A * 4.0;
		iirAmount = pow (B, 3) / overallscale;
		output    = C;
		wet       = D;
		dry       = 1.0 - wet;
		out       = fabs (density);
		density   = density * fabs (density);
		while (--sampleFrames >= 0) {
			int expon;
			inputSampleL = *in1;
			if (fabs (inputSampleL) < 1.18e-23)
				inputSampleL = pp->fpdL * 1.18e-17;
			drySampleL = inputSampleL;
			if (pp->fpFlip) {
				pp->iirSampleAL = (pp->iirSampleAL * (1.0 - iirAmount)) + (inputSampleL * iirAmount);
				inputSampleL -= pp->iirSampleAL;
			} else {
				pp->iirSampleBL = (pp->iirSampleBL * (1.0 - iirAmount)) + (inputSampleL * iirAmount);
				inputSampleL -= pp->iirSampleBL;
			}
			pp->fpFlip = !pp->fpFlip;
			count      = density;
			while (count > 1.0) {
				bridgerectifier = fabs (inputSampleL) * 1.57079633;
				if (bridgerectifier > 1.57079633)
					bridgerectifier = 1.57079633;
				bridgerectifier = sin (bridgerectifier);
				if (inputSampleL > 0.0)
					inputSampleL = bridgerectifier;
				else
					inputSampleL = -bridgerectifier;
				count = count - 1.0;
			}
			while (out > 1.0)
				out = out - 1.0;
			bridgerectifier = fabs (inputSampleL) * 1.57079633;
			if (bridgerectifier > 1.57079633)
				bridgerectifier = 1.57079633;
			if (density > 0)
				bridgerectifier = sin (bridgerectifier);
			else
				bridgerectifier = 1 - cos (bridgerectifier);
			if (inputSampleL > 0)
				inputSampleL = (inputSampleL * (1 - out)) + (bridgerectifier * out);
			else
				inputSampleL = (inputSampleL * (1 - out)) - (bridgerectifier * out);
			if (output < 1.0)
				inputSampleL *= output;
			if (wet < 1.0)
				inputSampleL = (drySampleL * dry) + (inputSampleL * wet);
			frexpf ((float)inputSampleL, &expon);
			pp->fpdL ^= pp->fpdL << 13;
			pp->fpdL ^= pp->fpdL >> 17;
			pp->fpdL ^= pp->fpdL << 5;
			/* x87 long double, exactly as the reference's 5.5e-36l literal */
			inputSampleL += ((double)(pp->fpdL) - (uint32_t)0x7fffffff) * 5.5e-36L * pow (2, expon + 62);
			*out1 = (float)inputSampleL;
			in1++;
			out1++;
		}
	}
}

/* ------------------------------------------------------------------ reverb */

/* allocated ring lengths, src/reverb.h:36-62 (A..M) */
static const int rv_alloc[13] = {8111, 7511, 7311, 6911, 6311, 6111, 5511, 4911, 4511, 4311, 3911, 3311, 3111};

/* src/reverb.cpp:81-224 b_reverb::b_reverb, 260-266 initReverb */
struct orc_reverb* orc_reverb_alloc (orc_rand* rnd, double sr)
{
	static const int    d0[13]    = {79, 73, 71, 67, 61, 59, 53, 47, 43, 41, 37, 31, 29};
	static const double depth[8]  = {0.003251, 0.002999, 0.002917, 0.002749, 0.002503, 0.002423, 0.002146, 0.002088};
	struct orc_reverb*  r         = (struct orc_reverb*)calloc (1, sizeof (*r));
	int                 c, i;
	for (c = 0; c < 2; c++)
		for (i = 0; i < 13; i++)
			r->ring[c][i] = (double*)calloc ((size_t)rv_alloc[i], sizeof (double));
	for (i = 0; i < 13; i++) {
		r->count[i] = 1;
		r->delay[i] = d0[i];
	}
	for (i = 0; i < 8; i++)
		r->depth[i] = depth[i];
	for (i = 0; i < 8; i++)
		r->vib[0][i] = orc_rand_next (rnd) - 2147483647 / 2;
	for (i = 0; i < 8; i++)
		r->vib[1][i] = orc_rand_next (rnd) - 2147483647 / 2;
	r->A    = 1.0f;
	r->B    = 0.2f;
	r->C    = 0.0f;
	r->D    = 0.0f;
	r->E    = 0.4f;
	r->F    = 0.8f;
	r->G    = 0.1f;
	r->fpdL = 1;
	while (r->fpdL < 16386)
		r->fpdL = (uint32_t)orc_rand_next (rnd) * 0xFFFFFFFFu;
	r->fpdR = 1;
	while (r->fpdR < 16386)
		r->fpdR = (uint32_t)orc_rand_next (rnd) * 0xFFFFFFFFu;
	r->SampleRateD = sr;
	return r;
}

static void rv_free (struct orc_reverb* r)
{
	int c, i;
	for (c = 0; c < 2; c++)
		for (i = 0; i < 13; i++)
			free (r->ring[c][i]);
	free (r);
}

/* biquad "like mono AU" (src/reverb.cpp:361-369, 733-741, 756-764), state at [7+2c],[8+2c] */
static inline double rv_biquad (double* bq, int c, double x)
{
	double t    = (x * bq[2]) + bq[7 + 2 * c];
	bq[7 + 2 * c] = (x * bq[3]) - (t * bq[5]) + bq[8 + 2 * c];
	bq[8 + 2 * c] = (x * bq[4]) - (t * bq[6]);
	return t;
}

static inline void rv_inc (int* count, int delay)
{
	(*count)++;
	if (*count < 0 || *count > delay)
		*count = 0;
}

/* src/reverb.cpp:274-794 b_reverb::reverb; lines A..H = 0..7, allpasses I..L = 8..11,
 * predelay M = 12.  Both channels use the mono input (in1 == in2). */
void orc_reverb_run (struct orc_reverb* r, const float* in1, float* out1, int sampleFrames)
{
	double       K, norm, vibSpeed, vibDepth, size, depthFactor, blend, crossmod, regen, wet;
	double*      bA = r->biquadA;
	double*      bB = r->biquadB;
	double*      bC = r->biquadC;
	static const int dmul[12] = {79, 73, 71, 67, 61, 59, 53, 47, 43, 41, 37, 31};
	int          i, c;

	bC[0] = bB[0] = bA[0] = ((r->A * 9000.0) + 1000.0) / r->SampleRateD;
	bA[1]                 = 1.618033988749894848204586;
	bB[1]                 = 0.618033988749894848204586;
	bC[1]                 = 0.5;
	K                     = tan (M_PI * bA[0]);
	norm                  = 1.0 / (1.0 + K / bA[1] + K * K);
	bA[2]                 = K * K * norm;
	bA[3]                 = 2.0 * bA[2];
	bA[4]                 = bA[2];
	bA[5]                 = 2.0 * (K * K - 1.0) * norm;
	bA[6]                 = (1.0 - K / bA[1] + K * K) * norm;
	K                     = tan (M_PI * bA[0]);
	norm                  = 1.0 / (1.0 + K / bB[1] + K * K);
	bB[2]                 = K * K * norm;
	bB[3]                 = 2.0 * bB[2];
	bB[4]                 = bB[2];
	bB[5]                 = 2.0 * (K * K - 1.0) * norm;
	bB[6]                 = (1.0 - K / bB[1] + K * K) * norm;
	K                     = tan (M_PI * bC[0]);
	norm                  = 1.0 / (1.0 + K / bC[1] + K * K);
	bC[2]                 = K * K * norm;
	bC[3]                 = 2.0 * bC[2];
	bC[4]                 = bC[2];
	bC[5]                 = 2.0 * (K * K - 1.0) * norm;
	bC[6]                 = (1.0 - K / bC[1] + K * K) * norm;

	vibSpeed    = 0.06 + r->C;
	vibDepth    = (0.027 + pow (r->D, 3)) * 100.0;
	size        = (pow (r->E, 2) * 90.0) + 10.0;
	depthFactor = 1.0 - pow ((1.0 - (0.82 - ((r->B * 0.5) + (size * 0.002)))), 4);
	blend       = 0.955 - (size * 0.007);
	crossmod    = (r->F - 0.5) * 2.0;
	crossmod    = pow (crossmod, 3) * 0.5;
	regen       = depthFactor * (0.5 - (fabs (crossmod) * 0.031));
	wet         = r->G;

	for (i = 0; i < 12; i++)
		r->delay[i] = (int)(dmul[i] * size);
	r->delay[12] = (int)((29 * size) - (56 * size * fabs (crossmod)));

	while (--sampleFrames >= 0) {
		double in[2], dry[2], ap[2][4], interpol[2][8], fb[2][8], x;
		int    expon, l;
		in[0] = *in1;
		in[1] = *in1;
		if (fabs (in[0]) < 1.18e-23)
			in[0] = r->fpdL * 1.18e-17;
		if (fabs (in[1]) < 1.18e-23)
			in[1] = r->fpdR * 1.18e-17;
		dry[0] = in[0];
		dry[1] = in[1];

		/* predelay M */
		r->ring[0][12][r->count[12]] = in[0];
		r->ring[1][12][r->count[12]] = in[1];
		rv_inc (&r->count[12], r->delay[12]);
		in[0] = r->ring[0][12][r->count[12]];
		in[1] = r->ring[1][12][r->count[12]];

		for (c = 0; c < 2; c++) {
			in[c] = rv_biquad (bA, c, in[c]);
			in[c] *= wet;
			in[c] = sin (in[c]);
		}

		/* allpasses I, J, K, L (each fed by the same input) */
		for (l = 8; l < 12; l++) {
			int    d = r->delay[l];
			int    tmp = r->count[l] + 1;
			double* aL = r->ring[0][l];
			double* aR = r->ring[1][l];
			double apL = in[0], apR = in[1];
			if (tmp < 0 || tmp > d)
				tmp = 0;
			apL -= aL[tmp] * 0.5;
			aL[r->count[l]] = apL;
			apL *= 0.5;
			apR -= aR[tmp] * 0.5;
			aR[r->count[l]] = apR;
			apR *= 0.5;
			rv_inc (&r->count[l], d);
			apL += (aL[r->count[l]]);
			apR += (aR[r->count[l]]);
			ap[0][l - 8] = apL;
			ap[1][l - 8] = apR;
		}

		/* writes into the 8 modulated delay lines: A<-L, B<-K, C<-J, D<-I, E<-I, F<-J, G<-K, H<-L */
		{
			static const int src[8] = {3, 2, 1, 0, 0, 1, 2, 3};
			for (c = 0; c < 2; c++)
				for (l = 0; l < 8; l++)
					r->ring[c][l][r->count[l]] = ap[c][src[l]] + r->feedback[c][l];
		}
		for (l = 0; l < 8; l++)
			rv_inc (&r->count[l], r->delay[l]);

		for (c = 0; c < 2; c++)
			for (l = 0; l < 8; l++)
				r->vib[c][l] += (r->depth[l] * vibSpeed);

		for (c = 0; c < 2; c++) {
			double off[8];
			int    wk[8];
			for (l = 0; l < 8; l++)
				off[l] = (sin (r->vib[c][l]) + 1.0) * vibDepth;
			for (l = 0; l < 8; l++)
				wk[l] = (int)(r->count[l] + off[l]);
			for (l = 0; l < 8; l++) {
				const double* a  = r->ring[c][l];
				const int     d  = r->delay[l];
				const int     w0 = wk[l] - ((wk[l] > d) ? d + 1 : 0);
				const int     w1 = wk[l] + 1 - ((wk[l] + 1 > d) ? d + 1 : 0);
				double        v  = (a[w0] * (1 - (off[l] - floor (off[l]))));
				v += (a[w1] * ((off[l] - floor (off[l]))));
				interpol[c][l] = v;
			}
			for (l = 0; l < 8; l++) {
				const double* a  = r->ring[c][l];
				const int     d  = r->delay[l];
				const int     w0 = wk[l] - ((wk[l] > d) ? d + 1 : 0);
				interpol[c][l]   = ((1.0 - blend) * interpol[c][l]) + (a[w0] * blend);
			}
			interpol[c][0] = (interpol[c][0] * (1.0 - fabs (crossmod))) + (interpol[c][4] * crossmod);
			interpol[c][4] = (interpol[c][4] * (1.0 - fabs (crossmod))) + (interpol[c][0] * crossmod);
		}

		for (c = 0; c < 2; c++) {
			double* I = interpol[c];
			fb[c][0]  = (I[0] - (I[1] + I[2] + I[3])) * regen;
			fb[c][1]  = (I[1] - (I[0] + I[2] + I[3])) * regen;
			fb[c][2]  = (I[2] - (I[0] + I[1] + I[3])) * regen;
			fb[c][3]  = (I[3] - (I[0] + I[1] + I[2])) * regen;
			fb[c][4]  = (I[4] - (I[5] + I[6] + I[7])) * regen;
			fb[c][5]  = (I[5] - (I[4] + I[6] + I[7])) * regen;
			fb[c][6]  = (I[6] - (I[4] + I[5] + I[7])) * regen;
			fb[c][7]  = (I[7] - (I[4] + I[5] + I[6])) * regen;
			for (l = 0; l < 8; l++)
				r->feedback[c][l] = fb[c][l];
			in[c] = (I[0] + I[1] + I[2] + I[3] + I[4] + I[5] + I[6] + I[7]) / 8.0;
		}

		for (c = 0; c < 2; c++) {
			x = rv_biquad (bB, c, in[c]);
			if (x > 1.0)
				x = 1.0;
			if (x < -1.0)
				x = -1.0;
			x     = asin (x);
			in[c] = rv_biquad (bC, c, x);
		}

		if (wet != 1.0) {
			in[0] += (dry[0] * (1.0 - wet));
			in[1] += (dry[1] * (1.0 - wet));
		}

		frexpf ((float)in[0], &expon);
		r->fpdL ^= r->fpdL << 13;
		r->fpdL ^= r->fpdL >> 17;
		r->fpdL ^= r->fpdL << 5;
		in[0] += ((double)(r->fpdL) - (uint32_t)0x7fffffff) * 5.5e-36L * pow (2, expon + 62);
		frexpf ((float)in[1], &expon);
		r->fpdR ^= r->fpdR << 13;
		r->fpdR ^= r->fpdR >> 17;
		r->fpdR ^= r->fpdR << 5;
		in[1] += ((double)(r->fpdR) - (uint32_t)0x7fffffff) * 5.5e-36L * pow (2, expon + 62);

		*out1 = (float)(0.7071067811865476 * (in[0] + in[1]));
		in1++;
		out1++;
	}
}

/* ------------------------------------------------------------------ eqcomp */

/* src/eqcomp.cpp:98-203 eqCompute; C = {B0, B1, B2, A0, A1, A2} */
void orc_eq_compute (int type, double fqHz, double Q, double dbG, double* C, double SampleRateD)
{
	double A     = pow (10.0, (dbG / 40.0));
	double omega = (2.0 * M_PI * fqHz) / SampleRateD;
	double sin_  = sin (omega);
	double cos_  = cos (omega);
	double alpha = sin_ / (2.0 * Q);
	double beta  = sqrt (A) / Q;
	switch (type) {
		case 0:
			C[0] = (1.0 - cos_) / 2.0; C[1] = 1.0 - cos_; C[2] = (1.0 - cos_) / 2.0;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 1:
			C[0] = (1.0 + cos_) / 2.0; C[1] = -(1.0 + cos_); C[2] = (1.0 + cos_) / 2.0;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 2:
			C[0] = sin_ / 2.0; C[1] = 0.0; C[2] = -sin_ / 2.0;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 3:
			C[0] = alpha; C[1] = 0.0; C[2] = -alpha;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 4:
			C[0] = 1.0; C[1] = -2.0 * cos_; C[2] = 1.0;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 5:
			C[0] = 1.0 - alpha; C[1] = -2.0 * cos_; C[2] = 1.0 + alpha;
			C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha;
			break;
		case 6:
			C[0] = 1.0 + (alpha * A); C[1] = -2.0 * cos_; C[2] = 1.0 - (alpha * A);
			C[3] = 1.0 + (alpha / A); C[4] = -2.0 * cos_; C[5] = 1.0 - (alpha / A);
			break;
		case 7:
			C[0] = A * ((A + 1) - ((A - 1) * cos_) + (beta * sin_));
			C[1] = (2.0 * A) * ((A - 1) - ((A + 1) * cos_));
			C[2] = A * ((A + 1) - ((A - 1) * cos_) - (beta * sin_));
			C[3] = (A + 1) + ((A - 1) * cos_) + (beta * sin_);
			C[4] = -2.0 * ((A - 1) + ((A + 1) * cos_));
			C[5] = (A + 1) + ((A - 1) * cos_) - (beta * sin_);
			break;
		case 8:
			C[0] = A * ((A + 1) + ((A - 1) * cos_) + (beta * sin_));
			C[1] = -(2.0 * A) * ((A - 1) + ((A + 1) * cos_));
			C[2] = A * ((A + 1) + ((A - 1) * cos_) - (beta * sin_));
			C[3] = (A + 1) - ((A - 1) * cos_) + (beta * sin_);
			C[4] = 2.0 * ((A - 1) - ((A + 1) * cos_));
			C[5] = (A + 1) - ((A - 1) * cos_) - (beta * sin_);
			break;
	}
	C[0] /= C[3];
	C[1] /= C[3];
	C[2] /= C[3];
	C[4] /= C[3];
	C[5] /= C[3];
}

/* ------------------------------------------------------------------ whirl */
enum { fa0, fa1, fa2, fb0, fb1, fb2, fz0, fz1 };

/* src/whirl.cpp:147-172 setIIRFilter */
static void setIIRFilter (float W[], int T, const double F, const double Q, const double G, const double SR)
{
	double C[6];
	if (Q <= 0.1 || Q >= 6.00 || F / SR <= 0.0002 || F / SR >= 0.4998 || G <= -48.0 || G >= 48.0 || T < 0 || T > 8)
		return;
	orc_eq_compute (T, F, Q, G, C, SR);
	W[fa1] = (float)C[4];
	W[fa2] = (float)C[5];
	W[fb0] = (float)C[0];
	W[fb1] = (float)C[1];
	W[fb2] = (float)C[2];
}

/* the MIDI control functions initWhirl registers (src/whirl.cpp:966-981), setters 699-889:
 * the value mapped into the field's range in double, stored in the (float or double)
 * field, then UPDATE_A_FILTER / UPDATE_B_FILTER (679-689) for the horn filters.  The speed
 * ramps read hornAcc .. drumDec at every block (whirlProc2, 1255-1257).  Returns 0, or -1
 * for a name that is not one of them. */
int orc_whirl_control (struct orc_whirl* w, const char* fn, unsigned char uc)
{
	const double u = (double)uc;
	if (!strcmp (fn, "whirl.horn.filter.a.type"))
		w->haT = (int)(uc / 15);
	else if (!strcmp (fn, "whirl.horn.filter.a.hz"))
		w->haF = 250.0 + ((8000.0 - 250.0) * ((u * u) / 16129.0));
	else if (!strcmp (fn, "whirl.horn.filter.a.q"))
		w->haQ = 0.01 + ((6.00 - 0.01) * (u / 127.0));
	else if (!strcmp (fn, "whirl.horn.filter.a.gain"))
		w->haG = -48.0 + ((48.0 - -48.0) * (u / 127.0));
	else if (!strcmp (fn, "whirl.horn.filter.b.type"))
		w->hbT = (int)(uc / 15);
	else if (!strcmp (fn, "whirl.horn.filter.b.hz"))
		w->hbF = 250.0 + ((8000.0 - 250.0) * ((u * u) / 16129.0));
	else if (!strcmp (fn, "whirl.horn.filter.b.q"))
		w->hbQ = 0.01 + ((6.00 - 0.01) * (u / 127.0));
	else if (!strcmp (fn, "whirl.horn.filter.b.gain"))
		w->hbG = -48.0 + ((48.0 - -48.0) * (u / 127.0));
	else if (!strcmp (fn, "whirl.horn.brakepos"))
		w->hnBrakePos = u / 127.0;
	else if (!strcmp (fn, "whirl.drum.brakepos"))
		w->drBrakePos = u / 127.0;
	else if (!strcmp (fn, "whirl.horn.acceleration"))
		w->hornAcc = .01 + u / 80.0;
	else if (!strcmp (fn, "whirl.horn.deceleration"))
		w->hornDec = .01 + u / 80.0;
	else if (!strcmp (fn, "whirl.drum.acceleration"))
		w->drumAcc = .01 + u / 14.0;
	else if (!strcmp (fn, "whirl.drum.deceleration"))
		w->drumDec = .01 + u / 14.0;
	else
		return -1;
	if (!strncmp (fn, "whirl.horn.filter.a.", 20))
		setIIRFilter (w->hafw, (int)w->haT, w->haF, w->haQ, w->haG, w->SampleRateD);
	else if (!strncmp (fn, "whirl.horn.filter.b.", 20))
		setIIRFilter (w->hbfw, (int)w->hbT, w->hbF, w->hbQ, w->hbG, w->SampleRateD);
	return 0;
}

/* src/whirl.cpp:174-224 useRevOption */
void orc_whirl_use_rev_option (struct orc_whirl* w, int n, int signals)
{
	int i         = n % 9;
	w->hornTarget = w->revHorn[i];
	w->drumTarget = w->revDrum[i];
	if (w->hornIncr < w->hornTarget)
		w->hornAcDc = 1;
	else if (w->hornTarget < w->hornIncr)
		w->hornAcDc = -1;
	if (w->drumIncr < w->drumTarget)
		w->drumAcDc = 1;
	else if (w->drumTarget < w->drumIncr)
		w->drumAcDc = -1;
	if (signals & 2) {
		const int hr = (n / 3) % 3;
		w->revSelect = hr == 2 ? 2 : hr == 1 ? 0 : 1;
	}
}

/* src/whirl.cpp:295-327 _ipoldraw */
static void ipoldraw (struct orc_whirl* sw, double degrees, double level, int partial, double* ipx, double* ipy)
{
	double d, e, range;
	int    fromIndex, toIndex, i;
	d = *ipx;
	while (d < 0.0)
		d += 360.0;
	fromIndex = (int)((d * (double)16384) / 360.0);
	*ipx      = degrees;
	e         = *ipx;
	while (e < d)
		e += 360.0;
	toIndex = (int)((e * (double)16384) / 360.0);
	range   = (double)(toIndex - fromIndex);
	for (i = fromIndex; i <= toIndex; i++) {
		double x                       = (double)(i - fromIndex);
		double wv                      = (*ipy) + ((x / range) * (level - (*ipy)));
		sw->bfw[i & 16383].b[partial] = (float)wv;
	}
	*ipy = level;
}

/* angular impulse-response drawing data, src/whirl.cpp:366-490 */
static const double ir0[][2] = {{-180.0, 1.052}, {-166.4, .881}, {-150.5, .881}, {-135.3, .881}, {-122.4, .792}, {-106.5, .792}, {-91.2, .836}, {-75.8, .881}, {-59.4, .851}, {-44.7, .941}, {-30.0, 1.298}, {-14.7, 2.119}, {0.0, 2.820}, {15.6, 2.313}, {30.0, 1.492}, {44.7, .926}, {60.0, .836}, {74.7, .866}, {90.6, .792}, {100.0, .777}, {105.0, .777}, {120.0, .836}, {135.3, .836}, {150.0, .881}, {164.5, .874}, {180.0, 1.052}};
static const double ir1[][2] = {{-180.0, -0.07}, {-150.0, 0.10}, {-135.0, -0.10}, {-122.2, 0.16}, {-105.0, 0.15}, {-91.2, 0.37}, {-75.3, 0.32}, {-60.1, 0.39}, {-44.5, 0.70}, {-30.0, 0.53}, {-12.0, -0.40}, {0.0, -0.81}, {2.7, -0.77}, {15.0, -0.52}, {33.1, 0.38}, {43.7, 0.68}, {57.7, 0.49}, {74.1, 0.19}, {89.4, 0.33}, {105.0, 0.03}, {120.0, 0.12}, {134.0, -0.13}, {153.3, 0.08}, {180.0, -0.07}};
static const double ir2[][2] = {{-180.0, 0.40}, {-165.0, 0.20}, {-150.0, 0.48}, {-135.0, 0.27}, {-121.2, 0.22}, {-89.2, 0.30}, {-69.2, 0.22}, {-58.0, 0.11}, {-40.2, -0.43}, {-29.0, -0.53}, {-15.6, -0.43}, {0.0, 0.00}, {14.3, -0.44}, {30.3, -0.60}, {60.3, 0.11}, {74.9, 0.32}, {91.5, 0.23}, {104.9, 0.32}, {121.7, 0.19}, {135.0, 0.27}, {150.0, 0.45}, {165.0, 0.20}, {180.0, 0.40}};
static const double ir3[][2] = {{-180.0, -0.08}, {-165.2, -0.19}, {-150.0, 0.00}, {-133.9, -0.20}, {-120.0, -0.15}, {-106.0, 0.09}, {-89.3, -0.15}, {-76.3, 0.00}, {-60.3, 0.29}, {-44.6, -0.02}, {-15.6, -0.22}, {0.0, 0.24}, {14.5, 0.11}, {30.1, -0.10}, {44.6, 0.17}, {60.4, 0.22}, {75.9, 0.16}, {90.4, -0.05}, {104.9, 0.07}, {122.8, -0.07}, {136.2, -0.07}, {150.0, 0.08}, {165.0, -0.19}, {180.0, -0.08}};
static const double ir4[][2] = {{-180.0, 0.13}, {-165.2, 0.00}, {-150.0, 0.17}, {-135.2, -0.20}, {-120.5, 0.00}, {-105.0, 0.00}, {-90.0, 0.04}, {-75.0, -0.09}, {-60.3, -0.14}, {-45.0, 0.16}, {-15.6, 0.00}, {0.0, 0.22}, {15.6, -0.21}, {30.1, -0.09}, {45.0, 0.10}, {60.3, -0.07}, {74.8, -0.15}, {90.4, -0.03}, {104.9, -0.14}, {120.5, 0.00}, {135.2, -0.26}, {150.0, 0.16}, {165.0, -0.02}, {180.0, 0.13}};

static void drawIR (struct orc_whirl* w, const double (*pts)[2], int n, int partial)
{
	double ipx = pts[0][0], ipy = pts[0][1];
	int    i;
	for (i = 1; i < n; i++)
		ipoldraw (w, pts[i][0], pts[i][1], partial, &ipx, &ipy);
}

/* src/whirl.cpp:338-517 initTables */
static void initTables (struct orc_whirl* w)
{
	unsigned int i, j;
	double       sum = 0.0;
	drawIR (w, ir0, (int)(sizeof (ir0) / sizeof (ir0[0])), 0);
	drawIR (w, ir1, (int)(sizeof (ir1) / sizeof (ir1[0])), 1);
	drawIR (w, ir2, (int)(sizeof (ir2) / sizeof (ir2[0])), 2);
	drawIR (w, ir3, (int)(sizeof (ir3) / sizeof (ir3[0])), 3);
	drawIR (w, ir4, (int)(sizeof (ir4) / sizeof (ir4[0])), 4);
	for (i = 0; i < 16384; i++) {
		double colsum = 0.0;
		for (j = 0; j < 5; j++)
			colsum += fabs (w->bfw[i].b[j]);
		if (sum < colsum)
			sum = colsum;
	}
	for (i = 0; i < 16384; i++)
		for (j = 0; j < 5; j++) {
			w->bfw[i].b[j]               = (float)(w->bfw[i].b[j] * (1.0 / sum));
			w->bbw[16384 - i - 1].b[j] = w->bfw[i].b[j];
		}
}

/* src/whirl.cpp:534-624 computeOffsets */
static void computeOffsets (struct orc_whirl* w)
{
	unsigned int i;
	static const float hs[6] = {12.0f, 18.0f, 53.0f, 50.0f, 106.0f, 116.0f};
	static const float ds[6] = {36.0f, 39.0f, 79.0f, 86.0f, 123.0f, 116.0f};
	const double hornR = (w->hornRadiusCm * w->SampleRateD / 100.0) / w->airSpeed;
	const double drumR = (w->drumRadiusCm * w->SampleRateD / 100.0) / w->airSpeed;
	const double micD  = (w->micDistCm * w->SampleRateD / 100.0) / w->airSpeed;
	const double micX  = (w->hornXOffsetCm * w->SampleRateD / 100.0) / w->airSpeed;
	const double micZ  = (w->hornZOffsetCm * w->SampleRateD / 100.0) / w->airSpeed;
	w->adi0 = w->adi1 = w->adi2 = 0;
	w->outpos                   = 0;
	memset (w->HLbuf, 0, sizeof (w->HLbuf));
	memset (w->HRbuf, 0, sizeof (w->HRbuf));
	memset (w->DLbuf, 0, sizeof (w->DLbuf));
	memset (w->DRbuf, 0, sizeof (w->DRbuf));
	memset (w->adx0, 0, sizeof (w->adx0));
	memset (w->adx1, 0, sizeof (w->adx1));
	memset (w->adx2, 0, sizeof (w->adx2));
	for (i = 0; i < 16384; i++) {
		double v = (2.0 * M_PI * (double)i) / (double)16384;
		double a = micD - (hornR * cos (v));
		double b = micZ + hornR * sin (v);
		const double dist = sqrt ((a * a) + (b * b));
		w->hnFwdDispl[i]               = (float)(dist + micX);
		w->hnBwdDispl[16384 - (i + 1)] = (float)(dist - micX);
		a                              = micD - (drumR * cos (v));
		b                              = drumR * sin (v);
		w->drFwdDispl[i]               = (float)sqrt ((a * a) + (b * b));
		w->drBwdDispl[16384 - (i + 1)] = w->drFwdDispl[i];
	}
	w->hornPhase[0] = 0;
	w->hornPhase[1] = 16384 >> 1;
	w->hornPhase[2] = ((16384 * 2) / 6);
	w->hornPhase[3] = ((16384 * 5) / 6);
	w->hornPhase[4] = ((16384 * 1) / 6);
	w->hornPhase[5] = ((16384 * 4) / 6);
	for (i = 0; i < 6; i++)
		w->hornSpacing[i] = (float)(hs[i] * w->SampleRateD / 22100.0 + hornR + 1.0);
	for (i = 0; i < 6; i++)
		w->drumPhase[i] = w->hornPhase[i];
	for (i = 0; i < 6; i++)
		w->drumSpacing[i] = (float)(ds[i] * w->SampleRateD / 22100.0 + drumR + 1.0);
}

/* src/whirl.cpp:43-134 initValues, 956-986 initWhirl (initialize + computeRotationSpeeds) */
struct orc_whirl* orc_whirl_alloc (double sr, const orc_cfg* c)
{
	struct orc_whirl* w = (struct orc_whirl*)calloc (1, sizeof (*w));
	double            hfast, hslow, dfast, dslow;
	orc_cfg           dflt;
	if (!c) {
		orc_cfg_default (&dflt);
		c = &dflt;
	}
	/* initValues (43-134), then the cfg's whirlConfig assignments (992-1160) */
	w->hornRPMslow      = c->hornRPMslow;
	w->hornRPMfast      = c->hornRPMfast;
	w->drumRPMslow      = c->drumRPMslow;
	w->drumRPMfast      = c->drumRPMfast;
	w->hornAcc          = c->hornAcc;
	w->hornDec          = c->hornDec;
	w->drumAcc          = c->drumAcc;
	w->drumDec          = c->drumDec;
	w->airSpeed         = 340.0f;
	w->micDistCm        = c->micDistCm;
	w->hornXOffsetCm    = c->hornXOffsetCm;
	w->hornZOffsetCm    = c->hornZOffsetCm;
	w->hornRadiusCm     = c->hornRadiusCm;
	w->drumRadiusCm     = c->drumRadiusCm;
	w->lpT              = c->lpT;
	w->lpF              = c->lpF;
	w->lpQ              = c->lpQ;
	w->lpG              = c->lpG;
	w->haT              = c->haT;
	w->haF              = c->haF;
	w->haQ              = c->haQ;
	w->haG              = c->haG;
	w->hbT              = c->hbT;
	w->hbF              = c->hbF;
	w->hbQ              = c->hbQ;
	w->hbG              = c->hbG;
	w->hornMic_hll = w->drumMic_dll = 1.0f;
	w->hornMic_hlr = w->drumMic_dlr = 0.0f;
	w->hornMic_hrl = w->drumMic_drl = 0.0f;
	w->hornMic_hrr = w->drumMic_drr = 1.0f;
	if (c->drumMicWidth != 0.0f) { /* fsetDrumMicWidth (912-930; no-op at the current width 0) */
		const float dw = c->drumMicWidth;
		const float dwP = dw > 0.f ? (dw > 1.f ? 1.f : dw) : 0.f;
		const float dwN = dw < 0.f ? (dw < -1.f ? 1.f : -dw) : 0.f;
		w->drumMic_dll  = sqrtf (1.f - dwP);
		w->drumMic_dlr  = sqrtf (0.f + dwP);
		w->drumMic_drl  = sqrtf (0.f + dwN);
		w->drumMic_drr  = sqrtf (1.f - dwN);
	}
	if (c->hornMicWidth != 0.0f) { /* fsetHornMicWidth (932-949) */
		const float hw = c->hornMicWidth;
		const float hwP = hw > 0.f ? (hw > 1.f ? 1.f : hw) : 0.f;
		const float hwN = hw < 0.f ? (hw < -1.f ? 1.f : -hw) : 0.f;
		w->hornMic_hll  = sqrtf (1.f - hwP);
		w->hornMic_hlr  = sqrtf (0.f + hwP);
		w->hornMic_hrl  = sqrtf (0.f + hwN);
		w->hornMic_hrr  = sqrtf (1.f - hwN);
	}
	w->hornLevel        = c->hornLevel;
	w->leakLevel        = c->leakLevel;
	w->bypass           = c->bypass;
	w->revSelect        = c->revSelect;
	w->micAngle         = c->micAngle;
	w->hnBrakePos       = c->hnBrakePos;
	w->drBrakePos       = c->drBrakePos;
	w->SampleRateD      = sr;
	/* initialize (626-662) */
	w->leakage = w->leakLevel * w->hornLevel;
	setIIRFilter (w->drfL, w->lpT, w->lpF, w->lpQ, w->lpG, w->SampleRateD);
	setIIRFilter (w->drfR, w->lpT, w->lpF, w->lpQ, w->lpG, w->SampleRateD);
	setIIRFilter (w->hafw, (int)w->haT, w->haF, w->haQ, w->haG, w->SampleRateD);
	setIIRFilter (w->hbfw, (int)w->hbT, w->hbF, w->hbQ, w->hbG, w->SampleRateD);
	computeOffsets (w);
	initTables (w);
	/* computeRotationSpeeds (270-293) */
	hfast = w->hornRPMfast / (w->SampleRateD * 60.0);
	hslow = w->hornRPMslow / (w->SampleRateD * 60.0);
	dfast = w->drumRPMfast / (w->SampleRateD * 60.0);
	dslow = w->drumRPMslow / (w->SampleRateD * 60.0);
	w->revHorn[8] = hfast; w->revDrum[8] = dfast;
	w->revHorn[7] = hfast; w->revDrum[7] = dslow;
	w->revHorn[6] = hfast; w->revDrum[6] = 0;
	w->revHorn[5] = hslow; w->revDrum[5] = dfast;
	w->revHorn[4] = hslow; w->revDrum[4] = dslow;
	w->revHorn[3] = hslow; w->revDrum[3] = 0;
	w->revHorn[2] = 0;     w->revDrum[2] = dfast;
	w->revHorn[1] = 0;     w->revDrum[1] = dslow;
	w->revHorn[0] = 0;     w->revDrum[0] = 0;
	w->revselects[0] = 4;
	w->revselects[1] = 0;
	w->revselects[2] = 8;
	/* setRevSelect (226-233) */
	w->revSelect = w->revSelect % 3;
	orc_whirl_use_rev_option (w, w->revselects[w->revSelect], 1);
	return w;
}

#define EQ_IIR(W, X, Y)                                                        \
	{                                                                          \
		float temp = (X) - (W[fa1] * W[fz0]) - (W[fa2] * W[fz1]);               \
		Y          = (temp * W[fb0]) + (W[fb1] * W[fz0]) + (W[fb2] * W[fz1]);  \
		W[fz1]     = W[fz0];                                                   \
		W[fz0]     = temp;                                                     \
	}

/* src/whirl.cpp:1191-1638 whirlProc2 (outputs as used by whirlProc3) and
 * 1653-1681 whirlProc3 */
void orc_whirl_run3 (struct orc_whirl* w, const float* inbuffer, float* outL, float* outR, float* outDL,
                     float* outDR, size_t bufferLengthSamples)
{
	unsigned int i;
	if (w->bypass) {
		for (i = 0; i < bufferLengthSamples; i++) {
			outL[i]  = inbuffer[i];
			outR[i]  = inbuffer[i];
			outDL[i] = 0;
			outDR[i] = 0;
		}
	} else {
		if (w->hornAcDc) {
			int         flywheel = 0;
			const float hardstop = (float)(10.f / (60.f * w->SampleRateD));
			if (w->hnBrakePos > 0 && w->hornTarget == 0 && w->hornIncr > 0 && w->hornIncr < hardstop) {
				const double targetPos = fmod (1.25 - w->hnBrakePos, 1.0);
				if (fabs (w->hornAngleGRD - targetPos) < (2.0 / 16384)) {
					w->hornAngleGRD = targetPos;
					w->hornIncr     = 0;
				} else {
					const float minspeed = (float)(3.f / (60.f * w->SampleRateD));
					const float diffinc  = (float)(fmod (1. + targetPos - w->hornAngleGRD, 1.0) / (float)bufferLengthSamples);
					if (w->hornIncr > diffinc)
						w->hornIncr = diffinc;
					else if (w->hornIncr < minspeed)
						w->hornIncr = minspeed;
					flywheel = 1;
				}
			}
			if (!flywheel) {
				const double l = exp (-1.0 / (w->SampleRateD / bufferLengthSamples * (w->hornAcDc > 0 ? w->hornAcc : w->hornDec)));
				w->hornIncr += (1 - l) * (w->hornTarget - w->hornIncr);
			}
			if (fabs (w->hornTarget - w->hornIncr) < (.05 / (60.f * w->SampleRateD))) {
				w->hornAcDc = 0;
				w->hornIncr = w->hornTarget;
			}
		}
		if (w->drumAcDc) {
			int         flywheel = 0;
			const float hardstop = (float)(8.f / (60.f * w->SampleRateD));
			if (w->drBrakePos > 0 && w->drumTarget == 0 && w->drumIncr > 0 && w->drumIncr < hardstop) {
				const double targetPos = fmod (w->drBrakePos + .75, 1.0);
				if (fabs (w->drumAngleGRD - targetPos) < (2.0 / 16384)) {
					w->drumAngleGRD = targetPos;
					w->drumIncr     = 0;
				} else {
					const float minspeed = (float)(3.f / (60.f * w->SampleRateD));
					const float diffinc  = (float)(fmod (1. + targetPos - w->drumAngleGRD, 1.0) / (float)bufferLengthSamples);
					if (w->drumIncr > diffinc)
						w->drumIncr = diffinc;
					else if (w->drumIncr < minspeed)
						w->drumIncr = minspeed;
					flywheel = 1;
				}
			}
			if (!flywheel) {
				const double l = exp (-1.0 / (w->SampleRateD / bufferLengthSamples * (w->drumAcDc > 0 ? w->drumAcc : w->drumDec)));
				w->drumIncr += (1 - l) * (w->drumTarget - w->drumIncr);
			}
			if (fabs (w->drumTarget - w->drumIncr) < (.05 / (60.f * w->SampleRateD))) {
				w->drumAcDc = 0;
				w->drumIncr = w->drumTarget;
			}
		}
		{
			int brake = 0;
			if (w->hnBrakePos > 0) {
				const double targetPos = fmod (1.25 - w->hnBrakePos, 1.0);
				if (!w->hornAcDc && w->hornIncr == 0 && w->hornAngleGRD != targetPos) {
					brake |= 1;
					if (fabs (w->hornAngleGRD - targetPos) < (2.0 / 16384)) {
						w->hornAngleGRD = targetPos;
					} else {
						const float limit = (float)(60.f / (60. * w->SampleRateD));
						w->hornIncr       = fmod (1. + targetPos - w->hornAngleGRD, 1.0) / (float)bufferLengthSamples;
						if (w->hornIncr > limit)
							w->hornIncr = limit;
					}
				}
			}
			if (w->drBrakePos > 0) {
				const double targetPos = fmod (w->drBrakePos + .75, 1.0);
				if (!w->drumAcDc && w->drumIncr == 0 && w->drumAngleGRD != targetPos) {
					brake |= 2;
					if (fabs (w->drumAngleGRD - targetPos) < (2.0 / 16384)) {
						w->drumAngleGRD = targetPos;
					} else {
						const float limit = (float)(100.f / (60. * w->SampleRateD));
						w->drumIncr       = fmod (1. + targetPos - w->drumAngleGRD, 1.0) / (float)bufferLengthSamples;
						if (w->drumIncr > limit)
							w->drumIncr = limit;
					}
				}
			}
			{
				double       hornAngleGRD = w->hornAngleGRD;
				double       drumAngleGRD = w->drumAngleGRD;
				unsigned int outpos       = w->outpos;
				const double fwAng        = w->micAngle * .25;
				const double bwAng        = 1. + w->micAngle * -.25;
				const float  leakage      = w->leakage;
				const float  hornLevel    = w->hornLevel;
				const double hornIncr     = w->hornIncr;
				const double drumIncr     = w->drumIncr;
				float*       z            = w->z;

#define HN_MOTION(P, BUF, DSP, BW, DX, DI, ANG)                                                   \
	{                                                                                             \
		const float        h1   = (float)((ANG) * (unsigned int)16384 + w->hornPhase[(P)]);        \
		const float        hd   = fmodf (h1, 1.f);                                                \
		const unsigned int hl   = ((unsigned int)floorf (h1)) & 16383;                             \
		const unsigned int hh   = (hl + 1) & 16383;                                               \
		const float        intp = w->DSP[hl] * (1.f - hd) + hd * w->DSP[hh];                       \
		const unsigned int k    = ((unsigned int)roundf (h1)) & 16383;                             \
		const float        t    = w->hornSpacing[(P)] + intp + (float)outpos;                      \
		const float        r    = floorf (t);                                                     \
		float              xa;                                                                    \
		xa = w->BW[k].b[0] * x;                                                                   \
		xa += w->BW[k].b[1] * w->DX[(DI)];                                                        \
		xa += w->BW[k].b[2] * w->DX[((DI) + 1) & 7];                                              \
		xa += w->BW[k].b[3] * w->DX[((DI) + 2) & 7];                                              \
		xa += w->BW[k].b[4] * w->DX[((DI) + 3) & 7];                                              \
		{                                                                                         \
			const float q = xa * (t - r);                                                         \
			n             = ((unsigned int)r) & 2047;                                              \
			w->BUF[n] += xa - q;                                                                  \
			n = (n + 1) & 2047;                                                                   \
			w->BUF[n] += q;                                                                       \
		}                                                                                         \
	}
#define DR_MOTION(P, BUF, DSP)                                                                  \
	{                                                                                           \
		const float        d1   = (float)(drumAngleGRD * (unsigned int)16384 + w->drumPhase[(P)]); \
		const float        dd   = fmodf (d1, 1.f);                                              \
		const unsigned int dl   = ((unsigned int)floorf (d1)) & 16383;                           \
		const unsigned int dh   = (dl + 1) & 16383;                                             \
		const float        intp = w->DSP[dl] * (1.f - dd) + dd * w->DSP[dh];                     \
		const float        t    = w->drumSpacing[(P)] + intp + (float)outpos;                    \
		const float        r    = floorf (t);                                                   \
		const float        q    = x * (t - r);                                                  \
		n                       = ((unsigned int)r) & 2047;                                      \
		w->BUF[n] += x - q;                                                                     \
		n = (n + 1) & 2047;                                                                     \
		w->BUF[n] += q;                                                                         \
	}
#define FILTER_C(W0, W1, I)                              \
	{                                                    \
		float temp = x;                                  \
		x          = (float)(((W0) * x) + ((W1) * z[(I)])); \
		z[(I)]     = temp;                               \
	}
#define ADDHIST(DX, DI, XS)           \
	{                                 \
		DI     = (DI + 7) & 7;        \
		DX[DI] = XS;                  \
	}
				for (i = 0; i < bufferLengthSamples; i++) {
					unsigned int n;
					float        x    = (float)((double)inbuffer[i] + 1e-14);
					float        xx   = x;
					float        leak = 0;
					EQ_IIR (w->hafw, x, x);
					EQ_IIR (w->hbfw, x, x);
					leak = x * leakage;
					HN_MOTION (0, HLbuf, hnFwdDispl, bbw, adx0, w->adi0, hornAngleGRD + fwAng);
					HN_MOTION (1, HRbuf, hnBwdDispl, bfw, adx0, w->adi0, hornAngleGRD + bwAng);
					ADDHIST (w->adx0, w->adi0, x);
					FILTER_C (0.4, 0.4, 0);
					HN_MOTION (2, HLbuf, hnBwdDispl, bfw, adx1, w->adi1, hornAngleGRD + fwAng);
					HN_MOTION (3, HRbuf, hnFwdDispl, bbw, adx1, w->adi1, hornAngleGRD + bwAng);
					ADDHIST (w->adx1, w->adi1, x);
					FILTER_C (0.4, 0.4, 1);
					HN_MOTION (4, HLbuf, hnFwdDispl, bbw, adx2, w->adi2, hornAngleGRD + fwAng);
					HN_MOTION (5, HRbuf, hnBwdDispl, bfw, adx2, w->adi2, hornAngleGRD + bwAng);
					ADDHIST (w->adx2, w->adi2, x);
					x = xx;
					DR_MOTION (0, DLbuf, drFwdDispl);
					DR_MOTION (1, DRbuf, drBwdDispl);
					FILTER_C (0.4, 0.4, 2);
					DR_MOTION (2, DLbuf, drBwdDispl);
					DR_MOTION (3, DRbuf, drFwdDispl);
					FILTER_C (0.4, 0.4, 3);
					DR_MOTION (4, DLbuf, drFwdDispl);
					DR_MOTION (5, DRbuf, drBwdDispl);
					{
						float y;
						EQ_IIR (w->drfL, w->DLbuf[outpos], y);
						outL[i]  = hornLevel * w->HLbuf[outpos] + leak;
						outDL[i] = y;
						EQ_IIR (w->drfR, w->DRbuf[outpos], y);
						outR[i]  = hornLevel * w->HRbuf[outpos] + leak;
						outDR[i] = y;
					}
					w->HLbuf[outpos] = 0.0f;
					w->HRbuf[outpos] = 0.0f;
					w->DLbuf[outpos] = 0.0f;
					w->DRbuf[outpos] = 0.0f;
					outpos           = (outpos + 1) & 2047;
					hornAngleGRD     = fmod (hornAngleGRD + hornIncr, 1.0);
					drumAngleGRD     = fmod (drumAngleGRD + drumIncr, 1.0);
				}
#undef HN_MOTION
#undef DR_MOTION
#undef FILTER_C
#undef ADDHIST
				if (isnan (w->hafw[fz0])) w->hafw[fz0] = 0;
				if (isnan (w->hafw[fz1])) w->hafw[fz1] = 0;
				if (isnan (w->hbfw[fz0])) w->hbfw[fz0] = 0;
				if (isnan (w->hbfw[fz1])) w->hbfw[fz1] = 0;
				if (isnan (w->drfL[fz0])) w->drfL[fz0] = 0;
				if (isnan (w->drfL[fz1])) w->drfL[fz1] = 0;
				if (isnan (w->drfR[fz0])) w->drfR[fz0] = 0;
				if (isnan (w->drfR[fz1])) w->drfR[fz1] = 0;
				for (i = 0; i < 4; i++)
					if (isnan (z[i]))
						z[i] = 0;
				w->hornAngleGRD = hornAngleGRD;
				w->drumAngleGRD = drumAngleGRD;
				if (brake & 1)
					w->hornIncr = 0;
				if (brake & 2)
					w->drumIncr = 0;
				w->outpos = outpos;
			}
		}
	}
	/* whirlProc3 mic-width mix */
	for (i = 0; i < bufferLengthSamples; ++i) {
		const float tmp = outL[i];
		outL[i]         = outL[i] * w->hornMic_hll + outR[i] * w->hornMic_hlr + outDL[i] * w->drumMic_dll + outDR[i] * w->drumMic_dlr;
		outR[i]         = tmp * w->hornMic_hrl + outR[i] * w->hornMic_hrr + outDL[i] * w->drumMic_drl + outDR[i] * w->drumMic_drr;
	}
}

/* ------------------------------------------------------------------ standalone stage API */
orc_whirl* orc_whirl_new (double sr) { return orc_whirl_alloc (sr, NULL); }
void       orc_whirl_free (orc_whirl* w) { free (w); }
void       orc_whirl_rev_option (orc_whirl* w, int n) { orc_whirl_use_rev_option (w, n, 2); }
void       orc_whirl_proc3 (orc_whirl* w, const float* in, float* L, float* R, int n)
{
	float tl[4096], tr[4096];
	while (n > 0) {
		int m = n > 4096 ? 4096 : n;
		orc_whirl_run3 (w, in, L, R, tl, tr, (size_t)m);
		in += m;
		L += m;
		R += m;
		n -= m;
	}
}
orc_reverb* orc_reverb_new (double sr, unsigned int seed)
{
	orc_rand rnd;
	orc_srand (&rnd, seed);
	return orc_reverb_alloc (&rnd, sr);
}
void orc_reverb_free (orc_reverb* r) { rv_free (r); }
void orc_reverb_set_mix (orc_reverb* r, float g) { r->G = g; }
void orc_reverb_proc (orc_reverb* r, const float* in, float* out, int n) { orc_reverb_run (r, in, out, n); }
orc_preamp* orc_preamp_new (double sr, unsigned int seed)
{
	orc_rand    rnd;
	orc_preamp* p = (orc_preamp*)calloc (1, sizeof (*p));
	orc_srand (&rnd, seed);
	orc_preamp_init (p, &rnd, sr);
	return p;
}
void orc_preamp_free (orc_preamp* p) { free (p); }
void orc_preamp_set (orc_preamp* p, int clean, float character)
{
	p->isClean = clean;
	orc_preamp_set_character (p, character);
}
void orc_preamp_proc (orc_preamp* p, const float* in, float* out, int n) { orc_preamp_run (p, in, out, n); }
