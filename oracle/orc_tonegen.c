/*
 * oracle/orc_tonegen.c -- TEST INFRASTRUCTURE ONLY (see orc.h).
 * Restatement of the tone generator (src/tonegen.cpp) and vibrato scanner
 * (src/vibrato.cpp): table builders, regression dumps and the block renderer.
 */
#include "orc_internal.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define NW ORC_NOF_WHEELS
#define BSS ORC_BLK

/* ------------------------------------------------------------------ lists */
static void lst_push (orc_list* l, short sa, short sb, float fc)
{
	if (l->n == l->cap) {
		l->cap = l->cap ? 2 * l->cap : 8;
		l->v   = (orc_le*)realloc (l->v, sizeof (orc_le) * l->cap);
	}
	l->v[l->n].sa = sa;
	l->v[l->n].sb = sb;
	l->v[l->n].fc = fc;
	l->n++;
}

static void lst_insert (orc_list* l, int at, orc_le e)
{
	if (l->n == l->cap) {
		l->cap = l->cap ? 2 * l->cap : 8;
		l->v   = (orc_le*)realloc (l->v, sizeof (orc_le) * l->cap);
	}
	memmove (&l->v[at + 1], &l->v[at], sizeof (orc_le) * (l->n - at));
	l->v[at] = e;
	l->n++;
}

/* src/tonegen.cpp:337 */
static double dBToGain (double dB) { return pow (10.0, (dB / 20.0)); }

/* src/tonegen.cpp:205-233 (data tables) */
static const short northTransformers[] = {
	85, 66, 90, 71, 47, 64, 86, 69, 45, 62, 86, 67, 91, 72, 48, 65, 89, 70,
	46, 63, 87, 68, 44, 61, 0};
static const short southTransformers[] = {
	78, 54, 83, 59, 76, 52, 81, 57, 74, 50, 79, 55, 84, 60, 77, 53, 82, 58,
	75, 51, 80, 56, 73, 49, 0};
static const short terminalStrip[] = {
	85, 42, 30, 76, 66, 18, 6, 54, 90, 35, 83, 71, 23, 11, 59, 47, 40,
	28, 76, 64, 16, 4, 52, 88, 33, 81, 69, 21, 9, 57, 45, 34, 26, 74,
	62, 14, 2, 50, 86, 43, 31, 79, 67, 19, 7, 55, 91, 36, 84, 72, 24,
	12, 60, 48, 41, 29, 77, 65, 17, 5, 53, 89, 34, 82, 70, 22, 10, 58,
	46, 39, 27, 75, 63, 15, 3, 51, 87, 32, 80, 68, 20, 8, 56, 44, 37,
	25, 73, 61, 13, 1, 49, 0};

/* src/tonegen.cpp:502-692 taperingModel (dB steps -10,-7,-3.5,0,3.5,7) */
static double taperingModel (int key, int bus)
{
	double tp = 0.0;
	key       = key - 36;
	switch (bus) {
		case 0: tp = key < 12 ? -10.0 : key < 17 ? -7.0 : key < 24 ? -3.5 : key < 36 ? 0.0 : key < 48 ? 3.5 : 7.0; break;
		case 1: tp = key < 15 ? -3.5 : key < 38 ? 0.0 : key < 50 ? 3.5 : 7.0; break;
		case 2: tp = key < 17 ? -7.0 : key < 22 ? -3.5 : key < 37 ? 0.0 : key < 49 ? 3.5 : 7.0; break;
		case 3: tp = key < 17 ? -3.5 : key < 39 ? 0.0 : -3.5; break;
		case 4: tp = key < 14 ? 7.0 : key < 20 ? 3.5 : key < 40 ? 0.0 : key < 50 ? -3.5 : -7.0; break;
		case 5: tp = key < 12 ? 7.0 : key < 15 ? 3.5 : key < 41 ? 0.0 : key < 54 ? -3.5 : -7.0; break;
		case 6: tp = key < 14 ? 3.5 : key < 42 ? 0.0 : key < 50 ? -3.5 : -7.0; break;
		case 7: tp = key < 43 ? 0.0 : key < 48 ? -3.5 : -7.0; break;
		case 8: tp = key < 43 ? 0.0 : -7.0; break;
	}
	return dBToGain (tp);
}

/* src/tonegen.cpp:694-702 */
static double oscFreq (const orc_template* t, int i)
{
	return fmin (fmax (t->frequency[i - 1], 12.0), 2.5e10);
}

/* src/tonegen.cpp:707-802 applyManualDefaults: nearest-cents wheel per drawbar ratio */
static void applyManualDefaults (orc_template* t, int keyOffset, int busOffset)
{
	double of[NW + 1];
	int    i, k, b, tn, best;
	float  ratio, centDiff, smallest;
	for (i = 1; i <= NW; i++)
		of[i] = oscFreq (t, i);
	for (k = 0; k < 128; k++) {
		int kn = k + keyOffset;
		if (t->keyTaper[kn].n != 0)
			continue;
		for (b = 0; b < 9; b++) {
			smallest = INFINITY;
			best     = 0;
			for (tn = 1; tn <= NW; tn++) {
				ratio    = (float)(of[tn] / t->frequency[k]);
				centDiff = (float)(1200 * fabs (log2 (t->targetRatio[b] / ratio)));
				if (centDiff < smallest) {
					smallest = centDiff;
					best     = tn;
				}
			}
			if (best != 1 && best != NW)
				lst_push (&t->keyTaper[kn], (short)best, (short)(b + busOffset), (float)taperingModel (k, b));
		}
	}
}

/* src/tonegen.cpp:810-841 applyPedalDefaults */
static void applyPedalDefaults (orc_template* t, int nofPedals)
{
	static const int PDoffset[9] = {-12, 7, 0, 12, 19, 24, 28, 31, 36};
	int              k, b;
	for (k = 0; k < nofPedals; k++) {
		int kn = k + 256;
		if (t->keyTaper[kn].n != 0)
			continue;
		for (b = 0; b < 9; b++) {
			int tn = (k + 1) + PDoffset[b];
			if (tn < 1 || NW < tn)
				continue;
			lst_push (&t->keyTaper[kn], (short)tn, (short)(b + 18), (float)dBToGain (0.0));
		}
	}
}

/* src/tonegen.cpp:849-879 applyDefaultCrosstalk (defaultWiringCrosstalk) */
static void applyDefaultCrosstalk (orc_template* t, int keyOffset, int busOffset, double wiring)
{
	int k, b, e;
	for (k = 0; k < 128; k++) {
		int kn = k + keyOffset;
		if (t->keyCrosstalk[kn].n != 0)
			continue;
		for (b = 0; b < 9; b++) {
			int busNumber = busOffset + b;
			for (e = 0; e < t->keyTaper[kn].n; e++) {
				const orc_le* lep = &t->keyTaper[kn].v[e];
				if (lep->sb == busNumber)
					continue;
				lst_push (&t->keyCrosstalk[kn], lep->sa, (short)busNumber,
				          (float)((wiring * lep->fc) / abs (busNumber - lep->sb)));
			}
		}
	}
}

/* src/tonegen.cpp:884-909 */
static int findEastWest (const short* v, int w, int* ep, int* wp)
{
	int i;
	*ep = 0;
	*wp = 0;
	for (i = 0; 0 < v[i]; i++) {
		if (v[i] == (short)w) {
			if (0 < i)
				*ep = v[i - 1];
			*wp = v[i + 1];
			return 1;
		}
	}
	return 0;
}

/* src/tonegen.cpp:933-1041 applyDefaultConfiguration (defaults: compartment 0.01,
 * transformer 0, terminal strip 0.01, wiring 0.01) */
static void applyDefaultConfiguration (orc_template* t, const orc_cfg* c)
{
	const double compartment = c->compartmentXT, transformer = c->transformerXT, strip = c->stripXT;
	int          i;
	for (i = 1; i <= NW; i++) {
		if (t->terminalMix[i].n == 0) {
			lst_push (&t->terminalMix[i], (short)i, 0, (float)(1.0 - compartment));
			if (0.0 < compartment) {
				short pw = orc_paired_wheel ((short)i);
				if (0 < pw && pw <= NW)
					lst_push (&t->terminalMix[i], pw, 0, (float)compartment);
			}
		}
	}
	if (0.0 < transformer) {
		for (i = 44; i <= NW; i++) {
			int east = 0, west = 0;
			if (!findEastWest (northTransformers, i, &east, &west))
				findEastWest (southTransformers, i, &east, &west);
			if (0 < east)
				lst_push (&t->terminalMix[i], (short)east, 0, (float)transformer);
			if (0 < west)
				lst_push (&t->terminalMix[i], (short)west, 0, (float)transformer);
		}
	}
	if (0.0 < strip) {
		for (i = 1; i <= NW; i++) {
			int east = 0, west = 0;
			findEastWest (terminalStrip, i, &east, &west);
			if (0 < east)
				lst_push (&t->terminalMix[i], (short)east, 0, (float)strip);
			if (0 < west)
				lst_push (&t->terminalMix[i], (short)west, 0, (float)strip);
		}
	}
	applyManualDefaults (t, 0, 0);
	applyManualDefaults (t, 128, 9);
	applyPedalDefaults (t, 32);
	applyDefaultCrosstalk (t, 0, 0, c->wiringXT);
	applyDefaultCrosstalk (t, 128, 9, c->wiringXT);
}

/* src/tonegen.cpp:1061-1111 cpmInsert */
static void cpmInsert (const orc_template* t, const orc_le* lep, unsigned char cpmBus[][ORC_NOF_BUSES],
                       float cpmGain[][ORC_NOF_BUSES], short* wheelNumber, short* rowLength, int* endRowp)
{
	int           endRow   = *endRowp;
	int           terminal = lep->sa;
	unsigned char bus      = (unsigned char)lep->sb;
	int           e, r, c, b;
	for (e = 0; e < t->terminalMix[terminal].n; e++) {
		const orc_le* tl   = &t->terminalMix[terminal].v[e];
		float         gain = tl->fc * lep->fc;
		short         wnr  = tl->sa;
		if (gain == 0.0)
			continue;
		wheelNumber[endRow] = wnr;
		for (r = 0; wheelNumber[r] != wnr; r++)
			;
		if (r == endRow) {
			rowLength[r] = 0;
			endRow += 1;
		}
		c           = rowLength[r];
		cpmBus[r][c] = bus;
		for (b = 0; cpmBus[r][b] != bus; b++)
			;
		if (b == c) {
			rowLength[r] += 1;
			cpmGain[r][b] = gain;
		} else {
			cpmGain[r][b] += gain;
		}
	}
	*endRowp = endRow;
}

/* src/tonegen.cpp:1122-1213 compilePlayMatrix (contribution floor / minimum: defaults
 * 0.0000158 / 0.0) */
static void compilePlayMatrix (orc_template* t, const orc_cfg* cfg)
{
	static unsigned char cpmBus[NW + 1][ORC_NOF_BUSES];
	static float         cpmGain[NW][ORC_NOF_BUSES];
	short                wheelNumber[NW + 1];
	short                rowLength[NW];
	const double         floorLevel = cfg->contribFloor, minLevel = cfg->contribMin;
	int                  k, w, c, e;
	for (k = 0; k < ORC_MAX_KEYS; k++) {
		int endRow = 0;
		for (e = 0; e < t->keyTaper[k].n; e++)
			cpmInsert (t, &t->keyTaper[k].v[e], cpmBus, cpmGain, wheelNumber, rowLength, &endRow);
		for (e = 0; e < t->keyCrosstalk[k].n; e++)
			cpmInsert (t, &t->keyCrosstalk[k].v[e], cpmBus, cpmGain, wheelNumber, rowLength, &endRow);
		for (w = 0; w < endRow; w++) {
			for (c = 0; c < rowLength[w]; c++) {
				orc_le rep;
				int    at;
				if (cpmGain[w][c] < floorLevel)
					continue;
				rep.sa = wheelNumber[w];
				rep.sb = cpmBus[w][c];
				rep.fc = cpmGain[w][c];
				if (rep.fc < minLevel)
					rep.fc = (float)minLevel;
				for (at = 0; at < t->keyContrib[k].n; at++) {
					const orc_le* P = &t->keyContrib[k].v[at];
					if (rep.sa < P->sa)
						break;
					if (rep.sa == P->sa && rep.sb < P->sb)
						break;
				}
				lst_insert (&t->keyContrib[k], at, rep);
			}
		}
	}
}

/* src/tonegen.cpp:1223-1233 damperCurve */
static double damperCurve (int thisTG, int firstTG, int lastTG, double w, double v, double u)
{
	double x = ((double)(thisTG - firstTG)) / ((double)(lastTG - firstTG));
	double z = (x * (u - v)) - u;
	return 1.0 - w * z * z;
}

/* src/tonegen.cpp:1266-1311 applyOscEQ_peak24 / applyOscEQ_peak46 */
static void applyPeak (orc_template* t, int nofOscillators, int peak46)
{
	int i;
	for (i = 1; i <= 43; i++)
		t->watt[i] = peak46 ? damperCurve (i, 1, 43, 0.3, 0.4, 1.0) : damperCurve (i, 1, 43, 0.2, -0.8, 1.0);
	for (i = 44; i <= 48; i++)
		t->watt[i] = peak46 ? damperCurve (i, 44, 48, 0.1, -0.4, 0.4) : damperCurve (i, 44, 48, 1.6, -0.4, -0.3);
	for (i = 49; i <= nofOscillators; i++)
		t->watt[i] = peak46 ? damperCurve (i, 49, nofOscillators, 0.8, -1.0, -0.3)
		                    : damperCurve (i, 49, nofOscillators, 0.9, -1.0, -0.7);
}

/* src/tonegen.cpp:1240-1261 apply_CH_Spline (defaults p1y=1, r1y=0, p4y=1, r4y=0) */
static void applySpline (orc_template* tg, int nofOscillators, double p1y, double r1y, double p4y, double r4y)
{
	int    i;
	double k = nofOscillators - 1;
	for (i = 1; i <= nofOscillators; i++) {
		double t   = ((double)(i - 1)) / k;
		double tSq = t * t;
		double tCb = tSq * t;
		double r   = p1y * (2.0 * tCb - 3.0 * tSq + 1.0) + p4y * (-2.0 * tCb + 3.0 * tSq) +
		           r1y * (tCb - 2.0 * tSq + t) + r4y * (tCb - tSq);
		tg->watt[i] = (r < 0.0) ? 0.0 : (1.0 < r) ? 1.0 : r;
	}
}

/* src/tonegen.cpp:1335-1369 fitWave */
size_t orc_fitwave (double Hz, double precision, int minSamples, int maxSamples, double rate)
{
	double minErr = 99999.9, minSpn = 0.0;
	int    i, minWaves, maxWaves;
	minWaves = (int)ceil ((Hz * (double)minSamples) / rate);
	maxWaves = (int)floor ((Hz * (double)maxSamples) / rate);
	for (i = minWaves; i <= maxWaves; i++) {
		double nws = (rate * i) / Hz;
		double spn = rint (nws);
		double err = fabs (nws - spn);
		if (err < minErr) {
			minErr = err;
			minSpn = spn;
		}
		if (err < precision)
			break;
	}
	return (size_t)minSpn;
}

/* src/tonegen.cpp:1402-1457 writeSamples: 12 partials, Nyquist mute, random LSB */
static void writeSamples (float* buf, size_t len, const double* ap, double attenuation, double f1Hz,
                          double rate, orc_rand* rnd)
{
	const double fullCircle = 2.0 * M_PI;
	double       apl[ORC_MAX_PARTIALS], plHz[ORC_MAX_PARTIALS], aplSum, U;
	unsigned int i;
	for (i = 0, aplSum = 0.0; i < ORC_MAX_PARTIALS; i++) {
		apl[i] = ap[i];
		aplSum += fabs (apl[i]);
		plHz[i] = f1Hz * ((double)(i + 1));
		if ((rate * 0.5) <= plHz[i])
			apl[i] = 0.0;
	}
	U = attenuation / aplSum;
	for (i = 0; i < len; i++) {
		int    j;
		double s = 0.0;
		for (j = 0; j < ORC_MAX_PARTIALS; j++)
			s += apl[j] * sin (remainder ((plHz[j] * fullCircle * (double)i) / rate, fullCircle));
		buf[i] = (orc_rand_next (rnd) < (2147483647 >> 1)) ? (float)(1.0 / 32767.0) : 0.0f;
		buf[i] = (float)((double)buf[i] + (U * s));
	}
}

/* src/tonegen.cpp:1939-1966 initKeyCompTable */
static void initKeyCompTable (orc_template* t)
{
	int   i;
	float u = -5.0f, v = -9.0f;
	float m = (float)(1.0 / (128 - 12));
	t->keyCompTable[0] = t->keyCompTable[1] = 1.0f;
	t->keyCompTable[2]                      = (float)dBToGain (-1.1598);
	t->keyCompTable[3]                      = (float)dBToGain (-2.0291);
	t->keyCompTable[4]                      = (float)dBToGain (-2.4987);
	t->keyCompTable[5]                      = (float)dBToGain (-2.9952);
	t->keyCompTable[6]                      = (float)dBToGain (-3.5218);
	t->keyCompTable[7]                      = (float)dBToGain (-4.0823);
	t->keyCompTable[8]                      = (float)dBToGain (-4.6815);
	t->keyCompTable[9]                      = (float)dBToGain (-4.9975);
	t->keyCompTable[10]                     = (float)dBToGain (-4.9998);
	for (i = 11; i < 128; i++) {
		float a            = (float)(i - 11);
		t->keyCompTable[i] = (float)dBToGain (u + ((v - u) * a * m));
	}
}

/* src/tonegen.cpp:2562-2728 initEnvelopes with the default models
 * (attack = ENV_CLICK level 0.5, release = ENV_LINEAR; tonegen.cpp:247-251) */
static void initEnvelopes (orc_template* t, orc_rand* rnd, const orc_cfg* c)
{
	const double T = (double)(BSS - 1);
	int          b, i, burst, bound, start;
	for (b = 0; b < 9; b++) {
		if (c->envAttackModel == ORC_ENV_CLICK) {
			bound = t->envAtkClkMaxLength - t->envAtkClkMinLength;
			if (bound < 1)
				bound = 1;
			burst = t->envAtkClkMinLength + (orc_rand_next (rnd) % bound);
			if (BSS <= burst)
				burst = BSS - 1;
			start = (orc_rand_next (rnd) % (BSS - burst));
			for (i = 0; i < start; i++)
				t->attackEnv[b][i] = 0.0f;
			for (; i < (start + burst); i++) {
				double drnd        = ((double)orc_rand_next (rnd)) / (double)2147483647;
				t->attackEnv[b][i] = (float)(1.0 - (c->envAttackClickLevel * drnd));
			}
			for (; i < BSS; i++)
				t->attackEnv[b][i] = 1.0f;
			t->attackEnv[b][0] = (float)(t->attackEnv[b][0] / 2.0);
			for (i = 1; i < BSS; i++)
				t->attackEnv[b][i] = (float)((float)(t->attackEnv[b][i - 1] + t->attackEnv[b][i]) / 2.0);
		}
		if (c->envAttackModel == ORC_ENV_SHELF) {
			bound = t->envAtkClkMaxLength - t->envAtkClkMinLength;
			if (bound < 1)
				bound = 1;
			start = orc_rand_next (rnd) % bound;
			if ((BSS - 2) <= start)
				start = BSS - 2;
			for (i = 0; i < start; i++)
				t->attackEnv[b][i] = 0.0f;
			t->attackEnv[b][i + 0] = (float)0.33333333;
			t->attackEnv[b][i + 1] = (float)0.66666666;
			for (i = i + 2; i < BSS; i++)
				t->attackEnv[b][i] = 1.0f;
		}
		if (c->envReleaseModel == ORC_ENV_SHELF) {
			bound = t->envAtkClkMaxLength - t->envAtkClkMinLength;
			if (bound < 1)
				bound = 1;
			start = orc_rand_next (rnd) % bound;
			if ((BSS - 2) <= start)
				start = BSS - 2;
			for (i = 0; i < start; i++)
				t->releaseEnv[b][i] = 0.0f;
			t->releaseEnv[b][i + 0] = (float)0.33333333;
			t->releaseEnv[b][i + 1] = (float)0.66666666;
			for (i = i + 2; i < BSS; i++)
				t->releaseEnv[b][i] = 1.0f;
		}
		if (c->envReleaseModel == ORC_ENV_CLICK) {
			burst = 8 + (orc_rand_next (rnd) % 32);
			start = (orc_rand_next (rnd) % (BSS - burst));
			for (i = 0; i < start; i++)
				t->releaseEnv[b][i] = 0.0f;
			for (; i < (start + burst); i++) {
				double drnd         = ((double)orc_rand_next (rnd)) / (double)2147483647;
				t->releaseEnv[b][i] = (float)(1.0 - (c->envReleaseClickLevel * drnd));
			}
			for (; i < BSS; i++)
				t->releaseEnv[b][i] = 1.0f;
			t->releaseEnv[b][0] = (float)(t->releaseEnv[b][0] / 2.0);
			for (i = 1; i < BSS; i++)
				t->releaseEnv[b][i] = (float)((float)(t->releaseEnv[b][i - 1] + t->releaseEnv[b][i]) / 2.0);
		}
		if (c->envAttackModel == ORC_ENV_COSINE)
			for (i = 0; i < BSS; i++) {
				int    d          = BSS - (i + 1);
				double a          = (M_PI * (double)d) / T;
				t->attackEnv[b][i] = (float)(0.5 + (0.5 * cos (a)));
			}
		if (c->envReleaseModel == ORC_ENV_COSINE)
			for (i = 0; i < BSS; i++) {
				double a           = (M_PI * (double)i) / T;
				t->releaseEnv[b][i] = (float)(0.5 - (0.5 * cos (a)));
			}
		if (c->envAttackModel == ORC_ENV_LINEAR)
			for (i = 0; i < BSS; i++)
				t->attackEnv[b][i] = ((float)i) / (float)BSS;
		if (c->envReleaseModel == ORC_ENV_LINEAR)
			for (i = 0; i < BSS; i++)
				t->releaseEnv[b][i] = ((float)i) / (float)BSS;
	}
}

/* initToneGenerator (src/tonegen.cpp:2905-3066) minus the instance-runtime parts, with
 * the rand() stream seeded explicitly (batch protocol). */
orc_template* orc_template_new (double sr, const double* mts128, const double* ratio9, unsigned int seed)
{
	return orc_template_new_cfg (sr, mts128, ratio9, seed, NULL);
}

orc_template* orc_template_new_cfg (double sr, const double* mts128, const double* ratio9, unsigned int seed,
                                    const orc_cfg* cfg)
{
	static const double defaultRatio[9] = {0.5, 1.5, 1, 2, 3, 4, 5, 6, 8};
	orc_template*       t               = (orc_template*)calloc (1, sizeof (orc_template));
	orc_rand            rnd;
	orc_cfg             dflt;
	int                 i, j;
	double              harm[ORC_MAX_PARTIALS];
	if (!cfg) {
		orc_cfg_default (&dflt);
		cfg = &dflt;
	}
	orc_srand (&rnd, seed);
	t->sr                 = sr;
	t->envAtkClkMinLength = cfg->envAtkClkMinLength;
	t->envAtkClkMaxLength = cfg->envAtkClkMaxLength;
	if (t->envAtkClkMinLength < 0)
		t->envAtkClkMinLength = (int)floor (sr * 8.0 / 22050.0);
	if (t->envAtkClkMaxLength < 0)
		t->envAtkClkMaxLength = (int)ceil (sr * 40.0 / 22050.0);
	if (t->envAtkClkMinLength > BSS)
		t->envAtkClkMinLength = BSS;
	if (t->envAtkClkMaxLength > BSS)
		t->envAtkClkMaxLength = BSS;
	orc_get_frequencies (t->frequency, mts128);
	for (i = 0; i < 9; i++)
		t->targetRatio[i] = ratio9 ? ratio9[i] : defaultRatio[i];
	/* the cfg's terminal / taper / crosstalk lists, in file order (oscConfig) */
	for (j = 0; j < cfg->nle; j++) {
		const int k = cfg->le[j].idx;
		switch (cfg->le[j].kind) {
			case ORC_LE_TERMINAL: lst_push (&t->terminalMix[k], cfg->le[j].sa, 0, cfg->le[j].fc); break;
			case ORC_LE_TAPER: lst_push (&t->keyTaper[k], cfg->le[j].sa, cfg->le[j].sb, cfg->le[j].fc); break;
			case ORC_LE_XTALK: lst_push (&t->keyCrosstalk[k], cfg->le[j].sa, cfg->le[j].sb, cfg->le[j].fc); break;
		}
	}
	applyDefaultConfiguration (t, cfg);
	compilePlayMatrix (t, cfg);
	/* initOscillators (tonegen.cpp:1470-1630) */
	if (cfg->eqMacro == ORC_EQ_SPLINE)
		applySpline (t, NW, cfg->eqP1y, cfg->eqR1y, cfg->eqP4y, cfg->eqR4y);
	else
		applyPeak (t, NW, cfg->eqMacro == ORC_EQ_PEAK46);
	for (i = 1; i <= NW; i++) {
		int e;
		t->wfreq[i] = oscFreq (t, i);
		t->wlen[i]  = orc_fitwave (t->wfreq[i], cfg->tgPrecision, 3 * BSS, (int)(ceil (sr / 48000.0) * 4096), sr);
		t->wave[i]  = (float*)malloc (sizeof (float) * t->wlen[i]);
		/* compile-time harmonics, then the cfg's global ones, then this wheel's */
		for (j = 0; j < ORC_MAX_PARTIALS; j++)
			harm[j] = j == 0 ? 1.0 : 0.0;
		for (e = 0; e < cfg->nle; e++)
			if (cfg->le[e].kind == ORC_LE_HARMONIC && cfg->le[e].idx == 0 && cfg->le[e].sa - 1 < ORC_MAX_PARTIALS)
				harm[cfg->le[e].sa - 1] += cfg->le[e].fc;
		for (e = 0; e < cfg->nle; e++)
			if (cfg->le[e].kind == ORC_LE_HARMONIC && cfg->le[e].idx == i && cfg->le[e].sa - 1 < ORC_MAX_PARTIALS)
				harm[cfg->le[e].sa - 1] += cfg->le[e].fc;
		writeSamples (t->wave[i], t->wlen[i], harm, t->watt[i], t->wfreq[i], sr, &rnd);
	}
	initKeyCompTable (t);
	initEnvelopes (t, &rnd, cfg);
	return t;
}

void orc_template_free (orc_template* t)
{
	int i;
	if (!t)
		return;
	for (i = 0; i <= NW; i++) {
		free (t->wave[i]);
		free (t->terminalMix[i].v);
	}
	for (i = 0; i < ORC_MAX_KEYS; i++) {
		free (t->keyTaper[i].v);
		free (t->keyCrosstalk[i].v);
		free (t->keyContrib[i].v);
	}
	free (t);
}

size_t orc_template_bank_size (const orc_template* t)
{
	size_t n = 0;
	int    i;
	for (i = 1; i <= NW; i++)
		n += t->wlen[i];
	return n;
}

void orc_template_bank (const orc_template* t, float* out, uint32_t* lens)
{
	size_t o = 0;
	int    i;
	for (i = 1; i <= NW; i++) {
		memcpy (out + o, t->wave[i], sizeof (float) * t->wlen[i]);
		lens[i - 1] = (uint32_t)t->wlen[i];
		o += t->wlen[i];
	}
}

void orc_template_envs (const orc_template* t, float* a, float* r, float* kc)
{
	memcpy (a, t->attackEnv, sizeof (t->attackEnv));
	memcpy (r, t->releaseEnv, sizeof (t->releaseEnv));
	memcpy (kc, t->keyCompTable, sizeof (t->keyCompTable));
}

/* DEBUG_TONEGEN_OSC dumps: src/tonegen.cpp:1974-2084, 2089-2134, 2139-2166 */
int orc_template_dump (const orc_template* t, const char* dir)
{
	char  fn[4096];
	FILE* fp;
	int   i, j, k;
	snprintf (fn, sizeof (fn), "%s/osc_cfglists.txt", dir);
	if (!(fp = fopen (fn, "w")))
		return -1;
	fprintf (fp, "%s\n\n", "Array wheelHarmonics (index is wheel number)");
	for (i = 0; i <= NW; i++)
		fprintf (fp, "wheelHarmonics[%2d]=NULL\n", i);
	fprintf (fp, "\n%s\n\n", "Array terminalMix (index is terminal number)");
	for (i = 0; i <= NW; i++) {
		fprintf (fp, "terminalMix[%2d]=", i);
		if (t->terminalMix[i].n == 0)
			fprintf (fp, "NULL");
		for (j = 0; j < t->terminalMix[i].n; j++) {
			if (j)
				fprintf (fp, ", ");
			fprintf (fp, "w%d:%f", t->terminalMix[i].v[j].sa, t->terminalMix[i].v[j].fc);
		}
		fprintf (fp, "\n");
	}
	fprintf (fp, "\n%s\n\n", "Array keyTaper (index is keynumber)");
	for (i = 0; i < ORC_MAX_KEYS; i++) {
		fprintf (fp, "keyTaper[%2d]=", i);
		if (t->keyTaper[i].n == 0)
			fprintf (fp, "NULL");
		for (j = 0; j < t->keyTaper[i].n; j++) {
			if (j)
				fprintf (fp, ", ");
			fprintf (fp, "t%d:b%d:g%f", t->keyTaper[i].v[j].sa, t->keyTaper[i].v[j].sb, t->keyTaper[i].v[j].fc);
		}
		fprintf (fp, "\n");
	}
	fprintf (fp, "\n%s\n\n", "Array keyCrosstalk (index is keynumber)");
	for (i = 0; i < ORC_MAX_KEYS; i++) {
		fprintf (fp, "keyCrosstalk[%2d]=", i);
		if (t->keyCrosstalk[i].n == 0)
			fprintf (fp, "NULL");
		for (j = 0; j < t->keyCrosstalk[i].n; j++) {
			if (j)
				fprintf (fp, ", ");
			fprintf (fp, "b%d:t%d:g%f", t->keyCrosstalk[i].v[j].sb, t->keyCrosstalk[i].v[j].sa,
			         t->keyCrosstalk[i].v[j].fc);
		}
		fprintf (fp, "\n");
	}
	fprintf (fp, "\nEnd of dump\n");
	fclose (fp);

	snprintf (fn, sizeof (fn), "%s/osc_runtime.txt", dir);
	if (!(fp = fopen (fn, "w")))
		return -1;
	fprintf (fp, "%s\n\n", "Array keyContrib (index is key number)");
	for (k = 0; k < ORC_MAX_KEYS; k++) {
		int wcount = 0, lastWheel = -1;
		fprintf (fp, "keyContrib[%3d]=", k);
		for (j = 0; j < t->keyContrib[k].n; j++) {
			const orc_le* rep     = &t->keyContrib[k].v[j];
			double        dbLevel = 20.0 * log10 (rep->fc);
			int           x;
			if (j)
				fprintf (fp, "%16c", ' ');
			fprintf (fp, "[w%2d:b%2d:g%f] % 10.6lf dB  ", rep->sa, rep->sb, rep->fc, dbLevel);
			if (-60.0 < dbLevel) {
				int len = (int)(25.0 * rep->fc / 3.0);
				for (x = 0; x < len; x++)
					fprintf (fp, "I");
			}
			fprintf (fp, "\n");
			if (lastWheel != rep->sa) {
				wcount++;
				lastWheel = rep->sa;
			}
		}
		fprintf (fp, "%2d wheels, %3d entries\n", wcount, t->keyContrib[k].n);
	}
	fclose (fp);

	snprintf (fn, sizeof (fn), "%s/osc.txt", dir);
	if (!(fp = fopen (fn, "w")))
		return -1;
	{
		size_t total = 0;
		fprintf (fp, "Oscillator dump\n");
		fprintf (fp, "[%3s]:%10s:%5s:%6s:%5s\n", "OSC", "Frequency", "Sampl", "Bytes", "Gain");
		for (i = 0; i < NW; i++) {
			fprintf (fp, "[%3d]:%7.2lf Hz:%5zu:%6zu:%5.2lf\n", i, i ? t->wfreq[i] : 0.0, i ? t->wlen[i] : 0,
			         (i ? t->wlen[i] : 0) * sizeof (float), i ? t->watt[i] : 0.0);
			total += i ? t->wlen[i] : 0;
		}
		fprintf (fp, "TOTAL MEMORY: %zu samples, %zu bytes\n", total, total * sizeof (float));
	}
	fclose (fp);
	return 0;
}

/* ------------------------------------------------------------------ vibrato */

/* src/vibrato.cpp:312-329 reset_vibrato + init_vibrato (setScannerFrequency 91-95,
 * initIncrementTables 224-283, setVibrato(v, 0)) */
void orc_vibrato_init (orc_vibrato* v, double rate, const orc_cfg* c)
{
	int    i;
	double S = 65536.0;
	memset (v, 0, sizeof (*v));
	v->offsetTable     = v->offset3Table;
	v->stator          = 0;
	v->outPos          = 1023 / 2;
	v->vib1OffAmp      = c->vib1OffAmp;
	v->vib2OffAmp      = c->vib2OffAmp;
	v->vib3OffAmp      = c->vib3OffAmp;
	v->vibFqHertz      = c->vibFqHertz;
	v->statorIncrement = (unsigned int)(((v->vibFqHertz * 2048) / rate) * 65536.0);
	for (i = 0; i < 2048; i++) {
		double m           = sin ((2.0 * M_PI * i) / 2048);
		v->offset1Table[i] = (unsigned int)((1.0 + v->vib1OffAmp + (m * v->vib1OffAmp)) * S);
		v->offset2Table[i] = (unsigned int)((1.0 + v->vib2OffAmp + (m * v->vib2OffAmp)) * S);
		v->offset3Table[i] = (unsigned int)((1.0 + v->vib3OffAmp + (m * v->vib3OffAmp)) * S);
	}
	v->effectEnabled = 0;
	v->mixedBuffers  = 0;
}

/* src/vibrato.cpp:97-129 setVibrato / setVibratoFromInt */
static void setVibrato (orc_vibrato* v, int select)
{
	switch (select & 3) {
		case 0: v->effectEnabled = 0; break;
		case 1: v->effectEnabled = 1; v->offsetTable = v->offset1Table; break;
		case 2: v->effectEnabled = 1; v->offsetTable = v->offset2Table; break;
		case 3: v->effectEnabled = 1; v->offsetTable = v->offset3Table; break;
	}
	v->mixedBuffers = select & 0x80;
}

void orc_tg_set_vibrato_from_int (orc_tonegen* t, int param)
{
	static const int map[6] = {0x01, 0x81, 0x02, 0x82, 0x03, 0x83};
	if (param >= 0 && param < 6)
		setVibrato (&t->vib, map[param]);
}

/* src/vibrato.cpp:365-411 vibratoProc */
void orc_vibrato_proc (orc_vibrato* v, const float* in, float* out, size_t n)
{
	const float  fnorm   = (float)(1.0 / 65536.0);
	const float  mixnorm = (float)0.7071067811865475;
	unsigned int i;
	for (i = 0; i < n; i++) {
		const float        x = in[i];
		const unsigned int j = ((v->outPos << 16) + v->offsetTable[v->stator >> 16]) & 0x03FFFFFF;
		const int          h = j >> 16;
		const int          k = (h + 1) & 0x3FF;
		const float        f = fnorm * ((float)(j & 0xFFFF));
		const float        g = f * x;
		v->vibBuffer[h] += x - g;
		v->vibBuffer[k] += g;
		if (v->mixedBuffers)
			out[i] = (x + v->vibBuffer[v->outPos]) * mixnorm;
		else
			out[i] = v->vibBuffer[v->outPos];
		v->vibBuffer[v->outPos] = 0;
		v->outPos               = (v->outPos + 1) & 0x3FF;
		v->stator               = (v->stator + v->statorIncrement) & 0x07ffffff;
	}
}

/* ------------------------------------------------------------------ tonegen runtime */

/* src/tonegen.cpp:2738-2750 setDrawBar */
void orc_tg_set_drawbar (orc_tonegen* t, int bus, unsigned int setting)
{
	t->drawBarChange = 1;
	if (bus == t->percTriggerBus) {
		t->percTrigRestore = setting;
		if (t->percEnabled)
			return;
	}
	t->drawBarGain[bus] = t->drawBarLevel[bus][setting];
}

/* src/tonegen.cpp:2752-2756 */
static void setMIDIDrawBar (orc_tonegen* t, int bus, unsigned char v)
{
	int val = 127 - v;
	orc_tg_set_drawbar (t, bus, (unsigned int)rint (val * 8.0 / 127.0));
}

/* src/tonegen.cpp:1635-1660 */
void orc_tg_set_vibrato_upper (orc_tonegen* t, int on)
{
	if (on)
		t->newRouting |= 0x02;
	else
		t->newRouting &= ~0x02u;
}
void orc_tg_set_vibrato_lower (orc_tonegen* t, int on)
{
	if (on)
		t->newRouting |= 0x01;
	else
		t->newRouting &= ~0x01u;
}

/* src/tonegen.cpp:1678-1765 percussion setters */
void orc_tg_set_perc_enabled (orc_tonegen* t, int on)
{
	if (on) {
		t->newRouting |= 0x0C;
		if (-1 < t->percTriggerBus) {
			t->drawBarGain[t->percTriggerBus] = 0.0f;
			t->drawBarChange                  = 1;
		}
	} else {
		t->newRouting &= ~0x0Cu;
		if (-1 < t->percTriggerBus) {
			t->drawBarGain[t->percTriggerBus] = t->drawBarLevel[t->percTriggerBus][t->percTrigRestore];
			t->drawBarChange                  = 1;
		}
	}
	t->percEnabled = on;
}
static void setPercussionResets (orc_tonegen* t)
{
	if (t->percIsFast)
		t->percEnvGainDecay = t->percIsSoft ? t->percEnvGainDecayFastSoft : t->percEnvGainDecayFastNorm;
	else
		t->percEnvGainDecay = t->percIsSoft ? t->percEnvGainDecaySlowSoft : t->percEnvGainDecaySlowNorm;
}
void orc_tg_set_perc_fast (orc_tonegen* t, int isFast)
{
	t->percIsFast = isFast;
	setPercussionResets (t);
}
void orc_tg_set_perc_volume (orc_tonegen* t, int isSoft)
{
	t->percIsSoft       = isSoft;
	t->percEnvGainReset = t->percEnvScaling * (isSoft ? t->percEnvGainResetSoft : t->percEnvGainResetNorm);
	t->percDrawbarGain  = isSoft ? t->percDrawbarSoftGain : t->percDrawbarNormalGain;
	setPercussionResets (t);
}
void orc_tg_set_perc_first (orc_tonegen* t, int isFirst)
{
	t->percSendBus = isFirst ? t->percSendBusA : t->percSendBusB;
}

/* allocTonegen (initValues, tonegen.cpp:238-331; resetVibrato) + the per-instance
 * part of initToneGenerator (tonegen.cpp:2914-3021) on a shared template. */
void orc_tg_init (orc_tonegen* t, const orc_template* tpl, const orc_cfg* c)
{
	int i, s;
	memset (t, 0, sizeof (*t));
	t->tpl                      = tpl;
	t->percSendBus              = 4;
	t->percSendBusA             = c->percSendBusA;
	t->percSendBusB             = c->percSendBusB;
	t->swellPedalGain           = 0.07f;
	t->outputLevelTrim          = 0.07f;
	t->percTriggerBus           = c->percTriggerBus;
	t->percEnvScaling           = c->percEnvScaling;
	t->percEnvGainResetNorm     = c->percEnvGainResetNorm;
	t->percEnvGainResetSoft     = c->percEnvGainResetSoft;
	t->percEnvGainDecayFastNorm = 0.9995f;
	t->percEnvGainDecayFastSoft = 0.9995f;
	t->percEnvGainDecaySlowNorm = 0.9999f;
	t->percEnvGainDecaySlowSoft = 0.9999f;
	t->percDrawbarNormalGain    = 0.60512f;
	t->percDrawbarSoftGain      = 1.0f;
	t->percDrawbarGain          = 1.0f;
	t->outputGain               = 1.0f;
	t->keyCompLevel             = 1.0f;
	for (i = 0; i <= NW; i++)
		t->aclPos[i] = -1;
	memcpy (t->keyCompTable, tpl->keyCompTable, sizeof (t->keyCompTable));
	for (i = 0; i < ORC_NOF_BUSES; i++)
		for (s = 0; s < 9; s++) {
			float u               = (float)s;
			t->drawBarLevel[i][s] = (float)(u / 8.0);
		}
	setMIDIDrawBar (t, 0, 8);
	setMIDIDrawBar (t, 1, 8);
	setMIDIDrawBar (t, 2, 6);
	setMIDIDrawBar (t, 9, 8);
	setMIDIDrawBar (t, 10, 3);
	setMIDIDrawBar (t, 11, 8);
	setMIDIDrawBar (t, 18, 8);
	setMIDIDrawBar (t, 20, 6);
	orc_tg_set_perc_first (t, 0);
	orc_tg_set_perc_volume (t, 0);
	orc_tg_set_perc_fast (t, 1);
	orc_tg_set_perc_enabled (t, 0);
	orc_vibrato_init (&t->vib, tpl->sr, c);
}

/* src/tonegen.cpp:3096-3166 oscKeyOff / oscKeyOn (msgQueue 1024 u16) */
void orc_tg_key_off (orc_tonegen* t, int key)
{
	if (key < 0 || ORC_MAX_KEYS <= key)
		return;
	if (t->activeKeys[key] != 0) {
		t->activeKeys[key] = 0;
		if (key < 128)
			t->upperKeyCount--;
		t->keyDownCount--;
		t->msgQueue[t->msgW++] = (unsigned short)(0x0000 | (key & 0x0fff));
		if (t->msgW == 1024)
			t->msgW = 0;
	}
}

void orc_tg_key_on (orc_tonegen* t, int key)
{
	if (key < 0 || ORC_MAX_KEYS <= key)
		return;
	if (t->activeKeys[key] != 0)
		orc_tg_key_off (t, key);
	t->activeKeys[key] = 1;
	if (key < 128)
		t->upperKeyCount++;
	t->keyDownCount++;
	t->msgQueue[t->msgW++] = (unsigned short)(0x1000 | (key & 0x0fff));
	if (t->msgW == 1024)
		t->msgW = 0;
}

/* src/tonegen.cpp:3218-3778 oscGenerateFragment */
void orc_tg_generate (orc_tonegen* t, float* buf)
{
	const orc_template* tpl = t->tpl;
	int                 i;
	unsigned int        copyDone = 0, recomputeRouting;
	int                 removedEnd = 0;
	orc_coreins*        cw         = t->corePgm;
	const float         keyComp    = t->keyCompTable[t->keyDownCount];
	const float         keyCompDelta = (keyComp - t->keyCompLevel) / (float)BSS;

	/* message queue (3257-3327) */
	while (t->msgR != t->msgW) {
		unsigned short msg = t->msgQueue[t->msgR++];
		int            kn, e;
		if (t->msgR == 1024)
			t->msgR = 0;
		kn = msg & 0x0fff;
		if ((msg & 0xf000) == 0x1000) {
			for (e = 0; e < tpl->keyContrib[kn].n; e++) {
				const orc_le* lep = &tpl->keyContrib[kn].v[e];
				int           wn  = lep->sa;
				if (t->aot[wn].refCount == 0) {
					t->rflags[wn] = 0x0006;
					if (t->aclPos[wn] == -1) {
						t->aclPos[wn]                          = t->activeOscLEnd;
						t->activeOscList[t->activeOscLEnd++] = wn;
					}
				} else {
					t->rflags[wn] |= 0x0004;
				}
				t->aot[wn].busLevel[lep->sb] += lep->fc;
				t->aot[wn].keyCount[lep->sb] += 1;
				t->aot[wn].refCount += 1;
			}
		} else {
			for (e = 0; e < tpl->keyContrib[kn].n; e++) {
				const orc_le* lep = &tpl->keyContrib[kn].v[e];
				int           wn  = lep->sa;
				t->aot[wn].busLevel[lep->sb] -= lep->fc;
				t->aot[wn].keyCount[lep->sb] -= 1;
				t->aot[wn].refCount -= 1;
				if (t->aot[wn].refCount == 0)
					t->rflags[wn] = 0x0005;
				else
					t->rflags[wn] |= 0x0004;
			}
		}
	}

	/* activated list (3333-3566) */
	if ((recomputeRouting = (t->oldRouting != t->newRouting)))
		t->oldRouting = t->newRouting;

	for (i = 0; i < t->activeOscLEnd; i++) {
		int      on  = t->activeOscList[i];
		orc_aot* aop = &t->aot[on];
		size_t   len = tpl->wlen[on];
		if (t->rflags[on] & 0x0001) {
			t->removedList[removedEnd++] = (unsigned short)on;
			cw->envRow                   = 8 + (i & 7);
			cw->envOff                   = 0;
			if (copyDone)
				cw->opr = 3;
			else {
				cw->opr  = 2;
				copyDone = 1;
			}
			cw->wheel  = on;
			cw->src    = t->pos[on];
			cw->off    = 0;
			cw->sgain  = aop->sumSwell;
			cw->pgain  = aop->sumPercn;
			cw->vgain  = aop->sumScanr;
			cw->nsgain = cw->npgain = cw->nvgain = 0.0f;
			if (len < (t->pos[on] + BSS)) {
				orc_coreins* prev = cw;
				cw->cnt           = (int)(len - t->pos[on]);
				t->pos[on]        = BSS - cw->cnt;
				cw += 1;
				*cw        = *prev;
				cw->src    = 0;
				cw->off    = prev->cnt;
				cw->envOff = prev->envOff + prev->cnt;
				cw->cnt    = (int)t->pos[on];
			} else {
				cw->cnt = BSS;
				t->pos[on] += BSS;
			}
			cw += 1;
		} else {
			int reroute = 0;
			if (t->rflags[on] & 0x0002) {
				cw->sgain = cw->pgain = cw->vgain = 0.0f;
			} else {
				cw->sgain = aop->sumSwell;
				cw->pgain = aop->sumPercn;
				cw->vgain = aop->sumScanr;
			}
			if ((t->rflags[on] & 0x0004) || t->drawBarChange) {
				int   d;
				float sum = 0.0f;
				for (d = 0; d < 9; d++)
					sum += aop->busLevel[d] * t->drawBarGain[d];
				aop->sumUpper = sum;
				sum           = 0.0f;
				for (d = 9; d < 18; d++)
					sum += aop->busLevel[d] * t->drawBarGain[d];
				aop->sumLower = sum;
				sum           = 0.0f;
				for (d = 18; d < 27; d++)
					sum += aop->busLevel[d] * t->drawBarGain[d];
				aop->sumPedal = sum;
				reroute       = 1;
			}
			if (reroute || recomputeRouting) {
				if (t->oldRouting & 0x0C)
					aop->sumPercn = aop->busLevel[t->percSendBus];
				else
					aop->sumPercn = 0.0f;
				aop->sumScanr = 0.0f;
				aop->sumSwell = aop->sumPedal;
				if (t->oldRouting & 0x02)
					aop->sumScanr += aop->sumUpper;
				else
					aop->sumSwell += aop->sumUpper;
				if (t->oldRouting & 0x01)
					aop->sumScanr += aop->sumLower;
				else
					aop->sumSwell += aop->sumLower;
			}
			if (t->rflags[on] & 0x0006) {
				cw->envRow = i & 7;
				cw->envOff = 0;
				cw->nsgain = aop->sumSwell;
				cw->npgain = aop->sumPercn;
				cw->nvgain = aop->sumScanr;
				if (copyDone)
					cw->opr = 3;
				else {
					cw->opr  = 2;
					copyDone = 1;
				}
			} else {
				cw->envRow = -1;
				cw->envOff = 0;
				if (copyDone)
					cw->opr = 1;
				else {
					cw->opr  = 0;
					copyDone = 1;
				}
			}
			cw->wheel = on;
			cw->src   = t->pos[on];
			cw->off   = 0;
			if (len < (t->pos[on] + BSS)) {
				orc_coreins* prev = cw;
				cw->cnt           = (int)(len - t->pos[on]);
				t->pos[on]        = BSS - cw->cnt;
				cw += 1;
				*cw     = *prev;
				cw->src = 0;
				cw->off = prev->cnt;
				if (cw->opr & 2)
					cw->envOff = prev->envOff + prev->cnt;
				cw->cnt = (int)t->pos[on];
			} else {
				cw->cnt = BSS;
				t->pos[on] += BSS;
			}
			cw += 1;
		}
		t->rflags[on] = 0;
	}
	t->drawBarChange = 0;

	/* removal list (3576-3594) */
	for (i = 0; i < removedEnd; i++) {
		int vic = t->removedList[i];
		int act = t->aclPos[vic];
		t->aclPos[vic] = -1;
		t->activeOscLEnd--;
		if (0 < t->activeOscLEnd) {
			int mov = t->activeOscList[t->activeOscLEnd];
			if (mov != vic) {
				t->activeOscList[act] = mov;
				t->aclPos[mov]        = act;
			}
		}
	}

	t->corePgmLen = (int)(cw - t->corePgm);
	/* core interpreter (3607-3687) */
	if (cw == t->corePgm) {
		for (i = 0; i < BSS; i++)
			t->swlBuffer[i] = t->vibBuffer[i] = t->prcBuffer[i] = 0.0f;
	}
	{
		orc_coreins* cr;
		for (cr = t->corePgm; cr < cw; cr++) {
			short        opr = cr->opr;
			int          n   = cr->cnt;
			float*       ys  = t->swlBuffer + cr->off;
			float*       yv  = t->vibBuffer + cr->off;
			float*       yp  = t->prcBuffer + cr->off;
			const float  gs  = cr->sgain;
			const float  gv  = cr->vgain;
			const float  gp  = cr->pgain;
			const float  ds  = cr->nsgain - gs;
			const float  dv  = cr->nvgain - gv;
			const float  dp  = cr->npgain - gp;
			const float* xp  = tpl->wave[cr->wheel] + cr->src;
			const float* ep  = cr->envRow < 0 ? NULL
			                 : (cr->envRow < 8 ? tpl->attackEnv[cr->envRow] : tpl->releaseEnv[cr->envRow - 8]) + cr->envOff;
			if (opr & 1) {
				if (opr & 2) {
					for (; 0 < n; n--) {
						float       x = *xp++;
						const float e = *ep++;
						*ys++ += x * (gs + (e * ds));
						*yv++ += x * (gv + (e * dv));
						*yp++ += x * (gp + (e * dp));
					}
				} else {
					for (; 0 < n; n--) {
						const float x = *xp++;
						*ys++ += x * gs;
						*yv++ += x * gv;
						*yp++ += x * gp;
					}
				}
			} else {
				if (opr & 2) {
					for (; 0 < n; n--) {
						const float x = *xp++;
						const float e = *ep++;
						*ys++         = x * (gs + (e * ds));
						*yv++         = x * (gv + (e * dv));
						*yp++         = x * (gp + (e * dp));
					}
				} else {
					for (; 0 < n; n--) {
						const float x = *xp++;
						*ys++         = x * gs;
						*yv++         = x * gv;
						*yp++         = x * gp;
					}
				}
			}
		}
	}

	/* mixdown (3699-3777) */
	if (t->oldRouting & 0x03)
		orc_vibrato_proc (&t->vib, t->vibBuffer, t->vibYBuffr, BSS);
	{
		const float* xp = t->swlBuffer;
		const float* vp = t->vibYBuffr;
		const float* pp = t->prcBuffer;
		float*       yp = buf;
		if (t->oldRouting & 0x0C) {
			float* tp   = &(t->prcBuffer[BSS - 1]);
			float  temp = *tp;
			float* qq   = tp - 1;
			for (i = 1; i < BSS; i++) {
				*tp = *qq - *tp;
				tp--;
				qq--;
			}
			*tp   = t->pz - *tp;
			t->pz = temp;
			pp    = t->prcBuffer;
			t->outputGain = t->swellPedalGain * t->percDrawbarGain;
			if (t->oldRouting & 0x03) {
				for (i = 0; i < BSS; i++) {
					*yp++ = (t->outputGain * t->keyCompLevel * ((*xp++) + (*vp++) + ((*pp++) * t->percEnvGain)));
					t->percEnvGain *= t->percEnvGainDecay;
					t->keyCompLevel += keyCompDelta;
				}
			} else {
				for (i = 0; i < BSS; i++) {
					*yp++ = (t->outputGain * t->keyCompLevel * ((*xp++) + ((*pp++) * t->percEnvGain)));
					t->percEnvGain *= t->percEnvGainDecay;
					t->keyCompLevel += keyCompDelta;
				}
			}
		} else if (t->oldRouting & 0x03) {
			for (i = 0; i < BSS; i++) {
				*yp++ = (t->swellPedalGain * t->keyCompLevel * ((*xp++) + (*vp++)));
				t->keyCompLevel += keyCompDelta;
			}
		} else {
			for (i = 0; i < BSS; i++) {
				*yp++ = (t->swellPedalGain * t->keyCompLevel * (*xp++));
				t->keyCompLevel += keyCompDelta;
			}
		}
	}
	if (t->upperKeyCount == 0)
		t->percEnvGain = t->percEnvGainReset;
}

int orc_template_contrib (const orc_template* t, int key, int16_t* wheel, int16_t* bus, float* level, int cap)
{
	int i;
	for (i = 0; i < t->keyContrib[key].n && i < cap; i++) {
		wheel[i] = t->keyContrib[key].v[i].sa;
		bus[i]   = t->keyContrib[key].v[i].sb;
		level[i] = t->keyContrib[key].v[i].fc;
	}
	return t->keyContrib[key].n;
}
