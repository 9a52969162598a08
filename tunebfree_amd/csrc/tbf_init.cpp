/*
 * tbf_init.cpp -- host table builders and tonegen control plane (see tbf_host.h).
 * Each function cites the reference code whose arithmetic it reproduces.
 */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <limits>

#include "tbf_host.h"
#include "tbf_rand.h"

namespace tbf {

/* glibc srandom_r/random_r TYPE_3 (degree 31, separation 3) */
GlibcRand::GlibcRand (unsigned int seed)
{
	if (seed == 0)
		seed = 1;
	int32_t word = (int32_t)seed;
	s[0]         = word;
	for (int i = 1; i < 31; ++i) {
		int64_t hi = word / 127773;
		int64_t lo = word % 127773;
		int64_t w  = 16807 * lo - 2836 * hi;
		if (w < 0)
			w += 2147483647;
		word = (int32_t)w;
		s[i] = word;
	}
	f = 3;
	r = 0;
	for (int i = 0; i < 310; ++i)
		next ();
}

int32_t GlibcRand::next ()
{
	uint32_t val = (uint32_t)s[f] + (uint32_t)s[r];
	s[f]         = (int32_t)val;
	if (++f >= 31) {
		f = 0;
		++r;
	} else if (++r >= 31) {
		r = 0;
	}
	return (int32_t)(val >> 1);
}

void GlibcRand::window (uint32_t* W) const
{
	for (int j = 0; j < 31; j++)
		W[j] = (uint32_t)s[(f + j) % 31];
}

void GlibcRand::discard (uint64_t k)
{
	uint32_t W[31], E[61], W2[31];
	window (W);
	gr_extend (W, E);
	gr_jump_window (E, k, W2);
	for (int j = 0; j < 31; j++)
		s[j] = (int32_t)W2[j];
	f = 0;
	r = 28;
}

static double dBToGain (double dB) { return pow (10.0, (dB / 20.0)); }

/* src/tuning.cpp:48-147 */
static void frequencies (double* f, const double* mts128)
{
	for (int i = 0; i < 128; i++)
		f[i] = mts128 ? mts128[i] : 440. * pow (2., (i - 69.) / 12.);
	int   scaleSize = -1;
	float period    = -1.0f;
	bool  found     = false;
	for (float p = 2.0f; p < 10.0f && !found; p++)
		for (int s = 1; s < 128 && !found; s++) {
			bool mismatch = false;
			for (int i = 0; i < 128 - s; i++)
				if (fabs (f[i + s] / f[i] - p) > 1e-6) {
					mismatch = true;
					break;
				}
			if (!mismatch) {
				scaleSize = s;
				period    = p;
				found     = true;
			}
		}
	for (int s = 1; s < 128 && !found; s++) {
		float p        = (float)(f[s] / f[0]);
		bool  mismatch = false;
		for (int i = 0; i < 128 - s; i++)
			if (fabs (f[i + s] / f[i] - p) > 1e-6) {
				mismatch = true;
				break;
			}
		if (!mismatch) {
			scaleSize = s;
			period    = p;
			found     = true;
		}
	}
	for (int i = 128; i < 300; i++)
		f[i] = scaleSize > 0 ? period * f[i - scaleSize] : f[127];
}

/* src/tonegen.cpp:502-692 */
static double taper (int key, int bus)
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

/* src/tuning.cpp:153-174 (wheel pairs table is reference data) */
static short pairedWheel (short n)
{
	static const short wp[92] = {0, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63, 64, 65, 66, 67, 68, 69,
	                             70, 71, 72, 73, 74, 75, 76, 77, 78, 79, 80, 81, 82, 83, 84, 0, 0, 0, 0, 0, 85, 86,
	                             87, 88, 89, 90, 91, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
	                             19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 42, 43, 44,
	                             45, 46, 47, 48};
	return (short)((n / 92) * 92 + wp[n % 92]);
}

static const short kTerminalStrip[] = {
	85, 42, 30, 76, 66, 18, 6, 54, 90, 35, 83, 71, 23, 11, 59, 47, 40, 28, 76, 64, 16, 4, 52, 88, 33, 81, 69, 21, 9,
	57, 45, 34, 26, 74, 62, 14, 2, 50, 86, 43, 31, 79, 67, 19, 7, 55, 91, 36, 84, 72, 24, 12, 60, 48, 41, 29, 77, 65,
	17, 5, 53, 89, 34, 82, 70, 22, 10, 58, 46, 39, 27, 75, 63, 15, 3, 51, 87, 32, 80, 68, 20, 8, 56, 44, 37, 25, 73,
	61, 13, 1, 49, 0};

struct Le {
	short sa, sb;
	float fc;
};

/* the cfg's lists (cf.lists: a key / terminal with its own list keeps it and gets no
 * default) and the default terminal mix (src/tonegen.cpp:949-997) */
static void matrixLists (const Config& cf, std::vector<Le>* terminalMix, std::vector<Le>* keyTaper,
                         std::vector<Le>* keyCrosstalk)
{
	for (const Config::ListEntry& e : cf.lists) {
		if (e.kind == LE_TERMINAL)
			terminalMix[e.idx].push_back ({e.sa, 0, e.fc});
		else if (e.kind == LE_TAPER)
			keyTaper[e.idx].push_back ({e.sa, e.sb, e.fc});
		else if (e.kind == LE_XTALK)
			keyCrosstalk[e.idx].push_back ({e.sa, e.sb, e.fc});
	}
	for (int i = 1; i <= TBF_NW; i++) {
		if (!terminalMix[i].empty ())
			continue;
		terminalMix[i].push_back ({(short)i, 0, (float)(1.0 - cf.compartmentXT)});
		if (0.0 < cf.compartmentXT) {
			short pw = pairedWheel ((short)i);
			if (0 < pw && pw <= TBF_NW)
				terminalMix[i].push_back ({pw, 0, (float)cf.compartmentXT});
		}
	}
	/* transformer crosstalk (971-997): configSet admits only 0, see tbf_config.cpp */
	if (0.0 < cf.stripXT)
		for (int i = 1; i <= TBF_NW; i++) {
			for (int j = 0; kTerminalStrip[j] > 0; j++) {
				if (kTerminalStrip[j] == (short)i) {
					int east = j > 0 ? kTerminalStrip[j - 1] : 0;
					int west = kTerminalStrip[j + 1];
					if (east > 0)
						terminalMix[i].push_back ({(short)east, 0, (float)cf.stripXT});
					if (west > 0)
						terminalMix[i].push_back ({(short)west, 0, (float)cf.stripXT});
					break;
				}
			}
		}
}

void MatrixInputs::build (const Config& cf)
{
	std::vector<Le> terminalMix[TBF_NW + 1], keyTaper[384], keyCrosstalk[384];
	matrixLists (cf, terminalMix, keyTaper, keyCrosstalk);
	auto flat = [] (const std::vector<Le>* lists, int n, std::vector<tbf_le>& v, std::vector<uint32_t>& off) {
		v.clear ();
		off.assign (1, 0u);
		size_t longest = 0;
		for (int i = 0; i < n; i++) {
			for (const Le& e : lists[i])
				v.push_back ({e.sa, e.sb, e.fc});
			off.push_back ((uint32_t)v.size ());
			longest = std::max (longest, lists[i].size ());
		}
		return longest;
	};
	const size_t M = flat (terminalMix, TBF_NW + 1, tm, tmOff);
	tmOff.push_back (tmOff.back ()); /* terminal TBF_NW + 1: none */
	/* a key's events: its taper list (<= 9 defaults) and crosstalk list (<= 9 per taper
	 * element by default), each element times its terminal's mix; cells <= wheels x buses */
	const size_t T = std::max<size_t> (9, flat (keyTaper, 384, tp, tpOff));
	const size_t X = std::max<size_t> (9 * T, flat (keyCrosstalk, 384, xt, xtOff));
	cap            = (uint32_t)std::max<size_t> (1, std::min<size_t> ((size_t)TBF_NW * 27, (T + X) * M));
	for (int k = 0; k < 128; k++)
		for (int b = 0; b < 9; b++)
			taper[k][b] = (float)tbf::taper (k, b);
	wiringXT = cf.wiringXT;
	floor    = cf.contribFloor;
	minLevel = cf.contribMin;
}

/* src/tonegen.cpp:933-1213 applyDefaultConfiguration + compilePlayMatrix (the device
 * builder k_tpl_matrix, tbf_tpl.hip, restates the same steps per key) */
static void playMatrix (TgTemplate& t)
{
	const Config&   cf = t.cfg;
	std::vector<Le> terminalMix[TBF_NW + 1], keyTaper[384], keyCrosstalk[384];
	matrixLists (cf, terminalMix, keyTaper, keyCrosstalk);
	/* applyManualDefaults (707-802) */
	double of[TBF_NW + 1];
	for (int i = 1; i <= TBF_NW; i++)
		of[i] = fmin (fmax (t.frequency[i - 1], 12.0), 2.5e10);
	for (int man = 0; man < 2; man++) {
		const int keyOffset = man * 128, busOffset = man * 9;
		for (int k = 0; k < 128; k++) {
			if (!keyTaper[k + keyOffset].empty ())
				continue;
			for (int b = 0; b < 9; b++) {
				float smallest = std::numeric_limits<float>::infinity ();
				int   best     = 0;
				for (int tn = 1; tn <= TBF_NW; tn++) {
					float ratio    = (float)(of[tn] / t.frequency[k]);
					float centDiff = (float)(1200 * fabs (log2 (t.targetRatio[b] / ratio)));
					if (centDiff < smallest) {
						smallest = centDiff;
						best     = tn;
					}
				}
				if (best != 1 && best != TBF_NW)
					keyTaper[k + keyOffset].push_back ({(short)best, (short)(b + busOffset), (float)taper (k, b)});
			}
		}
	}
	/* applyPedalDefaults (810-841) */
	static const int PDoffset[9] = {-12, 7, 0, 12, 19, 24, 28, 31, 36};
	for (int k = 0; k < 32; k++) {
		if (!keyTaper[k + 256].empty ())
			continue;
		for (int b = 0; b < 9; b++) {
			int tn = (k + 1) + PDoffset[b];
			if (tn < 1 || TBF_NW < tn)
				continue;
			keyTaper[k + 256].push_back ({(short)tn, (short)(b + 18), (float)dBToGain (0.0)});
		}
	}
	/* applyDefaultCrosstalk (849-879) */
	for (int man = 0; man < 2; man++)
		for (int k = 0; k < 128; k++) {
			const int kn = k + man * 128;
			if (!keyCrosstalk[kn].empty ())
				continue;
			for (int b = 0; b < 9; b++) {
				const int busNumber = man * 9 + b;
				for (const Le& e : keyTaper[kn]) {
					if (e.sb == busNumber)
						continue;
					keyCrosstalk[kn].push_back (
					    {e.sa, (short)busNumber, (float)((cf.wiringXT * e.fc) / abs (busNumber - e.sb))});
				}
			}
		}
	/* compilePlayMatrix + cpmInsert (1061-1213) */
	static thread_local unsigned char cpmBus[TBF_NW + 1][27]; /* templates build in parallel */
	static thread_local float         cpmGain[TBF_NW][27];
	short                wheelNumber[TBF_NW + 1];
	short                rowLength[TBF_NW];
	for (int k = 0; k < 384; k++) {
		int  endRow = 0;
		auto ins    = [&] (const Le& lep) {
            const int           terminal = lep.sa;
            const unsigned char bus      = (unsigned char)lep.sb;
            for (const Le& tl : terminalMix[terminal]) {
                float gain = tl.fc * lep.fc;
                short wnr  = tl.sa;
                if (gain == 0.0)
                    continue;
                int r, b;
                wheelNumber[endRow] = wnr;
                for (r = 0; wheelNumber[r] != wnr; r++)
                    ;
                if (r == endRow) {
                    rowLength[r] = 0;
                    endRow += 1;
                }
                int c        = rowLength[r];
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
		};
		for (const Le& e : keyTaper[k])
			ins (e);
		for (const Le& e : keyCrosstalk[k])
			ins (e);
		std::vector<Contrib>& out = t.keyContrib[k];
		for (int w = 0; w < endRow; w++)
			for (int c = 0; c < rowLength[w]; c++) {
				if (cpmGain[w][c] < cf.contribFloor)
					continue;
				Contrib rep {wheelNumber[w], (int16_t)cpmBus[w][c], cpmGain[w][c]};
				if (rep.level < cf.contribMin)
					rep.level = (float)cf.contribMin;
				size_t  at = 0;
				for (; at < out.size (); at++) {
					if (rep.wheel < out[at].wheel)
						break;
					if (rep.wheel == out[at].wheel && rep.bus < out[at].bus)
						break;
				}
				out.insert (out.begin () + (long)at, rep);
			}
	}
}

/* src/tonegen.cpp:1335-1369 */
static size_t fitWave (double Hz, double precision, int minSamples, int maxSamples, double rate)
{
	double minErr = 99999.9, minSpn = 0.0;
	int    minWaves = (int)ceil ((Hz * (double)minSamples) / rate);
	int    maxWaves = (int)floor ((Hz * (double)maxSamples) / rate);
	for (int i = minWaves; i <= maxWaves; i++) {
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

void TgTemplate::build (double rate, const double* mts128, const double* ratio9, unsigned int seed, const Config& c)
{
	GlibcRand rnd (seed);
	prepare (rate, mts128, ratio9, c);
	synthHost (rnd);
	finish (rnd);
}

void TgTemplate::prepare (double rate, const double* mts128, const double* ratio9, const Config& c, bool matrix)
{
	static const double defaultRatio[9] = {0.5, 1.5, 1, 2, 3, 4, 5, 6, 8};
	sr     = rate;
	cfg    = c;
	/* initToneGenerator (tonegen.cpp:2938-2955): click lengths from the rate unless set */
	envMin = c.envAtkClkMinLength < 0 ? (int)floor (sr * 8.0 / 22050.0) : c.envAtkClkMinLength;
	envMax = c.envAtkClkMaxLength < 0 ? (int)ceil (sr * 40.0 / 22050.0) : c.envAtkClkMaxLength;
	envMin = std::min (envMin, TBF_BLK);
	envMax = std::min (envMax, TBF_BLK);
	frequencies (frequency, mts128);
	for (int i = 0; i < 9; i++)
		targetRatio[i] = ratio9 ? ratio9[i] : defaultRatio[i];
	for (auto& v : keyContrib)
		v.clear ();
	if (matrix)
		playMatrix (*this);

	/* initOscillators (1470-1630): wheel EQ (apply_CH_Spline 1240-1261 or the legacy
	 * peak24 / peak46 damper curves 1223-1311), fitWave, the harmonics list (compile-time
	 * fundamental + the cfg's global harmonics + this wheel's), writeSamples with one
	 * rand() LSB per sample, wheels 1..256 in order */
	auto damper = [] (int thisTG, int firstTG, int lastTG, double w, double v, double u) {
		double x = ((double)(thisTG - firstTG)) / ((double)(lastTG - firstTG));
		double z = (x * (u - v)) - u;
		return 1.0 - w * z * z;
	};
	total = 0;
	for (int i = 1; i <= TBF_NW; i++) {
		double att;
		if (c.eqMacro == EQ_SPLINE) {
			double k   = TBF_NW - 1;
			double tt  = ((double)(i - 1)) / k;
			double tSq = tt * tt;
			double tCb = tSq * tt;
			double r   = c.eqP1y * (2.0 * tCb - 3.0 * tSq + 1.0) + c.eqP4y * (-2.0 * tCb + 3.0 * tSq) +
			           c.eqR1y * (tCb - 2.0 * tSq + tt) + c.eqR4y * (tCb - tSq);
			att = (r < 0.0) ? 0.0 : (1.0 < r) ? 1.0 : r;
		} else if (c.eqMacro == EQ_PEAK24) {
			att = i <= 43 ? damper (i, 1, 43, 0.2, -0.8, 1.0)
			    : i <= 48 ? damper (i, 44, 48, 1.6, -0.4, -0.3)
			              : damper (i, 49, TBF_NW, 0.9, -1.0, -0.7);
		} else {
			att = i <= 43 ? damper (i, 1, 43, 0.3, 0.4, 1.0)
			    : i <= 48 ? damper (i, 44, 48, 0.1, -0.4, 0.4)
			              : damper (i, 49, TBF_NW, 0.8, -1.0, -0.3);
		}
		const double wf  = fmin (fmax (frequency[i - 1], 12.0), 2.5e10);
		const size_t wl  = fitWave (wf, c.tgPrecision, 3 * TBF_BLK, (int)(ceil (sr / 48000.0) * 4096), sr);
		off[i]           = (uint32_t)total;
		len[i]           = (uint32_t)wl;
		total += wl;
		double harm[12];
		for (int j = 0; j < 12; j++)
			harm[j] = j == 0 ? 1.0 : 0.0;
		for (int pass = 0; pass < 2; pass++) /* wheelHarmonics[0], then wheelHarmonics[i] */
			for (const Config::ListEntry& e : c.lists)
				if (e.kind == LE_HARMONIC && e.idx == (pass ? i : 0) && e.sa - 1 < 12)
					harm[e.sa - 1] += e.fc;
		double apl[12], plHz[12], aplSum = 0.0;
		for (int j = 0; j < 12; j++) {
			apl[j] = harm[j];
			aplSum += fabs (apl[j]);
			plHz[j] = wf * ((double)(j + 1));
			if ((sr * 0.5) <= plHz[j])
				apl[j] = 0.0;
		}
		U[i] = att / aplSum;
		/* a partial of amplitude 0 adds 0 * sin (finite) = +-0 to the sum, which leaves
		 * it unchanged, so only the nonzero partials are kept (the default spectrum
		 * has one) */
		nPartials[i] = 0;
		for (int j = 0; j < 12; j++)
			if (apl[j] != 0.0) {
				pAmp[i][nPartials[i]] = apl[j];
				pHz[i][nPartials[i]]  = plHz[j];
				nPartials[i]++;
			}
	}
}

void TgTemplate::synthHost (GlibcRand& rnd)
{
	const double fullCircle = 2.0 * M_PI;
	bank.assign (total, 0.f);
	for (int i = 1; i <= TBF_NW; i++) {
		float* y = bank.data () + off[i];
		for (size_t n = 0; n < len[i]; n++) {
			double s = 0.0;
			for (int q = 0; q < nPartials[i]; q++)
				s += pAmp[i][q] * sin (remainder ((pHz[i][q] * fullCircle * (double)n) / sr, fullCircle));
			float v = (rnd.next () < (2147483647 >> 1)) ? (float)(1.0 / 32767.0) : 0.0f;
			y[n]    = (float)((double)v + (U[i] * s));
		}
	}
}

void TgTemplate::finish (GlibcRand& rnd)
{
	/* initKeyCompTable (1939-1966) */
	{
		float u = -5.0f, v = -9.0f, m = (float)(1.0 / (128 - 12));
		keyCompTable[0] = keyCompTable[1] = 1.0f;
		static const double t2[9] = {-1.1598, -2.0291, -2.4987, -2.9952, -3.5218, -4.0823, -4.6815, -4.9975, -4.9998};
		for (int i = 0; i < 9; i++)
			keyCompTable[2 + i] = (float)dBToGain (t2[i]);
		for (int i = 11; i < 128; i++) {
			float a         = (float)(i - 11);
			keyCompTable[i] = (float)dBToGain (u + ((v - u) * a * m));
		}
	}
	/* initEnvelopes (2562-2728): the four attack / release models; the default pair is
	 * click (level 0.5) / linear */
	const int    bss = TBF_BLK;
	const double T   = (double)(TBF_BLK - 1);
	for (int b = 0; b < 9; b++) {
		float* A = attackEnv[b];
		float* R = releaseEnv[b];
		int    i, bound, burst, start;
		if (cfg.envAttackModel == ENV_CLICK) {
			bound = std::max (envMax - envMin, 1);
			burst = envMin + (rnd.next () % bound);
			if (bss <= burst)
				burst = bss - 1;
			start = (rnd.next () % (bss - burst));
			for (i = 0; i < start; i++)
				A[i] = 0.0f;
			for (; i < start + burst; i++) {
				double d = ((double)rnd.next ()) / (double)2147483647;
				A[i]     = (float)(1.0 - (cfg.envAttackClickLevel * d));
			}
			for (; i < bss; i++)
				A[i] = 1.0f;
			A[0] = (float)(A[0] / 2.0);
			for (i = 1; i < bss; i++)
				A[i] = (float)((float)(A[i - 1] + A[i]) / 2.0);
		}
		if (cfg.envAttackModel == ENV_SHELF || cfg.envReleaseModel == ENV_SHELF) {
			for (int pass = 0; pass < 2; pass++) { /* attack's draw first, then release's */
				float* E = pass == 0 ? A : R;
				if ((pass == 0 ? cfg.envAttackModel : cfg.envReleaseModel) != ENV_SHELF)
					continue;
				bound = std::max (envMax - envMin, 1);
				start = rnd.next () % bound;
				if ((bss - 2) <= start)
					start = bss - 2;
				for (i = 0; i < start; i++)
					E[i] = 0.0f;
				E[i + 0] = (float)0.33333333;
				E[i + 1] = (float)0.66666666;
				for (i = i + 2; i < bss; i++)
					E[i] = 1.0f;
			}
		}
		if (cfg.envReleaseModel == ENV_CLICK) {
			burst = 8 + (rnd.next () % 32);
			start = (rnd.next () % (bss - burst));
			for (i = 0; i < start; i++)
				R[i] = 0.0f;
			for (; i < start + burst; i++) {
				double d = ((double)rnd.next ()) / (double)2147483647;
				R[i]     = (float)(1.0 - (cfg.envReleaseClickLevel * d));
			}
			for (; i < bss; i++)
				R[i] = 1.0f;
			R[0] = (float)(R[0] / 2.0);
			for (i = 1; i < bss; i++)
				R[i] = (float)((float)(R[i - 1] + R[i]) / 2.0);
		}
		if (cfg.envAttackModel == ENV_COSINE)
			for (i = 0; i < bss; i++)
				A[i] = (float)(0.5 + (0.5 * cos ((M_PI * (double)(bss - (i + 1))) / T)));
		if (cfg.envReleaseModel == ENV_COSINE)
			for (i = 0; i < bss; i++)
				R[i] = (float)(0.5 - (0.5 * cos ((M_PI * (double)i) / T)));
		if (cfg.envAttackModel == ENV_LINEAR)
			for (i = 0; i < bss; i++)
				A[i] = ((float)i) / (float)bss;
		if (cfg.envReleaseModel == ENV_LINEAR)
			for (i = 0; i < bss; i++)
				R[i] = ((float)i) / (float)bss;
	}
}

/* ------------------------------------------------------------------ whirl tables */
static void ipoldraw (std::vector<float>& bfw, double degrees, double level, int partial, double* ipx, double* ipy)
{
	double d = *ipx;
	while (d < 0.0)
		d += 360.0;
	int fromIndex = (int)((d * (double)16384) / 360.0);
	*ipx          = degrees;
	double e      = *ipx;
	while (e < d)
		e += 360.0;
	int    toIndex = (int)((e * (double)16384) / 360.0);
	double range   = (double)(toIndex - fromIndex);
	for (int i = fromIndex; i <= toIndex; i++) {
		double x                              = (double)(i - fromIndex);
		double w                              = (*ipy) + ((x / range) * (level - (*ipy)));
		bfw[(size_t)(i & 16383) * 5 + partial] = (float)w;
	}
	*ipy = level;
}

/* src/whirl.cpp:366-490 angular impulse-response drawing (reference data) */
static const double kIr[5][26][2] = {
	{{-180.0, 1.052}, {-166.4, .881}, {-150.5, .881}, {-135.3, .881}, {-122.4, .792}, {-106.5, .792}, {-91.2, .836}, {-75.8, .881}, {-59.4, .851}, {-44.7, .941}, {-30.0, 1.298}, {-14.7, 2.119}, {0.0, 2.820}, {15.6, 2.313}, {30.0, 1.492}, {44.7, .926}, {60.0, .836}, {74.7, .866}, {90.6, .792}, {100.0, .777}, {105.0, .777}, {120.0, .836}, {135.3, .836}, {150.0, .881}, {164.5, .874}, {180.0, 1.052}},
	{{-180.0, -0.07}, {-150.0, 0.10}, {-135.0, -0.10}, {-122.2, 0.16}, {-105.0, 0.15}, {-91.2, 0.37}, {-75.3, 0.32}, {-60.1, 0.39}, {-44.5, 0.70}, {-30.0, 0.53}, {-12.0, -0.40}, {0.0, -0.81}, {2.7, -0.77}, {15.0, -0.52}, {33.1, 0.38}, {43.7, 0.68}, {57.7, 0.49}, {74.1, 0.19}, {89.4, 0.33}, {105.0, 0.03}, {120.0, 0.12}, {134.0, -0.13}, {153.3, 0.08}, {180.0, -0.07}},
	{{-180.0, 0.40}, {-165.0, 0.20}, {-150.0, 0.48}, {-135.0, 0.27}, {-121.2, 0.22}, {-89.2, 0.30}, {-69.2, 0.22}, {-58.0, 0.11}, {-40.2, -0.43}, {-29.0, -0.53}, {-15.6, -0.43}, {0.0, 0.00}, {14.3, -0.44}, {30.3, -0.60}, {60.3, 0.11}, {74.9, 0.32}, {91.5, 0.23}, {104.9, 0.32}, {121.7, 0.19}, {135.0, 0.27}, {150.0, 0.45}, {165.0, 0.20}, {180.0, 0.40}},
	{{-180.0, -0.08}, {-165.2, -0.19}, {-150.0, 0.00}, {-133.9, -0.20}, {-120.0, -0.15}, {-106.0, 0.09}, {-89.3, -0.15}, {-76.3, 0.00}, {-60.3, 0.29}, {-44.6, -0.02}, {-15.6, -0.22}, {0.0, 0.24}, {14.5, 0.11}, {30.1, -0.10}, {44.6, 0.17}, {60.4, 0.22}, {75.9, 0.16}, {90.4, -0.05}, {104.9, 0.07}, {122.8, -0.07}, {136.2, -0.07}, {150.0, 0.08}, {165.0, -0.19}, {180.0, -0.08}},
	{{-180.0, 0.13}, {-165.2, 0.00}, {-150.0, 0.17}, {-135.2, -0.20}, {-120.5, 0.00}, {-105.0, 0.00}, {-90.0, 0.04}, {-75.0, -0.09}, {-60.3, -0.14}, {-45.0, 0.16}, {-15.6, 0.00}, {0.0, 0.22}, {15.6, -0.21}, {30.1, -0.09}, {45.0, 0.10}, {60.3, -0.07}, {74.8, -0.15}, {90.4, -0.03}, {104.9, -0.14}, {120.5, 0.00}, {135.2, -0.26}, {150.0, 0.16}, {165.0, -0.02}, {180.0, 0.13}},
};
static const int kIrN[5] = {26, 24, 23, 24, 24};

/* RBJ designer, src/eqcomp.cpp:98-203 (only the types the whirl uses by default are
 * exercised, all nine are kept for configurability) */
static void eqCompute (int type, double fqHz, double Q, double dbG, double* C, double SampleRateD)
{
	double A = pow (10.0, (dbG / 40.0)), omega = (2.0 * M_PI * fqHz) / SampleRateD;
	double sin_ = sin (omega), cos_ = cos (omega), alpha = sin_ / (2.0 * Q), beta = sqrt (A) / Q;
	switch (type) {
		case 0: C[0] = (1.0 - cos_) / 2.0; C[1] = 1.0 - cos_; C[2] = (1.0 - cos_) / 2.0; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 1: C[0] = (1.0 + cos_) / 2.0; C[1] = -(1.0 + cos_); C[2] = (1.0 + cos_) / 2.0; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 2: C[0] = sin_ / 2.0; C[1] = 0.0; C[2] = -sin_ / 2.0; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 3: C[0] = alpha; C[1] = 0.0; C[2] = -alpha; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 4: C[0] = 1.0; C[1] = -2.0 * cos_; C[2] = 1.0; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 5: C[0] = 1.0 - alpha; C[1] = -2.0 * cos_; C[2] = 1.0 + alpha; C[3] = 1.0 + alpha; C[4] = -2.0 * cos_; C[5] = 1.0 - alpha; break;
		case 6: C[0] = 1.0 + (alpha * A); C[1] = -2.0 * cos_; C[2] = 1.0 - (alpha * A); C[3] = 1.0 + (alpha / A); C[4] = -2.0 * cos_; C[5] = 1.0 - (alpha / A); break;
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

/* setIIRFilter (src/whirl.cpp:147-172) -> {a1, a2, b0, b1, b2}: out-of-range settings
 * leave the coefficients as they were */
static void iirSet (float* W, int T, double F, double Q, double G, double SR)
{
	double C[6];
	if (Q <= 0.1 || Q >= 6.00 || F / SR <= 0.0002 || F / SR >= 0.4998 || G <= -48.0 || G >= 48.0 || T < 0 || T > 8)
		return;
	eqCompute (T, F, Q, G, C, SR);
	W[0] = (float)C[4];
	W[1] = (float)C[5];
	W[2] = (float)C[0];
	W[3] = (float)C[1];
	W[4] = (float)C[2];
}

/* ... on the zeroed filter of allocWhirl's calloc (src/whirl.cpp:136-143) */
static void iirCoef (float* W, int T, double F, double Q, double G, double SR)
{
	W[0] = W[1] = W[2] = W[3] = W[4] = 0.f;
	iirSet (W, T, F, Q, G, SR);
}

void WhirlTables::build (double rate, const Config& c)
{
	sr = rate;
	displ.assign (4 * 16384, 0.f);
	bw.assign (2 * 16384 * 5, 0.f);
	/* initValues (src/whirl.cpp:43-134) geometry and filters, as the cfg left them */
	const float  hornRadiusCm = c.hornRadiusCm, drumRadiusCm = c.drumRadiusCm, airSpeed = 340.0f,
	            micDistCm = c.micDistCm;
	const float  hornXOffsetCm = c.hornXOffsetCm, hornZOffsetCm = c.hornZOffsetCm;
	const double hornR = (hornRadiusCm * sr / 100.0) / airSpeed;
	const double drumR = (drumRadiusCm * sr / 100.0) / airSpeed;
	const double micD  = (micDistCm * sr / 100.0) / airSpeed;
	const double micX  = (hornXOffsetCm * sr / 100.0) / airSpeed;
	const double micZ  = (hornZOffsetCm * sr / 100.0) / airSpeed;
	float*       hnFwd = displ.data (), *hnBwd = hnFwd + 16384, *drFwd = hnBwd + 16384, *drBwd = drFwd + 16384;
	float        maxhn = 0.f, maxdr = 0.f;
	for (int i = 0; i < 16384; i++) {
		double       v    = (2.0 * M_PI * (double)i) / (double)16384;
		double       a    = micD - (hornR * cos (v));
		double       b    = micZ + hornR * sin (v);
		const double dist = sqrt ((a * a) + (b * b));
		hnFwd[i]                  = (float)(dist + micX);
		hnBwd[16384 - (i + 1)]    = (float)(dist - micX);
		a                         = micD - (drumR * cos (v));
		b                         = drumR * sin (v);
		drFwd[i]                  = (float)sqrt ((a * a) + (b * b));
		drBwd[16384 - (i + 1)]    = drFwd[i];
		maxhn                     = std::max (maxhn, std::max (hnFwd[i], hnBwd[16384 - (i + 1)]));
		maxdr                     = std::max (maxdr, drFwd[i]);
	}
	static const float hs[6] = {12.0f, 18.0f, 53.0f, 50.0f, 106.0f, 116.0f};
	static const float ds[6] = {36.0f, 39.0f, 79.0f, 86.0f, 123.0f, 116.0f};
	static const int   ph[6] = {0, 16384 >> 1, (16384 * 2) / 6, (16384 * 5) / 6, (16384 * 1) / 6, (16384 * 4) / 6};
	maxAhead                 = 0.f;
	for (int i = 0; i < 6; i++) {
		hornSpacing[i] = (float)(hs[i] * sr / 22100.0 + hornR + 1.0);
		drumSpacing[i] = (float)(ds[i] * sr / 22100.0 + drumR + 1.0);
		phase[i]       = ph[i];
		maxAhead       = std::max (maxAhead, std::max (hornSpacing[i] + maxhn, drumSpacing[i] + maxdr));
	}
	/* initTables (338-517) */
	std::vector<float> bfw (16384 * 5, 0.f);
	for (int p = 0; p < 5; p++) {
		double ipx = kIr[p][0][0], ipy = kIr[p][0][1];
		for (int i = 1; i < kIrN[p]; i++)
			ipoldraw (bfw, kIr[p][i][0], kIr[p][i][1], p, &ipx, &ipy);
	}
	double sum = 0.0;
	for (int i = 0; i < 16384; i++) {
		double colsum = 0.0;
		for (int j = 0; j < 5; j++)
			colsum += fabs (bfw[(size_t)i * 5 + j]);
		if (sum < colsum)
			sum = colsum;
	}
	float* obfw = bw.data ();
	float* obbw = obfw + 16384 * 5;
	for (int i = 0; i < 16384; i++)
		for (int j = 0; j < 5; j++) {
			float v                                  = (float)(bfw[(size_t)i * 5 + j] * (1.0 / sum));
			obfw[(size_t)i * 5 + j]                  = v;
			obbw[(size_t)(16384 - i - 1) * 5 + j] = v;
		}
	/* initialize (626-662): drum hi-shelf (the horn filters: WhirlRt) */
	iirCoef (drf, c.lpT, c.lpF, c.lpQ, c.lpG, sr);
	/* computeRotationSpeeds (270-293) */
	const float  hornRPMslow = c.hornRPMslow, hornRPMfast = c.hornRPMfast;
	const float  drumRPMslow = c.drumRPMslow, drumRPMfast = c.drumRPMfast;
	const double hfast = hornRPMfast / (sr * 60.0), hslow = hornRPMslow / (sr * 60.0);
	const double dfast = drumRPMfast / (sr * 60.0), dslow = drumRPMslow / (sr * 60.0);
	const double H[9]  = {0, 0, 0, hslow, hslow, hslow, hfast, hfast, hfast};
	const double D[9]  = {0, dslow, dfast, 0, dslow, dfast, 0, dslow, dfast};
	for (int i = 0; i < 9; i++) {
		revHorn[i] = H[i];
		revDrum[i] = D[i];
	}
}

void WhirlRt::init (double rate, const Config& c)
{
	sr         = rate;
	haT        = c.haT;
	haF        = c.haF;
	haQ        = c.haQ;
	haG        = c.haG;
	hbT        = c.hbT;
	hbF        = c.hbF;
	hbQ        = c.hbQ;
	hbG        = c.hbG;
	hornAcc    = c.hornAcc;
	hornDec    = c.hornDec;
	drumAcc    = c.drumAcc;
	drumDec    = c.drumDec;
	/* initialize (626-662): horn A low-pass, horn B low-shelf */
	iirCoef (cur.hafw, (int)haT, haF, haQ, haG, sr);
	iirCoef (cur.hbfw, (int)hbT, hbF, hbQ, hbG, sr);
	ramps ();
	cur.hnBrakePos = c.hnBrakePos;
	cur.drBrakePos = c.drBrakePos;
}

/* the speed-ramp factors of whirlProc2 (1255-1257, 1306-1308), block = 128 */
void WhirlRt::ramps ()
{
	const float acc[4] = {hornAcc, hornDec, drumAcc, drumDec};
	for (int i = 0; i < 4; i++)
		cur.lAcc[i] = exp (-1.0 / (sr / (size_t)TBF_BLK * acc[i]));
}

/* the MIDI control functions initWhirl registers (src/whirl.cpp:966-981), setters 699-889:
 * each maps the 7-bit value into the field's range in double and stores it in the field */
bool WhirlRt::control (const char* fn, unsigned char uc)
{
	static const char pre[] = "whirl.";
	if (strncmp (fn, pre, sizeof (pre) - 1))
		return false;
	const char*  f = fn + sizeof (pre) - 1;
	const double u = (double)uc;
	for (int ab = 0; ab < 2; ab++) {
		float* T = ab ? &hbT : &haT;
		float* F = ab ? &hbF : &haF;
		float* Q = ab ? &hbQ : &haQ;
		float* G = ab ? &hbG : &haG;
		char   nm[32];
		snprintf (nm, sizeof (nm), "horn.filter.%c.", ab ? 'b' : 'a');
		const size_t l = strlen (nm);
		if (strncmp (f, nm, l))
			continue;
		const char* k = f + l;
		if (!strcmp (k, "type")) /* setHornFilterAType / BType */
			*T = (float)(int)(uc / 15);
		else if (!strcmp (k, "hz")) /* ... Frequency: 250 .. 8000, quadratic */
			*F = (float)(250.0 + ((8000.0 - 250.0) * ((u * u) / 16129.0)));
		else if (!strcmp (k, "q")) /* ... Q: 0.01 .. 6 */
			*Q = (float)(0.01 + ((6.00 - 0.01) * (u / 127.0)));
		else if (!strcmp (k, "gain")) /* ... Gain: -48 .. 48 dB */
			*G = (float)(-48.0 + ((48.0 - -48.0) * (u / 127.0)));
		else
			return false;
		/* UPDATE_A_FILTER / UPDATE_B_FILTER (679-689) */
		iirSet (ab ? cur.hbfw : cur.hafw, (int)*T, *F, *Q, *G, sr);
		return true;
	}
	if (!strcmp (f, "horn.brakepos")) /* setHornBrakePosition */
		cur.hnBrakePos = u / 127.0;
	else if (!strcmp (f, "drum.brakepos")) /* setDrumBrakePosition */
		cur.drBrakePos = u / 127.0;
	else if (!strcmp (f, "horn.acceleration")) /* setHornAcceleration */
		hornAcc = (float)(.01 + u / 80.0);
	else if (!strcmp (f, "horn.deceleration"))
		hornDec = (float)(.01 + u / 80.0);
	else if (!strcmp (f, "drum.acceleration")) /* setDrumAcceleration */
		drumAcc = (float)(.01 + u / 14.0);
	else if (!strcmp (f, "drum.deceleration"))
		drumDec = (float)(.01 + u / 14.0);
	else
		return false;
	ramps ();
	return true;
}

/* ------------------------------------------------------------------ tonegen control */
void TgControl::init (const TgTemplate* t, const Config& c)
{
	*this = TgControl (); /* allocTonegen: initValues (src/tonegen.cpp:238-331) */
	tpl   = t;
	/* oscConfig's runtime keys (src/tonegen.cpp:2206-2237), set before initToneGenerator's
	 * setters below read them */
	percSendBusA         = (unsigned)c.percSendBusA;
	percSendBusB         = (unsigned)c.percSendBusB;
	percTriggerBus       = c.percTriggerBus;
	percEnvGainResetNorm = c.percEnvGainResetNorm;
	percEnvGainResetSoft = c.percEnvGainResetSoft;
	percEnvScaling       = c.percEnvScaling;
	memset (keyBits, 0, sizeof (keyBits));
	memset (drawBarGain, 0, sizeof (drawBarGain));
	for (int i = 0; i < 27; i++)
		for (int s = 0; s < 9; s++) {
			float u            = (float)s;
			drawBarLevel[i][s] = (float)(u / 8.0);
		}
	/* initToneGenerator temporary drawbars (tonegen.cpp:3006-3015) via setMIDIDrawBar */
	static const int midiBus[8] = {0, 1, 2, 9, 10, 11, 18, 20};
	static const int midiVal[8] = {8, 8, 6, 8, 3, 8, 8, 6};
	for (int i = 0; i < 8; i++)
		setDrawBar (midiBus[i], (unsigned)rint ((127 - midiVal[i]) * 8.0 / 127.0));
	setPercFirst (0);
	setPercVolume (0);
	setPercFast (1);
	setPercEnabled (0);
	/* LV2 initSynth: setDrawBars (inst, 0, {8,8,6,0,...}) (b_synth/lv2.cpp:167-180) */
	static const unsigned preset[9] = {8, 8, 6, 0, 0, 0, 0, 0, 0};
	for (int i = 0; i < 9; i++)
		setDrawBar (i, preset[i]);
}

/* src/tonegen.cpp:3096-3166 */
void TgControl::keyOff (int key)
{
	if (key < 0 || key >= 384 || !keyActive (key))
		return;
	keyClear (key);
	if (key < 128)
		upperKeyCount--;
	keyDownCount--;
	msg.push_back ((uint16_t)(key & 0x0fff));
}

void TgControl::keyOn (int key)
{
	if (key < 0 || key >= 384)
		return;
	if (keyActive (key))
		keyOff (key);
	keySet (key);
	if (key < 128)
		upperKeyCount++;
	keyDownCount++;
	msg.push_back ((uint16_t)(0x1000 | (key & 0x0fff)));
}

int TgControl::noteCount (int key, bool on)
{
	if (key < 0 || key >= 384)
		return 0;
	int m = 0;
	if (keyActive (key)) { /* keyOff, or keyOn's release of a held key first */
		keyClear (key);
		if (key < 128)
			upperKeyCount--;
		keyDownCount--;
		m++;
	}
	if (on) {
		keySet (key);
		if (key < 128)
			upperKeyCount++;
		keyDownCount++;
		m++;
	}
	return m;
}

/* src/tonegen.cpp:2738-2750 */
void TgControl::setDrawBar (int bus, unsigned setting)
{
	if (bus < 0 || bus >= 27 || setting > 8)
		return;
	drawBarChange = 1;
	if (bus == percTriggerBus) {
		percTrigRestore = (int)setting;
		if (percEnabled)
			return;
	}
	drawBarGain[bus] = drawBarLevel[bus][setting];
	gainMask |= 1u << bus;
}

void TgControl::setVibratoUpper (int on) { newRouting = on ? (newRouting | 0x02u) : (newRouting & ~0x02u); }
void TgControl::setVibratoLower (int on) { newRouting = on ? (newRouting | 0x01u) : (newRouting & ~0x01u); }

/* src/vibrato.cpp:97-129: param 0..5 = V1 C1 V2 C2 V3 C3 */
void TgControl::setVibratoFromInt (int p)
{
	if (p < 0 || p > 5)
		return;
	vibTable = (uint32_t)(p / 2);
	vibMixed = (uint32_t)(p & 1);
}

/* src/tonegen.cpp:1678-1765 */
void TgControl::setPercEnabled (int on)
{
	if (on) {
		newRouting |= 0x0C;
		if (-1 < percTriggerBus) {
			drawBarGain[percTriggerBus] = 0.0f;
			gainMask |= 1u << percTriggerBus;
			drawBarChange               = 1;
		}
	} else {
		newRouting &= ~0x0Cu;
		if (-1 < percTriggerBus) {
			drawBarGain[percTriggerBus] = drawBarLevel[percTriggerBus][percTrigRestore];
			gainMask |= 1u << percTriggerBus;
			drawBarChange               = 1;
		}
	}
	percEnabled = on;
}

static void percResets (TgControl& t)
{
	if (t.percIsFast)
		t.percEnvGainDecay = t.percIsSoft ? t.percEnvGainDecayFastSoft : t.percEnvGainDecayFastNorm;
	else
		t.percEnvGainDecay = t.percIsSoft ? t.percEnvGainDecaySlowSoft : t.percEnvGainDecaySlowNorm;
}

void TgControl::setPercFast (int isFast)
{
	percIsFast = isFast;
	percResets (*this);
}

void TgControl::setPercVolume (int isSoft)
{
	percIsSoft       = isSoft;
	percEnvGainReset = percEnvScaling * (isSoft ? percEnvGainResetSoft : percEnvGainResetNorm);
	percDrawbarGain  = isSoft ? percDrawbarSoftGain : percDrawbarNormalGain;
	percResets (*this);
}

void TgControl::setPercFirst (int isFirst) { percSendBus = isFirst ? percSendBusA : percSendBusB; }

bool TgControl::dirty () const
{
	return !msg.empty () || drawBarChange || oldRouting != newRouting || steadyPending;
}

/* src/tonegen.cpp:3250-3594: message queue, active list + program emission, removal.
 * The wrap split of each instruction (3376-3402, 3524-3555) is applied on the device
 * from the wheel position it tracks. */
TgControl::Wheels::Wheels ()
{
	memset (aot, 0, sizeof (aot));
	for (int i = 0; i <= TBF_NW; i++) {
		aclPos[i] = -1;
		rflags[i] = 0;
	}
}

void TgControl::step (std::vector<tbf_prog_entry>& prog, tbf_seg_ctl& ctl)
{
	if (wh.empty ())
		wh.resize (1);
	Wheels&   W             = wh[0];
	Aot*      aot           = W.aot;
	int*      activeOscList = W.activeOscList;
	int&      activeOscLEnd = W.activeOscLEnd;
	int*      aclPos        = W.aclPos;
	uint16_t* rflags        = W.rflags;
	prog.clear ();
	int      removed[TBF_NW + 1];
	int      removedEnd = 0;
	bool     anyEnv     = false;
	bool     anyRoute   = false; /* some wheel's routed sums changed: its next entry differs */
	for (uint16_t m : msg) {
		const int kn = m & 0x0fff;
		if ((m & 0xf000) == 0x1000) {
			for (const Contrib& c : tpl->keyContrib[kn]) {
				const int wn = c.wheel;
				if (aot[wn].refCount == 0) {
					rflags[wn] = 0x0006;
					if (aclPos[wn] == -1) {
						aclPos[wn]                       = activeOscLEnd;
						activeOscList[activeOscLEnd++] = wn;
					}
				} else {
					rflags[wn] |= 0x0004;
				}
				aot[wn].busLevel[c.bus] += c.level;
				aot[wn].keyCount[c.bus] += 1;
				aot[wn].refCount += 1;
			}
		} else {
			for (const Contrib& c : tpl->keyContrib[kn]) {
				const int wn = c.wheel;
				aot[wn].busLevel[c.bus] -= c.level;
				aot[wn].keyCount[c.bus] -= 1;
				aot[wn].refCount -= 1;
				if (aot[wn].refCount == 0)
					rflags[wn] = 0x0005;
				else
					rflags[wn] |= 0x0004;
			}
		}
	}
	msg.clear ();
	const bool recomputeRouting = (oldRouting != newRouting);
	if (recomputeRouting)
		oldRouting = newRouting;

	for (int i = 0; i < activeOscLEnd; i++) {
		const int      on  = activeOscList[i];
		Aot&           a   = aot[on];
		tbf_prog_entry e;
		memset (&e, 0, sizeof (e));
		e.wheel = (uint16_t)on;
		if (rflags[on] & 0x0001) {
			removed[removedEnd++] = on;
			e.env                 = 2;
			e.row                 = (uint8_t)(i & 7);
			e.sg                  = a.sumSwell;
			e.pg                  = a.sumPercn;
			e.vg                  = a.sumScanr;
			e.nsg = e.npg = e.nvg = 0.0f;
			anyEnv                = true;
		} else {
			bool reroute = false;
			if (rflags[on] & 0x0002) {
				e.sg = e.pg = e.vg = 0.0f;
			} else {
				e.sg = a.sumSwell;
				e.pg = a.sumPercn;
				e.vg = a.sumScanr;
			}
			if ((rflags[on] & 0x0004) || drawBarChange) {
				float sum = 0.0f;
				for (int d = 0; d < 9; d++)
					sum += a.busLevel[d] * drawBarGain[d];
				a.sumUpper = sum;
				sum        = 0.0f;
				for (int d = 9; d < 18; d++)
					sum += a.busLevel[d] * drawBarGain[d];
				a.sumLower = sum;
				sum        = 0.0f;
				for (int d = 18; d < 27; d++)
					sum += a.busLevel[d] * drawBarGain[d];
				a.sumPedal = sum;
				reroute    = true;
			}
			if (reroute || recomputeRouting) {
				anyRoute   = true;
				a.sumPercn = (oldRouting & 0x0C) ? a.busLevel[percSendBus] : 0.0f;
				a.sumScanr = 0.0f;
				a.sumSwell = a.sumPedal;
				if (oldRouting & 0x02)
					a.sumScanr += a.sumUpper;
				else
					a.sumSwell += a.sumUpper;
				if (oldRouting & 0x01)
					a.sumScanr += a.sumLower;
				else
					a.sumSwell += a.sumLower;
			}
			if (rflags[on] & 0x0006) {
				e.env  = 1;
				e.row  = (uint8_t)(i & 7);
				e.nsg  = a.sumSwell;
				e.npg  = a.sumPercn;
				e.nvg  = a.sumScanr;
				anyEnv = true;
			}
		}
		rflags[on] = 0;
		prog.push_back (e);
	}
	drawBarChange = 0;
	for (int i = 0; i < removedEnd; i++) {
		const int vic = removed[i];
		const int act = aclPos[vic];
		aclPos[vic]   = -1;
		activeOscLEnd--;
		if (0 < activeOscLEnd) {
			const int mov = activeOscList[activeOscLEnd];
			if (mov != vic) {
				activeOscList[act] = mov;
				aclPos[mov]        = act;
			}
		}
	}
	/* the next block's program differs from this one's when an envelope ends, a wheel
	 * left the active list, or a steady wheel was rerouted (a drawbar or routing change
	 * with no key event: this block still plays the old sums, the next the new ones) */
	steadyPending = anyEnv || removedEnd > 0 || anyRoute;

	mixCtl (ctl);
}

void TgControl::stepFront (uint16_t* msgDst, uint32_t msgOff, float* gainDst, uint32_t gainOff, tbf_tgc_rec& rec,
                           tbf_seg_ctl& ctl)
{
	const uint32_t ng = gainPairs (); /* gainDst holds ng (bus, gain) pairs */
	memset (&rec, 0, sizeof (rec));
	rec.msgOff = msgOff;
	rec.nMsg   = (uint32_t)msg.size (); /* every message of the block, as the host path */
	std::copy (msg.begin (), msg.begin () + rec.nMsg, msgDst);
	const bool recompute = oldRouting != newRouting;
	if (recompute)
		oldRouting = newRouting;
	rec.flags       = (uint8_t)(0x80 | (drawBarChange ? 1 : 0) | (recompute ? 2 : 0) | (ng ? 4 : 0));
	rec.oldRouting  = (uint8_t)oldRouting;
	rec.percSendBus = (uint8_t)percSendBus;
	if (ng) {
		const uint32_t m = gainsSent ? gainMask : (1u << 27) - 1u;
		uint32_t       j = 0;
		for (uint32_t bus = 0; bus < 27; bus++)
			if ((m >> bus) & 1u) {
				gainDst[2 * j]     = __builtin_bit_cast (float, bus);
				gainDst[2 * j + 1] = drawBarGain[bus];
				j++;
			}
		rec.gainOff = gainOff;
		rec.pad     = (uint8_t)ng;
	}
	gainsSent = true;
	gainMask  = 0;
	/* a block with inputs makes the next block's program differ (envelopes end, released
	 * wheels leave, rerouted sums take over: the device's steadyPending); a block with
	 * none leaves it unchanged, so stepping once after each input block is exact */
	steadyPending = rec.nMsg > 0 || (rec.flags & 3) != 0;
	msg.clear ();
	drawBarChange = 0;
	mixCtl (ctl);
}

/* mixdown control (src/tonegen.cpp:3712-3777) */
void TgControl::mixCtl (tbf_seg_ctl& ctl) const
{
	ctl.routing          = oldRouting;
	ctl.swellPedalGain   = swellPedalGain;
	ctl.outputGain       = swellPedalGain * percDrawbarGain;
	ctl.percEnvGainDecay = percEnvGainDecay;
	ctl.percEnvGainReset = percEnvGainReset;
	ctl.keyCompTarget    = tpl->keyCompTable[keyDownCount < 0 ? 0 : (keyDownCount > 127 ? 127 : keyDownCount)];
	ctl.resetPercAtEnd   = upperKeyCount == 0;
	ctl.vibTable         = vibTable;
	ctl.vibMixed         = vibMixed;
}

} // namespace tbf
