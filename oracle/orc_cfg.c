/*
 * oracle/orc_cfg.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The cfg keys of the hot path: defaults and per-key assignments restated from
 *   whirlConfig   src/whirl.cpp:992-1160 (defaults: initValues 43-134)
 *   oscConfig     src/tonegen.cpp:2173-2555: the scalar keys, the wheel EQ, the default
 *                 crosstalk levels and the list keys (defaults: initValues 238-331)
 *   scannerConfig src/vibrato.cpp:334-357 (defaults: reset_vibrato 296-300)
 *   reverbConfig  src/reverb.cpp:242-256 (default: the ctor's G, 217)
 * Value parsing follows getConfigParameter_d/_dr/_i/_ir (src/cfgParser.cpp:453-620):
 * sscanf %lf / %d, inclusive ranges, a failed parse or range check assigns nothing.
 */
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include "orc.h"

size_t orc_cfg_size (void) { return sizeof (orc_cfg); }

void orc_cfg_default (orc_cfg* c)
{
	memset (c, 0, sizeof (*c));
	c->hornRPMslow   = (float)(60.0 * 0.672);
	c->hornRPMfast   = (float)(60.0 * 7.056);
	c->drumRPMslow   = (float)(60.0 * 0.600);
	c->drumRPMfast   = (float)(60.0 * 5.955);
	c->hornAcc       = 0.161f;
	c->hornDec       = 0.321f;
	c->drumAcc       = 4.127f;
	c->drumDec       = 1.371f;
	c->hornRadiusCm  = 19.2f;
	c->drumRadiusCm  = 22.0f;
	c->micDistCm     = 42.0f;
	c->hornXOffsetCm = 0.0f;
	c->hornZOffsetCm = 0.0f;
	c->hornLevel     = 0.7f;
	c->leakLevel     = 0.15f;
	c->drumMicWidth  = 0.0f;
	c->hornMicWidth  = 0.0f;
	c->lpT           = 8; /* EQC_HIGH */
	c->lpF           = 811.9695;
	c->lpQ           = 1.6016;
	c->lpG           = -38.9291;
	c->haT           = 0; /* EQC_LPF */
	c->haF           = 4500;
	c->haQ           = 2.7456f;
	c->haG           = -30.0f;
	c->hbT           = 7; /* EQC_LOW */
	c->hbF           = 300.0f;
	c->hbQ           = 1.0f;
	c->hbG           = -30.0f;
	c->revSelect     = 0;
	c->bypass        = 0;
	c->micAngle      = 0;
	c->hnBrakePos    = 0;
	c->drBrakePos    = 0;
	c->vibFqHertz    = 7.25;
	c->vib1OffAmp    = 3.0;
	c->vib2OffAmp    = 6.0;
	c->vib3OffAmp    = 9.0;
	c->reverbMix     = 0.1f;
	c->tgPrecision          = 0.001;
	c->percFastDecaySeconds = 1.0;
	c->percSlowDecaySeconds = 4.0;
	c->percEnvGainResetNorm = 1.0f;
	c->percEnvGainResetSoft = 0.5012f;
	c->percEnvScaling       = 11.0f; /* HIPASS_PERCUSSION */
	c->percSendBusA         = 3;
	c->percSendBusB         = 4;
	c->percTriggerBus       = 8;
	c->envAttackClickLevel  = 0.50f;
	c->envReleaseClickLevel = 0.25f;
	c->envAtkClkMinLength   = -1;
	c->envAtkClkMaxLength   = -1;
	c->envAttackModel       = ORC_ENV_CLICK;
	c->envReleaseModel      = ORC_ENV_LINEAR;
	c->eqMacro              = ORC_EQ_SPLINE;
	c->eqP1y                = 1.0;
	c->eqR1y                = 0.0;
	c->eqP4y                = 1.0;
	c->eqR4y                = 0.0;
	c->compartmentXT        = 0.01;
	c->transformerXT        = 0.0;
	c->stripXT              = 0.01;
	c->wiringXT             = 0.01;
	c->contribFloor         = 0.0000158;
	c->contribMin           = 0.0;
	c->nle                  = 0;
}

static int le_push (orc_cfg* c, int kind, int idx, int sa, int sb, double fc)
{
	if (c->nle >= ORC_CFG_MAX_LE)
		return -1;
	c->le[c->nle].kind = (short)kind;
	c->le[c->nle].idx  = (short)idx;
	c->le[c->nle].sa   = (short)sa;
	c->le[c->nle].sb   = (short)sb;
	c->le[c->nle].fc   = (float)fc;
	c->nle++;
	return 1;
}

/* oscConfig's list keys (src/tonegen.cpp:2296-2474).  The reference appends every
 * well-formed element and only warns about the rest; here a key with any malformed or
 * out-of-range part assigns nothing and returns -1.  A harmonic number below 1 would
 * fail initOscillators' assert (1604-1605), so it is refused here. */
static int osc_list_key (orc_cfg* c, const char* k, const char* v)
{
	int    n, w, b, kk;
	double x;
	if (!strncasecmp (k, "osc.harmonic.", 13)) {
		if (sscanf (k + 13, "%d", &n) == 1) {
			if (sscanf (v, "%lf", &x) != 1 || n < 1 || 32767 < n)
				return -1;
			return le_push (c, ORC_LE_HARMONIC, 0, n, 0, x);
		}
		if (sscanf (k + 13, "w%d.f%d", &w, &n) == 2) {
			if (!(0 < w && w <= ORC_NOF_WHEELS) || n < 1 || 32767 < n || sscanf (v, "%lf", &x) != 1)
				return -1;
			return le_push (c, ORC_LE_HARMONIC, w, n, 0, x);
		}
		return -1;
	}
	if (!strncasecmp (k, "osc.terminal.", 13)) {
		if (sscanf (k + 13, "t%d.w%d", &n, &w) != 2 || !(0 < n && n <= ORC_NOF_WHEELS) ||
		    !(0 < w && w <= ORC_NOF_WHEELS) || sscanf (v, "%lf", &x) != 1)
			return -1;
		return le_push (c, ORC_LE_TERMINAL, n, w, 0, x);
	}
	if (!strncasecmp (k, "osc.taper.", 10)) {
		/* bus 0 is refused, as the reference's 0 < b test does */
		if (sscanf (k + 10, "k%d.b%d.t%d", &kk, &b, &w) != 3 || !(0 < kk && kk < ORC_MAX_KEYS) ||
		    !(0 < b && b < ORC_NOF_BUSES) || !(0 < w && w <= ORC_NOF_WHEELS) || sscanf (v, "%lf", &x) != 1)
			return -1;
		return le_push (c, ORC_LE_TAPER, kk, w, b, x);
	}
	if (!strncasecmp (k, "osc.crosstalk.", 14)) {
		const char* p;
		int         cnt = 0;
		if (sscanf (k + 14, "k%d", &kk) != 1 || !(0 < kk && kk < ORC_MAX_KEYS))
			return -1;
		for (p = v; p; p = strchr (p, ','), p = p ? p + 1 : p) { /* validate first */
			if (sscanf (p, "%d:%d:%lf", &b, &w, &x) != 3 || !(0 < b && b < ORC_NOF_BUSES) ||
			    !(0 < w && w <= ORC_NOF_WHEELS))
				return -1;
			cnt++;
		}
		if (c->nle + cnt > ORC_CFG_MAX_LE)
			return -1;
		for (p = v; p; p = strchr (p, ','), p = p ? p + 1 : p) {
			sscanf (p, "%d:%d:%lf", &b, &w, &x);
			le_push (c, ORC_LE_XTALK, kk, w, b, x);
		}
		return 1;
	}
	return 0;
}

/* getConfigParameter_d / _dr / _i / _ir: 1 assigned, -1 parse or range failure */
static int get_d (const char* v, double* out, int ranged, double lo, double hi)
{
	double a;
	if (sscanf (v, "%lf", &a) != 1)
		return -1;
	if (ranged && !(lo <= a && a <= hi))
		return -1;
	*out = a;
	return 1;
}

static int get_i (const char* v, int* out, int ranged, int lo, int hi)
{
	int a;
	if (sscanf (v, "%d", &a) != 1)
		return -1;
	if (ranged && !(lo <= a && a <= hi))
		return -1;
	*out = a;
	return 1;
}

static int env_model (const char* v, int* m)
{
	if (!strcasecmp (v, "click"))
		*m = ORC_ENV_CLICK;
	else if (!strcasecmp (v, "cosine"))
		*m = ORC_ENV_COSINE;
	else if (!strcasecmp (v, "linear"))
		*m = ORC_ENV_LINEAR;
	else if (!strcasecmp (v, "shelf"))
		*m = ORC_ENV_SHELF;
	return 1; /* the reference acknowledges the key whatever the value */
}

/* setEnvAtkClkLength (src/tonegen.cpp:1893-1902) */
static void clk_length (int* p, double u)
{
	if (0.0 <= u && u <= 1.0)
		*p = (int)(((double)128) * u);
}

int orc_cfg_set (orc_cfg* c, const char* k, const char* v)
{
	double d = 0;
	int    i = 0, r;
#define D(name) (!strcasecmp (k, name) && (r = get_d (v, &d, 0, 0, 0)) != 0)
#define DR(name, lo, hi) (!strcasecmp (k, name) && (r = get_d (v, &d, 1, lo, hi)) != 0)
#define I(name) (!strcasecmp (k, name) && (r = get_i (v, &i, 0, 0, 0)) != 0)
#define IR(name, lo, hi) (!strcasecmp (k, name) && (r = get_i (v, &i, 1, lo, hi)) != 0)
#define SET(stmt) \
	do {          \
		if (r == 1) \
			stmt;   \
		return r;   \
	} while (0)
	/* whirl.* */
	if (D ("whirl.horn.slowrpm")) SET (c->hornRPMslow = (float)d);
	if (D ("whirl.horn.fastrpm")) SET (c->hornRPMfast = (float)d);
	if (D ("whirl.horn.acceleration")) SET (c->hornAcc = (float)d);
	if (D ("whirl.horn.deceleration")) SET (c->hornDec = (float)d);
	if (D ("whirl.drum.slowrpm")) SET (c->drumRPMslow = (float)d);
	if (D ("whirl.drum.fastrpm")) SET (c->drumRPMfast = (float)d);
	if (D ("whirl.drum.acceleration")) SET (c->drumAcc = (float)d);
	if (D ("whirl.drum.deceleration")) SET (c->drumDec = (float)d);
	if (D ("whirl.horn.radius")) SET (c->hornRadiusCm = (float)d);
	if (D ("whirl.drum.radius")) SET (c->drumRadiusCm = (float)d);
	if (D ("whirl.horn.level")) SET (c->hornLevel = (float)d);
	if (D ("whirl.horn.leak")) SET (c->leakLevel = (float)d);
	if (D ("whirl.drum.width")) SET (c->drumMicWidth = (float)d);
	if (D ("whirl.horn.width")) SET (c->hornMicWidth = (float)d);
	if (D ("whirl.mic.distance")) SET (c->micDistCm = (float)d);
	if (D ("whirl.horn.offset.x")) SET (c->hornXOffsetCm = (float)d);
	if (D ("whirl.horn.offset.z")) SET (c->hornZOffsetCm = (float)d);
	if (IR ("whirl.drum.filter.type", 0, 8)) SET (c->lpT = i);
	if (D ("whirl.drum.filter.q")) SET (c->lpQ = d);
	if (D ("whirl.drum.filter.hz")) SET (c->lpF = d);
	if (D ("whirl.drum.filter.gain")) SET (c->lpG = d);
	if (IR ("whirl.horn.filter.a.type", 0, 8)) SET (c->haT = (float)i);
	if (D ("whirl.horn.filter.a.hz")) SET (c->haF = (float)d);
	if (D ("whirl.horn.filter.a.q")) SET (c->haQ = (float)d);
	if (D ("whirl.horn.filter.a.gain")) SET (c->haG = (float)d);
	if (IR ("whirl.horn.filter.b.type", 0, 8)) SET (c->hbT = (float)i);
	if (D ("whirl.horn.filter.b.hz")) SET (c->hbF = (float)d);
	if (D ("whirl.horn.filter.b.q")) SET (c->hbQ = (float)d);
	if (D ("whirl.horn.filter.b.gain")) SET (c->hbG = (float)d);
	if (I ("whirl.speed-preset")) SET (c->revSelect = i % 3);
	if (IR ("whirl.bypass", 0, 1)) SET (c->bypass = i);
	if (DR ("whirl.horn.mic.angle", 0, 180.0)) SET (c->micAngle = 1.0 - d / 180.0);
	if (DR ("whirl.horn.brakepos", 0, 1.0) || DR ("whirl.horn.breakpos", 0, 1.0)) SET (c->hnBrakePos = d);
	if (DR ("whirl.drum.brakepos", 0, 1.0) || DR ("whirl.drum.breakpos", 0, 1.0)) SET (c->drBrakePos = d);
	/* scanner.* */
	if (DR ("scanner.hz", 4.0, 22.0)) SET (c->vibFqHertz = d);
	if (DR ("scanner.modulation.v1", 0.0, 12.0)) SET (c->vib1OffAmp = d);
	if (DR ("scanner.modulation.v2", 0.0, 12.0)) SET (c->vib2OffAmp = d);
	if (DR ("scanner.modulation.v3", 0.0, 12.0)) SET (c->vib3OffAmp = d);
	/* reverb.mix */
	if (DR ("reverb.mix", 0, 1.0)) SET (c->reverbMix = (float)d);
	/* osc.* scalar keys */
	if (D ("osc.x-precision")) SET (if (0.0 < d) c->tgPrecision = d);
	if (D ("osc.perc.fast")) SET (c->percFastDecaySeconds = d);
	if (D ("osc.perc.slow")) SET (c->percSlowDecaySeconds = d);
	if (D ("osc.perc.normal")) SET (c->percEnvGainResetNorm = (float)d);
	if (D ("osc.perc.soft")) SET (c->percEnvGainResetSoft = (float)d);
	if (D ("osc.perc.gain")) SET (c->percEnvScaling = (float)d);
	if (IR ("osc.perc.bus.a", 0, 8)) SET (c->percSendBusA = i);
	if (IR ("osc.perc.bus.b", 0, 8)) SET (c->percSendBusB = i);
	if (IR ("osc.perc.bus.trig", -1, 8)) SET (c->percTriggerBus = i);
	if (DR ("osc.attack.click.level", 0.0, 1.0)) SET (c->envAttackClickLevel = (float)d);
	if (DR ("osc.attack.click.maxlength", 0.0, 1.0)) SET (clk_length (&c->envAtkClkMaxLength, d));
	if (DR ("osc.attack.click.minlength", 0.0, 1.0)) SET (clk_length (&c->envAtkClkMinLength, d));
	if (DR ("osc.release.click.level", 0.0, 1.0)) SET (c->envReleaseClickLevel = (float)d);
	if (DR ("osc.compartment-crosstalk", 0.0, 1.0)) SET (c->compartmentXT = d);
	/* a level above 0 makes initToneGenerator abort: findTransformerNeighbours asserts
	 * for every wheel above 91 (src/tonegen.cpp:914-927, called for 44..256 at 973-978),
	 * so only 0 is a usable value */
	if (DR ("osc.transformer-crosstalk", 0.0, 0.0)) SET (c->transformerXT = d);
	if (DR ("osc.terminalstrip-crosstalk", 0.0, 1.0)) SET (c->stripXT = d);
	if (DR ("osc.wiring-crosstalk", 0.0, 1.0)) SET (c->wiringXT = d);
	if (DR ("osc.contribution-floor", 0.0, 1.0)) SET (c->contribFloor = d);
	if (DR ("osc.contribution-min", 0.0, 1.0)) SET (c->contribMin = d);
	if (D ("osc.eq.p1y")) SET (c->eqP1y = d);
	if (D ("osc.eq.r1y")) SET (c->eqR1y = d);
	if (D ("osc.eq.p4y")) SET (c->eqP4y = d);
	if (D ("osc.eq.r4y")) SET (c->eqR4y = d);
	if (!strcasecmp (k, "osc.eq.macro")) {
		if (!strcasecmp (v, "chspline"))
			c->eqMacro = ORC_EQ_SPLINE;
		else if (!strcasecmp (v, "peak24"))
			c->eqMacro = ORC_EQ_PEAK24;
		else if (!strcasecmp (v, "peak46"))
			c->eqMacro = ORC_EQ_PEAK46;
		else
			return -1;
		return 1;
	}
	if ((r = osc_list_key (c, k, v)) != 0)
		return r;
	if (!strcasecmp (k, "osc.release.model"))
		return env_model (v, &c->envReleaseModel);
	if (!strcasecmp (k, "osc.attack.model"))
		return env_model (v, &c->envAttackModel);
#undef D
#undef DR
#undef I
#undef IR
#undef SET
	return 0;
}
