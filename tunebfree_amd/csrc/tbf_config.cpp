/*
 * tbf_config.cpp -- the hot path's cfg keys (tbf_config_set / tbf_config_parse).
 *
 * The reference routes each `key=value` cfg line to every module's config function
 * (distributeParameter, src/cfgParser.cpp:61-92); the ones that reach this engine's
 * tables are whirlConfig (src/whirl.cpp:992-1160), oscConfig (src/tonegen.cpp:2173-2555),
 * scannerConfig (src/vibrato.cpp:334-357) and reverbConfig (src/reverb.cpp:242-256).
 * Values parse like getConfigParameter_d/_dr/_i/_ir (src/cfgParser.cpp:453-620): sscanf
 * %lf / %d, inclusive ranges, and a value that fails either assigns nothing.  Keys the
 * reference stores but never reads on this path are ignored: overdrive.* / xov.*
 * (ampConfig, src/overdrive.cpp:395-433: legacy fields airwindows_density never reads),
 * osc.tuning / osc.temperament (the wheel frequencies come from MTS-ESP; the gear code
 * that read them is compiled out, src/tonegen.cpp:1518-1556), osc.eqv.* (cleared by
 * initToneGenerator before initOscillators reads them, 2933-2937) and
 * whirl.horn.comb.* (the comb filter is compiled out, src/whirl.cpp:1527-1533).
 */
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include "tbf_host.h"

namespace tbf {

namespace {

int getD (const char* v, double& out, bool ranged = false, double lo = 0, double hi = 0)
{
	double a;
	if (sscanf (v, "%lf", &a) != 1 || (ranged && !(lo <= a && a <= hi)))
		return -1;
	out = a;
	return 1;
}

int getI (const char* v, int& out, bool ranged = false, int lo = 0, int hi = 0)
{
	int a;
	if (sscanf (v, "%d", &a) != 1 || (ranged && !(lo <= a && a <= hi)))
		return -1;
	out = a;
	return 1;
}

/* setEnvAttackModel / setEnvReleaseModel by name (src/tonegen.cpp:2515-2555) */
void envModel (const char* v, int& m)
{
	if (!strcasecmp (v, "click"))
		m = ENV_CLICK;
	else if (!strcasecmp (v, "cosine"))
		m = ENV_COSINE;
	else if (!strcasecmp (v, "linear"))
		m = ENV_LINEAR;
	else if (!strcasecmp (v, "shelf"))
		m = ENV_SHELF;
}

int push (Config& c, int kind, int idx, int sa, int sb, double fc)
{
	c.lists.push_back ({(int16_t)kind, (int16_t)idx, (int16_t)sa, (int16_t)sb, (float)fc});
	return 1;
}

/* oscConfig's list keys (src/tonegen.cpp:2296-2474).  The reference appends every
 * well-formed element and warns about the rest; here a key with any malformed or
 * out-of-range part assigns nothing (-1).  A harmonic number below 1 would fail
 * initOscillators' assert (1604-1605) and is refused. */
int listKey (Config& c, const char* k, const char* v)
{
	int    n, w, b, kk;
	double x;
	if (!strncasecmp (k, "osc.harmonic.", 13)) {
		if (sscanf (k + 13, "%d", &n) == 1) {
			if (sscanf (v, "%lf", &x) != 1 || n < 1 || 32767 < n)
				return -1;
			return push (c, LE_HARMONIC, 0, n, 0, x);
		}
		if (sscanf (k + 13, "w%d.f%d", &w, &n) == 2) {
			if (!(0 < w && w <= TBF_NW) || n < 1 || 32767 < n || sscanf (v, "%lf", &x) != 1)
				return -1;
			return push (c, LE_HARMONIC, w, n, 0, x);
		}
		return -1;
	}
	if (!strncasecmp (k, "osc.terminal.", 13)) {
		if (sscanf (k + 13, "t%d.w%d", &n, &w) != 2 || !(0 < n && n <= TBF_NW) || !(0 < w && w <= TBF_NW) ||
		    sscanf (v, "%lf", &x) != 1)
			return -1;
		return push (c, LE_TERMINAL, n, w, 0, x);
	}
	if (!strncasecmp (k, "osc.taper.", 10)) { /* bus 0 refused, as the reference's 0 < b */
		if (sscanf (k + 10, "k%d.b%d.t%d", &kk, &b, &w) != 3 || !(0 < kk && kk < 384) || !(0 < b && b < 27) ||
		    !(0 < w && w <= TBF_NW) || sscanf (v, "%lf", &x) != 1)
			return -1;
		return push (c, LE_TAPER, kk, w, b, x);
	}
	if (!strncasecmp (k, "osc.crosstalk.", 14)) { /* "bus:terminal:level, ..." */
		if (sscanf (k + 14, "k%d", &kk) != 1 || !(0 < kk && kk < 384))
			return -1;
		std::vector<Config::ListEntry> add;
		for (const char* p = v; p; p = strchr (p, ',') ? strchr (p, ',') + 1 : nullptr) {
			if (sscanf (p, "%d:%d:%lf", &b, &w, &x) != 3 || !(0 < b && b < 27) || !(0 < w && w <= TBF_NW))
				return -1;
			add.push_back ({LE_XTALK, (int16_t)kk, (int16_t)w, (int16_t)b, (float)x});
		}
		c.lists.insert (c.lists.end (), add.begin (), add.end ());
		return 1;
	}
	return 0;
}

} // namespace

int configSet (Config& c, const char* k, const char* v, int* scope)
{
	double d  = 0;
	int    i  = 0;
	int    sc = 0;
	struct Key {
		const char* name;
		char        kind; /* d: double, r: ranged double, i: int, j: ranged int */
		double      lo, hi;
		int         scope;
		void (*apply) (Config&, double, int);
	};
	static const Key keys[] = {
		/* whirl.*: engine-wide tables (displacement, filters, speeds) ... */
		{"whirl.horn.slowrpm", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornRPMslow = (float)d; }},
		{"whirl.horn.fastrpm", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornRPMfast = (float)d; }},
		{"whirl.horn.acceleration", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornAcc = (float)d; }},
		{"whirl.horn.deceleration", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornDec = (float)d; }},
		{"whirl.drum.slowrpm", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.drumRPMslow = (float)d; }},
		{"whirl.drum.fastrpm", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.drumRPMfast = (float)d; }},
		{"whirl.drum.acceleration", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.drumAcc = (float)d; }},
		{"whirl.drum.deceleration", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.drumDec = (float)d; }},
		{"whirl.horn.radius", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornRadiusCm = (float)d; }},
		{"whirl.drum.radius", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.drumRadiusCm = (float)d; }},
		{"whirl.mic.distance", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.micDistCm = (float)d; }},
		{"whirl.horn.offset.x", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornXOffsetCm = (float)d; }},
		{"whirl.horn.offset.z", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hornZOffsetCm = (float)d; }},
		{"whirl.drum.filter.type", 'j', 0, 8, CFG_SHARED, [] (Config& c, double, int i) { c.lpT = i; }},
		{"whirl.drum.filter.q", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.lpQ = d; }},
		{"whirl.drum.filter.hz", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.lpF = d; }},
		{"whirl.drum.filter.gain", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.lpG = d; }},
		{"whirl.horn.filter.a.type", 'j', 0, 8, CFG_SHARED, [] (Config& c, double, int i) { c.haT = (float)i; }},
		{"whirl.horn.filter.a.hz", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.haF = (float)d; }},
		{"whirl.horn.filter.a.q", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.haQ = (float)d; }},
		{"whirl.horn.filter.a.gain", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.haG = (float)d; }},
		{"whirl.horn.filter.b.type", 'j', 0, 8, CFG_SHARED, [] (Config& c, double, int i) { c.hbT = (float)i; }},
		{"whirl.horn.filter.b.hz", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hbF = (float)d; }},
		{"whirl.horn.filter.b.q", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hbQ = (float)d; }},
		{"whirl.horn.filter.b.gain", 'd', 0, 0, CFG_SHARED, [] (Config& c, double d, int) { c.hbG = (float)d; }},
		/* ... and per-instance constants */
		{"whirl.horn.level", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.hornLevel = (float)d; }},
		{"whirl.horn.leak", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.leakLevel = (float)d; }},
		{"whirl.drum.width", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.drumMicWidth = (float)d; }},
		{"whirl.horn.width", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.hornMicWidth = (float)d; }},
		{"whirl.speed-preset", 'i', 0, 0, CFG_INSTANCE, [] (Config& c, double, int i) { c.revSelect = i % 3; }},
		{"whirl.bypass", 'j', 0, 1, CFG_INSTANCE, [] (Config& c, double, int i) { c.bypass = i; }},
		{"whirl.horn.mic.angle", 'r', 0, 180.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.micAngle = 1.0 - d / 180.0; }},
		{"whirl.horn.brakepos", 'r', 0, 1.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.hnBrakePos = d; }},
		{"whirl.drum.brakepos", 'r', 0, 1.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.drBrakePos = d; }},
		{"whirl.horn.breakpos", 'r', 0, 1.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.hnBrakePos = d; }},
		{"whirl.drum.breakpos", 'r', 0, 1.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.drBrakePos = d; }},
		/* scanner.*: the engine's offset tables and stator increment */
		{"scanner.hz", 'r', 4.0, 22.0, CFG_SHARED, [] (Config& c, double d, int) { c.vibFqHertz = d; }},
		{"scanner.modulation.v1", 'r', 0.0, 12.0, CFG_SHARED, [] (Config& c, double d, int) { c.vib1OffAmp = d; }},
		{"scanner.modulation.v2", 'r', 0.0, 12.0, CFG_SHARED, [] (Config& c, double d, int) { c.vib2OffAmp = d; }},
		{"scanner.modulation.v3", 'r', 0.0, 12.0, CFG_SHARED, [] (Config& c, double d, int) { c.vib3OffAmp = d; }},
		/* reverb.mix */
		{"reverb.mix", 'r', 0, 1.0, CFG_INSTANCE, [] (Config& c, double d, int) { c.reverbMix = (float)d; }},
		/* osc.*: templates ... */
		{"osc.x-precision", 'd', 0, 0, CFG_TEMPLATE, [] (Config& c, double d, int) { if (0.0 < d) c.tgPrecision = d; }},
		{"osc.attack.click.level", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.envAttackClickLevel = (float)d; }},
		{"osc.attack.click.maxlength", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.envAtkClkMaxLength = (int)(128.0 * d); }},
		{"osc.attack.click.minlength", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.envAtkClkMinLength = (int)(128.0 * d); }},
		{"osc.release.click.level", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.envReleaseClickLevel = (float)d; }},
		{"osc.eq.p1y", 'd', 0, 0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.eqP1y = d; }},
		{"osc.eq.r1y", 'd', 0, 0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.eqR1y = d; }},
		{"osc.eq.p4y", 'd', 0, 0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.eqP4y = d; }},
		{"osc.eq.r4y", 'd', 0, 0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.eqR4y = d; }},
		{"osc.compartment-crosstalk", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.compartmentXT = d; }},
		/* above 0 initToneGenerator aborts: findTransformerNeighbours asserts for every
		 * wheel above 91 (src/tonegen.cpp:914-927, called for 44..256 at 973-978) */
		{"osc.transformer-crosstalk", 'r', 0.0, 0.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.transformerXT = d; }},
		{"osc.terminalstrip-crosstalk", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.stripXT = d; }},
		{"osc.wiring-crosstalk", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.wiringXT = d; }},
		{"osc.contribution-floor", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.contribFloor = d; }},
		{"osc.contribution-min", 'r', 0.0, 1.0, CFG_TEMPLATE, [] (Config& c, double d, int) { c.contribMin = d; }},
		/* ... and instances (percussion) */
		{"osc.perc.fast", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.percFastDecaySeconds = d; }},
		{"osc.perc.slow", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.percSlowDecaySeconds = d; }},
		{"osc.perc.normal", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.percEnvGainResetNorm = (float)d; }},
		{"osc.perc.soft", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.percEnvGainResetSoft = (float)d; }},
		{"osc.perc.gain", 'd', 0, 0, CFG_INSTANCE, [] (Config& c, double d, int) { c.percEnvScaling = (float)d; }},
		{"osc.perc.bus.a", 'j', 0, 8, CFG_INSTANCE, [] (Config& c, double, int i) { c.percSendBusA = i; }},
		{"osc.perc.bus.b", 'j', 0, 8, CFG_INSTANCE, [] (Config& c, double, int i) { c.percSendBusB = i; }},
		{"osc.perc.bus.trig", 'j', -1, 8, CFG_INSTANCE, [] (Config& c, double, int i) { c.percTriggerBus = i; }},
	};
	if (scope)
		*scope = 0;
	for (const Key& q : keys) {
		if (strcasecmp (k, q.name))
			continue;
		int r = (q.kind == 'd' || q.kind == 'r') ? getD (v, d, q.kind == 'r', q.lo, q.hi)
		                                         : getI (v, i, q.kind == 'j', (int)q.lo, (int)q.hi);
		if (r == 1) {
			q.apply (c, d, i);
			sc = q.scope;
		}
		if (scope)
			*scope = sc;
		return r;
	}
	if (!strcasecmp (k, "osc.attack.model")) {
		envModel (v, c.envAttackModel);
		if (scope)
			*scope = CFG_TEMPLATE;
		return 1;
	}
	if (!strcasecmp (k, "osc.release.model")) {
		envModel (v, c.envReleaseModel);
		if (scope)
			*scope = CFG_TEMPLATE;
		return 1;
	}
	if (!strcasecmp (k, "osc.eq.macro")) {
		if (!strcasecmp (v, "chspline"))
			c.eqMacro = EQ_SPLINE;
		else if (!strcasecmp (v, "peak24"))
			c.eqMacro = EQ_PEAK24;
		else if (!strcasecmp (v, "peak46"))
			c.eqMacro = EQ_PEAK46;
		else
			return -1;
		if (scope)
			*scope = CFG_TEMPLATE;
		return 1;
	}
	if (int r = listKey (c, k, v)) {
		if (scope)
			*scope = r == 1 ? CFG_TEMPLATE : 0;
		return r;
	}
	/* everything else, including the keys with no effect on this path (header), is
	 * ignored like any other module's keys */
	return 0;
}

} // namespace tbf
