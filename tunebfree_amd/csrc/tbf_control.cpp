/*
 * tbf_control.cpp -- the reference's host control surface for the hot path, on the
 * engine's instances: MIDI control functions by name (callMIDIControlFunction,
 * src/midi.cpp:535-545), programme files in the .pgm syntax (src/pgmParser.cpp,
 * bindToProgram src/program.cpp:308-603) and programme installation (installProgram,
 * src/program.cpp:735-921).
 *
 * Everything here runs on the host between render calls and only changes what the
 * next block renders (b_synth/lv2.cpp:1130-1134), exactly like tbf_note/tbf_set_param.
 */
#include <ctype.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <strings.h>

#include <string>

#include "tbf_engine_impl.h"

using namespace tbf;

namespace {

/* programme flags, src/program.h:58-101 */
enum : uint32_t {
	FL_INUSE  = 0x0001,
	FL_DRAWBR = 0x0002,
	FL_SCANNR = 0x0100,
	FL_PRCENA = 0x0200,
	FL_PRCVOL = 0x0400,
	FL_PRCSPD = 0x0800,
	FL_PRCHRM = 0x1000,
	FL_OVRSEL = 0x2000,
	FL_ROTENA = 0x4000,
	FL_ROTSPS = 0x8000,
	FL_RVBMIX = 0x00010000,
	FL_DRWRND = 0x00020000,
	FL_KSPLTL = 0x00040000,
	FL_LOWDRW = 0x00080000,
	FL_PDLDRW = 0x00100000,
	FL_KSPLTP = 0x00200000,
	FL_TRA_PD = 0x00400000,
	FL_TRA_LM = 0x00800000,
	FL_TRA_UM = 0x01000000,
	FL_TRANSP = 0x02000000,
	FL_TRCH_A = 0x04000000,
	FL_TRCH_B = 0x08000000,
	FL_TRCH_C = 0x10000000,
	FL_VCRUPR = 0x20000000,
	FL_VCRLWR = 0x40000000,
};

/* scanner selections, src/vibrato.h:30-36; whirl revSelect, src/whirl.h:251-254 */
enum { VIB1 = 0x01, VIB2 = 0x02, VIB3 = 0x03, CHO_ = 0x80, CHO1 = 0x81, CHO2 = 0x82, CHO3 = 0x83 };
enum { WHIRL_SLOW = 0, WHIRL_STOP = 1, WHIRL_FAST = 2 };
static const int revselects[3] = {4, 0, 8}; /* computeRotationSpeeds, src/whirl.cpp:289-291 */

/* useRevOption (src/whirl.cpp:174-224), queued for the next block; `signals & 2`
 * updates revSelect from the horn speed */
void useRevOption (Instance& in, int n, int signals)
{
	in.revOpt = n % 9;
	if (signals & 2) {
		const int hr = (n / 3) % 3;
		in.revSelect = hr == 2 ? WHIRL_FAST : (hr == 1 ? WHIRL_SLOW : WHIRL_STOP);
	}
	in.ctlDirty = true;
}

/* setRevSelect (src/whirl.cpp:226-233) */
void setRevSelect (Instance& in, int n)
{
	in.revSelect = n % 3;
	useRevOption (in, revselects[in.revSelect], 1);
}

/* setVibrato (src/vibrato.cpp:91-116) through the knob index of setVibratoFromInt */
void setVibratoKnob (Instance& in, int knob) { in.tg.setVibratoFromInt (knob); }

/* callMIDIControlFunction targets on the hot path (src/midi.cpp:100-170 names) */
bool controlFunction (Instance& in, const char* fn, unsigned char u)
{
	static const char* bars[9] = {"16", "513", "8", "4", "223", "2", "135", "113", "1"};
	static const char* manuals[3] = {"upper.drawbar", "lower.drawbar", "pedal.drawbar"};
	for (int m = 0; m < 3; m++) {
		const size_t l = strlen (manuals[m]);
		if (!strncmp (fn, manuals[m], l))
			for (int b = 0; b < 9; b++)
				if (!strcmp (fn + l, bars[b])) {
					/* setMIDIDrawBar, src/tonegen.cpp:2752-2756 */
					const int val = 127 - u;
					in.tg.setDrawBar (m * 9 + b, (unsigned)rint (val * 8.0 / 127.0));
					in.ctlDirty = true;
					return true;
				}
	}
	if (!strcmp (fn, "percussion.enable")) /* src/tonegen.cpp:2850-2880 */
		in.tg.setPercEnabled (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "percussion.decay"))
		in.tg.setPercFast (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "percussion.harmonic"))
		in.tg.setPercFirst (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "percussion.volume"))
		in.tg.setPercVolume (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "swellpedal1") || !strcmp (fn, "swellpedal2")) /* 2885-2900 */
		in.tg.swellPedalGain = (float)((in.tg.outputLevelTrim * ((double)u)) / 127.0);
	else if (!strcmp (fn, "vibrato.knob")) { /* src/vibrato.cpp:148-172 */
		const int k = u / 23;
		if (k <= 5)
			setVibratoKnob (in, k);
	} else if (!strcmp (fn, "vibrato.routing")) { /* 177-202 */
		const int r = u / 32;
		in.tg.setVibratoUpper ((r & 2) ? 1 : 0);
		in.tg.setVibratoLower ((r & 1) ? 1 : 0);
	} else if (!strcmp (fn, "vibrato.upper")) /* 204-210 */
		in.tg.setVibratoUpper (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "vibrato.lower")) /* 212-218 */
		in.tg.setVibratoLower (u < 64 ? 0 : 1);
	else if (!strcmp (fn, "overdrive.enable")) /* setCleanCC, src/overdrive.cpp:392 */
		in.odClean = u > 63 ? 0 : 1;
	else if (!strcmp (fn, "overdrive.character")) /* setCharacter, 576-580 */
		setCharacter (in, (float)(0.001 + ((1.0 - 0.001) * (((float)u) / 127.0))));
	else if (!strcmp (fn, "reverb.mix")) /* setReverbMixFromMIDI, src/reverb.cpp:236-240 */
		in.rvG = (float)((float)u / 127.0);
	else if (!strcmp (fn, "rotary.speed-preset")) /* revControl, src/whirl.cpp:244-249 */
		setRevSelect (in, (int)(u / 43));
	else if (!strcmp (fn, "rotary.speed-select")) /* revControlAll, 237-241 */
		useRevOption (in, (int)(u / 15), 2);
	else if (!strcmp (fn, "rotary.speed-toggle")) { /* setWhirlSustainPedal, 252-261 */
		if (u > 63)
			useRevOption (in, in.revSelect == WHIRL_SLOW ? revselects[WHIRL_FAST] : revselects[WHIRL_SLOW], 3);
	} else if (in.whr.control (fn, u)) /* whirl.horn.filter.*, brakepos, acceleration (src/whirl.cpp:699-889) */
		in.whDirty = true;
	else
		return false;
	in.ctlDirty = true;
	return true;
}

/* control function ids of TBF_EV_CONTROL events (tbf_midi_control_id) */
const char* const kControlNames[] = {
    "upper.drawbar16", "upper.drawbar513", "upper.drawbar8", "upper.drawbar4", "upper.drawbar223",
    "upper.drawbar2", "upper.drawbar135", "upper.drawbar113", "upper.drawbar1",
    "lower.drawbar16", "lower.drawbar513", "lower.drawbar8", "lower.drawbar4", "lower.drawbar223",
    "lower.drawbar2", "lower.drawbar135", "lower.drawbar113", "lower.drawbar1",
    "pedal.drawbar16", "pedal.drawbar513", "pedal.drawbar8", "pedal.drawbar4", "pedal.drawbar223",
    "pedal.drawbar2", "pedal.drawbar135", "pedal.drawbar113", "pedal.drawbar1",
    "percussion.enable", "percussion.decay", "percussion.harmonic", "percussion.volume",
    "swellpedal1", "swellpedal2", "vibrato.knob", "vibrato.routing", "vibrato.upper", "vibrato.lower",
    "overdrive.enable", "overdrive.character", "reverb.mix",
    "rotary.speed-preset", "rotary.speed-select", "rotary.speed-toggle",
    "whirl.horn.filter.a.type", "whirl.horn.filter.a.hz", "whirl.horn.filter.a.q", "whirl.horn.filter.a.gain",
    "whirl.horn.filter.b.type", "whirl.horn.filter.b.hz", "whirl.horn.filter.b.q", "whirl.horn.filter.b.gain",
    "whirl.horn.brakepos", "whirl.drum.brakepos", "whirl.horn.acceleration", "whirl.horn.deceleration",
    "whirl.drum.acceleration", "whirl.drum.deceleration"};
const int kNControls = (int)(sizeof (kControlNames) / sizeof (kControlNames[0]));

/* ---------------------------------------------------------------- .pgm parser */
enum { TKN_EOF = -1, TKN_ERROR = -2, TKN_STRING = 256 };

struct PgmLexer {
	const char* p;
	int         line = 1;
	int         tok  = 0;
	std::string buf;
	std::string err;

	/* getToken, src/pgmParser.cpp:80-190: '{' '}' '=' ',' or a string (quoted with
	 * backslash escapes, or a run of alnum - . _ +); '#' comments to end of line */
	int next ()
	{
		buf.clear ();
		int c;
		for (;;) {
			c = (unsigned char)*p;
			if (!c)
				return tok = TKN_EOF;
			p++;
			if (c == '\n') {
				line++;
				continue;
			}
			if (isspace (c))
				continue;
			if (c == '#') {
				while (*p && *p != '\n')
					p++;
				continue;
			}
			break;
		}
		if (c == '{' || c == '}' || c == '=' || c == ',') {
			buf = (char)c;
			return tok = c;
		}
		if (c == '"') {
			for (;;) {
				c = (unsigned char)*p;
				if (!c) {
					err = "End of file in quoted string";
					return tok = TKN_ERROR;
				}
				p++;
				if (c == '"')
					break;
				if (c == '\\') {
					if (!*p) {
						err = "End of file in quoted string";
						return tok = TKN_ERROR;
					}
					c = (unsigned char)*p++;
				}
				if (c == '\n')
					line++;
				buf += (char)c;
			}
			return tok = TKN_STRING;
		}
		buf += (char)c;
		while (isalnum ((unsigned char)*p) || *p == '-' || *p == '.' || *p == '_' || *p == '+')
			buf += *p++;
		return tok = TKN_STRING;
	}
};

bool isAffirmative (const char* v)
{
	return !strcasecmp (v, "on") || !strcasecmp (v, "yes") || !strcasecmp (v, "true") || !strcasecmp (v, "enabled");
}

bool isNegatory (const char* v)
{
	return !strcasecmp (v, "off") || !strcasecmp (v, "no") || !strcasecmp (v, "none") || !strcasecmp (v, "false") ||
	       !strcasecmp (v, "disabled");
}

/* parseDrawbarRegistration, src/program.cpp:203-240 */
bool parseDrawbars (const char* d, unsigned bar[9], std::string& err)
{
	int bus = 0;
	for (const char* t = d; bus < 9;) {
		if (!*t) {
			err = std::string ("Drawbar registration incomplete '") + d + "'";
			return false;
		}
		if (isspace ((unsigned char)*t) || *t == '-' || *t == '_') {
			t++;
			continue;
		}
		if ('0' <= *t && *t <= '8') {
			bar[bus++] = (unsigned)(*t++ - '0');
			continue;
		}
		err = std::string ("Illegal char in drawbar registration '") + *t + "'";
		return false;
	}
	return true;
}

/* parseTranspose, src/program.cpp:289-306 */
bool parseTranspose (const char* v, int* out, std::string& err)
{
	int iv;
	if (sscanf (v, "%d", &iv) == 0) {
		err = std::string ("Unparseable transpose value '") + v + "'";
		return false;
	}
	if (iv < -127 || 127 < iv) {
		err = std::string ("Transpose value out of range '") + v + "'";
		return false;
	}
	*out = iv;
	return true;
}

/* bindToProgram, src/program.cpp:308-603 (property table 133-167) */
bool bindToProgram (tbf_engine* e, int& prevPgm, int pgm, const char* sym, const char* val, std::string& err)
{
	if (pgm < 0 || (int)e->progs.size () <= pgm) {
		err = "Program number " + std::to_string (pgm) + " out of range";
		return false;
	}
	Programme& P = e->progs[pgm];
	if (pgm != prevPgm) {
		P.flags = 0;
		prevPgm = pgm;
	}
	auto is = [&] (const char* s) { return !strcasecmp (sym, s); };
	auto v  = [&] (const char* s) { return !strcasecmp (val, s); };
	if (is ("name")) {
		strncpy (P.name, val, sizeof (P.name) - 1);
		P.name[sizeof (P.name) - 1] = 0;
		P.flags |= FL_INUSE;
	} else if (is ("drawbars") || is ("drawbarsupper") || is ("drawbarslower") || is ("drawbarspedals")) {
		const bool     low = is ("drawbarslower"), ped = is ("drawbarspedals");
		const uint32_t fl  = low ? FL_LOWDRW : (ped ? FL_PDLDRW : FL_DRAWBR);
		unsigned*      bar = low ? P.lowerDrawbars : (ped ? P.pedalDrawbars : P.drawbars);
		if (v ("random"))
			P.flags |= FL_INUSE | fl | FL_DRWRND;
		else if (parseDrawbars (val, bar, err))
			P.flags |= FL_INUSE | fl;
		else
			return false;
	} else if (is ("vibrato") || is ("vibratoknob")) {
		static const struct { const char* n; int s; } m[6] = {{"v1", VIB1}, {"v2", VIB2}, {"v3", VIB3},
		                                                      {"c1", CHO1}, {"c2", CHO2}, {"c3", CHO3}};
		int sel = -1;
		for (auto& x : m)
			if (v (x.n))
				sel = x.s;
		if (sel < 0) {
			err = std::string ("Unrecognized vibrato value '") + val + "'";
			return false;
		}
		P.scanner = (P.scanner & 0xFF00) | (uint32_t)sel;
		P.flags |= FL_INUSE | FL_SCANNR;
	} else if (is ("vibratoupper") || is ("vibratolower")) {
		const uint32_t bit = is ("vibratoupper") ? 0x200 : 0x100;
		const uint32_t fl  = is ("vibratoupper") ? FL_VCRUPR : FL_VCRLWR;
		if (isNegatory (val))
			P.scanner &= ~bit;
		else if (isAffirmative (val))
			P.scanner |= bit;
		else {
			err = std::string ("Unrecognized keyword '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | fl;
	} else if (is ("perc")) {
		if (isAffirmative (val))
			P.percussionEnabled = 1;
		else if (isNegatory (val))
			P.percussionEnabled = 0;
		else {
			err = std::string ("Unrecognized percussion enabled value '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_PRCENA;
	} else if (is ("percvol")) {
		if (v ("normal") || v ("high") || v ("hi"))
			P.percussionVolume = 0;
		else if (v ("soft") || v ("low") || v ("lo"))
			P.percussionVolume = 1;
		else {
			err = std::string ("Unrecognized percussion volume argument '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_PRCVOL;
	} else if (is ("percspeed")) {
		if (v ("fast") || v ("high") || v ("hi"))
			P.percussionSpeed = 1;
		else if (v ("slow") || v ("low") || v ("lo"))
			P.percussionSpeed = 0;
		else {
			err = std::string ("Unrecognized percussion speed argument '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_PRCSPD;
	} else if (is ("percharm")) {
		if (v ("second") || v ("2nd") || v ("low") || v ("lo"))
			P.percussionHarmonic = 1;
		else if (v ("third") || v ("3rd") || v ("high") || v ("hi"))
			P.percussionHarmonic = 0;
		else {
			err = std::string ("Unrecognized percussion harmonic option '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_PRCHRM;
	} else if (is ("overdrive")) {
		if (isNegatory (val))
			P.overdriveSelect = 0;
		else if (isAffirmative (val))
			P.overdriveSelect = 1;
		else {
			err = std::string ("Unrecognized overdrive select argument '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_OVRSEL;
	} else if (is ("rotaryspeed")) {
		if (v ("tremolo") || v ("fast") || v ("high") || v ("hi"))
			P.rotarySpeedSelect = WHIRL_FAST;
		else if (v ("chorale") || v ("slow") || v ("low") || v ("lo"))
			P.rotarySpeedSelect = WHIRL_SLOW;
		else if (v ("stop") || v ("zero") || v ("break") || v ("stopped"))
			P.rotarySpeedSelect = WHIRL_STOP;
		else {
			err = std::string ("Unrecognized rotary speed argument '") + val + "'";
			return false;
		}
		P.flags |= FL_INUSE | FL_ROTSPS;
	} else if (is ("reverbmix")) {
		float fv;
		P.flags |= FL_INUSE | FL_RVBMIX;
		if (sscanf (val, "%f", &fv) == 0) {
			err = std::string ("Unrecognized reverb mix value : '") + val + "'";
			return false;
		}
		if (fv < 0.0 || 1.0 < fv) {
			err = "Reverb mix value out of range : " + std::to_string (fv);
			return false;
		}
		P.reverbMix = fv;
	} else if (is ("keysplitlower") || is ("keysplitpedals")) {
		int iv;
		P.flags |= FL_INUSE | (is ("keysplitlower") ? FL_KSPLTL : FL_KSPLTP);
		if (sscanf (val, "%d", &iv) == 0 || iv < 0 || 127 < iv) {
			err = std::string ("split: bad MIDI note number '") + val + "'";
			return false;
		}
		(is ("keysplitlower") ? P.keyboardSplitLower : P.keyboardSplitPedals) = iv;
	} else if (is ("trssplitpedals") || is ("trssplitlower") || is ("trssplitupper") || is ("transpose") ||
	           is ("transposeupper") || is ("transposelower") || is ("transposepedals")) {
		static const struct { const char* n; uint32_t f; int i; } m[7] = {
		    {"trssplitpedals", FL_TRA_PD, 0}, {"trssplitlower", FL_TRA_LM, 1}, {"trssplitupper", FL_TRA_UM, 2},
		    {"transpose", FL_TRANSP, 3},      {"transposeupper", FL_TRCH_A, 4}, {"transposelower", FL_TRCH_B, 5},
		    {"transposepedals", FL_TRCH_C, 6}};
		for (auto& x : m)
			if (is (x.n)) {
				P.flags |= FL_INUSE | x.f;
				if (!parseTranspose (val, &P.transpose[x.i], err))
					return false;
			}
	} else if (is ("attackenv") || is ("attacklvl") || is ("attackdur") || is ("rotary")) {
		/* in the property table but without a case in bindToProgram: accepted, no effect */
	} else {
		err = std::string ("Unrecognized property '") + sym + "'";
		return false;
	}
	return true;
}

/* randomizeDrawbars, src/program.cpp:716-729 (the instance's control rand stream) */
void randomizeDrawbars (Instance& in, unsigned bar[9])
{
	for (int i = 0; i < 9; i++)
		bar[i] = (unsigned)(in.ctlRand.next () % 9);
}

} // namespace

int tbf::controlById (Instance& in, int id, int value)
{
	if (id < 0 || id >= kNControls || value < 0)
		return -1;
	controlFunction (in, kControlNames[id], (unsigned char)(value > 127 ? 127 : value));
	return 0;
}

extern "C" {

int tbf_midi_control_id (const char* fn)
{
	if (!fn)
		return -1;
	for (int i = 0; i < kNControls; i++)
		if (!strcmp (fn, kControlNames[i]))
			return i;
	return -1;
}

int tbf_midi_control (tbf_engine* e, uint32_t inst, const char* fn, int32_t value)
{
	if (!e || !fn || inst >= e->inst.size ())
		return fail (-22, "bad argument");
	if (value < 0)
		return fail (-22, "control value must be 0..127");
	const unsigned char u = (unsigned char)(value > 127 ? 127 : value);
	markActive (e, inst);
	return controlFunction (e->inst[inst], fn, u) ? 0 : 1;
}

int tbf_program_parse (tbf_engine* e, const char* text)
{
	if (!e || !text)
		return fail (-22, "null argument");
	PgmLexer    L;
	std::string err;
	int         prev = -1;
	L.p              = text;
	L.next ();
	/* parseProgramDefinitionList, src/pgmParser.cpp:360-375 */
	while (L.tok != TKN_EOF) {
		if (L.tok == TKN_ERROR)
			return fail (-22, "line " + std::to_string (L.line) + ": " + L.err);
		int pgm;
		if (L.tok != TKN_STRING || sscanf (L.buf.c_str (), "%d", &pgm) != 1)
			return fail (-22, "line " + std::to_string (L.line) + ": program number expected");
		L.next ();
		if (L.tok != '{')
			return fail (-22, "line " + std::to_string (L.line) + ": assignment list expected");
		L.next ();
		while (L.tok != '}') {
			if (L.tok != TKN_STRING)
				return fail (-22, "line " + std::to_string (L.line) + ": identifier expected.");
			const std::string sym = L.buf;
			L.next ();
			if (L.tok != '=')
				return fail (-22, "line " + std::to_string (L.line) + ": '=' expected after '" + sym + "'");
			L.next ();
			if (L.tok != TKN_STRING)
				return fail (-22, "line " + std::to_string (L.line) + ": bad expression after '" + sym + "='");
			const std::string val = L.buf;
			if (!bindToProgram (e, prev, pgm, sym.c_str (), val.c_str (), err))
				return fail (-22, "line " + std::to_string (L.line) + ": " + err);
			L.next ();
			if (L.tok == ',')
				L.next ();
			if (L.tok == TKN_EOF || L.tok == TKN_ERROR)
				return fail (-22, "line " + std::to_string (L.line) + ": '}' expected");
		}
		L.next ();
	}
	int used = 0;
	for (auto& P : e->progs)
		used += (P.flags & FL_INUSE) ? 1 : 0;
	return used;
}

int tbf_program_install (tbf_engine* e, uint32_t inst, uint32_t pc)
{
	if (!e || inst >= e->inst.size ())
		return fail (-22, "bad instance");
	Instance& in = e->inst[inst];
	const int p  = (int)(pc & 0x7f) + e->pgmOffset;
	markActive (e, inst);
	if (!(0 < p && p < (int)e->progs.size ()))
		return 0;
	Programme&     P  = e->progs[p];
	const uint32_t f0 = P.flags;
	if (!(f0 & FL_INUSE))
		return 0;
	if (f0 & FL_DRWRND) {
		if (f0 & FL_DRAWBR) randomizeDrawbars (in, P.drawbars);
		if (f0 & FL_LOWDRW) randomizeDrawbars (in, P.lowerDrawbars);
		if (f0 & FL_PDLDRW) randomizeDrawbars (in, P.pedalDrawbars);
	}
	/* setDrawBars (inst, manual, bars) */
	const unsigned* bars[3] = {P.drawbars, P.lowerDrawbars, P.pedalDrawbars};
	const uint32_t  fl[3]   = {FL_DRAWBR, FL_LOWDRW, FL_PDLDRW};
	for (int m = 0; m < 3; m++)
		if (f0 & fl[m])
			for (int b = 0; b < 9; b++)
				in.tg.setDrawBar (m * 9 + b, bars[m][b]);
	if (f0 & FL_SCANNR) {
		const int knob = (int)(((P.scanner & 0xf) << 1) - ((P.scanner & CHO_) ? 1 : 2));
		controlFunction (in, "vibrato.knob", (unsigned char)(knob * 23));
	}
	if (f0 & FL_VCRUPR) {
		int rt = (in.tg.newRouting & 0x01 ? 1 : 0) | (in.tg.newRouting & 0x02 ? 2 : 0);
		rt     = (rt & ~0x2) | ((P.scanner & 0x200) ? 2 : 0);
		controlFunction (in, "vibrato.routing", (unsigned char)(rt << 5));
	}
	if (f0 & FL_VCRLWR) {
		int rt = (in.tg.newRouting & 0x01 ? 1 : 0) | (in.tg.newRouting & 0x02 ? 2 : 0);
		rt     = (rt & ~0x1) | ((P.scanner & 0x100) ? 1 : 0);
		controlFunction (in, "vibrato.routing", (unsigned char)(rt << 5));
	}
	if (f0 & FL_PRCENA) {
		in.tg.setPercEnabled (P.percussionEnabled);
		controlFunction (in, "percussion.enable", P.percussionEnabled ? 127 : 0);
	}
	if (f0 & FL_PRCVOL)
		controlFunction (in, "percussion.volume", P.percussionVolume ? 127 : 0);
	if (f0 & FL_PRCSPD)
		controlFunction (in, "percussion.decay", P.percussionSpeed ? 127 : 0);
	if (f0 & FL_PRCHRM)
		controlFunction (in, "percussion.harmonic", P.percussionHarmonic ? 127 : 0);
	if (f0 & FL_OVRSEL)
		controlFunction (in, "overdrive.enable", P.overdriveSelect ? 127 : 0);
	if (f0 & FL_ROTSPS)
		controlFunction (in, "rotary.speed-preset", (unsigned char)ceilf (P.rotarySpeedSelect * 63.5f));
	/* FL_RVBMIX: installProgram calls the control function "reverb.mix-preset", which is
	 * not a registered name (src/midi.cpp:100-170), so the reference applies nothing.
	 * Keyboard split / transpose (FL_KSPLT*, FL_TRA*, FL_TRCH*) remap MIDI notes to keys:
	 * host-side MIDI routing, outside the engine (its input is keys). */
	in.ctlDirty = true;
	return 0;
}

int tbf_program_name (tbf_engine* e, uint32_t pc, char* out, uint32_t cap)
{
	if (!e || !out || cap == 0)
		return fail (-22, "bad argument");
	const int p = (int)(pc & 0x7f) + e->pgmOffset;
	out[0]      = 0;
	if (!(0 < p && p < (int)e->progs.size ()) || !(e->progs[p].flags & FL_INUSE))
		return 0;
	strncpy (out, e->progs[p].name, cap - 1);
	out[cap - 1] = 0;
	return 1;
}

/* test hook: the instance's control state as doubles (see include/tbf.h) */
int tbf_debug_control (tbf_engine* e, uint32_t inst, double* out, uint32_t cap)
{
	if (!e || !out || inst >= e->inst.size ())
		return fail (-22, "bad argument");
	const Instance& in = e->inst[inst];
	const TgControl& t = in.tg;
	double v[64];
	int    k = 0;
	v[k++] = in.odClean;
	v[k++] = in.odA;
	v[k++] = in.odC;
	v[k++] = in.rvG;
	v[k++] = in.revOpt;
	v[k++] = in.revSelect;
	v[k++] = in.whBypass;
	v[k++] = t.newRouting;
	v[k++] = t.swellPedalGain;
	v[k++] = t.percEnabled;
	v[k++] = t.percIsSoft;
	v[k++] = t.percIsFast;
	v[k++] = t.percSendBus;
	v[k++] = t.vibTable;
	v[k++] = t.vibMixed;
	v[k++] = t.percDrawbarGain;
	for (int b = 0; b < 27; b++)
		v[k++] = t.drawBarGain[b];
	const WhirlRt& w = in.whr;
	for (float f : {w.haT, w.haF, w.haQ, w.haG, w.hbT, w.hbF, w.hbQ, w.hbG, w.hornAcc, w.hornDec, w.drumAcc, w.drumDec})
		v[k++] = f;
	v[k++] = w.cur.hnBrakePos;
	v[k++] = w.cur.drBrakePos;
	const uint32_t n = (uint32_t)k < cap ? (uint32_t)k : cap;
	for (uint32_t i = 0; i < n; i++)
		out[i] = v[i];
	return k;
}

} /* extern "C" */
