/*
 * tbf_host.h -- host-side table builders and the tonegen control plane.
 *
 * Everything here runs once per template / instance / event on the CPU, in the
 * reference's FP64/FP32 arithmetic with glibc libm, so the tables the device consumes
 * are bit-identical to what the reference's init code builds:
 *   - TgTemplate: initToneGenerator's shared part (src/tonegen.cpp:2905-3066):
 *     frequencies (src/tuning.cpp:142), play matrix (1122-1213), wave bank
 *     (1470-1630), key-compression table (1939-1966), envelopes (2562-2728);
 *   - WhirlTables: computeOffsets/initTables (src/whirl.cpp:534-624, 338-517);
 *   - TgControl: the message-queue / active-list / routing part of
 *     oscGenerateFragment (src/tonegen.cpp:3257-3594) which turns key and drawbar
 *     events into per-block core programs for the device.
 */
#ifndef TBF_HOST_H
#define TBF_HOST_H

#include <stdint.h>

#include <vector>

#include "tbf_types.h"

namespace tbf {

/* glibc rand() (TYPE_3) -- srand(seed) stream of the reference hosts */
struct GlibcRand {
	int32_t s[31];
	int     f = 3, r = 0;
	explicit GlibcRand (unsigned int seed);
	int32_t next ();
	/* the 31 words y[i-31 .. i-1] before the next draw y[i] (oldest first) */
	void window (uint32_t* W) const;
	/* skip k draws by the polynomial jump of tbf_rand.h (same state as k next () calls) */
	void discard (uint64_t k);
};

struct Contrib {
	int16_t wheel, bus;
	float   level;
};

/* The hot path's cfg keys (parseConfigurationLine / distributeParameter,
 * src/cfgParser.cpp:61-160) with the reference's defaults and field types:
 * whirlConfig (src/whirl.cpp:992-1160; initValues 43-134), oscConfig
 * (src/tonegen.cpp:2173-2555; initValues 238-331), scannerConfig (src/vibrato.cpp:334-357)
 * and reverbConfig (src/reverb.cpp:242-256). */
enum { ENV_CLICK = 0, ENV_COSINE = 1, ENV_LINEAR = 2, ENV_SHELF = 3 };
enum { EQ_SPLINE = 0, EQ_PEAK24 = 1, EQ_PEAK46 = 2 };                 /* src/tonegen.cpp:143-145 */
enum { LE_HARMONIC = 0, LE_TERMINAL = 1, LE_TAPER = 2, LE_XTALK = 3 }; /* which list */
struct Config {
	/* whirl.* */
	float  hornRPMslow = (float)(60.0 * 0.672), hornRPMfast = (float)(60.0 * 7.056);
	float  drumRPMslow = (float)(60.0 * 0.600), drumRPMfast = (float)(60.0 * 5.955);
	float  hornAcc = 0.161f, hornDec = 0.321f, drumAcc = 4.127f, drumDec = 1.371f;
	float  hornRadiusCm = 19.2f, drumRadiusCm = 22.0f, micDistCm = 42.0f, hornXOffsetCm = 0.0f, hornZOffsetCm = 0.0f;
	float  hornLevel = 0.7f, leakLevel = 0.15f;
	float  drumMicWidth = 0.0f, hornMicWidth = 0.0f;
	int    lpT = 8;
	double lpF = 811.9695, lpQ = 1.6016, lpG = -38.9291;
	float  haT = 0, haF = 4500, haQ = 2.7456f, haG = -30.0f;
	float  hbT = 7, hbF = 300.0f, hbQ = 1.0f, hbG = -30.0f;
	int    revSelect = 0, bypass = 0;
	double micAngle = 0, hnBrakePos = 0, drBrakePos = 0;
	/* scanner.* */
	double vibFqHertz = 7.25, vib1OffAmp = 3.0, vib2OffAmp = 6.0, vib3OffAmp = 9.0;
	/* reverb.mix */
	float  reverbMix = 0.1f;
	/* osc.* (scalar keys) */
	double tgPrecision = 0.001, percFastDecaySeconds = 1.0, percSlowDecaySeconds = 4.0;
	float  percEnvGainResetNorm = 1.0f, percEnvGainResetSoft = 0.5012f, percEnvScaling = 11.0f;
	int    percSendBusA = 3, percSendBusB = 4, percTriggerBus = 8;
	float  envAttackClickLevel = 0.50f, envReleaseClickLevel = 0.25f;
	int    envAtkClkMinLength = -1, envAtkClkMaxLength = -1; /* -1: from the sample rate */
	int    envAttackModel = ENV_CLICK, envReleaseModel = ENV_LINEAR;
	/* osc.* tone-generator model keys (initValues 302-316): wheel EQ, the default
	 * crosstalk model's levels, the play matrix contribution floor / minimum */
	int    eqMacro = EQ_SPLINE;
	double eqP1y = 1.0, eqR1y = 0.0, eqP4y = 1.0, eqR4y = 0.0;
	double compartmentXT = 0.01, transformerXT = 0.0, stripXT = 0.01, wiringXT = 0.01;
	double contribFloor = 0.0000158, contribMin = 0.0;
	/* osc.harmonic.* / osc.terminal.* / osc.taper.* / osc.crosstalk.*: one element per
	 * appendListElement of oscConfig (src/tonegen.cpp:2296-2474), in file order */
	struct ListEntry {
		int16_t kind, idx; /* LE_*, list index (wheel / terminal / key) */
		int16_t sa, sb;    /* harmonic number | wheel | terminal ; bus */
		float   fc;        /* level */
	};
	std::vector<ListEntry> lists;
};

/* what a cfg key touches (configSet's `scope` out-parameter) */
enum { CFG_SHARED = 1, /* engine-wide tables: whirl.*, scanner.* */
       CFG_TEMPLATE = 2, /* templates created afterwards: osc.x-precision, envelopes */
       CFG_INSTANCE = 4 /* instances added afterwards: perc, reverb.mix, per-instance whirl */ };
/* one key=value: 1 applied, 0 not a key of the hot path or a key with no effect on it,
 * -1 unparsable / out of range (nothing assigned) */
int configSet (Config& c, const char* key, const char* value, int* scope);

struct TgTemplate {
	double                            sr = 48000.0;
	double                            frequency[300];
	double                            targetRatio[9];
	int                               envMin = 0, envMax = 0;
	std::vector<Contrib>              keyContrib[384];
	std::vector<float>                bank; /* wheels 1..256 concatenated */
	uint32_t                          off[TBF_NW + 1] = {0};
	uint32_t                          len[TBF_NW + 1] = {0};
	float                             keyCompTable[128];
	float                             attackEnv[9][TBF_BLK];
	float                             releaseEnv[9][TBF_BLK];
	/* writeSamples spectrum per wheel: y[n] = (float)(lsb (draw off + n) + U sum_q
	 * amp[q] sin (remainder (hz[q] 2 pi n / sr, 2 pi))) over the nonzero partials */
	double                            U[TBF_NW + 1];
	int                               nPartials[TBF_NW + 1];
	double                            pAmp[TBF_NW + 1][12], pHz[TBF_NW + 1][12];
	size_t                            total = 0; /* bank samples = rand() draws of the bank */
	Config                            cfg; /* the osc.* template keys it was built with */
	void build (double sr, const double* mts128, const double* ratio9, unsigned int seed, const Config& c);
	/* the steps of build: prepare (tables, play matrix unless matrix is false, wheel
	 * lengths and spectra), synthHost (the bank, one draw per sample), finish (key
	 * compression, envelopes: the draws after the bank) */
	void prepare (double sr, const double* mts128, const double* ratio9, const Config& c, bool matrix = true);
	void synthHost (GlibcRand& rnd);
	void finish (GlibcRand& rnd);
};

/* the template-independent inputs of the play matrix for the device builder (k_tpl_matrix,
 * tbf_tpl.hip): the terminal mix of applyDefaultConfiguration (src/tonegen.cpp:933-1003),
 * the cfg's taper and crosstalk lists per key, the manual taper levels (taper (),
 * 502-692), and the bound on a key's list length that sizes the device staging */
struct MatrixInputs {
	std::vector<tbf_le>   tm, tp, xt;          /* flattened lists */
	std::vector<uint32_t> tmOff, tpOff, xtOff; /* TBF_NW + 2, 385, 385 offsets */
	float                 taper[128][9];
	double                wiringXT = 0, floor = 0, minLevel = 0;
	uint32_t              cap = 0;
	void build (const Config& c);
};

struct WhirlTables {
	double             sr = 0;
	std::vector<float> displ; /* hnFwd, hnBwd, drFwd, drBwd: 4 x 16384 */
	std::vector<float> bw;    /* bfw, bbw: 2 x 16384 x 5 */
	float              hornSpacing[6], drumSpacing[6];
	int32_t            phase[6];
	float              drf[5];
	double             revHorn[9], revDrum[9];
	float              maxAhead; /* largest write-ahead in samples */
	void build (double sr, const Config& c);
};

/* the whirl fields the MIDI control functions set (struct b_whirl, src/whirl.h; setters
 * src/whirl.cpp:699-889), with the reference's field types, and the parameter set k_whirl
 * renders with: the horn filters through setIIRFilter (UPDATE_A_FILTER / UPDATE_B_FILTER),
 * the speed-ramp factors of whirlProc2 (1255-1257, 1306-1308) */
struct WhirlRt {
	float         haT = 0, haF = 0, haQ = 0, haG = 0, hbT = 0, hbF = 0, hbQ = 0, hbG = 0;
	float         hornAcc = 0, hornDec = 0, drumAcc = 0, drumDec = 0;
	double        sr = 0;
	tbf_wh_params cur = {}; /* the set as of the last setter (hnBrakePos / drBrakePos live here) */
	void init (double sr, const Config& c); /* initValues + whirlConfig + initialize */
	bool control (const char* fn, unsigned char u); /* false: not a whirl parameter */
	void ramps ();
};

/* per-instance tonegen control state (runtime fields of struct b_tonegen) */
struct TgControl {
	struct Aot {
		float busLevel[27];
		int   keyCount[27];
		int   refCount;
		float sumUpper, sumLower, sumPedal, sumPercn, sumSwell, sumScanr;
	};
	/* per-wheel state of the host control path (step).  The device path (stepFront) keeps
	 * it in tbf_tgc_state instead, so it is allocated by the first step () only: an
	 * instance's per-block fields then sit a few KB from the next instance's, not 70 KB
	 * (host worker threads stepping thousands of instances are bound by that footprint) */
	struct Wheels {
		Aot      aot[TBF_NW + 1];
		int      activeOscList[TBF_NW + 1];
		int      activeOscLEnd = 0;
		int      aclPos[TBF_NW + 1];
		uint16_t rflags[TBF_NW + 1];
		Wheels ();
	};
	const TgTemplate*     tpl = nullptr;
	std::vector<Wheels>   wh; /* empty until step () */
	std::vector<uint16_t> msg;
	int               keyDownCount = 0;
	unsigned          upperKeyCount = 0;
	unsigned          newRouting = 0, oldRouting = 0;
	unsigned          percSendBus = 4, percSendBusA = 3, percSendBusB = 4;
	float             swellPedalGain = 0.07f, outputLevelTrim = 0.07f;
	uint32_t          keyBits[12]; /* activeKeys[384] (src/tonegen.cpp:3096-3166) as bits */
	float             drawBarGain[27];
	float             drawBarLevel[27][9];
	uint16_t          drawBarChange = 0;
	int               percEnabled = 0, percTriggerBus = 8, percTrigRestore = 0, percIsSoft = 0, percIsFast = 0;
	float             percEnvGainReset = 0, percEnvGainDecay = 0, percEnvScaling = 11.0f;
	float             percEnvGainResetNorm = 1.0f, percEnvGainResetSoft = 0.5012f;
	float             percEnvGainDecayFastNorm = 0.9995f, percEnvGainDecayFastSoft = 0.9995f;
	float             percEnvGainDecaySlowNorm = 0.9999f, percEnvGainDecaySlowSoft = 0.9999f;
	float             percDrawbarNormalGain = 0.60512f, percDrawbarSoftGain = 1.0f, percDrawbarGain = 1.0f;
	/* vibrato knob (setVibrato, src/vibrato.cpp:97-129) */
	uint32_t          vibTable = 2, vibMixed = 0;
	bool              steadyPending = false; /* last block emitted env entries / removals */
	bool              gainsSent = false;     /* the device holds drawBarGain (stepFront) */
	uint32_t          gainMask  = 0;         /* buses whose drawBarGain changed since the last send */

	void init (const TgTemplate* t, const Config& c);
	void keyOn (int key);
	void keyOff (int key);
	/* keyOn / keyOff without queueing the messages (the device front end derives them):
	 * returns the number of messages the key event makes */
	int noteCount (int key, bool on);
	bool keyActive (int key) const { return (keyBits[key >> 5] >> (key & 31)) & 1u; }
	void keySet (int key) { keyBits[key >> 5] |= 1u << (key & 31); }
	void keyClear (int key) { keyBits[key >> 5] &= ~(1u << (key & 31)); }
	void setDrawBar (int bus, unsigned setting);
	void setVibratoUpper (int on);
	void setVibratoLower (int on);
	void setVibratoFromInt (int param);
	void setPercEnabled (int on);
	void setPercVolume (int isSoft);
	void setPercFast (int isFast);
	void setPercFirst (int isFirst);
	bool dirty () const;
	/* one block of control: returns the block's program and mixdown control */
	void step (std::vector<tbf_prog_entry>& prog, tbf_seg_ctl& ctl);
	/* the same block with the per-wheel part left to the device (k_tgctl): the block's
	 * key messages (msg.size () of them, written to msgDst = the chunk's message array
	 * at msgOff) and drawbar / routing inputs in rec, the mixdown control in ctl.
	 * wh (aot / active list / rflags) is not used. */
	void stepFront (uint16_t* msgDst, uint32_t msgOff, float* gainDst, uint32_t gainOff, tbf_tgc_rec& rec,
	                tbf_seg_ctl& ctl);
	/* the (bus, gain) pairs stepFront sends on this step (gainDst: 2 words each): the changed
	 * buses, or all 27 until the device holds them */
	uint32_t gainPairs () const { return !gainsSent ? 27u : (uint32_t)__builtin_popcount (gainMask); }
	void mixCtl (tbf_seg_ctl& ctl) const;
};

} // namespace tbf

#endif
