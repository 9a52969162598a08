/*
 * oracle/orc.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the tuneBfree per-sample DSP chain
 *   oscGenerateFragment -> preamp -> b_reverb::reverb -> whirlProc3
 * (reference: /root/reference/src/{tonegen,vibrato,overdrive,reverb,whirl,eqcomp,tuning}.cpp).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code, and only as the checker.  The product (tunebfree_amd/) never links
 * or calls it.  Every function cites the reference file:line it restates.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - init tables: the 6 tests/regression_test_data fixture sets (byte-exact dumps)
 *     plus the reference doctest known answers (fitWave, tuning, crosstalk);
 *   - runtime (all five stages): bit-exact against the reference's own
 *     translation units compiled from /root/reference/src by oracle/Makefile
 *     into oracle/_ref/ (strict IEEE, -ffp-contract=off), see oracle/ref_harness.cpp.
 *
 * Float discipline: compiled with -O2 -ffp-contract=off, no fast-math; every
 * float/double expression keeps the reference's literal evaluation order.
 */
#ifndef TBF_ORACLE_H
#define TBF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_BLK 128
#define ORC_NOF_WHEELS 256
#define ORC_NOF_FREQS 300
#define ORC_MAX_KEYS 384
#define ORC_NOF_BUSES 27
#define ORC_MAX_PARTIALS 12

/* ---------------- glibc-compatible rand() (TYPE_3 additive feedback) ------------- */
typedef struct orc_rand {
	int32_t state[31];
	int     f, r;
} orc_rand;

void    orc_srand (orc_rand* s, unsigned int seed);
int32_t orc_rand_next (orc_rand* s);

/* ---------------- tuning (src/tuning.cpp) ---------------- */
/* 128 MTS-ESP note frequencies -> 300-entry table. mts128 == NULL -> MTS-ESP with
 * no master connected (12-TET, A4 = 440 Hz). */
void orc_get_frequencies (double* out300, const double* mts128);
void orc_infer_scale_size (const double* f128, int* scaleSize, float* period);
short orc_paired_wheel (short n);

/* ---------------- list element (src/tonegen.h:59-71) ---------------- */
typedef struct {
	short sa, sb;
	float fc;
} orc_le;

typedef struct {
	orc_le* v;
	int     n, cap;
} orc_list;

/* ---------------- configuration: the cfg keys of the hot path ----------------
 * Restates the assignments of whirlConfig (src/whirl.cpp:992-1160), oscConfig
 * (src/tonegen.cpp:2173-2555, the scalar keys), scannerConfig (src/vibrato.cpp:334-357)
 * and reverbConfig (src/reverb.cpp:242-256), with the defaults of initValues
 * (src/whirl.cpp:43-134, src/tonegen.cpp:238-331, src/vibrato.cpp:296-300) and the
 * reverb ctor (src/reverb.cpp:217).  overdrive.* / xov.* (ampConfig,
 * src/overdrive.cpp:395-433) only write legacy fields airwindows_density never reads,
 * so they are accepted and have no effect, as in the reference. */
#define ORC_ENV_CLICK 0
#define ORC_ENV_COSINE 1
#define ORC_ENV_LINEAR 2
#define ORC_ENV_SHELF 3
#define ORC_EQ_SPLINE 0 /* src/tonegen.h eqMacro values (EQ_SPLINE, EQ_PEAK24, EQ_PEAK46) */
#define ORC_EQ_PEAK24 1
#define ORC_EQ_PEAK46 2
#define ORC_LE_HARMONIC 0 /* wheelHarmonics[idx] (idx 0: every wheel) */
#define ORC_LE_TERMINAL 1 /* terminalMix[idx] */
#define ORC_LE_TAPER 2    /* keyTaper[idx] */
#define ORC_LE_XTALK 3    /* keyCrosstalk[idx] */
#define ORC_CFG_MAX_LE 8192
typedef struct orc_cfg {
	/* whirl.* (struct b_whirl field types) */
	float  hornRPMslow, hornRPMfast, drumRPMslow, drumRPMfast;
	float  hornAcc, hornDec, drumAcc, drumDec;
	float  hornRadiusCm, drumRadiusCm, micDistCm, hornXOffsetCm, hornZOffsetCm;
	float  hornLevel, leakLevel;
	float  drumMicWidth, hornMicWidth;
	int    lpT;
	double lpF, lpQ, lpG;
	float  haT, haF, haQ, haG, hbT, hbF, hbQ, hbG;
	int    revSelect, bypass;
	double micAngle, hnBrakePos, drBrakePos;
	/* scanner.* */
	double vibFqHertz, vib1OffAmp, vib2OffAmp, vib3OffAmp;
	/* reverb.mix */
	float  reverbMix;
	/* osc.* */
	double tgPrecision, percFastDecaySeconds, percSlowDecaySeconds;
	float  percEnvGainResetNorm, percEnvGainResetSoft, percEnvScaling;
	int    percSendBusA, percSendBusB, percTriggerBus;
	float  envAttackClickLevel, envReleaseClickLevel;
	int    envAtkClkMinLength, envAtkClkMaxLength; /* -1: from the sample rate */
	int    envAttackModel, envReleaseModel;
	/* osc.* tone-generator model keys (struct b_tonegen fields, initValues 302-316):
	 * wheel EQ macro and spline points, the default crosstalk levels, the play matrix
	 * contribution floor / minimum */
	int    eqMacro; /* ORC_EQ_* */
	double eqP1y, eqR1y, eqP4y, eqR4y;
	double compartmentXT, transformerXT, stripXT, wiringXT;
	double contribFloor, contribMin;
	/* the list keys (osc.harmonic.*, osc.terminal.*, osc.taper.*, osc.crosstalk.*) in
	 * file order: each becomes one ListElement appended to its list, exactly as
	 * oscConfig's appendListElement calls (src/tonegen.cpp:2296-2474) */
	int    nle;
	struct {
		short kind, idx; /* ORC_LE_*, list index (wheel / terminal / key) */
		short sa, sb;    /* harmonic number | wheel | terminal ; bus */
		float fc;        /* level */
	} le[ORC_CFG_MAX_LE];
} orc_cfg;

void   orc_cfg_default (orc_cfg* c);
size_t orc_cfg_size (void);
/* one cfg line's key and value: 1 applied, 0 not a key of the hot path (ignored), -1
 * unparsable or out of range (not applied), as getConfigParameter_* (src/cfgParser.cpp) */
int  orc_cfg_set (orc_cfg* c, const char* key, const char* value);

/* ---------------- tonegen template: everything initToneGenerator builds ---------------- */
typedef struct orc_template {
	double sr;
	double frequency[ORC_NOF_FREQS];
	double targetRatio[9];
	int    envAtkClkMinLength, envAtkClkMaxLength;
	orc_list terminalMix[ORC_NOF_WHEELS + 1];
	orc_list keyTaper[ORC_MAX_KEYS];
	orc_list keyCrosstalk[ORC_MAX_KEYS];
	orc_list keyContrib[ORC_MAX_KEYS];
	float*   wave[ORC_NOF_WHEELS + 1];
	size_t   wlen[ORC_NOF_WHEELS + 1];
	double   wfreq[ORC_NOF_WHEELS + 1];
	double   watt[ORC_NOF_WHEELS + 1];
	float    keyCompTable[128];
	float    attackEnv[9][ORC_BLK];
	float    releaseEnv[9][ORC_BLK];
} orc_template;

orc_template* orc_template_new (double sr, const double* mts128, const double* ratio9, unsigned int seed);
/* the same with the osc.* template keys of cfg (x-precision, envelope models/levels/lengths) */
orc_template* orc_template_new_cfg (double sr, const double* mts128, const double* ratio9, unsigned int seed,
                                    const orc_cfg* cfg);
void          orc_template_free (orc_template* t);
int           orc_template_dump (const orc_template* t, const char* dir);
/* flat export of the wave bank (wheels 1..256 concatenated) for product cross-checks */
size_t        orc_template_bank_size (const orc_template* t);
void          orc_template_bank (const orc_template* t, float* out, uint32_t* lens);
void          orc_template_envs (const orc_template* t, float* attack9x128, float* release9x128, float* keycomp128);
size_t        orc_fitwave (double hz, double precision, int minS, int maxS, double rate);
int           orc_template_contrib (const orc_template* t, int key, int16_t* wheel, int16_t* bus, float* level, int cap);

/* ---------------- instances ---------------- */
typedef struct orc_inst orc_inst;

/* LV2 construction protocol (b_synth/lv2.cpp:336-353, 164-193) with the tonegen
 * template shared: srand(seed) -> allocReverb (18+ rand) -> allocPreamp (1+ rand);
 * then initSynth: tonegen runtime init, init_vibrato, initPreamp, initReverb,
 * initWhirl, setDrawBars(upper, {8,8,6,0,...}). */
orc_inst* orc_inst_new (const orc_template* tpl, unsigned int seed);
/* the same with cfg applied before each module's init, as the reference's startup
 * parses the cfg between alloc* and init* (whirl, scanner, percussion, reverb.mix) */
orc_inst* orc_inst_new_cfg (const orc_template* tpl, unsigned int seed, const orc_cfg* cfg);
void      orc_inst_free (orc_inst* p);
/* the CLAP reinitToneGen on a new template (MTS-ESP retune / drawbar ratios), see
 * orc_chain.c; takes effect from the next orc_render block */
void      orc_inst_retune (orc_inst* p, const orc_template* tpl, const orc_cfg* cfg);
void      orc_param_defaults (double* params64);
void      orc_note (orc_inst* p, int key, int on);                 /* oscKeyOn/Off */
void      orc_set_param (orc_inst* p, int pid, double value);      /* CLAP setParam */
void      orc_set_chain (orc_inst* p, int mode);                   /* 0 full, 1 tonegen only */
/* a MIDI control function by name, value 0..127: the whirl's runtime parameters
 * (whirl.horn.filter.{a,b}.{type,hz,q,gain}, whirl.{horn,drum}.brakepos,
 * whirl.{horn,drum}.{acceleration,deceleration}); -1 for any other name */
int       orc_control (orc_inst* p, const char* name, int value);
/* the whirl fields the control functions write (test hook, for the setter pin
 * oracle/ref_whirl_pin.cpp): haT haF haQ haG hafw[1..5] hbT hbF hbQ hbG hbfw[1..5]
 * hnBrakePos drBrakePos hornAcc hornDec drumAcc drumDec; returns the count (24) */
int       orc_whirl_fields (const orc_inst* p, double* out);
/* render nblocks of the synthSound quartet; any output pointer may be NULL.
 * sA/sB/sC receive the tonegen, preamp and reverb stage outputs. */
void orc_render (orc_inst* p, int nblocks, float* L, float* R, float* sA, float* sB, float* sC);
/* the core program of the last orc_render block: 9 floats per instruction
 * {wheel, opr, envRow, sg, pg, vg, nsg, npg, nvg} (wrap-split halves included) */
int           orc_debug_program (const orc_inst* p, float* out9, int cap);
/* test hook: set the reverb vibrato phase vib[c][l] (lines 0..7) */
void          orc_debug_rv_phase (orc_inst* p, int c, int l, double value);

/* parameter ids (src/clap.cpp:31-48) */
#define ORC_P_DRAWBAR_MIN 0
#define ORC_P_DRAWBAR_MAX 8
#define ORC_P_VIBRATO 9
#define ORC_P_VIBRATO_TYPE 10
#define ORC_P_DRUM 11
#define ORC_P_HORN 12
#define ORC_P_OVERDRIVE 13
#define ORC_P_CHARACTER 14
#define ORC_P_REVERB 15
#define ORC_P_PERCUSSION 16
#define ORC_P_PERCUSSION_VOLUME 17
#define ORC_P_PERCUSSION_DECAY 18
#define ORC_P_PERCUSSION_HARMONIC 19
/* extension ids beyond the CLAP set (lower/pedal drawbars via setDrawBar bus index,
 * vibrato lower routing, swell pedal, whirl bypass) */
#define ORC_P_BUS_DRAWBAR_BASE 100 /* 100+bus (0..26), value 0..8 */
#define ORC_P_VIBRATO_LOWER 130
#define ORC_P_SWELL 131           /* swellPedalGain, value 0..1 of outputLevelTrim */
#define ORC_P_WHIRL_BYPASS 132

/* ---------------- single-stage access (unit parity against oracle/_ref) ---------------- */
typedef struct orc_whirl  orc_whirl;
typedef struct orc_reverb orc_reverb;
typedef struct orc_preamp orc_preamp;

orc_whirl*  orc_whirl_new (double sr);
void        orc_whirl_free (orc_whirl* w);
void        orc_whirl_rev_option (orc_whirl* w, int n);
void        orc_whirl_proc3 (orc_whirl* w, const float* in, float* L, float* R, int n);
orc_reverb* orc_reverb_new (double sr, unsigned int seed);
void        orc_reverb_free (orc_reverb* r);
void        orc_reverb_set_mix (orc_reverb* r, float g);
void        orc_reverb_proc (orc_reverb* r, const float* in, float* out, int n);
orc_preamp* orc_preamp_new (double sr, unsigned int seed);
void        orc_preamp_free (orc_preamp* p);
void        orc_preamp_set (orc_preamp* p, int clean, float character);
void        orc_preamp_proc (orc_preamp* p, const float* in, float* out, int n);

#ifdef __cplusplus
}
#endif
#endif
