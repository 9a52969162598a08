/*
 * oracle/orc_internal.h -- TEST INFRASTRUCTURE ONLY (see orc.h).
 * State layouts of the restated reference structs.
 */
#ifndef TBF_ORC_INTERNAL_H
#define TBF_ORC_INTERNAL_H

#include "orc.h"

/* src/vibrato.h:42-68 struct b_vibrato */
typedef struct orc_vibrato {
	unsigned int  offset1Table[2048];
	unsigned int  offset2Table[2048];
	unsigned int  offset3Table[2048];
	unsigned int* offsetTable;
	unsigned int  stator;
	unsigned int  statorIncrement;
	unsigned int  outPos;
	float         vibBuffer[1024];
	double        vib1OffAmp, vib2OffAmp, vib3OffAmp;
	double        vibFqHertz;
	int           mixedBuffers;
	int           effectEnabled;
} orc_vibrato;

/* src/tonegen.h:98-109 AOTElement */
typedef struct {
	float        busLevel[ORC_NOF_BUSES];
	int          keyCount[ORC_NOF_BUSES];
	int          refCount;
	float        sumUpper, sumLower, sumPedal, sumPercn, sumSwell, sumScanr;
	unsigned int flags;
} orc_aot;

/* src/tonegen.h:114-129 CoreIns (pointers replaced by wheel/offset indices) */
typedef struct {
	short  opr;
	int    cnt;
	size_t off;
	int    wheel;
	size_t src;  /* offset into wave */
	int    envRow; /* -1: none; 0..7 attack; 8..15 release */
	int    envOff;
	float  sgain, nsgain, pgain, npgain, vgain, nvgain;
} orc_coreins;

/* runtime part of src/tonegen.h:176-563 struct b_tonegen */
typedef struct orc_tonegen {
	const orc_template* tpl;
	orc_aot             aot[ORC_NOF_WHEELS + 1];
	int                 activeOscList[ORC_NOF_WHEELS + 1];
	int                 activeOscLEnd;
	unsigned short      msgQueue[1024];
	int                 msgW, msgR;
	float               keyCompTable[128];
	int                 keyDownCount;
	orc_coreins         corePgm[256 * 2 + 8];
	int                 corePgmLen;
	unsigned int        newRouting, oldRouting;
	unsigned int        percSendBus, percSendBusA, percSendBusB;
	unsigned int        upperKeyCount;
	float               swellPedalGain, outputLevelTrim;
	size_t              pos[ORC_NOF_WHEELS + 1];
	int                 aclPos[ORC_NOF_WHEELS + 1];
	unsigned short      rflags[ORC_NOF_WHEELS + 1];
	unsigned int        activeKeys[ORC_MAX_KEYS];
	float               drawBarGain[ORC_NOF_BUSES];
	float               drawBarLevel[ORC_NOF_BUSES][9];
	unsigned short      drawBarChange;
	int                 percEnabled, percTriggerBus, percTrigRestore, percIsSoft, percIsFast;
	float               percEnvGain, percEnvGainReset, percEnvGainDecay, percEnvScaling;
	float               percEnvGainResetNorm, percEnvGainResetSoft;
	float               percEnvGainDecayFastNorm, percEnvGainDecayFastSoft;
	float               percEnvGainDecaySlowNorm, percEnvGainDecaySlowSoft;
	float               percDrawbarNormalGain, percDrawbarSoftGain, percDrawbarGain;
	unsigned short      removedList[ORC_NOF_WHEELS + 1];
	float               swlBuffer[ORC_BLK], vibBuffer[ORC_BLK], vibYBuffr[ORC_BLK], prcBuffer[ORC_BLK];
	float               outputGain, pz, keyCompLevel;
	orc_vibrato         vib;
} orc_tonegen;

/* src/overdrive.h:38-76 struct b_preamp (Airwindows Density subset) */
struct orc_preamp {
	double   iirSampleAL, iirSampleBL;
	int      fpFlip;
	uint32_t fpdL;
	float    A, B, C, D;
	int      isClean;
	double   SampleRateD;
};

/* src/reverb.h:27-110 struct b_reverb, rings indexed A..M = 0..12 */
struct orc_reverb {
	double   biquadA[11], biquadB[11], biquadC[11];
	double*  ring[2][13]; /* [L/R][A..M] */
	int      count[13], delay[13];
	double   feedback[2][8], vib[2][8], depth[8];
	uint32_t fpdL, fpdR;
	float    A, B, C, D, E, F, G;
	double   SampleRateD;
};

/* src/whirl.h:65-221 struct b_whirl */
struct orc_bw {
	float b[5];
};
struct orc_whirl {
	double SampleRateD;
	int    bypass;
	double hnBrakePos, drBrakePos;
	float  hnFwdDispl[16384], drFwdDispl[16384], hnBwdDispl[16384], drBwdDispl[16384];
	struct orc_bw bfw[16384], bbw[16384];
	float  adx0[8], adx1[8], adx2[8];
	int    adi0, adi1, adi2;
	int    hornPhase[6], drumPhase[6];
	double hornAngleGRD, drumAngleGRD, micAngle;
	float  hornRPMslow, hornRPMfast, drumRPMslow, drumRPMfast;
	float  hornAcc, hornDec, drumAcc, drumDec;
	double revHorn[9], revDrum[9];
	int    revselects[3];
	int    revSelect;
	int    hornAcDc, drumAcDc;
	double hornIncr, drumIncr, hornTarget, drumTarget;
	float  hornSpacing[6];
	float  hornRadiusCm, drumRadiusCm, airSpeed, micDistCm, hornXOffsetCm, hornZOffsetCm;
	float  drumSpacing[6];
	float  HLbuf[2048], HRbuf[2048], DLbuf[2048], DRbuf[2048];
	unsigned int outpos;
	float  z[4];
	float  drfL[8], drfR[8];
	int    lpT;
	double lpF, lpQ, lpG;
	float  hafw[8];
	float  haT, haF, haQ, haG;
	float  hbfw[8];
	float  hbT, hbF, hbQ, hbG;
	float  hornLevel, leakLevel, leakage;
	float  drumMic_dll, drumMic_dlr, drumMic_drl, drumMic_drr;
	float  hornMic_hll, hornMic_hlr, hornMic_hrl, hornMic_hrr;
};

struct orc_inst {
	orc_tonegen       tg;
	struct orc_preamp pre;
	struct orc_reverb* rev;
	struct orc_whirl*  wh;
	int               chain;
	double            params[64];
	float             bufA[ORC_BLK], bufB[ORC_BLK], bufC[ORC_BLK];
	float             bufL[ORC_BLK], bufR[ORC_BLK], bufDL[ORC_BLK], bufDR[ORC_BLK];
};

/* tonegen runtime (orc_tonegen.c) */
void orc_tg_init (orc_tonegen* t, const orc_template* tpl, const orc_cfg* c);
void orc_tg_key_on (orc_tonegen* t, int key);
void orc_tg_key_off (orc_tonegen* t, int key);
void orc_tg_set_drawbar (orc_tonegen* t, int bus, unsigned int setting);
void orc_tg_set_vibrato_upper (orc_tonegen* t, int on);
void orc_tg_set_vibrato_lower (orc_tonegen* t, int on);
void orc_tg_set_vibrato_from_int (orc_tonegen* t, int param);
void orc_tg_set_perc_enabled (orc_tonegen* t, int on);
void orc_tg_set_perc_volume (orc_tonegen* t, int isSoft);
void orc_tg_set_perc_fast (orc_tonegen* t, int isFast);
void orc_tg_set_perc_first (orc_tonegen* t, int isFirst);
void orc_tg_generate (orc_tonegen* t, float* buf);
void orc_vibrato_init (orc_vibrato* v, double rate, const orc_cfg* c);
void orc_vibrato_proc (orc_vibrato* v, const float* in, float* out, size_t n);

/* effects (orc_fx.c) */
void orc_preamp_init (struct orc_preamp* p, orc_rand* rnd, double sr);
void orc_preamp_set_character (struct orc_preamp* p, float A);
void orc_preamp_run (struct orc_preamp* p, const float* in, float* out, int n);
struct orc_reverb* orc_reverb_alloc (orc_rand* rnd, double sr);
void orc_reverb_run (struct orc_reverb* r, const float* in, float* out, int n);
struct orc_whirl* orc_whirl_alloc (double sr, const orc_cfg* c);
void orc_whirl_use_rev_option (struct orc_whirl* w, int n, int signals);
int  orc_whirl_control (struct orc_whirl* w, const char* fn, unsigned char uc);
void orc_whirl_run3 (struct orc_whirl* w, const float* in, float* L, float* R, float* tL, float* tR, size_t n);
void orc_eq_compute (int type, double fqHz, double Q, double dbG, double* C, double sr);

#endif
