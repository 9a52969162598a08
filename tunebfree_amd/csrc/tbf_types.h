/*
 * tbf_types.h -- POD layouts shared by the host control plane (tbf_engine.cpp) and
 * the gfx950 render kernel (tbf_render.hip).
 *
 * Naming follows the reference's domain: wheels, buses, programs (the tonegen "core
 * program", src/tonegen.cpp:3333-3566), delay lines, rings, rotors.
 */
#ifndef TBF_TYPES_H
#define TBF_TYPES_H

#include <stdint.h>

#define TBF_BLK 128   /* BUFFER_SIZE_SAMPLES, src/tonegen.h:53 */
#define TBF_SUB 64    /* sub-block for reverb/whirl: one sample per lane of a wave64 */
#define TBF_NW 256    /* NOF_WHEELS, src/tonegen.h:79 */
#define TBF_VRING 256
#define TBF_WH_TSTRIDE 16388 /* device stride of the whirl displacement tables (16-byte aligned rows) */
#define TBF_XS_JUMP 129 /* dither jump table columns: k = 0 .. 128 steps */ /* compact vibrato ring (reference 1024; live window <= 21+128) */

/* one core-program entry = one wheel's contribution for one block
 * (CoreIns, src/tonegen.h:114-129; wrap splitting is done on the device) */
typedef struct tbf_prog_entry {
	uint16_t wheel;
	uint8_t  env; /* 0 plain (CR_CPY/ADD), 1 attack env, 2 release env */
	uint8_t  row; /* envelope row i & 7 */
	float    sg, pg, vg;    /* sgain, pgain, vgain */
	float    nsg, npg, nvg; /* next gains (env entries) */
	uint32_t pad;
} tbf_prog_entry;

/* A program slot is a header entry (wheel = 0xFFFF, pad = entry count) followed by the
 * entries; seg_ctl.prog_off indexes the header.  TBF_PROG_SLOT entries per slot. */
#define TBF_PROG_SLOT (TBF_NW + 2)
/* persistent program slots per instance (device control): k_tgctl of chunk c writes the
 * instance's final program into the slot after the current one (mod 3), which neither
 * chunk c nor chunk c - 1 renders from, so it may run beside chunk c - 1's k_tonegen */
#define TBF_PROG_PSLOTS 3

/* device-side tone-generator control (k_tgctl): the per-wheel part
 * of oscGenerateFragment's control (src/tonegen.cpp:3257-3594: the message queue's
 * activated-oscillator-table updates, the active list, routing sums and the core
 * program) runs on the device; the host keeps the key / drawbar / routing front end and
 * hands each stepped block this record */
typedef struct tbf_tgc_rec {
	uint32_t msgOff;         /* the block's key messages (0x1000 | key: on, key: off) ... */
	uint32_t nMsg;           /* ... msgs[msgOff .. msgOff + nMsg), all of the block's */
	uint32_t gainOff;        /* flags & 4: pad (bus, drawBarGain[bus]) pairs at gains[gainOff ..], the
	                          * bus as the float's bits (the buses that changed; k_tgctl keeps all 27
	                          * in tbf_tgc_state) */
	uint32_t full;           /* > 0: the delta's control entry is fulls[full - 1]; 0: the instance's
	                          * entry before it with the fields below (a key / drawbar step changes
	                          * no others), so only these 24 B cross PCIe, not the 120-B entry */
	float    keyCompTarget;  /* (full == 0) keyCompTable[keyDownCount] */
	uint8_t  flags;          /* 1 drawBarChange, 2 recomputeRouting, 4 gains follow, 8 resetPercAtEnd
	                          * (full == 0), 0x80 stepped */
	uint8_t  oldRouting;     /* routing word after this block's update */
	uint8_t  percSendBus;    /* a bus index (< 27) */
	uint8_t  pad;            /* flags & 4: the number of gain pairs */
} tbf_tgc_rec;

/* device front end (chunks of note, drawbar, vibrato-switch and percussion-switch events,
 * k_front): an instance's tone-generator front state at the chunk start */
typedef struct tbf_front_state {
	uint32_t keys[12];       /* activeKeys, 384 bits */
	int32_t  keyDown;        /* keyDownCount */
	int32_t  upperDown;      /* upperKeyCount */
	uint32_t pending;        /* steadyPending: the block before had inputs */
	uint32_t percSendBus;
	uint32_t routing;        /* the routing word (oldRouting == newRouting at the chunk start) */
	int32_t  percEnabled;
	int32_t  percTrigRestore;
	int32_t  percTriggerBus; /* < 0: none */
	uint32_t percSendBusA, percSendBusB;
	uint32_t gainOff;        /* the instance's slots for (bus, gain) pairs in gains (floats) */
	/* effect setters (TBF_FEV_EFFECT): the instance's percussion constants (percEnvScaling
	 * applied, src/tonegen.cpp:1725-1765) and the switches and swell at the chunk start */
	float    percReset[2];   /* percEnvGainReset, [isSoft] */
	float    percDrawbar[2]; /* percDrawbarGain, [isSoft] */
	float    percDecay[4];   /* percEnvGainDecay, [isFast * 2 + isSoft] */
	int32_t  percSoft, percFast;
	float    swell;          /* swellPedalGain */
	uint32_t pad;
} tbf_front_state;

/* a front-end event, 4 bytes: block << 16 | low 16 bits
 *   note   key (12 bits; 0x0fff: outside [0, 384), ignored) | on << 12
 *   param  0x8000 | op << 12 | flag << 9 | setting << 5 | bus, op:
 *          TBF_FEV_DRAWBAR (setting 0..8, 15: out of range, ignored), TBF_FEV_VIB_UPPER /
 *          TBF_FEV_VIB_LOWER / TBF_FEV_PERC (flag: on), TBF_FEV_PERC_FIRST (flag: first),
 *          TBF_FEV_EFFECT (bus = TBF_FX_*: a setter of the block's control entry; its value,
 *          as the host derives it from the parameter, is fevVal[event]) */
#define TBF_FEV_PARAM 0x8000u
#define TBF_FEV_DRAWBAR 0u
#define TBF_FEV_VIB_UPPER 1u
#define TBF_FEV_VIB_LOWER 2u
#define TBF_FEV_PERC 3u
#define TBF_FEV_PERC_FIRST 4u
#define TBF_FEV_EFFECT 5u
/* effect setters (src/clap.cpp:162-207 setParam) and their fevVal */
#define TBF_FX_ROTOR 0u      /* useRevOption (src/whirl.cpp:174-196): the option, a one-shot */
#define TBF_FX_CLEAN 1u      /* setClean (src/overdrive.cpp:387): the clean flag */
#define TBF_FX_CHARACTER 2u  /* fsetCharacter (src/overdrive.cpp:552-574): A in [0, 1] */
#define TBF_FX_REVERB 3u     /* setReverbMix (src/reverb.cpp:233): G */
#define TBF_FX_PERC_SOFT 4u  /* setPercussionVolume (src/tonegen.cpp:1740-1752): isSoft */
#define TBF_FX_PERC_FAST 5u  /* setPercussionFast (1727-1732): isFast */
#define TBF_FX_SWELL 6u      /* the swell pedal: swellPedalGain */
#define TBF_FX_BYPASS 7u     /* whirl bypass */
#define TBF_FX_VIBTYPE 8u    /* setVibrato knob (src/vibrato.cpp:97-129): 0..5 */

/* one keyContrib element on the device (Contrib): a key's list is sorted by wheel, then
 * bus (compilePlayMatrix's insertion sort, src/tonegen.cpp:1183-1201) */
typedef struct tbf_contrib {
	uint16_t wheel, bus;
	float    level;
} tbf_contrib;

/* one element of a play-matrix list (struct _list_element, src/tonegen.cpp:444-450):
 * terminal | wheel, bus, level -- the inputs of the device builder k_tpl_matrix */
typedef struct tbf_le {
	int16_t sa, sb;
	float   fc;
} tbf_le;

#define TBF_BL_ROW 28 /* floats per wheel row of tbf_tgc_state.busLevel */

/* per instance device control state (the runtime fields of struct b_tonegen that the
 * per-wheel control touches); aclPos1 = aclPos + 1 so that zeroed memory is the initial
 * state (no wheel in the list) */
typedef struct alignas (16) tbf_tgc_state {
	float    busLevel[TBF_NW + 1][TBF_BL_ROW]; /* 27 buses, rows padded to 16 B (k_tgctl's 16-B row loads) */
	float    sums[TBF_NW + 1][6]; /* sumUpper, sumLower, sumPedal, sumPercn, sumSwell, sumScanr */
	int32_t  refCount[TBF_NW + 1];
	uint16_t list[TBF_NW + 1];    /* activeOscList */
	int16_t  aclPos1[TBF_NW + 1];
	uint8_t  rflags[TBF_NW + 1];
	uint8_t  pad0[3];
	uint32_t listEnd;             /* activeOscLEnd */
	float    gain[27];            /* drawBarGain as of the last record that carried it */
	uint32_t pad1[4];
} tbf_tgc_state;

/* per instance, per launch segment: control state that is constant over the
 * segment's blocks (events land on segment boundaries) */
typedef struct tbf_seg_ctl {
	uint32_t prog_off, prog_len;
	uint32_t routing;        /* oldRouting after this block's update */
	float    outputGain;     /* swellPedalGain * percDrawbarGain */
	float    swellPedalGain;
	float    percEnvGainDecay;
	float    percEnvGainReset;
	float    keyCompTarget;  /* keyCompTable[keyDownCount] */
	uint32_t resetPercAtEnd; /* upperKeyCount == 0 */
	uint32_t vibTable;       /* 0..2 -> offset1/2/3Table */
	uint32_t vibMixed;       /* chorus */
	uint32_t odClean;
	int32_t  odIter;         /* sin iterations of the density loop */
	uint32_t odDensityPos;   /* density > 0 */
	uint32_t whBypass;
	int32_t  whRevOption;    /* >= 0: useRevOption(n) before the first block */
	uint32_t whSet;          /* > 0: the whirl takes whSets[whSet - 1] before this block */
	uint32_t pad0;
	double   odOut, odOutput, odWet, odDry, odIir;
	double   rvWet;
} tbf_seg_ctl;

/* the whirl parameters the MIDI control functions set (src/whirl.cpp:699-889: the horn
 * filters' coefficients, brake positions and the speed-ramp factors derived from the
 * acceleration / deceleration times).  k_whirl keeps the current set in tbf_wh_state and
 * replaces it before a block whose control entry carries one (tbf_seg_ctl.whSet). */
typedef struct tbf_wh_params {
	float    hafw[5], hbfw[5]; /* horn filters A, B: a1, a2, b0, b1, b2 */
	double   lAcc[4];          /* exp() speed-ramp factors: horn acc, horn dec, drum acc, drum dec */
	double   hnBrakePos, drBrakePos;
} tbf_wh_params;

/* per instance, constant over its lifetime */
typedef struct tbf_inst_const {
	uint32_t tpl;
	uint32_t vibRingPad;
	/* reverb (src/reverb.cpp:283-336 per-block constants; A..F never change) */
	double   bq[3][5]; /* biquadA/B/C [2..6] */
	double   vibDelta[8];
	double   vibDepth, blend, crossmod, oneMinusAbsCm, regen;
	int32_t  delay[13];
	uint32_t ringOff[26]; /* [c*13 + line] offset (doubles) inside the instance slab */
	uint32_t slabLen;
	uint32_t vibClosedForm; /* 1: phase increments have no rounding ties (host-checked) */
	/* whirl (src/whirl.cpp init) */
	float    drf[5];  /* drum shelf: a1, a2, b0, b1, b2 (the horn filters: tbf_wh_params) */
	float    hornSpacing[6], drumSpacing[6];
	int32_t  hornPhase[6];
	float    leakage, hornLevel;
	float    mic[8]; /* hll hlr dll dlr hrl hrr drl drr */
	double   fwAng, bwAng;
	double   deadzone;
	double   revHorn[9], revDrum[9];
	float    hnHardstop, drHardstop, minspeed, hnLimit, drLimit;
	float    pad0;
	double   sr;
} tbf_inst_const;

/* per instance device-resident DSP state, one sub-struct per render kernel (each
 * kernel stages only its own part in LDS); sizes are multiples of 8 bytes */
typedef struct tbf_tg_state { /* tonegen interpreter + vibrato: k_tonegen */
	uint32_t pos[TBF_NW + 1];
	float    pz;
	uint32_t stator, outPos;
	float    vring[TBF_VRING];
} tbf_tg_state;

typedef struct tbf_mo_state { /* mixdown gain chases + preamp: k_mixpre */
	float    keyCompLevel, percEnvGain; /* tone generator (a retune resets them) ... */
	double   iirA, iirB;                /* ... preamp (goes on through a retune) */
	uint32_t fpFlip, odFpd;
} tbf_mo_state;

typedef struct tbf_rv_chan { /* one channel of the feedback network: k_rv_core wave */
	int32_t  count[12]; /* delay-line counters A..L (lines 0-11) */
	uint32_t pad[4];
	double   fb[8];     /* feedback of the channel's last sample */
	double   vib[8];    /* vibrato phases */
	double   phD[8];    /* cached closed-form phase step of each line (0: none; valid for the
	                       instance's fixed vibDelta, zero it if that ever changes) ... */
	double   phLo[8];   /* ... and the |phase| range of the binade it is valid in */
	double   phHi[8];
} tbf_rv_chan;

/* the predelay (src/reverb.cpp:350-358) as a history of raw inputs: the ring slot read at
 * sample m holds the guarded input of sample m - delayM, so k_rv_pre reads the chunk's
 * input (or this history, for the first delayM samples of a chunk) delayM samples back
 * and guards it with the dither state of that sample.  TBF_PD_HIST floats per instance,
 * indexed by absolute sample position mod TBF_PD_HIST, in the slab's line-12 region. */
#define TBF_PD_HIST 1024
/* blocks of a render chunk: a chunk with control deltas has at most 64 (TBF_CHUNK, the
 * kernels keep a launch's per-block controls one per lane); a chunk without (every block
 * plays each instance's current control) up to TBF_STEADY_MAX, so the per-launch state
 * traffic (above all the reverb network's LDS rings) spreads over more samples */
#ifndef TBF_STEADY_MAX
#define TBF_STEADY_MAX 2048
#endif
/* the default: 512 blocks keep the stage buffers at 15 GB for 4096 instances (56 B per
 * stereo sample, tbf_engine.cpp stageBuffers) at the speed of 2048-block chunks (128.6 vs
 * 128.3 ms per 2048-block step, profiles/r05/s20_groups) */
#ifndef TBF_STEADY_DEFAULT
#define TBF_STEADY_DEFAULT 512
#endif
/* each reverb line of the slab starts on a 128-B boundary (16 doubles): a wave's 64
 * consecutive doubles then cover exactly four whole cache lines */
#define TBF_RING_ALIGN 16

typedef struct tbf_rv_state { /* reverb: k_rv_pre / k_rv_core / k_rv_post */
	int32_t     pdAge;        /* samples rendered, saturating at delayM (the predelay reads 0 before) */
	uint32_t    fpdL, fpdR;   /* dither streams as advanced by k_rv_pre: the state delayM samples back ... */
	uint32_t    fpdL2, fpdR2; /* ... and the stream itself, advanced by k_rv_post */
	uint32_t    pdPos;        /* history position of the next input (mod TBF_PD_HIST) */
	uint32_t    pad0[2];
	double      bq[3][4]; /* [A/B/C][L7, L8, R9, R10] */
	tbf_rv_chan ch[2];
} tbf_rv_state;

typedef struct tbf_wh_state { /* whirl: k_whirl */
	double   hornAngle, drumAngle, hornIncr, drumIncr, hornTarget, drumTarget;
	int32_t  hornAcDc, drumAcDc;
	uint32_t outpos;
	float    z[4];
	float    fz[4][2]; /* hafw, hbfw, drfL, drfR: z0, z1 */
	float    adx[3][8];
	int32_t  adi[3];
	int32_t  pad1[2];
	tbf_wh_params prm; /* the current runtime parameters */
} tbf_wh_state;

typedef struct tbf_inst_state {
	tbf_tg_state tg;
	tbf_mo_state mo;
	tbf_rv_state rv;
	tbf_wh_state wh;
} tbf_inst_state;

/* per template (tuning x sample rate): offsets into the shared wave bank */
typedef struct tbf_tpl_desc {
	uint32_t off[TBF_NW + 1];
	uint32_t len[TBF_NW + 1];
	float    attackEnv[8][TBF_BLK];  /* rows 0..7 used (i & 7) */
	float    releaseEnv[8][TBF_BLK];
} tbf_tpl_desc;

/* kernel launch parameters */
typedef struct tbf_launch {
	const float*          bank;
	const tbf_tpl_desc*   tpls;
	const tbf_inst_const* cst;
	tbf_inst_state*       st;
	float*                wring; /* [inst][4][wring_len] */
	float*                mid0;  /* [inst][midStride][2] k_tonegen -> k_mixpre: {bus sum, percussion difference} */
	float*                mid1;  /* [inst][midStride] preamp output of the chunk */
	float*                mid2;  /* [inst][midStride] reverb output of the chunk */
	double*               rvA;   /* [inst][2][midStride] k_rv_pre -> k_rv_core: sin(biquadA * wet) */
	double*               rvB;   /* [inst][2][midStride] k_rv_core -> k_rv_post: tap mix */
	uint64_t              midStride;
	double*               rslab; /* [inst][slabLen] */
	const tbf_seg_ctl*    ctl;    /* control pool: [0, nInst) current per instance, then this chunk's deltas */
	const uint32_t*       ctlIdx; /* [nBlocks][nInst] pool index per block, or NULL: entry inst */
	const tbf_prog_entry* prog;
	const uint32_t*       vibTab; /* [3][2048] */
	const uint32_t*       xsJump; /* [32][TBF_XS_JUMP]: xorshift32^k (1 << j), k = 0..128; then [8][16][TBF_XS_JUMP] nibble-sliced */
	const float*          whTab;  /* hnFwd, hnBwd, drFwd, drBwd [4][TBF_WH_TSTRIDE]: 16384 + [0] again + pad */
	const float*          whBw;   /* bfw, bbw [2][16384][5] */
	const tbf_wh_params*  whSets; /* the chunk's whirl parameter sets (tbf_seg_ctl.whSet) */
	float*                outL;
	float*                outR;
	uint64_t              outStride; /* floats between instances */
	uint64_t              outOffset; /* first sample index of this segment */
	uint32_t              nInst;
	uint32_t              nBlocks;
	uint32_t              wringLen;
	uint32_t              statorInc;
	uint32_t              chain;     /* TBF_CHAIN_*: 0 full, 1 tonegen, 2 preamp tap, 3 reverb tap */
	uint32_t              instBase;
	uint32_t              slabLen;
	uint32_t              dbg;       /* TBF_DEBUG_* bits of tbf_engine_config.debug_flags */
	uint32_t              whSplit;   /* k_whirl_split (two waves per instance) instead of k_whirl */
	uint32_t*             errFlags;  /* TBF_PATH_* bits: which rare paths a launch took */
	/* device-side control (k_tgctl) */
	tbf_tgc_state*        tgc;       /* [inst] */
	const tbf_tgc_rec*    rec;       /* [pool index - nInst]: inputs of the chunk's deltas */
	const uint16_t*       msgs;
	const float*          gains;  /* drawbar gain sets of the records with flags & 4 */
	const uint32_t*       ctlInst;   /* instances with a stepped delta in this chunk */
	uint32_t              nCtlInst;
	uint32_t              rvLds;     /* 1: the reverb core with its rings resident in LDS (k_rv_core_lds) */
	uint32_t              rvGrid;    /* k_rv_core_lds workgroups (persistent; 0: one per pair) */
	uint32_t              tgSplit;   /* k_tonegen block ranges per instance (chunks without deltas; <= nBlocks) */
	uint8_t*              mixFixed;  /* tonegen only: [inst] 1 when k_tonegen wrote the chunk's output (the
	                                  * mixdown's gain chases at a fixed point), so k_mixpre skips it */
	uint32_t*             rvWork;    /* k_rv_core_lds work counter */
	const uint32_t*       coff;      /* [tpl][385] keyContrib offsets into contrib */
	const tbf_contrib*    contrib;
	uint32_t              ctlNw;     /* k_tgctl's staged wheels: the largest wheel a play matrix names, + 1 */
	const tbf_seg_ctl*    fulls;     /* the chunk's full control entries (tbf_tgc_rec.full) */
	const tbf_front_state* front;    /* k_front: [inst] key state at the chunk start ... */
	const uint32_t*       fevOff;    /* ... [inst + 1] offsets into fev ... */
	const uint32_t*       fev;       /* ... an instance's events in order (TBF_FEV_*) ... */
	const float*          fevVal;    /* ... and the values of its TBF_FEV_EFFECT events */
	const float*          keyComp;   /* [tpl][128] keyCompTable */
	uint32_t              progBase;  /* program slot of delta d (pool index nInst + d): progBase + d * TBF_PROG_SLOT */
} tbf_launch;

#endif
