/*
 * oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives the reference's OWN translation units, compiled unmodified from
 * /root/reference/src/{tonegen,vibrato,overdrive,reverb,whirl,eqcomp}.cpp by
 * oracle/Makefile (target `ref`, outputs only into oracle/_ref/), to produce
 * reference outputs for pinning the oracle restatement.
 *
 * What is the reference here and what is not:
 *   - runtime: oscGenerateFragment, oscKeyOn/Off, the tonegen setters, init_vibrato,
 *     vibratoProc, allocPreamp/initPreamp/preamp, b_reverb ctor/reverb,
 *     allocWhirl/initWhirl/whirlProc3/useRevOption -- all reference code.
 *   - tonegen tables: initToneGenerator needs getFrequencies from src/tuning.cpp,
 *     which needs the un-vendored MTS-ESP client (libs/MTS-ESP is empty), so that one
 *     function is unbuildable here.  No stand-in is written for it: it is dropped by
 *     --gc-sections, and the b_tonegen fields it would fill (wave bank, play matrix,
 *     envelopes, key-compression table) are filled from the oracle's template, whose
 *     structure is itself pinned by the reference's regression fixtures.  The
 *     runtime-init steps of initToneGenerator (tonegen.cpp:2914-3021) are replayed
 *     here with the reference's exported setters.
 *
 * Construction protocol = LV2 allocSynth/initSynth order (b_synth/lv2.cpp:336-353,
 * 164-193) with glibc srand(seed) in place of srand(time(NULL)).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "eqcomp.h"
#include "overdrive.h"
#include "reverb.h"
#include "tonegen.h"
#include "whirl.h"

#include "orc.h"

#define API extern "C" __attribute__ ((visibility ("default")))

/* defined with external linkage in src/tonegen.cpp:1853-1866 (no header declaration) */
void setNormalPercussionGain (struct b_tonegen* t, double g);
void setSoftPercussionGain (struct b_tonegen* t, double g);
void setPercussionGainScaling (struct b_tonegen* t, double s);

struct ref_inst {
	b_tonegen*       t;
	struct b_preamp* p;
	b_reverb*        r;
	b_whirl*         w;
	int              chain;
	double           params[64];
	float            bufA[128], bufB[128], bufC[128], bufL[128], bufR[128], bufD0[128], bufD1[128];
};

static ListElement* mk_list (const orc_list* l)
{
	ListElement* head = NULL;
	ListElement* tail = NULL;
	for (int i = 0; i < l->n; i++) {
		ListElement* e = (ListElement*)calloc (1, sizeof (ListElement));
		e->u.ssf.sa    = l->v[i].sa;
		e->u.ssf.sb    = l->v[i].sb;
		e->u.ssf.fc    = l->v[i].fc;
		if (tail)
			tail->next = e;
		else
			head = e;
		tail = e;
	}
	return head;
}

static b_tonegen* ref_tonegen (const orc_template* tpl, const orc_cfg* c)
{
	b_tonegen* t = allocTonegen ();
	int        i;
	/* oscConfig's runtime keys (src/tonegen.cpp:2206-2237): field assignments and the
	 * exported setters, between allocTonegen and initToneGenerator as at startup */
	t->percFastDecaySeconds = c->percFastDecaySeconds;
	t->percSlowDecaySeconds = c->percSlowDecaySeconds;
	setNormalPercussionGain (t, c->percEnvGainResetNorm);
	setSoftPercussionGain (t, c->percEnvGainResetSoft);
	setPercussionGainScaling (t, c->percEnvScaling);
	t->percSendBusA   = c->percSendBusA;
	t->percSendBusB   = c->percSendBusB;
	t->percTriggerBus = c->percTriggerBus;
	/* initToneGenerator runtime part, tonegen.cpp:2909-2955 */
	t->SampleRateD  = tpl->sr;
	t->midi_cfg_ptr = NULL;
	t->percIsSoft = t->percIsFast = 0;
	t->percEnvGain                = 0;
	for (i = 0; i < NOF_BUSES; ++i) {
		t->drawBarGain[i] = 0;
		for (int j = 0; j < 9; ++j)
			t->drawBarLevel[i][j] = 0;
	}
	for (i = 0; i < MAX_KEYS; ++i)
		t->activeKeys[i] = 0;
	for (i = 0; i < MAX_KEYS / 32; ++i)
		t->_activeKeys[i] = 0;
	for (i = 0; i < CR_PGMMAX; ++i)
		memset ((void*)&t->corePgm[i], 0, sizeof (CoreIns));
	for (i = 0; i <= NOF_WHEELS; ++i)
		memset ((void*)&t->oscillators[i], 0, sizeof (struct _oscillator));
	t->envAtkClkMinLength = tpl->envAtkClkMinLength;
	t->envAtkClkMaxLength = tpl->envAtkClkMaxLength;
	memcpy (t->frequency, tpl->frequency, sizeof (t->frequency));
	memcpy (t->targetRatio, tpl->targetRatio, sizeof (t->targetRatio));
	/* tables from the oracle template (applyDefaultConfiguration/compilePlayMatrix,
	 * initOscillators, initKeyCompTable, initEnvelopes) */
	for (i = 0; i < MAX_KEYS; i++)
		t->keyContrib[i] = mk_list (&tpl->keyContrib[i]);
	for (i = 1; i <= NOF_WHEELS; i++) {
		struct _oscillator* osp = &t->oscillators[i];
		osp->wave               = (float*)malloc (sizeof (float) * tpl->wlen[i]);
		memcpy (osp->wave, tpl->wave[i], sizeof (float) * tpl->wlen[i]);
		osp->lengthSamples = tpl->wlen[i];
		osp->frequency     = tpl->wfreq[i];
		osp->attenuation   = tpl->watt[i];
		osp->aclPos        = -1;
		osp->rflags        = 0;
		osp->pos           = 0;
	}
	memcpy (t->keyCompTable, tpl->keyCompTable, sizeof (t->keyCompTable));
	memcpy (t->attackEnv, tpl->attackEnv, sizeof (t->attackEnv));
	memcpy (t->releaseEnv, tpl->releaseEnv, sizeof (t->releaseEnv));
	/* tonegen.cpp:2994-3021 */
	for (i = 0; i < NOF_BUSES; i++)
		for (int s = 0; s < 9; s++) {
			float u               = (float)s;
			t->drawBarLevel[i][s] = u / 8.0;
		}
	static const int midiBus[8] = {0, 1, 2, 9, 10, 11, 18, 20};
	static const int midiVal[8] = {8, 8, 6, 8, 3, 8, 8, 6};
	for (i = 0; i < 8; i++) /* setMIDIDrawBar (static) == setDrawBar(rint((127-v)*8/127)) */
		setDrawBar (t, midiBus[i], (unsigned int)rint ((127 - midiVal[i]) * 8.0 / 127.0));
	setPercussionFirst (t, 0);
	setPercussionVolume (t, 0);
	setPercussionFast (t, 1);
	setPercussionEnabled (t, 0);
	return t;
}

/* whirlConfig's assignments (src/whirl.cpp:992-1160) on the reference's own struct, between
 * allocWhirl and initWhirl as at startup.  The mic-width setters fsetHornMicWidth /
 * fsetDrumMicWidth (912-949) sit in the LV2-only part the CLAP define set compiles out;
 * their four assignments each are replayed here. */
static void ref_whirl_cfg (b_whirl* w, const orc_cfg* c)
{
	w->hornRPMslow   = c->hornRPMslow;
	w->hornRPMfast   = c->hornRPMfast;
	w->drumRPMslow   = c->drumRPMslow;
	w->drumRPMfast   = c->drumRPMfast;
	w->hornAcc       = c->hornAcc;
	w->hornDec       = c->hornDec;
	w->drumAcc       = c->drumAcc;
	w->drumDec       = c->drumDec;
	w->hornRadiusCm  = c->hornRadiusCm;
	w->drumRadiusCm  = c->drumRadiusCm;
	w->hornLevel     = c->hornLevel;
	w->leakLevel     = c->leakLevel;
	w->micDistCm     = c->micDistCm;
	w->hornXOffsetCm = c->hornXOffsetCm;
	w->hornZOffsetCm = c->hornZOffsetCm;
	w->lpT           = c->lpT;
	w->lpQ           = c->lpQ;
	w->lpF           = c->lpF;
	w->lpG           = c->lpG;
	w->haT           = c->haT;
	w->haF           = c->haF;
	w->haQ           = c->haQ;
	w->haG           = c->haG;
	w->hbT           = c->hbT;
	w->hbF           = c->hbF;
	w->hbQ           = c->hbQ;
	w->hbG           = c->hbG;
	w->revSelect     = c->revSelect;
	w->bypass        = c->bypass;
	w->micAngle      = c->micAngle;
	w->hnBrakePos    = c->hnBrakePos;
	w->drBrakePos    = c->drBrakePos;
	if (c->drumMicWidth != w->drumMicWidth) {
		const float dw = c->drumMicWidth;
		w->drumMicWidth = dw;
		const float dwP = dw > 0.f ? (dw > 1.f ? 1.f : dw) : 0.f;
		const float dwN = dw < 0.f ? (dw < -1.f ? 1.f : -dw) : 0.f;
		w->drumMic_dll  = sqrtf (1.f - dwP);
		w->drumMic_dlr  = sqrtf (0.f + dwP);
		w->drumMic_drl  = sqrtf (0.f + dwN);
		w->drumMic_drr  = sqrtf (1.f - dwN);
	}
	if (c->hornMicWidth != w->hornMicWidth) {
		const float hw = c->hornMicWidth;
		w->hornMicWidth = hw;
		const float hwP = hw > 0.f ? (hw > 1.f ? 1.f : hw) : 0.f;
		const float hwN = hw < 0.f ? (hw < -1.f ? 1.f : -hw) : 0.f;
		w->hornMic_hll  = sqrtf (1.f - hwP);
		w->hornMic_hlr  = sqrtf (0.f + hwP);
		w->hornMic_hrl  = sqrtf (0.f + hwN);
		w->hornMic_hrr  = sqrtf (1.f - hwN);
	}
}

API ref_inst* ref_inst_new_cfg (const orc_template* tpl, unsigned int seed, const orc_cfg* cfg)
{
	orc_cfg dflt;
	if (!cfg) {
		orc_cfg_default (&dflt);
		cfg = &dflt;
	}
	ref_inst* p = (ref_inst*)calloc (1, sizeof (ref_inst));
	srand (seed);
	p->r = allocReverb ();
	setReverbMix (p->r, cfg->reverbMix); /* reverbConfig (src/reverb.cpp:242-256) */
	p->w = allocWhirl ();
	ref_whirl_cfg (p->w, cfg);
	p->t = ref_tonegen (tpl, cfg);
	p->p = (struct b_preamp*)allocPreamp ();
	/* scannerConfig (src/vibrato.cpp:334-357): the fields init_vibrato reads */
	p->t->inst_vibrato.vibFqHertz = cfg->vibFqHertz;
	p->t->inst_vibrato.vib1OffAmp = cfg->vib1OffAmp;
	p->t->inst_vibrato.vib2OffAmp = cfg->vib2OffAmp;
	p->t->inst_vibrato.vib3OffAmp = cfg->vib3OffAmp;
	init_vibrato (&p->t->inst_vibrato, tpl->sr);
	initPreamp (p->p, NULL, tpl->sr);
	initReverb (p->r, NULL, tpl->sr);
	initWhirl (p->w, NULL, tpl->sr);
	static const unsigned int preset[9] = {8, 8, 6, 0, 0, 0, 0, 0, 0};
	for (int i = 0; i < 9; i++)
		setDrawBar (p->t, i, preset[i]);
	orc_param_defaults (p->params); /* the CLAP parameters' defaults (src/clap.cpp:383-545, 1062-1067) */
	return p;
}

/* the keyContrib lists ref_tonegen built, then the reference's freeToneGenerator */
static void ref_tonegen_free (b_tonegen* t)
{
	for (int i = 0; i < MAX_KEYS; i++)
		for (ListElement* e = t->keyContrib[i]; e;) {
			ListElement* n = e->next;
			free (e);
			e = n;
		}
	freeToneGenerator (t);
}

/* reinitToneGen (src/clap.cpp:129-157) with the reference's own calls: the tone
 * generator rebuilt on a new template, init_vibrato, setToneGenParam for the drawbars,
 * vibrato switch and vibrato type from the parameter values, newRouting kept */
API void ref_inst_retune (ref_inst* p, const orc_template* tpl, const orc_cfg* cfg)
{
	orc_cfg dflt;
	if (!cfg) {
		orc_cfg_default (&dflt);
		cfg = &dflt;
	}
	const unsigned int newRouting = p->t->newRouting;
	ref_tonegen_free (p->t);
	p->t                          = ref_tonegen (tpl, cfg);
	p->t->inst_vibrato.vibFqHertz = cfg->vibFqHertz;
	p->t->inst_vibrato.vib1OffAmp = cfg->vib1OffAmp;
	p->t->inst_vibrato.vib2OffAmp = cfg->vib2OffAmp;
	p->t->inst_vibrato.vib3OffAmp = cfg->vib3OffAmp;
	init_vibrato (&p->t->inst_vibrato, tpl->sr);
	for (int i = 0; i < 9; i++) {
		const float value = (float)p->params[i];
		setDrawBar (p->t, i, rint (value));
	}
	setVibratoUpper (p->t, rint ((float)p->params[9]));
	setVibratoFromInt (p->t, floor ((float)p->params[10]));
	p->t->newRouting = newRouting;
}

API ref_inst* ref_inst_new (const orc_template* tpl, unsigned int seed) { return ref_inst_new_cfg (tpl, seed, NULL); }

API void ref_inst_free (ref_inst* p)
{
	if (!p)
		return;
	freeReverb (p->r);
	freeWhirl (p->w);
	freePreamp (p->p);
	ref_tonegen_free (p->t);
	free (p);
}

API void ref_note (ref_inst* p, int key, int on)
{
	if (on)
		oscKeyOn (p->t, key, key);
	else
		oscKeyOff (p->t, key, key);
}

API void ref_set_chain (ref_inst* p, int mode) { p->chain = mode; }

/* src/clap.cpp:108-207 setToneGenParam + setParam, plus the extension ids of orc.h */
API void ref_set_param (ref_inst* p, int index, double v)
{
	float value = (float)v;
	if (index >= 0 && index < 64)
		p->params[index] = value;
	if (0 <= index && index <= 8)
		setDrawBar (p->t, index, (unsigned int)rint (value));
	else if (index == 9)
		setVibratoUpper (p->t, (int)rint (value));
	else if (index == 10)
		setVibratoFromInt (p->t, (int)floor (value));
	else if (index == 11 || index == 12)
		useRevOption (p->w, (int)(floor (p->params[11]) + 3 * floor (p->params[12])), 2);
	else if (index == 13)
		p->p->isClean = (int)rint (1.0f - value);
	else if (index == 14)
		fsetCharacter (p->p, value);
	else if (index == 15)
		setReverbMix (p->r, value);
	else if (index == 16)
		setPercussionEnabled (p->t, (int)rint (value));
	else if (index == 17)
		setPercussionVolume (p->t, (int)(1 - rint (value)));
	else if (index == 18)
		setPercussionFast (p->t, (int)rint (value));
	else if (index == 19)
		setPercussionFirst (p->t, (int)rint (value));
	else if (index >= 100 && index < 127)
		setDrawBar (p->t, index - 100, (unsigned int)rint (value));
	else if (index == 130)
		setVibratoLower (p->t, (int)rint (value));
	else if (index == 131) {
		unsigned char u     = (unsigned char)rint (value * 127.0);
		p->t->swellPedalGain = (p->t->outputLevelTrim * ((double)u)) / 127.0;
	} else if (index == 132)
		p->w->bypass = (int)rint (value);
}

/* The whirl's MIDI control functions (src/whirl.cpp:699-889) sit in the LV2-only part the
 * CLAP define compiles out, and registering them needs midi.cpp, so the harness sets the
 * reference struct's fields with the setters' mappings and recomputes the horn filters
 * with setIIRFilter's range guard (147-172) over the reference's own eqCompute; the
 * processing that reads the fields (whirlProc2/3) is the reference's. */
static void ref_iir (iir_t W[], int T, double F, double Q, double G, double SR)
{
	double C[6];
	if (Q <= 0.1 || Q >= 6.00 || F / SR <= 0.0002 || F / SR >= 0.4998 || G <= -48.0 || G >= 48.0 || T < EQC_LPF || T > EQC_HIGH)
		return;
	eqCompute (T, F, Q, G, C, SR);
	W[a1] = C[EQC_A1];
	W[a2] = C[EQC_A2];
	W[b0] = C[EQC_B0];
	W[b1] = C[EQC_B1];
	W[b2] = C[EQC_B2];
}

API int ref_control (ref_inst* p, const char* fn, int value)
{
	b_whirl*            w  = p->w;
	const unsigned char uc = (unsigned char)(value < 0 ? 0 : (value > 127 ? 127 : value));
	const double        u  = (double)uc;
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
		ref_iir (w->hafw, (int)w->haT, w->haF, w->haQ, w->haG, w->SampleRateD);
	else if (!strncmp (fn, "whirl.horn.filter.b.", 20))
		ref_iir (w->hbfw, (int)w->hbT, w->hbF, w->hbQ, w->hbG, w->SampleRateD);
	return 0;
}

API void ref_render (ref_inst* p, int nblocks, float* L, float* R, float* sA, float* sB, float* sC)
{
	for (int b = 0; b < nblocks; b++) {
		size_t o = (size_t)b * 128;
		oscGenerateFragment (p->t, p->bufA, 128);
		if (p->chain == 1) {
			memcpy (p->bufB, p->bufA, sizeof (p->bufA));
			memcpy (p->bufC, p->bufA, sizeof (p->bufA));
			memcpy (p->bufL, p->bufA, sizeof (p->bufA));
			memcpy (p->bufR, p->bufA, sizeof (p->bufA));
		} else {
			preamp (p->p, p->bufA, p->bufB, 128);
			p->r->reverb (p->bufB, p->bufC, 128);
			whirlProc3 (p->w, p->bufC, p->bufL, p->bufR, p->bufD0, p->bufD1, 128);
		}
		if (sA) memcpy (sA + o, p->bufA, sizeof (p->bufA));
		if (sB) memcpy (sB + o, p->bufB, sizeof (p->bufB));
		if (sC) memcpy (sC + o, p->bufC, sizeof (p->bufC));
		if (L) memcpy (L + o, p->bufL, sizeof (p->bufL));
		if (R) memcpy (R + o, p->bufR, sizeof (p->bufR));
	}
}

/* ---- single-stage access ---- */
API b_whirl* ref_whirl_new (double sr)
{
	b_whirl* w = allocWhirl ();
	initWhirl (w, NULL, sr);
	return w;
}
API void ref_whirl_free (b_whirl* w) { freeWhirl (w); }
API void ref_whirl_rev_option (b_whirl* w, int n) { useRevOption (w, n, 2); }
API void ref_whirl_proc3 (b_whirl* w, const float* in, float* L, float* R, int n)
{
	static float t0[4096], t1[4096];
	while (n > 0) {
		int m = n > 4096 ? 4096 : n;
		whirlProc3 (w, in, L, R, t0, t1, (size_t)m);
		in += m;
		L += m;
		R += m;
		n -= m;
	}
}
API b_reverb* ref_reverb_new (double sr, unsigned int seed)
{
	srand (seed);
	b_reverb* r = allocReverb ();
	initReverb (r, NULL, sr);
	return r;
}
API void ref_reverb_free (b_reverb* r) { freeReverb (r); }
API void ref_reverb_set_mix (b_reverb* r, float g) { setReverbMix (r, g); }
API void ref_reverb_proc (b_reverb* r, float* in, float* out, int n) { r->reverb (in, out, n); }
API void* ref_preamp_new (double sr, unsigned int seed)
{
	srand (seed);
	void* p = allocPreamp ();
	initPreamp (p, NULL, sr);
	return p;
}
API void ref_preamp_free (void* p) { freePreamp (p); }
API void ref_preamp_set (void* p, int clean, float character)
{
	((struct b_preamp*)p)->isClean = clean;
	fsetCharacter ((struct b_preamp*)p, character);
}
API void ref_preamp_proc (void* p, float* in, float* out, int n) { preamp (p, in, out, (size_t)n); }
