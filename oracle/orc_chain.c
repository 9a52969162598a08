/*
 * oracle/orc_chain.c -- TEST INFRASTRUCTURE ONLY (see orc.h).
 * Instance construction, the CLAP parameter surface and the synthSound quartet.
 */
#include "orc_internal.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* b_synth/lv2.cpp:336-353 allocSynth + 164-193 initSynth, with the tonegen template
 * shared between instances (batch protocol, SURVEY.md s7 "hard parts"). */
orc_inst* orc_inst_new (const orc_template* tpl, unsigned int seed) { return orc_inst_new_cfg (tpl, seed, NULL); }

orc_inst* orc_inst_new_cfg (const orc_template* tpl, unsigned int seed, const orc_cfg* cfg)
{
	static const unsigned int defaultPreset[9] = {8, 8, 6, 0, 0, 0, 0, 0, 0};
	orc_inst*                 p                = (orc_inst*)calloc (1, sizeof (orc_inst));
	orc_rand                  rnd;
	orc_cfg                   dflt;
	int                       i;
	if (!cfg) {
		orc_cfg_default (&dflt);
		cfg = &dflt;
	}
	orc_srand (&rnd, seed);
	p->rev = orc_reverb_alloc (&rnd, tpl->sr);   /* allocReverb: 18+ rand() */
	p->rev->G = cfg->reverbMix;                  /* reverbConfig: setReverbMix */
	p->wh  = orc_whirl_alloc (tpl->sr, cfg);     /* allocWhirl + whirlConfig + initWhirl (no rand) */
	orc_preamp_init (&p->pre, &rnd, tpl->sr);    /* allocPreamp: 1+ rand(), initPreamp */
	orc_tg_init (&p->tg, tpl, cfg);              /* allocTonegen + oscConfig/scannerConfig + initToneGenerator + init_vibrato */
	for (i = 0; i < 9; i++)                      /* setDrawBars (inst, 0, defaultPreset) */
		orc_tg_set_drawbar (&p->tg, i, defaultPreset[i]);
	orc_param_defaults (p->params);
	return p;
}

/* the CLAP parameters' default values (clap_plugin_params get_info, src/clap.cpp:383-545;
 * the plugin's init copies them into its parameter array, 1062-1067) */
void orc_param_defaults (double* params)
{
	static const float drawbar[9] = {7.0f, 8.0f, 8.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
	static const float top[9] = {1, 3, 1, 2, 3, 4, 5, 6, 8}, bottom[9] = {2, 2, 1, 1, 1, 1, 1, 1, 1};
	int                i;
	for (i = 0; i < 64; i++)
		params[i] = 0.0;
	for (i = 0; i < 9; i++) {
		params[ORC_P_DRAWBAR_MIN + i] = drawbar[i];
		params[20 + i]            = top[i];    /* P_RATIO_TOP_MIN */
		params[29 + i]            = bottom[i]; /* P_RATIO_BOTTOM_MIN */
	}
	params[ORC_P_DRUM]   = 1.0f;
	params[ORC_P_HORN]   = 1.0f;
	params[ORC_P_REVERB] = 0.1f;
}

/* reinitToneGen (src/clap.cpp:129-157), the CLAP plugin's response to an MTS-ESP tuning
 * or drawbar-ratio change: a fresh tone generator on the new template (allocTonegen +
 * initToneGenerator + init_vibrato), the drawbars, vibrato switch and vibrato type
 * restored from the parameter values, the routing word kept.  Preamp, reverb and whirl
 * go on. */
void orc_inst_retune (orc_inst* p, const orc_template* tpl, const orc_cfg* cfg)
{
	orc_cfg            dflt;
	const unsigned int newRouting = p->tg.newRouting;
	int                i;
	if (!cfg) {
		orc_cfg_default (&dflt);
		cfg = &dflt;
	}
	orc_tg_init (&p->tg, tpl, cfg);
	for (i = 0; i < 9; i++) /* setToneGenParam (108-121): float parameter values */
		orc_tg_set_drawbar (&p->tg, i, (unsigned int)rintf ((float)p->params[ORC_P_DRAWBAR_MIN + i]));
	orc_tg_set_vibrato_upper (&p->tg, (int)rintf ((float)p->params[ORC_P_VIBRATO]));
	orc_tg_set_vibrato_from_int (&p->tg, (int)floorf ((float)p->params[ORC_P_VIBRATO_TYPE]));
	p->tg.newRouting = newRouting;
}

void orc_inst_free (orc_inst* p)
{
	if (!p)
		return;
	orc_reverb_free (p->rev);
	free (p->wh);
	free (p);
}

void orc_note (orc_inst* p, int key, int on)
{
	if (on)
		orc_tg_key_on (&p->tg, key);
	else
		orc_tg_key_off (&p->tg, key);
}

void orc_set_chain (orc_inst* p, int mode) { p->chain = mode; }

/* callMIDIControlFunction (src/midi.cpp) for the whirl's registered functions */
int orc_control (orc_inst* p, const char* name, int value)
{
	const unsigned char uc = (unsigned char)(value < 0 ? 0 : (value > 127 ? 127 : value));
	return orc_whirl_control (p->wh, name, uc);
}

int orc_whirl_fields (const orc_inst* p, double* out)
{
	const struct orc_whirl* w = p->wh;
	int                     k = 0;
	out[k++]                  = w->haT;
	out[k++]                  = w->haF;
	out[k++]                  = w->haQ;
	out[k++]                  = w->haG;
	for (int i = 1; i <= 5; i++)
		out[k++] = w->hafw[i];
	out[k++] = w->hbT;
	out[k++] = w->hbF;
	out[k++] = w->hbQ;
	out[k++] = w->hbG;
	for (int i = 1; i <= 5; i++)
		out[k++] = w->hbfw[i];
	out[k++] = w->hnBrakePos;
	out[k++] = w->drBrakePos;
	out[k++] = w->hornAcc;
	out[k++] = w->hornDec;
	out[k++] = w->drumAcc;
	out[k++] = w->drumDec;
	return k;
}

/* src/clap.cpp:108-121 setToneGenParam and 162-207 setParam */
void orc_set_param (orc_inst* p, int index, double v)
{
	float value = (float)v;
	if (index >= 0 && index < 64)
		p->params[index] = value;
	if (ORC_P_DRAWBAR_MIN <= index && index <= ORC_P_DRAWBAR_MAX) {
		orc_tg_set_drawbar (&p->tg, index, (unsigned int)rint (value));
	} else if (index == ORC_P_VIBRATO) {
		orc_tg_set_vibrato_upper (&p->tg, (int)rint (value));
	} else if (index == ORC_P_VIBRATO_TYPE) {
		orc_tg_set_vibrato_from_int (&p->tg, (int)floor (value));
	} else if (index == ORC_P_DRUM || index == ORC_P_HORN) {
		orc_whirl_use_rev_option (p->wh, (int)(floor (p->params[ORC_P_DRUM]) + 3 * floor (p->params[ORC_P_HORN])), 2);
	} else if (index == ORC_P_OVERDRIVE) {
		p->pre.isClean = (int)rint (1.0f - value);
	} else if (index == ORC_P_CHARACTER) {
		orc_preamp_set_character (&p->pre, value);
	} else if (index == ORC_P_REVERB) {
		p->rev->G = value;
	} else if (index == ORC_P_PERCUSSION) {
		orc_tg_set_perc_enabled (&p->tg, (int)rint (value));
	} else if (index == ORC_P_PERCUSSION_VOLUME) {
		orc_tg_set_perc_volume (&p->tg, (int)(1 - rint (value)));
	} else if (index == ORC_P_PERCUSSION_DECAY) {
		orc_tg_set_perc_fast (&p->tg, (int)rint (value));
	} else if (index == ORC_P_PERCUSSION_HARMONIC) {
		orc_tg_set_perc_first (&p->tg, (int)rint (value));
	} else if (index >= ORC_P_BUS_DRAWBAR_BASE && index < ORC_P_BUS_DRAWBAR_BASE + 27) {
		orc_tg_set_drawbar (&p->tg, index - ORC_P_BUS_DRAWBAR_BASE, (unsigned int)rint (value));
	} else if (index == ORC_P_VIBRATO_LOWER) {
		orc_tg_set_vibrato_lower (&p->tg, (int)rint (value));
	} else if (index == ORC_P_SWELL) {
		/* src/tonegen.cpp:2885-2890 setSwellPedal1FromMIDI with u = value * 127 */
		unsigned char u        = (unsigned char)rint (value * 127.0);
		p->tg.swellPedalGain   = (float)((p->tg.outputLevelTrim * ((double)u)) / 127.0);
	} else if (index == ORC_P_WHIRL_BYPASS) {
		p->wh->bypass = (int)rint (value);
	}
}

/* synthSound block quartet: b_synth/lv2.cpp:220-228, src/clap.cpp:251-259 */
void orc_render (orc_inst* p, int nblocks, float* L, float* R, float* sA, float* sB, float* sC)
{
	int b;
	for (b = 0; b < nblocks; b++) {
		size_t o = (size_t)b * ORC_BLK;
		orc_tg_generate (&p->tg, p->bufA);
		if (p->chain == 1) {
			memcpy (p->bufB, p->bufA, sizeof (p->bufA));
			memcpy (p->bufC, p->bufA, sizeof (p->bufA));
			memcpy (p->bufL, p->bufA, sizeof (p->bufA));
			memcpy (p->bufR, p->bufA, sizeof (p->bufA));
		} else {
			orc_preamp_run (&p->pre, p->bufA, p->bufB, ORC_BLK);
			orc_reverb_run (p->rev, p->bufB, p->bufC, ORC_BLK);
			orc_whirl_run3 (p->wh, p->bufC, p->bufL, p->bufR, p->bufDL, p->bufDR, ORC_BLK);
		}
		if (sA)
			memcpy (sA + o, p->bufA, sizeof (p->bufA));
		if (sB)
			memcpy (sB + o, p->bufB, sizeof (p->bufB));
		if (sC)
			memcpy (sC + o, p->bufC, sizeof (p->bufC));
		if (L)
			memcpy (L + o, p->bufL, sizeof (p->bufL));
		if (R)
			memcpy (R + o, p->bufR, sizeof (p->bufR));
	}
}

/* test hook: the reverb vibrato phase vib[c][l] (tbf_debug_reverb_phase's counterpart) */
void orc_debug_rv_phase (orc_inst* p, int c, int l, double value)
{
	p->rev->vib[c][l] = value;
}

int orc_debug_program (const orc_inst* p, float* out, int cap)
{
	int i;
	for (i = 0; i < p->tg.corePgmLen && i < cap; i++) {
		const orc_coreins* c = &p->tg.corePgm[i];
		float*             o = out + 9 * i;
		o[0] = (float)c->wheel; o[1] = (float)c->opr; o[2] = (float)c->envRow;
		o[3] = c->sgain; o[4] = c->pgain; o[5] = c->vgain; o[6] = c->nsgain; o[7] = c->npgain; o[8] = c->nvgain;
	}
	return p->tg.corePgmLen;
}
