/*
 * oracle/ref_tpl_pin.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Pins the tonegen template tables (wave bank with its per-sample rand() LSBs, click and
 * release envelopes, key-compression table) to the reference's OWN code.
 * initToneGenerator (src/tonegen.cpp:2905-3066) is unbuildable here because its first
 * step, getFrequencies (src/tuning.cpp:142-147), needs the un-vendored MTS-ESP client.
 * Every later step is a `static` function of src/tonegen.cpp, which the reference's own
 * doctests reach by living inside that translation unit (src/tonegen.cpp:4136-4157);
 * this harness does the same: it #includes /root/reference/src/tonegen.cpp unmodified
 * (compiled by oracle/Makefile target `pin`, output only into oracle/_ref/) and replays
 * initToneGenerator's table steps with the 300-entry frequency table passed in (the
 * oracle's restatement of getFrequencies, itself pinned by the reference's osc.txt
 * fixtures):
 *     srand (seed); initOscillators; initKeyCompTable; initEnvelopes
 * and, for the play matrix, the steps of applyDefaultConfiguration (933-1041) and
 * compilePlayMatrix (1122-1213): the reference's own applyManualDefaults,
 * applyPedalDefaults, applyDefaultCrosstalk, findTransformerNeighbours /
 * findEastWestNeighbours and compilePlayMatrix.  The one piece replayed here is the
 * terminal-mix loop of applyDefaultConfiguration (941-1023), whose compartment step
 * calls getPairedWheel from the unbuildable src/tuning.cpp: its wheel-pair table is
 * taken from the oracle (orc_paired_wheel, src/tuning.cpp:153-174; the default play
 * matrix it yields is pinned by the reference's osc_runtime.txt fixtures).
 * cfg keys reach the reference's structs the way oscConfig (2173-2555) puts them
 * there: scalar fields and the reference's own setters, list keys as ListElements from
 * newConfigListElement / appendListElement, in file order, before the init steps.
 * No stand-in is written for anything: --gc-sections drops initToneGenerator,
 * applyDefaultConfiguration and the rest of the TU that the entry points below do not
 * reach, and --no-undefined proves nothing else is missing.
 */
#include "tonegen.cpp"

#include <stdint.h>

#include "orc.h"

#define PIN_API extern "C" __attribute__ ((visibility ("default")))

/* applyDefaultConfiguration's terminal-mix loop (src/tonegen.cpp:941-1023) */
static void pin_terminal_mix (struct b_tonegen* t)
{
	ListElement* lep;
	int          i;
	for (i = 1; i <= NOF_WHEELS; i++) {
		if (t->terminalMix[i] == NULL) {
			lep                     = newConfigListElement (t);
			LE_WHEEL_NUMBER_OF (lep) = (short)i;
			LE_WHEEL_LEVEL_OF (lep)  = 1.0 - t->defaultCompartmentCrosstalk;
			appendListElement (&(t->terminalMix[i]), lep);
			if (0.0 < t->defaultCompartmentCrosstalk) {
				short pw = orc_paired_wheel ((short)i);
				if ((0 < pw) && (pw <= NOF_WHEELS)) {
					lep                     = newConfigListElement (t);
					LE_WHEEL_NUMBER_OF (lep) = pw;
					LE_WHEEL_LEVEL_OF (lep)  = t->defaultCompartmentCrosstalk;
					appendListElement (&(t->terminalMix[i]), lep);
				}
			}
		}
	}
	if (0.0 < t->defaultTransformerCrosstalk)
		for (i = 44; i <= NOF_WHEELS; i++) {
			int east = 0, west = 0;
			findTransformerNeighbours (i, &east, &west);
			const int nb[2] = {east, west};
			for (int s = 0; s < 2; s++)
				if (0 < nb[s]) {
					lep                     = newConfigListElement (t);
					LE_WHEEL_NUMBER_OF (lep) = (short)nb[s];
					LE_WHEEL_LEVEL_OF (lep)  = t->defaultTransformerCrosstalk;
					appendListElement (&(t->terminalMix[i]), lep);
				}
		}
	if (0.0 < t->defaultTerminalStripCrosstalk)
		for (i = 1; i <= NOF_WHEELS; i++) {
			int east = 0, west = 0;
			findEastWestNeighbours (terminalStrip, i, &east, &west);
			const int nb[2] = {east, west};
			for (int s = 0; s < 2; s++)
				if (0 < nb[s]) {
					lep                     = newConfigListElement (t);
					LE_WHEEL_NUMBER_OF (lep) = (short)nb[s];
					LE_WHEEL_LEVEL_OF (lep)  = t->defaultTerminalStripCrosstalk;
					appendListElement (&(t->terminalMix[i]), lep);
				}
		}
}

/* oscConfig's template keys (src/tonegen.cpp:2173-2555) on the reference's struct:
 * its setters (479-485, 1868-1921), its fields, its list elements */
static void pin_apply_cfg (struct b_tonegen* t, const orc_cfg* cfg)
{
	setWavePrecision (t, cfg->tgPrecision);
	setEnvAttackModel (t, cfg->envAttackModel);
	setEnvReleaseModel (t, cfg->envReleaseModel);
	setEnvAttackClickLevel (t, cfg->envAttackClickLevel);
	setEnvReleaseClickLevel (t, cfg->envReleaseClickLevel);
	t->envAtkClkMinLength            = cfg->envAtkClkMinLength; /* setEnvAtkClkMinLength's result */
	t->envAtkClkMaxLength            = cfg->envAtkClkMaxLength;
	t->eqMacro                       = cfg->eqMacro;
	t->eqP1y                         = cfg->eqP1y;
	t->eqR1y                         = cfg->eqR1y;
	t->eqP4y                         = cfg->eqP4y;
	t->eqR4y                         = cfg->eqR4y;
	t->defaultCompartmentCrosstalk   = cfg->compartmentXT;
	t->defaultTransformerCrosstalk   = cfg->transformerXT;
	t->defaultTerminalStripCrosstalk = cfg->stripXT;
	t->defaultWiringCrosstalk        = cfg->wiringXT;
	t->contributionFloorLevel        = cfg->contribFloor;
	t->contributionMinLevel          = cfg->contribMin;
	for (int j = 0; j < cfg->nle; j++) {
		ListElement* lep = newConfigListElement (t);
		const int    k   = cfg->le[j].idx;
		switch (cfg->le[j].kind) {
			case ORC_LE_HARMONIC:
				LE_HARMONIC_NUMBER_OF (lep) = cfg->le[j].sa;
				LE_HARMONIC_LEVEL_OF (lep)  = cfg->le[j].fc;
				appendListElement (&(t->wheelHarmonics[k]), lep);
				break;
			case ORC_LE_TERMINAL:
				LE_WHEEL_NUMBER_OF (lep) = cfg->le[j].sa;
				LE_WHEEL_LEVEL_OF (lep)  = cfg->le[j].fc;
				appendListElement (&(t->terminalMix[k]), lep);
				break;
			case ORC_LE_TAPER:
				LE_TERMINAL_OF (lep)  = cfg->le[j].sa;
				LE_BUSNUMBER_OF (lep) = cfg->le[j].sb;
				LE_TAPER_OF (lep)     = cfg->le[j].fc;
				appendListElement (&t->keyTaper[k], lep);
				break;
			case ORC_LE_XTALK:
				LE_TERMINAL_OF (lep)  = cfg->le[j].sa;
				LE_BUSNUMBER_OF (lep) = cfg->le[j].sb;
				LE_LEVEL_OF (lep)     = cfg->le[j].fc;
				appendListElement (&(t->keyCrosstalk[k]), lep);
				break;
		}
	}
}

/* Build one template's tables the reference's way.  Outputs (any may be NULL):
 *   bank[cap]          wave samples of wheels 1..256 concatenated (returns the total)
 *   lens[256]          wave lengths; wfreq[256] wheel frequencies
 *   atk[9*128], rel[9*128], kc[128]   envelopes and key-compression table
 *   ncontrib[384], cwheel/cbus/clevel[ccap]   the play matrix (keyContrib lists, keys
 *                      0..383 concatenated; ncontrib = entries per key) */
PIN_API long refpin_template_full (double sr, const double* freq300, const double* ratio9, unsigned int seed,
                                   const orc_cfg* cfg, float* bank, uint64_t cap, uint32_t* lens, double* wfreq,
                                   float* atk, float* rel, float* kc, uint32_t* ncontrib, int16_t* cwheel,
                                   int16_t* cbus, float* clevel, uint32_t ccap)
{
	struct b_tonegen* t = allocTonegen ();
	int               i;
	if (cfg) /* between alloc and init, as at startup */
		pin_apply_cfg (t, cfg);
	/* initToneGenerator, src/tonegen.cpp:2909-2955 */
	t->SampleRateD  = sr;
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
	for (i = 0; i < 128; ++i) {
		t->eqvAtt[i] = 0.0;
		t->eqvSet[i] = '\0';
	}
	if (t->envAtkClkMinLength < 0)
		t->envAtkClkMinLength = floor (t->SampleRateD * 8.0 / 22050.0);
	if (t->envAtkClkMaxLength < 0)
		t->envAtkClkMaxLength = ceil (t->SampleRateD * 40.0 / 22050.0);
	if (t->envAtkClkMinLength > BUFFER_SIZE_SAMPLES)
		t->envAtkClkMinLength = BUFFER_SIZE_SAMPLES;
	if (t->envAtkClkMaxLength > BUFFER_SIZE_SAMPLES)
		t->envAtkClkMaxLength = BUFFER_SIZE_SAMPLES;
	/* getFrequencies (t->frequency, NOF_FREQS): the table passed in */
	memcpy (t->frequency, freq300, sizeof (double) * NOF_FREQS);
	static const double defaultTargetRatio[NOF_DRAWBARS] = {0.5, 1.5, 1, 2, 3, 4, 5, 6, 8};
	for (i = 0; i < NOF_DRAWBARS; i++)
		t->targetRatio[i] = ratio9 ? ratio9[i] : defaultTargetRatio[i];
	/* applyDefaultConfiguration (933-1041) + compilePlayMatrix: no rand() draws */
	pin_terminal_mix (t);
	applyManualDefaults (t, 0, 0);
	applyManualDefaults (t, NOF_MIDI_NOTES, 9);
	applyPedalDefaults (t, 32);
	applyDefaultCrosstalk (t, 0, 0);
	applyDefaultCrosstalk (t, NOF_MIDI_NOTES, 9);
	compilePlayMatrix (t);
	if (ncontrib) {
		uint32_t o = 0;
		for (int k = 0; k < MAX_KEYS; k++) {
			uint32_t n = 0;
			for (const ListElement* rep = t->keyContrib[k]; rep; rep = rep->next, n++, o++)
				if (o < ccap) {
					cwheel[o] = LE_WHEEL_NUMBER_OF (rep);
					cbus[o]   = LE_BUSNUMBER_OF (rep);
					clevel[o] = LE_LEVEL_OF (rep);
				}
			ncontrib[k] = n;
		}
	}
	/* the template's rand() stream (hosts: srand (time (NULL)), b_synth/lv2.cpp:949) */
	srand (seed);
	initOscillators (t, t->tgVariant, t->tgPrecision);
	initKeyCompTable (t);
	initEnvelopes (t);

	uint64_t total = 0;
	for (i = 1; i <= NOF_WHEELS; i++) {
		const struct _oscillator* o = &t->oscillators[i];
		if (bank && total + o->lengthSamples <= cap)
			memcpy (bank + total, o->wave, sizeof (float) * o->lengthSamples);
		total += o->lengthSamples;
		if (lens)
			lens[i - 1] = (uint32_t)o->lengthSamples;
		if (wfreq)
			wfreq[i - 1] = o->frequency;
	}
	if (atk)
		memcpy (atk, t->attackEnv, sizeof (t->attackEnv));
	if (rel)
		memcpy (rel, t->releaseEnv, sizeof (t->releaseEnv));
	if (kc)
		memcpy (kc, t->keyCompTable, sizeof (t->keyCompTable));
	for (i = 1; i <= NOF_WHEELS; i++)
		free (t->oscillators[i].wave);
	return (long)total;
}

PIN_API long refpin_template_cfg (double sr, const double* freq300, const double* ratio9, unsigned int seed,
                                  const orc_cfg* cfg, float* bank, uint64_t cap, uint32_t* lens, double* wfreq, float* atk,
                                  float* rel, float* kc)
{
	return refpin_template_full (sr, freq300, ratio9, seed, cfg, bank, cap, lens, wfreq, atk, rel, kc, NULL, NULL, NULL,
	                             NULL, 0);
}

PIN_API long refpin_template (double sr, const double* freq300, const double* ratio9, unsigned int seed, float* bank,
                              uint64_t cap, uint32_t* lens, double* wfreq, float* atk, float* rel, float* kc)
{
	return refpin_template_cfg (sr, freq300, ratio9, seed, NULL, bank, cap, lens, wfreq, atk, rel, kc);
}
