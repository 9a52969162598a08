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
 * The steps in between that the harness skips, applyDefaultConfiguration and
 * compilePlayMatrix, draw no rand() and feed none of these tables (initOscillators
 * reads only the frequencies and the EQ settings); they need getPairedWheel from the
 * unbuildable src/tuning.cpp, and the play matrix they build is pinned by the
 * reference's osc_cfglists.txt / osc_runtime.txt fixtures instead.
 * No stand-in is written for anything: --gc-sections drops initToneGenerator and the
 * rest of the TU that the entry point below does not reach, and --no-undefined proves
 * nothing else is missing.
 */
#include "tonegen.cpp"

#include <stdint.h>

#include "orc.h"

#define PIN_API extern "C" __attribute__ ((visibility ("default")))

/* Build one template's tables the reference's way.  Outputs (any may be NULL):
 *   bank[cap]          wave samples of wheels 1..256 concatenated (returns the total)
 *   lens[256]          wave lengths; wfreq[256] wheel frequencies
 *   atk[9*128], rel[9*128], kc[128]   envelopes and key-compression table */
PIN_API long refpin_template_cfg (double sr, const double* freq300, const double* ratio9, unsigned int seed,
                                  const orc_cfg* cfg, float* bank, uint64_t cap, uint32_t* lens, double* wfreq, float* atk,
                                  float* rel, float* kc)
{
	struct b_tonegen* t = allocTonegen ();
	int               i;
	if (cfg) { /* oscConfig's template keys, through the reference's own setters
	            * (src/tonegen.cpp:479-485, 1868-1921), between alloc and init as at startup */
		setWavePrecision (t, cfg->tgPrecision);
		setEnvAttackModel (t, cfg->envAttackModel);
		setEnvReleaseModel (t, cfg->envReleaseModel);
		setEnvAttackClickLevel (t, cfg->envAttackClickLevel);
		setEnvReleaseClickLevel (t, cfg->envReleaseClickLevel);
		t->envAtkClkMinLength = cfg->envAtkClkMinLength; /* setEnvAtkClkMinLength's result */
		t->envAtkClkMaxLength = cfg->envAtkClkMaxLength;
	}
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

PIN_API long refpin_template (double sr, const double* freq300, const double* ratio9, unsigned int seed, float* bank,
                              uint64_t cap, uint32_t* lens, double* wfreq, float* atk, float* rel, float* kc)
{
	return refpin_template_cfg (sr, freq300, ratio9, seed, NULL, bank, cap, lens, wfreq, atk, rel, kc);
}
