/*
 * lv2_synth.h -- the LV2 plugin's synthSound (b_synth/lv2.cpp:212-239) on the engine: the
 * binding INTEGRATION.md section 2 shows a maintainer adding to b_synth/lv2.cpp, compiled
 * here verbatim (tests/test_host_cpu.py checks that the document's block is this text).
 * hosts/lv2_bind.cpp builds it into libtbf_lv2.so, whose run() loop a GPU test drives
 * with irregular periods and MIDI events against the oracle.
 */
#ifndef TBF_LV2_SYNTH_H
#define TBF_LV2_SYNTH_H

#include <stdint.h>
#include <time.h>

#include "../../include/tbf.h"

/* --8<-- INTEGRATION.md section 2 */
struct B3S {
	/* ... existing fields ... */
	tbf_engine* tbf;     /* one engine per plugin instance, one instance inside */
};

static int tbf_instantiate_engine (B3S* b3s, double rate, const double* mts128)
{
	tbf_engine_config cfg = { rate, /*device*/ 0, TBF_CHAIN_FULL, /*debug_flags*/ 0, {0, 0, 0} };
	uint32_t tpl, first, seed = (uint32_t)time (NULL);   /* srand(time(NULL)), lv2.cpp:949 */
	b3s->tbf = NULL;
	if (tbf_engine_create (&cfg, &b3s->tbf)) return -1;
	if (tbf_template_create (b3s->tbf, mts128, NULL, seed, &tpl) ||
	    tbf_instances_add (b3s->tbf, 1, &tpl, &seed, &first)) {
		tbf_engine_destroy (b3s->tbf);   /* no half-built engine left behind */
		b3s->tbf = NULL;
		return -1;
	}
	/* initSynth's setDrawBars(inst, 0, {8,8,6,...}), lv2.cpp:167-180 */
	static const int bars[9] = {8, 8, 6, 0, 0, 0, 0, 0, 0};
	for (int i = 0; i < 9; ++i)
		tbf_set_param (b3s->tbf, 0, TBF_P_DRAWBAR_MIN + i, bars[i]);
	return 0;
}

/* replaces synthSound (lv2.cpp:212-239): same signature, slicing and return value (the
 * new `written`, which run() assigns: `written = synthSound (...)`, lv2.cpp:1133) */
static uint32_t synthSound (B3S* b3s, uint32_t written, uint32_t nframes, float** out)
{
	if (written >= nframes)
		return written;
	const uint32_t n = nframes - written;
	if (tbf_synth_sound (b3s->tbf, n, out[0] + written, out[1] + written, /*stride*/ n) != 0) {
		for (uint32_t i = 0; i < n; ++i) /* the reference cannot fail: play silence */
			out[0][written + i] = out[1][written + i] = 0.f;
	}
	return nframes;
}

/* process_midi_event -> note callbacks (src/midi.cpp:1095-1256) */
static void tbf_key (B3S* b3s, int key, int on) { tbf_note (b3s->tbf, 0, key, on); }
/* -->8-- */

#endif
