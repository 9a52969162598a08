/*
 * lv2_bind.cpp -- libtbf_lv2.so: the LV2 binding of hosts/lv2_synth.h behind a C entry
 * point, so a test can drive the plugin's run() loop (b_synth/lv2.cpp:1120-1140: render
 * up to each MIDI event's frame, apply the event, render the rest of the period) through
 * the exact synthSound a maintainer would add.
 */
#include "lv2_synth.h"

extern "C" {
/* synthSound (b3s with engine e, written, nframes, {L, R}) */
uint32_t tbf_lv2_synth_sound (tbf_engine* e, uint32_t written, uint32_t nframes, float* outL, float* outR)
{
	B3S    b3s = {e};
	float* out[2] = {outL, outR};
	return synthSound (&b3s, written, nframes, out);
}

/* tbf_key (b3s with engine e, key, on) */
void tbf_lv2_key (tbf_engine* e, int key, int on)
{
	B3S b3s = {e};
	tbf_key (&b3s, key, on);
}

/* tbf_instantiate_engine at the given rate (default tuning): returns the engine or NULL */
tbf_engine* tbf_lv2_instantiate (double rate)
{
	B3S b3s = {nullptr};
	return tbf_instantiate_engine (&b3s, rate, nullptr) == 0 ? b3s.tbf : nullptr;
}
}
