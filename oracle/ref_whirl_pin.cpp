/*
 * oracle/ref_whirl_pin.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Pins the whirl's MIDI control setters (src/whirl.cpp:699-909) to the reference's OWN
 * code.  They live in the LV2-only part of whirl.cpp (`#ifndef CLAP`), are `static`, and
 * reach the MIDI layer only through initWhirl's useMIDIControlFunction registrations
 * (961-982), which need the MIDI layer of src/midi.cpp.  This harness #includes
 * /root/reference/src/whirl.cpp unmodified WITHOUT the CLAP define (compiled by
 * oracle/Makefile target `wpin`, output only into oracle/_ref/), so the static setters
 * are in this translation unit, and calls them by the names initWhirl registers them
 * under.  Construction replays the part of initWhirl (956-986) that the setters' fields
 * depend on:
 *     allocWhirl; SampleRateD = rate; initialize
 * (not the registrations, nor computeRotationSpeeds: without CLAP its setRevSelect
 * notifies the MIDI layer, and no setter reads or writes the rotor speeds).
 * No stand-in is written: --gc-sections drops initWhirl, whirlConfig and the rest of the
 * TU the entry points below do not reach, and --no-undefined proves nothing else is
 * missing (eqcomp.o supplies eqCompute).
 *
 * tests/test_oracle_cpu.py compares the fields these setters write with the ones the
 * oracle's orc_control writes (orc_whirl_fields), value by value.
 */
#include "whirl.cpp"

#include <string.h>

#define PIN_API extern "C" __attribute__ ((visibility ("default")))

PIN_API void* wpin_new (double rate)
{
	struct b_whirl* w = allocWhirl ();
	if (!w)
		return NULL;
	w->SampleRateD = rate;
	initialize (w);
	return w;
}

PIN_API void wpin_free (void* w) { freeWhirl ((struct b_whirl*)w); }

/* the 14 functions initWhirl registers (src/whirl.cpp:970-981), by name */
PIN_API int wpin_control (void* d, const char* fn, int uc)
{
	static const struct {
		const char* name;
		void (*set) (void*, unsigned char);
	} tab[] = {
	    {"whirl.horn.filter.a.type", setHornFilterAType},
	    {"whirl.horn.filter.a.hz", setHornFilterAFrequency},
	    {"whirl.horn.filter.a.q", setHornFilterAQ},
	    {"whirl.horn.filter.a.gain", setHornFilterAGain},
	    {"whirl.horn.filter.b.type", setHornFilterBType},
	    {"whirl.horn.filter.b.hz", setHornFilterBFrequency},
	    {"whirl.horn.filter.b.q", setHornFilterBQ},
	    {"whirl.horn.filter.b.gain", setHornFilterBGain},
	    {"whirl.horn.brakepos", setHornBrakePosition},
	    {"whirl.drum.brakepos", setDrumBrakePosition},
	    {"whirl.horn.acceleration", setHornAcceleration},
	    {"whirl.horn.deceleration", setHornDeceleration},
	    {"whirl.drum.acceleration", setDrumAcceleration},
	    {"whirl.drum.deceleration", setDrumDeceleration},
	};
	for (const auto& t : tab)
		if (!strcmp (t.name, fn)) {
			t.set (d, (unsigned char)uc);
			return 0;
		}
	return -1;
}

/* the fields the setters write, in orc_whirl_fields' order:
 * haT haF haQ haG hafw[1..5] hbT hbF hbQ hbG hbfw[1..5]
 * hnBrakePos drBrakePos hornAcc hornDec drumAcc drumDec */
PIN_API int wpin_fields (const void* d, double* out)
{
	const struct b_whirl* w = (const struct b_whirl*)d;
	int                   k = 0;
	out[k++]                = w->haT;
	out[k++]                = w->haF;
	out[k++]                = w->haQ;
	out[k++]                = w->haG;
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
