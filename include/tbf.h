/*
 * tbf.h -- C-ABI of the MI355X batched render engine for tuneBfree's DSP chain.
 *
 * Drop-in boundary.  The reference evaluates one organ per plugin instance through
 * four per-block calls issued by synthSound (b_synth/lv2.cpp:212-239,
 * src/clap.cpp:244-270, src/main.cpp:243-292):
 *     oscGenerateFragment (struct b_tonegen*, float* buf, size_t)     src/tonegen.h:594
 *     preamp (void* pa, float* in, float* out, size_t)                 src/overdrive.h:35
 *     b_reverb::reverb (float* in, float* out, int)                    src/reverb.h:30
 *     whirlProc3 (struct b_whirl*, const float*, float*, float*,
 *                 float*, float*, size_t)                              src/whirl.h:245-249
 * tbf_render / tbf_synth_sound replace that quartet for a batch of instances; the
 * control surface replaces the host-side calls that mutate the DSP structs between
 * blocks:
 *     oscKeyOn / oscKeyOff                      src/tonegen.cpp:3096-3166 -> tbf_note
 *     CLAP setParam (drawbars, vibrato, rotary,
 *     overdrive, character, reverb, percussion) src/clap.cpp:162-207     -> tbf_set_param
 *     allocSynth + initSynth                    b_synth/lv2.cpp:336-353, 164-193
 *                                               -> tbf_template_create + tbf_instances_add
 * Event timing is the reference's: anything issued between two render calls takes
 * effect at the next 128-sample block boundary (b_synth/lv2.cpp:1130-1134).
 *
 * Conventions: plain C types, 0 on success, negative errno-style codes on failure
 * (tbf_last_error() has the message); one host thread per engine; no allocation
 * inside tbf_render_device once the instance set is fixed.
 */
#ifndef TBF_H
#define TBF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBF_ABI_VERSION 1
#define TBF_BLOCK_SAMPLES 128

/* parameter ids: CLAP ids of src/clap.cpp:31-48 ... */
#define TBF_P_DRAWBAR_MIN 0 /* upper manual drawbars 16' .. 1', value 0..8 */
#define TBF_P_DRAWBAR_MAX 8
#define TBF_P_VIBRATO 9            /* upper manual through the scanner, 0/1 */
#define TBF_P_VIBRATO_TYPE 10      /* 0..5 = V1 C1 V2 C2 V3 C3 */
#define TBF_P_DRUM 11              /* 0 stop, 1 slow, 2 fast */
#define TBF_P_HORN 12              /* 0 stop, 1 slow, 2 fast */
#define TBF_P_OVERDRIVE 13         /* 0 clean, 1 overdrive */
#define TBF_P_CHARACTER 14         /* 0..1 */
#define TBF_P_REVERB 15            /* reverb mix 0..1 */
#define TBF_P_PERCUSSION 16        /* 0/1 */
#define TBF_P_PERCUSSION_VOLUME 17 /* 1 normal, 0 soft (CLAP convention) */
#define TBF_P_PERCUSSION_DECAY 18  /* 1 fast, 0 slow */
#define TBF_P_PERCUSSION_HARMONIC 19 /* 1 second (bus A), 0 third (bus B) */
/* ... plus the setters the LV2/JACK hosts reach through MIDI CCs (src/midi.cpp) */
#define TBF_P_BUS_DRAWBAR_BASE 100 /* 100 + bus 0..26 (upper, lower, pedal), value 0..8 */
#define TBF_P_VIBRATO_LOWER 130    /* lower manual through the scanner, 0/1 */
#define TBF_P_SWELL 131            /* swell pedal 0..1 (setSwellPedal1FromMIDI) */
#define TBF_P_WHIRL_BYPASS 132     /* whirl.bypass 0/1 */

#define TBF_CHAIN_FULL 0     /* tonegen -> vibrato -> overdrive -> reverb -> whirl */
#define TBF_CHAIN_TONEGEN 1  /* oscGenerateFragment only, L = R = tonegen output */
#define TBF_CHAIN_TAP_PREAMP 2 /* parity tap: L = R = preamp output */
#define TBF_CHAIN_TAP_REVERB 3 /* parity tap: L = R = reverb output */

typedef struct tbf_engine tbf_engine;

/* tbf_engine_config.debug_flags */
#define TBF_DEBUG_FORCE_SERIAL 1u /* fail every fast-path precondition vote, so each guarded
                                   * stage takes its exact serial replay (parity tests of the
                                   * fallbacks; slow) */

typedef struct tbf_engine_config {
	double   sample_rate; /* Hz, 8000 .. 192000 */
	int32_t  device;      /* HIP device ordinal */
	uint32_t chain_mode;  /* TBF_CHAIN_* */
	uint32_t debug_flags; /* TBF_DEBUG_*, 0 in production */
	uint32_t reserved[3];
} tbf_engine_config;

int         tbf_abi_version (void);
const char* tbf_last_error (void);

int tbf_engine_create (const tbf_engine_config* cfg, tbf_engine** out);
int tbf_engine_destroy (tbf_engine* e);

/* ---- cfg keys (§8(f) row 4): the reference's `key=value` configuration lines ----
 * parseConfigurationLine / distributeParameter (src/cfgParser.cpp:61-160) hand each line
 * to every module; the ones that reach this engine are
 *   whirl.*   whirlConfig (src/whirl.cpp:992-1160): speeds, accelerations, geometry
 *             (horn/drum radius, mic distance, horn offsets), the three filters,
 *             horn level / leak, mic widths and angle, brake positions, speed preset,
 *             bypass.  Geometry re-derives the compact ring window (512 / 1024 / 2048)
 *   scanner.* scannerConfig (src/vibrato.cpp:334-357): scanner frequency, V1-V3 depths
 *   reverb.mix reverbConfig (src/reverb.cpp:242-256)
 *   osc.*     oscConfig (src/tonegen.cpp:2173-2555): x-precision, the key-click /
 *             release envelope models, levels and lengths, percussion gains, buses and
 *             trigger bus (osc.perc.fast / .slow are stored but, as in the reference,
 *             never reach the decay constants); the wheel EQ (osc.eq.macro, spline
 *             points), extra wheel harmonics (osc.harmonic.*), terminal mixes, key tapers
 *             and key crosstalk lists (osc.terminal.* / osc.taper.* / osc.crosstalk.*),
 *             the default crosstalk levels and the contribution floor / minimum
 * A setting applies to what is built after it: whirl.* tables and scanner.* shape
 * engine-wide tables and must precede tbf_instances_add (-16 after); osc.* template
 * keys apply to later tbf_template_create / tbf_templates_create; the rest to later
 * tbf_instances_add.  Returns 0 applied, 1 ignored: not a key of this path, or a key
 * the reference stores but never reads here (overdrive.* / xov.*: ampConfig,
 * src/overdrive.cpp:395-433, writes fields airwindows_density never reads;
 * osc.tuning / osc.temperament / osc.eqv.*; whirl.horn.comb.*), -22 bad value
 * (nothing assigned; a list key with any malformed part assigns none of it, where the
 * reference keeps the well-formed parts and warns; osc.transformer-crosstalk above 0,
 * with which the reference aborts in findTransformerNeighbours,
 * src/tonegen.cpp:914-927). */
int tbf_config_set (tbf_engine* e, const char* key, const char* value);
/* a cfg file's text (`name = value` lines, '#' comments): returns the number of keys
 * applied, or < 0 with tbf_last_error () = "line N: message".  All or nothing: a bad line
 * (or a table-shaping key after tbf_instances_add) applies none of the text's keys. */
int tbf_config_parse (tbf_engine* e, const char* text);

/* Tone-generator template (initToneGenerator's shared tables: wave bank, play matrix,
 * envelopes) for one tuning.  mts128: 128 MTS-ESP note frequencies or NULL for the
 * no-master 12-TET table; ratio9: drawbar target ratios or NULL for
 * {0.5,1.5,1,2,3,4,5,6,8}; seed: srand() seed of the template's rand() stream. */
int tbf_template_create (tbf_engine* e, const double* mts128, const double* ratio9, uint32_t seed,
                         uint32_t* tpl_id);

/* n templates built on the device (replaces n initToneGenerator
 * table builds, src/tonegen.cpp:1470-1630 initOscillators + 2562-2728 initEnvelopes):
 * the same tables as n tbf_template_create calls, with the wave bank's sines and its per-sample rand() draws
 * (each thread jumping the glibc stream to its chunk) computed on the engine's GPU.
 * mts128: n x 128 frequencies or NULL; ratio9: n x 9 or NULL; seeds[n]; ids[n] out.
 * Needs a device engine (-19 on a host-only engine). */
int tbf_templates_create (tbf_engine* e, uint32_t n, const double* mts128, const double* ratio9,
                          const uint32_t* seeds, uint32_t* tpl_ids);

/* Add n instances: instance k uses template tpl_ids[k] and per-instance seed seeds[k]
 * (srand before allocReverb/allocPreamp).  Returns the first new index in *first. */
int      tbf_instances_add (tbf_engine* e, uint32_t n, const uint32_t* tpl_ids, const uint32_t* seeds,
                            uint32_t* first);
uint32_t tbf_instance_count (const tbf_engine* e);

/* MTS-ESP retune (§8(f) row 3): the CLAP plugin's reinitToneGen (src/clap.cpp:129-157,
 * run from process() when MTS_NoteToFrequency or the drawbar ratios change,
 * src/clap.cpp:1133-1175) for instance inst on template tpl_id (built from the new
 * frequencies / ratios with tbf_template_create or tbf_templates_create).  From the next
 * block the instance plays a fresh tone generator on the new tables: no keys down,
 * initToneGenerator's defaults, then drawbars 16'..1', vibrato on/off and vibrato type
 * restored from the instance's CLAP parameter values (their get_info defaults when never
 * set, src/clap.cpp:383-545) and the routing word kept; preamp, reverb and whirl state
 * continue.  Events given after the call apply after the retune, as the reference
 * checks the tuning at the top of process() before the block's events.  The osc.* /
 * scanner.* cfg keys in force now apply to the new tone generator. */
int tbf_instance_retune (tbf_engine* e, uint32_t inst, uint32_t tpl_id);

int tbf_note (tbf_engine* e, uint32_t inst, int32_t key, int32_t on);
int tbf_set_param (tbf_engine* e, uint32_t inst, int32_t param, double value);

/* Render nblocks x 128 samples for every instance.  Host buffers; instance i writes
 * out[i * stride + 0 .. nblocks*128).  Synchronous. */
int tbf_render (tbf_engine* e, uint32_t nblocks, float* outL, float* outR, uint64_t stride);

/* Same into device memory on `stream` (hipStream_t, NULL = the engine's own
 * non-blocking stream); returns once the work is enqueued.  Outputs stay in HBM.
 * Ordering: the render is ordered after earlier work on `stream` and the outputs are
 * complete when `stream` reaches this point.  A NULL stream is NOT the legacy default
 * stream: a caller that consumes the outputs on another stream (e.g. torch's current
 * stream, whose handle is 0 on the default stream) must pass that stream's real handle
 * or call tbf_synchronize () first. */
int tbf_render_device (tbf_engine* e, uint32_t nblocks, float* d_outL, float* d_outR, uint64_t stride,
                       void* stream);

/* synthSound semantics (b_synth/lv2.cpp:212-239): serve nframes per instance out of
 * the 128-sample block FIFO, rendering blocks as needed.  Instance i writes
 * out[i * stride + 0 .. nframes); stride >= nframes (else -22). */
int tbf_synth_sound (tbf_engine* e, uint32_t nframes, float* outL, float* outR, uint64_t stride);

/* ---- host control surface (src/midi.cpp, src/program.cpp, src/pgmParser.cpp) ---- */
/* callMIDIControlFunction (src/midi.cpp:535-545) on one instance.  fn is a control
 * function name of src/midi.cpp:100-170 that reaches the DSP chain: upper|lower|pedal.
 * drawbar16/513/8/4/223/2/135/113/1, percussion.enable|volume|decay|harmonic,
 * vibrato.knob|routing|upper|lower, swellpedal1|2, overdrive.enable|character,
 * reverb.mix, rotary.speed-preset|speed-select|speed-toggle, and the whirl's
 * whirl.horn.filter.a|b.type|hz|q|gain, whirl.horn|drum.brakepos,
 * whirl.horn|drum.acceleration|deceleration (src/whirl.cpp:699-889, registered 966-981;
 * from the next block).  value 0..127 (clamped).  Returns 0 when applied, 1 for any
 * other name (ignored, as the reference ignores names without a registered function). */
int tbf_midi_control (tbf_engine* e, uint32_t inst, const char* fn, int32_t value);
/* programme definitions in the .pgm syntax (src/pgmParser.cpp:65-73, properties of
 * bindToProgram src/program.cpp:133-603) into the engine's programme table; returns the
 * number of programmes in use, or < 0 with tbf_last_error () = "line N: message" */
int tbf_program_parse (tbf_engine* e, const char* text);
/* installProgram (src/program.cpp:735-921): MIDI program change pc (0..127, plus the
 * reference's default pgm.controller.offset of 1) on one instance; random drawbars draw
 * from the instance's control rand() stream */
int tbf_program_install (tbf_engine* e, uint32_t inst, uint32_t pc);
/* name of the programme program change pc selects; returns 1 if in use, else 0 */
int tbf_program_name (tbf_engine* e, uint32_t pc, char* out, uint32_t cap);

/* ---- scheduled events (§8(f) row 1): a whole event script in one render ---- */
#define TBF_EV_NOTE 0    /* id = key 0..383 (oscKeyOn/Off), value != 0: on */
#define TBF_EV_PARAM 1   /* id = TBF_P_*, value as tbf_set_param */
#define TBF_EV_CONTROL 2 /* id = tbf_midi_control_id (name), value 0..127 */
#define TBF_EV_PROGRAM 3 /* id = program change 0..127 (tbf_program_install) */

typedef struct tbf_event {
	uint32_t block; /* block index (from the start of this call) before which it applies */
	uint32_t inst;
	int32_t  kind;  /* TBF_EV_* */
	int32_t  id;
	double   value;
} tbf_event;

/* id of a control function name for TBF_EV_CONTROL events, < 0 if not a hot-path name */
int tbf_midi_control_id (const char* fn);
/* render nblocks with events applied at their block boundaries (b_synth/lv2.cpp:
 * 1130-1134 timing), into device memory like tbf_render_device.  Events must be sorted
 * by block; within a block they apply in array order; events at or beyond nblocks apply
 * after the render.  The host steps the control plane per block and uploads only the
 * per-block control deltas, so one launch set covers a whole chunk of 64 blocks however
 * many events land in it. */
int tbf_render_events (tbf_engine* e, uint32_t nblocks, const tbf_event* ev, uint32_t nev, float* d_outL,
                       float* d_outR, uint64_t stride, void* stream);

int tbf_synchronize (tbf_engine* e);
/* Which exact-but-slow paths the kernels took since the engine's first render (cumulative,
 * informational; the results are bit-identical either way).  Waits for the engine's
 * own stream and the pipelined stage streams; a caller rendering on its own stream must
 * synchronize that stream first. */
#define TBF_PATH_VIB_SERIAL 1u   /* vibrato scatter: lane-serial replay (src/vibrato.cpp:380-409) */
#define TBF_PATH_WH_ANGLE 2u     /* whirl rotor angles: literal fmod recurrence (src/whirl.cpp:1428-1429) */
#define TBF_PATH_WH_MOTION 4u    /* whirl ring adds: sample-serial replay (src/whirl.cpp:1432-1469) */
#define TBF_PATH_RV_PHASE 8u     /* reverb LFO phases: literal recurrence + sin (src/reverb.cpp:479-496) */
#define TBF_PATH_RV_WINDOW 16u   /* reverb tap outside the staged window: direct ring reads */
int tbf_error_flags (tbf_engine* e, uint32_t* flags);
/* read back the wave bank of a template (wheels 1..256 concatenated) for checks */
int tbf_template_bank (tbf_engine* e, uint32_t tpl_id, float* out, uint64_t cap, uint32_t* lens256);

/* ---- test hooks (host only; used by the parity tests to pin the control plane) ---- */
/* play-matrix entries of one key (keyContrib, src/tonegen.cpp:1122-1213) */
int tbf_debug_contrib (tbf_engine* e, uint32_t tpl_id, int32_t key, int16_t* wheel, int16_t* bus, float* level,
                       uint32_t cap);
/* the program the instance's next block plays unless its control changes (the persistent
 * pool entry, read back from the device after synchronizing): 9 floats per instruction
 * as tbf_debug_render_program; works with either control path */
int tbf_debug_device_program (tbf_engine* e, uint32_t inst, float* entries9, uint32_t cap);
/* host control time: wall-clock the render calls spent stepping the control plane
 * (events, message queues, active lists, routing, per-block programmes) since the last
 * reset, and the blocks it covered */
int tbf_debug_host_time (tbf_engine* e, int32_t reset, double* ms, uint64_t* blocks);
/* self-check of the host worker pool the control plane's parallel sections run on: jobs
 * of 1..40 tasks back to back (jobs of them), each task counted; returns the number of
 * jobs in which a task ran other than exactly once (0: all good) */
int tbf_debug_pool_check (uint32_t jobs);
/* the cfg-derived HBM layout: the compact whirl ring window (512 / 1024 / 2048 samples
 * per ring, from the geometry's largest write-ahead) and the reverb slab length */
int tbf_debug_layout (const tbf_engine* e, uint32_t* wring_len, float* max_ahead, uint32_t* slab_len);
/* blocks per render chunk: with control deltas (64) and without (TBF_STEADY_CHUNK, up to 2048) */
int tbf_debug_chunks (const tbf_engine* e, uint32_t* delta_blocks, uint32_t* steady_blocks);
/* chunks with events since the engine was created, by the front end that stepped them:
 * the device's (k_front) and the host's */
int tbf_debug_front_chunks (const tbf_engine* e, uint64_t* device_chunks, uint64_t* host_chunks);
/* the longest render chunk without control deltas, in blocks (64 .. 2048, default 512).
 * The stage buffers hold one chunk per instance (56 B per instance and sample at the
 * default stage groups: 15 GB at 4096 instances and 512 blocks, 60 GB at 2048) and
 * grow to the longest chunk a call makes, so this bounds the engine's HBM footprint; longer
 * chunks spread each launch's state traffic over more samples.  The
 * value is clamped to what the device can hold for the instances added so far (halved
 * until the buffers fit the free memory plus the buffers held now), and a render that
 * still cannot allocate them halves it again (tbf_debug_chunks reports the value in
 * effect).  Takes effect at the next render (buffers larger than the new value are freed
 * then); returns the value in effect, or < 0 on error.  Renders are bit-identical at every
 * value. */
int tbf_set_steady_chunk (tbf_engine* e, uint32_t blocks);
/* test hook: set the reverb vibrato phase of line 0..7 of channel ch (b_reverb vib[ch][line],
 * src/reverb.cpp:479-496) of an instance, effective from the next block; parity tests use
 * it to place a phase just below a power of two (a binade crossing inside a launch) */
int tbf_debug_reverb_phase (tbf_engine* e, uint32_t inst, int32_t ch, int32_t line, double value);
/* envelopes (9 x 128 each) and key-compression table (128) of a template */
int tbf_debug_tables (tbf_engine* e, uint32_t tpl_id, float* attack, float* release, float* keycomp);
/* run one block of the tonegen control plane for an instance and return the core
 * program: per entry {wheel, env, row, sg, pg, vg, nsg, npg, nvg} as 9 floats */
int tbf_debug_step (tbf_engine* e, uint32_t inst, float* entries9, uint32_t cap);
/* the core program the instance's next rendered block uses, after the control-plane
 * step a render makes for that block (which steps only when something changed) */
int tbf_debug_render_program (tbf_engine* e, uint32_t inst, float* entries9, uint32_t cap);
/* an instance's host control state: odClean, odA, odC, rvG, revOpt, revSelect, whBypass,
 * newRouting, swellPedalGain, percEnabled, percIsSoft, percIsFast, percSendBus, vibTable,
 * vibMixed, percDrawbarGain, drawBarGain[27], the whirl's haT haF haQ haG hbT hbF hbQ hbG
 * hornAcc hornDec drumAcc drumDec hnBrakePos drBrakePos; returns the count (57) */
int tbf_debug_control (tbf_engine* e, uint32_t inst, double* out, uint32_t cap);
/* the kernel's exact shortcuts of serial recurrences, evaluated on the host (same source,
 * csrc/tbf_exact.h): op 0 phase_run (in: v0, d, m -> out: ok, D), op 1 cnt_adv (in: c0,
 * d, n -> out: count), op 2 wrap1 (in: x, -, - -> out: fmod (x, 1)), op 3 xorshift
 * dither jump (in: x0, k, - -> out: jump-table state, k literal steps), op 4 cached
 * phase steps along 4096 sub-blocks (in: v0, d, m -> out: mismatches vs phase_run, cache
 * hits), op 5 glibc rand() jump (in: seed, k, - -> out: next draw after GlibcRand::discard
 * (k), after k literal draws); n records */
int tbf_debug_exact (int32_t op, const double* in3, double* out2, uint32_t n);
/* per-stage kernel timing with HIP events on each launch's stream: enable 1 / -1 turns
 * recording on / off (1: as rendered, launches of neighbouring chunks overlapping; 2:
 * with the cross-chunk pipelining off, each kernel alone on the GPU); 0 returns the
 * summed milliseconds and launch counts of the six stage kernels k_tonegen, k_mixpre,
 * k_rv_pre, k_rv_core, k_rv_post, k_whirl since the last query (ms6[6], count6[6]) */
int tbf_debug_kernel_times (tbf_engine* e, int32_t enable, double* ms6, uint32_t* count6);
/* PMC calibration: op 0 streams n doubles from d_buf (8 B/lane reads, the reverb ring
 * pattern), op 1 writes them; ops 2 / 3 the same starting 64 B into a cache line (n >= 16);
 * op 4 (test hook for csrc/tbf_sin.h): d_buf holds n inputs x followed by room for 6 n
 * results: tbf_sin (x), sin (x), tbf_sin2's two results for (x, the input n / 2 further on),
 * the asin fast path and asin (x clamped to [-1, 1]); enqueued on `stream` (NULL = legacy
 * default stream) */
int tbf_debug_calibrate (int32_t op, void* d_buf, uint64_t n_doubles, void* stream);

#ifdef __cplusplus
}
#endif
#endif
