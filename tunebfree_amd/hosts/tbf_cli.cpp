/*
 * tbf_cli.cpp -- a headless host on the engine's C-ABI, the counterpart of the
 * reference's JACK CLI audio loop (src/main.cpp:206-292, headless with NO_JACK) and of
 * the LV2 synthSound path (b_synth/lv2.cpp:212-239).
 *
 * It loads a programme file (.pgm), builds one template and B organ instances, selects
 * a programme, plays a chord, and pulls audio buffer by buffer through tbf_synth_sound
 * exactly like a JACK/LV2 period: the engine renders 128-sample blocks and the FIFO
 * slices them into `--buffer` frames.  Instance 0 is written as a float32 stereo WAV,
 * or every instance as raw interleaved float32 with --raw.
 *
 *   tbf_cli --pgm FILE [--program N] [--instances B] [--rate HZ] [--buffer FRAMES]
 *           [--seconds S] [--notes 60,64,67,72] [--seed S] [--character X]
 *           [--out FILE.wav | --raw FILE]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/tbf.h"

static void usage ()
{
	fprintf (stderr,
	         "usage: tbf_cli --pgm FILE [--program N] [--instances B] [--rate HZ] [--buffer FRAMES]\n"
	         "               [--seconds S] [--notes K,K,...] [--seed S] [--character X] [--out F.wav | --raw F]\n");
}

static int check (int rc, const char* what)
{
	if (rc < 0) {
		fprintf (stderr, "tbf_cli: %s failed (%d): %s\n", what, rc, tbf_last_error ());
		exit (1);
	}
	return rc;
}

static void put32 (FILE* f, uint32_t v) { fwrite (&v, 4, 1, f); }
static void put16 (FILE* f, uint16_t v) { fwrite (&v, 2, 1, f); }

int main (int argc, char** argv)
{
	std::string pgm, out = "tbf_cli.wav", raw;
	int         program = 0, instances = 1, buffer = 256;
	double      rate = 48000.0, seconds = 2.0, character = -1.0;
	uint32_t    seed = 1;
	std::vector<int> notes = {60, 64, 67, 72};
	for (int i = 1; i < argc; i++) {
		std::string a = argv[i];
		auto        v = [&] () -> const char* {
			if (i + 1 >= argc) {
				usage ();
				exit (2);
			}
			return argv[++i];
		};
		if (a == "--pgm") pgm = v ();
		else if (a == "--program") program = atoi (v ());
		else if (a == "--instances") instances = atoi (v ());
		else if (a == "--rate") rate = atof (v ());
		else if (a == "--buffer") buffer = atoi (v ());
		else if (a == "--seconds") seconds = atof (v ());
		else if (a == "--seed") seed = (uint32_t)strtoul (v (), nullptr, 10);
		else if (a == "--character") character = atof (v ());
		else if (a == "--out") out = v ();
		else if (a == "--raw") raw = v ();
		else if (a == "--notes") {
			notes.clear ();
			for (char* t = strtok (const_cast<char*> (v ()), ","); t; t = strtok (nullptr, ","))
				notes.push_back (atoi (t));
		} else {
			usage ();
			return 2;
		}
	}
	if (instances < 1 || buffer < 1 || seconds <= 0) {
		usage ();
		return 2;
	}

	tbf_engine_config cfg;
	memset (&cfg, 0, sizeof (cfg));
	cfg.sample_rate = rate;
	cfg.device      = 0;
	cfg.chain_mode  = TBF_CHAIN_FULL;
	tbf_engine* e   = nullptr;
	check (tbf_engine_create (&cfg, &e), "tbf_engine_create");
	if (!pgm.empty ()) {
		FILE* f = fopen (pgm.c_str (), "rb");
		if (!f) {
			perror (pgm.c_str ());
			return 1;
		}
		std::string text;
		char        buf[4096];
		size_t      n;
		while ((n = fread (buf, 1, sizeof (buf), f)) > 0)
			text.append (buf, n);
		fclose (f);
		const int np = check (tbf_program_parse (e, text.c_str ()), "tbf_program_parse");
		fprintf (stderr, "tbf_cli: %d programmes\n", np);
	}
	uint32_t tpl = 0, first = 0;
	check (tbf_template_create (e, nullptr, nullptr, seed, &tpl), "tbf_template_create");
	std::vector<uint32_t> tpls (instances, tpl), seeds (instances);
	for (int i = 0; i < instances; i++)
		seeds[i] = seed + 1000u + (uint32_t)i;
	check (tbf_instances_add (e, instances, tpls.data (), seeds.data (), &first), "tbf_instances_add");
	char name[64] = "";
	if (!pgm.empty () && tbf_program_name (e, (uint32_t)program, name, sizeof (name)) == 1)
		fprintf (stderr, "tbf_cli: program %d \"%s\"\n", program, name);
	for (int i = 0; i < instances; i++) {
		if (!pgm.empty ())
			check (tbf_program_install (e, i, (uint32_t)program), "tbf_program_install");
		if (character >= 0)
			check (tbf_set_param (e, i, TBF_P_CHARACTER, character), "tbf_set_param");
		for (int k : notes)
			check (tbf_note (e, i, k, 1), "tbf_note");
	}

	/* the host period loop: one tbf_synth_sound per buffer of `buffer` frames */
	const uint64_t     total = (uint64_t)(seconds * rate);
	std::vector<float> L ((size_t)instances * buffer), R ((size_t)instances * buffer);
	std::vector<float> keepL, keepR; /* instance 0 (WAV) or all (raw) */
	FILE*              rf = raw.empty () ? nullptr : fopen (raw.c_str (), "wb");
	for (uint64_t done = 0; done < total;) {
		const uint32_t nf = (uint32_t)std::min<uint64_t> (buffer, total - done);
		check (tbf_synth_sound (e, nf, L.data (), R.data (), (uint64_t)buffer), "tbf_synth_sound");
		if (rf) {
			std::vector<float> il ((size_t)instances * nf * 2);
			for (int i = 0; i < instances; i++)
				for (uint32_t t = 0; t < nf; t++) {
					il[((size_t)i * nf + t) * 2]     = L[(size_t)i * buffer + t];
					il[((size_t)i * nf + t) * 2 + 1] = R[(size_t)i * buffer + t];
				}
			fwrite (il.data (), sizeof (float), il.size (), rf);
		} else {
			keepL.insert (keepL.end (), L.begin (), L.begin () + nf);
			keepR.insert (keepR.end (), R.begin (), R.begin () + nf);
		}
		done += nf;
	}
	if (rf)
		fclose (rf);
	else {
		FILE* f = fopen (out.c_str (), "wb");
		if (!f) {
			perror (out.c_str ());
			return 1;
		}
		const uint32_t frames = (uint32_t)keepL.size (), bytes = frames * 8;
		fwrite ("RIFF", 1, 4, f);
		put32 (f, 36 + bytes);
		fwrite ("WAVEfmt ", 1, 8, f);
		put32 (f, 16);
		put16 (f, 3); /* IEEE float */
		put16 (f, 2);
		put32 (f, (uint32_t)rate);
		put32 (f, (uint32_t)rate * 8);
		put16 (f, 8);
		put16 (f, 32);
		fwrite ("data", 1, 4, f);
		put32 (f, bytes);
		for (uint32_t t = 0; t < frames; t++) {
			fwrite (&keepL[t], 4, 1, f);
			fwrite (&keepR[t], 4, 1, f);
		}
		fclose (f);
	}
	fprintf (stderr, "tbf_cli: %llu frames x %d instances\n", (unsigned long long)total, instances);
	tbf_engine_destroy (e);
	return 0;
}
