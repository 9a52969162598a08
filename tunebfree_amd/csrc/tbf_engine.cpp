/*
 * tbf_engine.cpp -- the C-ABI of include/tbf.h: instance construction (LV2 allocSynth /
 * initSynth protocol with shared tonegen templates), the host control plane, and the
 * segmentation of a render into kernel launches at block boundaries where control
 * changes.
 */
#include <hip/hip_runtime.h>
#include <assert.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <stddef.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <memory>
#include <string>
#include <vector>

#include "../../include/tbf.h"
#include "tbf_engine_impl.h"
#include "tbf_rand.h"
#include "tbf_tpl.h"
#include "tbf_exact.h"
#include "tbf_host.h"
#include "tbf_types.h"

extern "C" int tbf_launch_stage (const tbf_launch* P, int k, hipStream_t stream);
extern "C" int tbf_chain_stages (uint32_t chain);
extern "C" int tbf_launch_tgctl (const tbf_launch* P, hipStream_t stream);
extern "C" int tbf_launch_front (const tbf_launch* P, hipStream_t stream);
extern "C" int tbf_launch_calibrate (int op, void* buf, uint64_t n, hipStream_t s);
extern "C" int tbf_rv_lds_fits (const tbf_inst_const* k);

using namespace tbf;

static thread_local std::string g_err;
thread_local std::vector<uint32_t>* tbf::tlAct = nullptr;

int tbf::fail (int code, const std::string& msg)
{
	g_err = msg;
	return code;
}

#define HIPCHK(x)                                                                        \
	do {                                                                                 \
		hipError_t _e = (x);                                                             \
		if (_e != hipSuccess)                                                            \
			return fail (-5, std::string (#x ": ") + hipGetErrorString (_e));           \
	} while (0)


/* program slots (tbf_types.h TBF_PROG_SLOT: header + entries).  The device program pool
 * holds two persistent slots per instance (2 i, 2 i + 1; the host-controlled path uses
 * the first), then the chunk's delta programs */
#define SLOT ((size_t)TBF_PROG_SLOT)
#define PSLOTS ((size_t)TBF_PROG_PSLOTS)
#define PERSIST(n) ((size_t)(n) * PSLOTS * SLOT)
/* blocks per kernel launch chunk: bounds the inter-stage buffers to
 * n_inst x TBF_CHUNK x 128 floats each (134 MB at 4096 instances) */
#ifndef TBF_CHUNK
#define TBF_CHUNK 64
#endif
/* host-controlled path: delta program entries one chunk may add (a chunk ends early when
 * they would not fit); the device-controlled path sizes its delta slots on demand */
#define DPROG_CAP(n) ((size_t)(n) * SLOT * 2 + 4096)
/* control pool region (one per chunk parity on the device-controlled path; the host path
 * uses region 0): n persistent entries + up to one delta per instance and block */
#define CTL_REGION(n) ((size_t)(n) * (TBF_CHUNK + 1))

/* ------------------------------------------------------------------ construction */

static void reverbConsts (tbf_inst_const& k, double sr, float A, float B, float C, float D, float E, float F)
{
	/* src/reverb.cpp:283-336 */
	double bq0  = ((A * 9000.0) + 1000.0) / sr;
	double b1[3] = {1.618033988749894848204586, 0.618033988749894848204586, 0.5};
	for (int q = 0; q < 3; q++) {
		double K    = tan (M_PI * bq0);
		double norm = 1.0 / (1.0 + K / b1[q] + K * K);
		k.bq[q][0]  = K * K * norm;
		k.bq[q][1]  = 2.0 * k.bq[q][0];
		k.bq[q][2]  = k.bq[q][0];
		k.bq[q][3]  = 2.0 * (K * K - 1.0) * norm;
		k.bq[q][4]  = (1.0 - K / b1[q] + K * K) * norm;
	}
	double vibSpeed    = 0.06 + C;
	double vibDepth    = (0.027 + pow (D, 3)) * 100.0;
	double size        = (pow (E, 2) * 90.0) + 10.0;
	double depthFactor = 1.0 - pow ((1.0 - (0.82 - ((B * 0.5) + (size * 0.002)))), 4);
	double blend       = 0.955 - (size * 0.007);
	double crossmod    = (F - 0.5) * 2.0;
	crossmod           = pow (crossmod, 3) * 0.5;
	double regen       = depthFactor * (0.5 - (fabs (crossmod) * 0.031));
	static const double depth[8] = {0.003251, 0.002999, 0.002917, 0.002749, 0.002503, 0.002423, 0.002146, 0.002088};
	static const int    dmul[12] = {79, 73, 71, 67, 61, 59, 53, 47, 43, 41, 37, 31};
	for (int l = 0; l < 8; l++)
		k.vibDelta[l] = depth[l] * vibSpeed;
	k.vibDepth      = vibDepth;
	k.blend         = blend;
	k.crossmod      = crossmod;
	k.oneMinusAbsCm = 1.0 - fabs (crossmod);
	k.regen         = regen;
	for (int l = 0; l < 12; l++)
		k.delay[l] = (int)(dmul[l] * size);
	k.delay[12] = (int)((29 * size) - (56 * size * fabs (crossmod)));
	uint32_t o  = 0;
	for (int c = 0; c < 2; c++)
		for (int l = 0; l < 13; l++) {
			k.ringOff[c * 13 + l] = o;
			/* line 12 of channel 0 holds the predelay history (TBF_PD_HIST floats) instead
			 * of a ring; channel 1's stays unused */
			const int len = (l == 12 && c == 0) ? std::max (k.delay[l] + 1, TBF_PD_HIST / 2) : k.delay[l] + 1;
			o += (uint32_t)((len + TBF_RING_ALIGN - 1) & ~(TBF_RING_ALIGN - 1));
		}
	k.slabLen = o;
}

static void whirlConsts (tbf_inst_const& k, const WhirlTables& wt, const Config& c)
{
	memcpy (k.drf, wt.drf, sizeof (k.drf));
	memcpy (k.hornSpacing, wt.hornSpacing, sizeof (k.hornSpacing));
	memcpy (k.drumSpacing, wt.drumSpacing, sizeof (k.drumSpacing));
	memcpy (k.hornPhase, wt.phase, sizeof (k.hornPhase));
	/* initialize (src/whirl.cpp:626-662): leakage = leakLevel * hornLevel */
	k.leakage   = c.leakLevel * c.hornLevel;
	k.hornLevel = c.hornLevel;
	/* mic widths (fsetHornMicWidth / fsetDrumMicWidth, src/whirl.cpp:912-949; width 0
	 * leaves the initValues gains hll dll hrr drr = 1, others 0) */
	float hll = 1.f, hlr = 0.f, hrl = 0.f, hrr = 1.f, dll = 1.f, dlr = 0.f, drl = 0.f, drr = 1.f;
	if (c.drumMicWidth != 0.f) {
		const float dw = c.drumMicWidth;
		const float dwP = dw > 0.f ? (dw > 1.f ? 1.f : dw) : 0.f;
		const float dwN = dw < 0.f ? (dw < -1.f ? 1.f : -dw) : 0.f;
		dll = sqrtf (1.f - dwP);
		dlr = sqrtf (0.f + dwP);
		drl = sqrtf (0.f + dwN);
		drr = sqrtf (1.f - dwN);
	}
	if (c.hornMicWidth != 0.f) {
		const float hw = c.hornMicWidth;
		const float hwP = hw > 0.f ? (hw > 1.f ? 1.f : hw) : 0.f;
		const float hwN = hw < 0.f ? (hw < -1.f ? 1.f : -hw) : 0.f;
		hll = sqrtf (1.f - hwP);
		hlr = sqrtf (0.f + hwP);
		hrl = sqrtf (0.f + hwN);
		hrr = sqrtf (1.f - hwN);
	}
	const float mic[8] = {hll, hlr, dll, dlr, hrl, hrr, drl, drr};
	memcpy (k.mic, mic, sizeof (mic));
	/* HN_MOTION / DR_MOTION angle offsets (src/whirl.cpp:1396-1400) */
	k.fwAng = c.micAngle * .25;
	k.bwAng = 1. + c.micAngle * -.25;
	k.deadzone = (.05 / (60.f * wt.sr));
	memcpy (k.revHorn, wt.revHorn, sizeof (k.revHorn));
	memcpy (k.revDrum, wt.revDrum, sizeof (k.revDrum));
	k.hnHardstop = (float)(10.f / (60.f * wt.sr));
	k.drHardstop = (float)(8.f / (60.f * wt.sr));
	k.minspeed   = (float)(3.f / (60.f * wt.sr));
	k.hnLimit    = (float)(60.f / (60. * wt.sr));
	k.drLimit    = (float)(100.f / (60. * wt.sr));
	k.sr         = wt.sr;
}

/* preamp per-block constants, src/overdrive.cpp:64-84 and the density/out loops */
static void odCtlCompute (const Instance& in, double sr, tbf_seg_ctl& c)
{
	double overallscale = 1.0;
	overallscale /= 44100.0;
	overallscale *= sr;
	double density = in.odA * 4.0;
	c.odIir        = pow (in.odB, 3) / overallscale;
	c.odOutput     = in.odC;
	c.odWet        = in.odD;
	c.odDry        = 1.0 - c.odWet;
	double out     = fabs (density);
	density        = density * fabs (density);
	double count   = density;
	int    iter    = 0;
	while (count > 1.0) {
		iter++;
		count = count - 1.0;
	}
	while (out > 1.0)
		out = out - 1.0;
	c.odIter       = iter;
	c.odOut        = out;
	c.odDensityPos = density > 0 ? 1u : 0u;
	c.odClean      = (uint32_t)in.odClean;
}

/* the preamp fields of a control entry, recomputed only when the preamp parameters changed
 * (the pow above costs more than the rest of a dense-event step per instance and block) */
static void odCtl (Instance& in, double sr, tbf_seg_ctl& c)
{
	Instance::OdCache& k = in.odc;
	if (!k.valid || k.A != in.odA || k.B != in.odB || k.C != in.odC || k.D != in.odD || k.clean != in.odClean) {
		odCtlCompute (in, sr, k.ctl);
		k.A     = in.odA;
		k.B     = in.odB;
		k.C     = in.odC;
		k.D     = in.odD;
		k.clean = in.odClean;
		k.valid = true;
	}
	c.odIir        = k.ctl.odIir;
	c.odOutput     = k.ctl.odOutput;
	c.odWet        = k.ctl.odWet;
	c.odDry        = k.ctl.odDry;
	c.odIter       = k.ctl.odIter;
	c.odOut        = k.ctl.odOut;
	c.odDensityPos = k.ctl.odDensityPos;
	c.odClean      = k.ctl.odClean;
}

/* fsetCharacter (src/overdrive.cpp:547-574): character A and the linear-segment output
 * level C */
void tbf::setCharacter (Instance& in, float value)
{
	static const double Aval[5] = {0.0, 0.25, 0.50, 0.75, 1.00};
	static const double Cval[5] = {1.0, 0.70, 0.25, 0.15, 0.13};
	in.odA                      = value;
	for (int q = 0; q < 4; q++)
		if (value <= Aval[q + 1]) {
			float a = (float)Aval[q], b = (float)Aval[q + 1], p = (float)Cval[q], qq = (float)Cval[q + 1];
			in.odC  = p + (value - a) * (qq - p) / (b - a);
			break;
		}
	in.ctlDirty = true;
}

/* the engine-wide tables the cfg shapes: whirl displacement / IR tables, filters and
 * speeds (initWhirl, src/whirl.cpp:956-986), the compact ring window derived from the
 * geometry, the scanner's offset tables and stator increment (init_vibrato,
 * src/vibrato.cpp:312-317) */
static int buildShared (tbf_engine* e)
{
	const double sr = e->cfg.sample_rate;
	e->wt.build (sr, e->conf);
	/* compact whirl ring: live window < maxAhead + 2 + one sub-block */
	uint32_t W = 512;
	while ((float)W < e->wt.maxAhead + 2.0f + TBF_SUB + 2.0f)
		W *= 2;
	if (W > 2048)
		return fail (-22, "whirl write-ahead exceeds the reference ring (2048 samples): geometry out of range");
	e->wringLen = W;
	/* vibrato tables (src/vibrato.cpp:91-95, 224-251) */
	e->vibTab.resize (3 * 2048);
	const double amp[3] = {e->conf.vib1OffAmp, e->conf.vib2OffAmp, e->conf.vib3OffAmp};
	for (int t = 0; t < 3; t++)
		for (int i = 0; i < 2048; i++) {
			double m                = sin ((2.0 * M_PI * i) / 2048);
			e->vibTab[t * 2048 + i] = (unsigned int)((1.0 + amp[t] + (m * amp[t])) * 65536.0);
		}
	e->statorInc = (unsigned int)(((e->conf.vibFqHertz * 2048) / sr) * 65536.0);
	return 0;
}

/* host worker threads for per-template work: the process's lease (OMP_NUM_THREADS, set
 * on the GPU boxes) or the hardware, at most TBF_MAX_HOST_THREADS (scanChunk sizes its
 * per-range stack arrays by it) */
#define TBF_MAX_HOST_THREADS 16u
static unsigned hostThreads ()
{
	unsigned    t   = std::thread::hardware_concurrency ();
	const char* omp = getenv ("OMP_NUM_THREADS");
	const char* ht  = getenv ("TBF_HOST_THREADS");
	if (ht && atoi (ht) > 0)
		t = (unsigned)atoi (ht);
	else if (omp && atoi (omp) > 0)
		t = (unsigned)atoi (omp);
	return std::max (1u, std::min (t, TBF_MAX_HOST_THREADS));
}

/* A persistent pool of hostThreads () - 1 workers (the caller is the last): a dense-event
 * chunk runs several parallel sections, and creating 16 threads for each cost ~0.3-0.8 ms.
 * One job at a time (the mutex), so engines driven from several host threads share it.
 * A job ends when its tasks are done, not when every worker has woken: each job is its own
 * object, so a worker the OS schedules late finds that job's tasks taken and leaves it. */
class HostPool {
  public:
	static HostPool& get ()
	{
		static HostPool p;
		return p;
	}
	void run (uint32_t n, const std::function<void (uint32_t)>& f)
	{
		std::lock_guard<std::mutex> job (jobM);
		auto                        j = std::make_shared<Job> ();
		j->fn                         = &f;
		j->cnt                        = n;
		{
			std::lock_guard<std::mutex> g (m);
			cur = j;
			gen++;
		}
		cv.notify_all ();
		work (*j);
		std::unique_lock<std::mutex> g (m);
		done.wait (g, [&] { return j->finished.load () == n; });
		cur.reset ();
	}
	unsigned workers () const { return (unsigned)th.size () + 1; }

  private:
	struct Job {
		const std::function<void (uint32_t)>* fn  = nullptr;
		uint32_t                              cnt = 0;
		std::atomic<uint32_t>                 next {0}, finished {0};
	};
	HostPool ()
	{
		const unsigned nt = hostThreads ();
		for (unsigned k = 1; k < nt; k++)
			th.emplace_back ([this] { loop (); });
	}
	~HostPool ()
	{
		{
			std::lock_guard<std::mutex> g (m);
			quit = true;
		}
		cv.notify_all ();
		for (auto& t : th)
			t.join ();
	}
	void work (Job& j)
	{
		for (uint32_t t; (t = j.next.fetch_add (1)) < j.cnt;) {
			(*j.fn) (t);
			if (j.finished.fetch_add (1) + 1 == j.cnt) {
				std::lock_guard<std::mutex> g (m);
				done.notify_all ();
			}
		}
	}
	void loop ()
	{
		uint64_t seen = 0;
		for (;;) {
			std::shared_ptr<Job> j;
			{
				std::unique_lock<std::mutex> g (m);
				cv.wait (g, [&] { return quit || gen != seen; });
				if (quit)
					return;
				seen = gen;
				j    = cur;
			}
			if (j)
				work (*j);
		}
	}
	std::vector<std::thread> th;
	std::mutex               m, jobM;
	std::condition_variable  cv, done;
	std::shared_ptr<Job>     cur;
	uint64_t                 gen  = 0;
	bool                     quit = false;
};

/* run f(t) for t < n on up to hostThreads () threads */
template <typename F>
static void parallelFor (uint32_t n, F f)
{
	if (n <= 1 || hostThreads () <= 1) {
		for (uint32_t t = 0; t < n; t++)
			f (t);
		return;
	}
	const std::function<void (uint32_t)> g (f);
	HostPool::get ().run (n, g);
}

extern "C" {

int tbf_abi_version (void) { return TBF_ABI_VERSION; }
const char* tbf_last_error (void) { return g_err.c_str (); }

int tbf_engine_create (const tbf_engine_config* cfg, tbf_engine** out)
{
	if (!cfg || !out)
		return fail (-22, "null argument");
	if (!(cfg->sample_rate >= 8000.0 && cfg->sample_rate <= 192000.0))
		return fail (-22, "sample_rate out of range");
	/* device -1: host-only engine (table builders and control plane; render refuses) */
	if (cfg->device != -1) {
		int ndev = 0;
		if (hipGetDeviceCount (&ndev) != hipSuccess || ndev <= 0)
			return fail (-19, "no HIP device available");
		if (cfg->device < 0 || cfg->device >= ndev)
			return fail (-19, "device ordinal out of range");
	}
	std::unique_ptr<tbf_engine> e (new tbf_engine ());
	e->cfg = *cfg;
	if (cfg->device >= 0) {
		HIPCHK (hipSetDevice (cfg->device));
		/* stream creation order matters: the process has GPU_MAX_HW_QUEUES (4) hardware
		 * queues and streams take them round-robin at creation.  The engine's own stream
		 * first, then the three stage-group streams: a caller's stream created after the
		 * engine shares the engine stream's queue (idle when the caller passes its
		 * stream); one created before shares the last stage group's, whose work the
		 * caller's stream waits for anyway.  A stage group's queue shared with the
		 * caller's stream would order the group's next launches behind the caller's
		 * end-of-call wait (measured with a fifth engine stream: steady step 6.7 -> 8.1 ms) */
		HIPCHK (hipStreamCreateWithFlags (&e->stream, hipStreamNonBlocking));
		if (const char* pg = getenv ("TBF_PIPE_GROUPS")) { /* "g0,...,g5": groups 0..5, non-decreasing, from 0 */
			/* stages 0 and 1 always share a stream: the tonegen-only chain's mixFixed flags
			 * (one buffer for every chunk) are written by k_tonegen and read by k_mixpre */
			for (int k = 0; k < TBF_NSTAGES && *pg; k++) {
				const int g = atoi (pg);
				if (g >= 0 && g < TBF_NSTAGES && (k == 0 ? g == 0 : k == 1 ? g == e->grp[0] : (g >= e->grp[k - 1] && g <= e->grp[k - 1] + 1)))
					e->grp[k] = g;
				while (*pg && *pg != ',')
					pg++;
				if (*pg == ',')
					pg++;
			}
		}
		/* stage-group stream priorities (TBF_GROUP_PRIO="p0,p1,...": HIP stream priorities,
		 * lower = higher, clamped to the device's range; default: the reverb group high).
		 * The reverb group is the step's critical path (k_rv_pre -> k_rv_core_lds ->
		 * k_rv_post, ~65 ms alone per 2048 blocks against ~46 for k_tonegen + k_mixpre and ~37
		 * for k_whirl); at equal priority the other groups' workgroups took the CUs first
		 * and k_rv_pre ran 4x slower than alone (tools/timeline.py, profiles/r05/s23) */
		int pLeast = 0, pGreatest = 0;
		HIPCHK (hipDeviceGetStreamPriorityRange (&pLeast, &pGreatest));
		int prio[TBF_NSTAGES] = {0, 0, 0, 0, 0, 0};
		if (e->grp[2] == e->grp[3] && e->grp[3] == e->grp[4] && e->grp[2] != e->grp[1] && e->grp[4] != e->grp[5])
			prio[e->grp[2]] = pGreatest;
		if (const char* gp = getenv ("TBF_GROUP_PRIO"))
			for (int g = 0; g < TBF_NSTAGES && *gp; g++) {
				prio[g] = atoi (gp);
				while (*gp && *gp != ',')
					gp++;
				if (*gp == ',')
					gp++;
			}
		for (int g = 0; g <= e->grp[TBF_NSTAGES - 1]; g++) {
			const int p = std::min (std::max (prio[g], std::min (pLeast, pGreatest)), std::max (pLeast, pGreatest));
			HIPCHK (hipStreamCreateWithPriority (&e->gs[g], hipStreamNonBlocking, p));
		}
		for (int k = 0; k < TBF_NSTAGES; k++) {
			HIPCHK (hipEventCreateWithFlags (&e->sdone[k], hipEventDisableTiming));
			for (int p = 0; p < 4; p++)
				HIPCHK (hipEventCreateWithFlags (&e->pev[p][k], hipEventDisableTiming));
		}
		HIPCHK (hipEventCreateWithFlags (&e->sjoin, hipEventDisableTiming));
		/* TBF_RV_LDS=0: the streaming reverb core (k_rv_core) instead of k_rv_core_lds */
		if (const char* rl = getenv ("TBF_RV_LDS"))
			e->rvLdsOn = rl[0] != '0';
		/* k_rv_core_lds runs one persistent workgroup per CU (TBF_RV_PERSIST=0: one per
		 * instance and channel, the round-2 grid) */
		int ncu = 0;
		HIPCHK (hipDeviceGetAttribute (&ncu, hipDeviceAttributeMultiprocessorCount, cfg->device));
		if (const char* ts = getenv ("TBF_TG_SPLIT"))
			e->tgSplit = atoi (ts);
		if (const char* sc = getenv ("TBF_STEADY_CHUNK")) /* A/B: blocks per chunk without deltas */
			e->steadyChunk = (uint32_t)std::min (std::max (atoi (sc), TBF_CHUNK), TBF_STEADY_MAX);
		const char* rp = getenv ("TBF_RV_PERSIST"); /* 0: per-pair grid; n > 0: n workgroups */
		e->rvGrid      = rp ? (uint32_t)std::max (atoi (rp), 0) : (uint32_t)std::max (ncu, 1);
		if (e->rvWork.ensure (1))
			return fail (-12, "out of device memory");
		HIPCHK (hipEventCreateWithFlags (&e->upEv, hipEventDisableTiming));
		HIPCHK (hipEventCreateWithFlags (&e->upEvB, hipEventDisableTiming));
		const char* pl = getenv ("TBF_PIPELINE");
		e->pipeline    = !(pl && pl[0] == '0');
		/* TBF_HOST_CONTROL=1: the per-wheel tone-generator control on the host (the
		 * reference path for A/B); default: on the device (k_tgctl) */
		const char* hc = getenv ("TBF_HOST_CONTROL");
		e->devCtl      = !(hc && hc[0] == '1');
		const char* hs = getenv ("TBF_HOST_SERIAL"); /* the serial loop (A/B); TBF_HOST_THREADS: workers */
		e->parCtl      = !(hs && hs[0] == '1');
		const char* df = getenv ("TBF_DEVICE_FRONT"); /* 0: note-only chunks step on the host too (A/B) */
		e->frontOn     = !(df && df[0] == '0');
		if (const char* sp = getenv ("TBF_WHIRL_SPLIT")) /* 0 / 1: k_whirl / k_whirl_split always */
			e->whSplit = sp[0] != '0' ? 1 : 0;
		e->nCU = (uint32_t)std::max (ncu, 1);
		if (const char* fm = getenv ("TBF_FRONT_MIN")) /* events a chunk needs for the device front end */
			e->frontMin = (uint32_t)std::max (atoi (fm), 1);
	}
	if (int rc = buildShared (e.get ()))
		return rc;
	*out = e.release ();
	return 0;
}

int tbf_engine_destroy (tbf_engine* e)
{
	if (!e)
		return 0;
	if (e->cfg.device >= 0)
		(void)hipSetDevice (e->cfg.device);
	if (e->stream)
		(void)hipStreamSynchronize (e->stream);
	for (hipStream_t q : e->gs)
		if (q)
			(void)hipStreamSynchronize (q);
	e->bank.release ();
	e->tplDesc.release ();
	e->cst.release ();
	e->st.release ();
	e->wring.release ();
	e->rslab.release ();
	e->ctl.release ();
	e->prog.release ();
	e->tgc.release ();
	e->drec.release ();
	e->dmsg.release ();
	e->dctlInst.release ();
	e->drecB.release ();
	e->dmsgB.release ();
	e->dgain.release ();
	e->dgainB.release ();
	e->dwh.release ();
	e->dwhB.release ();
	e->dctlInstB.release ();
	e->dfull.release ();
	e->dfullB.release ();
	e->dfront.release ();
	e->dfrontB.release ();
	e->dfev.release ();
	e->dfevB.release ();
	e->dfval.release ();
	e->dfvalB.release ();
	e->dfoff.release ();
	e->dfoffB.release ();
	e->dkeyComp.release ();
	e->dident.release ();
	e->coff.release ();
	e->contrib.release ();
	e->vib.release ();
	e->xsj.release ();
	e->whTab.release ();
	e->whBw.release ();
	e->err.release ();
	e->outL.release ();
	e->outR.release ();
	e->mid0.release ();
	e->mid1.release ();
	e->mid2.release ();
	e->rvA.release ();
	e->rvB.release ();
	e->rvWork.release ();
	e->mixFixed.release ();
	if (e->stream)
		(void)hipStreamDestroy (e->stream);
	for (hipStream_t q : e->gs)
		if (q)
			(void)hipStreamDestroy (q);
	for (int k = 0; k < TBF_NSTAGES; k++) {
		if (e->sdone[k])
			(void)hipEventDestroy (e->sdone[k]);
		for (int p = 0; p < 4; p++)
			if (e->pev[p][k])
				(void)hipEventDestroy (e->pev[p][k]);
	}
	if (e->sjoin)
		(void)hipEventDestroy (e->sjoin);
	for (hipEvent_t ev : {e->upEv, e->upEvB})
		if (ev)
			(void)hipEventDestroy (ev);
	delete e;
	return 0;
}

int tbf_template_create (tbf_engine* e, const double* mts128, const double* ratio9, uint32_t seed, uint32_t* id)
{
	if (!e || !id)
		return fail (-22, "null argument");
	std::unique_ptr<TgTemplate> t (new TgTemplate ());
	t->build (e->cfg.sample_rate, mts128, ratio9, seed, e->conf);
	*id = (uint32_t)e->tpls.size ();
	e->tpls.push_back (std::move (t));
	e->deviceReady = false;
	return 0;
}

int tbf_templates_create (tbf_engine* e, uint32_t n, const double* mts128, const double* ratio9, const uint32_t* seeds,
                          uint32_t* ids)
{
	if (!e || (n && (!seeds || !ids)))
		return fail (-22, "null argument");
	if (!e->stream)
		return fail (-19, "device template construction needs a device engine");
	if (n == 0)
		return 0;
	HIPCHK (hipSetDevice (e->cfg.device));
	const double                             sr = e->cfg.sample_rate;
	std::vector<std::unique_ptr<TgTemplate>> ts (n);
	std::vector<uint32_t>                    E (61 * (size_t)n);
	std::vector<uint64_t>                    total (n), base (n);
	std::vector<tbf_tpl_wheel>               wh ((size_t)n * TBF_NW);
	uint64_t                                 sum = 0;
	uint32_t                                 maxChunks = 0, maxLen = 0;
	/* the play matrices on the device (k_tpl_matrix) unless TBF_HOST_MATRIX=1 (A/B: the
	 * host builder of tbf_template_create, one template per host thread) */
	const char* hm         = getenv ("TBF_HOST_MATRIX");
	const bool  hostMatrix = hm && atoi (hm) != 0;
	/* the rand-free tables of each template (frequencies, wheel lengths and spectra) and
	 * its rand() window, one template per host thread */
	parallelFor (n, [&] (uint32_t t) {
		ts[t].reset (new TgTemplate ());
		ts[t]->prepare (sr, mts128 ? mts128 + 128 * (size_t)t : nullptr, ratio9 ? ratio9 + 9 * (size_t)t : nullptr,
		                e->conf, hostMatrix);
		uint32_t  W[31];
		GlibcRand rnd (seeds[t]);
		rnd.window (W);
		gr_extend (W, &E[61 * (size_t)t]);
	});
	for (uint32_t t = 0; t < n; t++) {
		TgTemplate& T = *ts[t];
		total[t] = T.total;
		base[t]  = sum;
		sum += T.total;
		maxChunks = std::max (maxChunks, (uint32_t)((T.total + 511) / 512));
		for (int i = 1; i <= TBF_NW; i++) {
			tbf_tpl_wheel& w = wh[(size_t)t * TBF_NW + i - 1];
			memset (&w, 0, sizeof (w));
			w.off = T.off[i];
			w.len = T.len[i];
			w.np  = T.nPartials[i];
			w.U   = T.U[i];
			for (int q = 0; q < w.np; q++) {
				w.amp[q] = T.pAmp[i][q];
				w.hz[q]  = T.pHz[i][q];
			}
			maxLen = std::max (maxLen, w.len);
		}
	}
	DevBuf<uint32_t>      dE;
	DevBuf<uint64_t>      dTot, dBase;
	DevBuf<tbf_tpl_wheel> dWh;
	DevBuf<uint8_t>       dLsb;
	DevBuf<float>         dBank;
	/* play matrix: the cfg-only inputs, each template's frequencies and bus ratios */
	MatrixInputs          mi;
	const size_t          nk = (size_t)n * 384;
	std::vector<double>   fr, ra;
	DevBuf<tbf_le>        dTm, dTp, dXt;
	DevBuf<uint32_t>      dTmOff, dTpOff, dXtOff, dCnt, dOff;
	DevBuf<float>         dTaper;
	DevBuf<double>        dFr, dRa;
	DevBuf<tbf_contrib>   dStage, dOut;
	std::vector<uint32_t> hCnt, hOff;
	std::vector<Contrib>  hOut;
	if (!hostMatrix) {
		mi.build (e->conf);
		fr.resize ((size_t)n * TBF_NW);
		ra.resize ((size_t)n * 9);
		for (uint32_t t = 0; t < n; t++) {
			memcpy (&fr[(size_t)t * TBF_NW], ts[t]->frequency, TBF_NW * sizeof (double));
			memcpy (&ra[(size_t)t * 9], ts[t]->targetRatio, 9 * sizeof (double));
		}
		if (dTm.ensure (mi.tm.size ()) || dTp.ensure (mi.tp.size ()) || dXt.ensure (mi.xt.size ()) ||
		    dTmOff.ensure (mi.tmOff.size ()) || dTpOff.ensure (mi.tpOff.size ()) || dXtOff.ensure (mi.xtOff.size ()) ||
		    dTaper.ensure (128 * 9) || dFr.ensure (fr.size ()) || dRa.ensure (ra.size ()) || dCnt.ensure (nk) ||
		    dOff.ensure (nk + 1) || dStage.ensure (nk * mi.cap) || dOut.ensure (nk * mi.cap))
			return fail (-12, "device play matrix buffers");
	}
	auto releaseAll = [&] () {
		dE.release (), dTot.release (), dBase.release (), dWh.release (), dLsb.release (), dBank.release ();
		dTm.release (), dTp.release (), dXt.release (), dTmOff.release (), dTpOff.release (), dXtOff.release ();
		dTaper.release (), dFr.release (), dRa.release (), dCnt.release (), dOff.release (), dStage.release ();
		dOut.release ();
	};
	if (dE.ensure (E.size ()) || dTot.ensure (n) || dBase.ensure (n) || dWh.ensure (wh.size ()) || dLsb.ensure (sum) ||
	    dBank.ensure (sum)) {
		releaseAll ();
		return fail (-12, "device template buffers");
	}
	int rc = 0;
	std::vector<float> hb (sum);
	do {
		hipStream_t s = e->stream;
		if (hipMemcpyAsync (dE.p, E.data (), E.size () * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
		    hipMemcpyAsync (dTot.p, total.data (), n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
		    hipMemcpyAsync (dBase.p, base.data (), n * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
		    hipMemcpyAsync (dWh.p, wh.data (), wh.size () * sizeof (tbf_tpl_wheel), hipMemcpyHostToDevice, s) != hipSuccess) {
			rc = fail (-5, "template upload");
			break;
		}
		if (tbf_tpl_launch (n, maxChunks, maxLen, dE.p, dTot.p, dBase.p, dWh.p, dLsb.p, dBank.p, sr, s)) {
			rc = fail (-5, "template kernels");
			break;
		}
		if (!hostMatrix) {
			auto up = [&] (void* d, const void* h, size_t bytes) {
				return bytes == 0 || hipMemcpyAsync (d, h, bytes, hipMemcpyHostToDevice, s) == hipSuccess;
			};
			if (!up (dTm.p, mi.tm.data (), mi.tm.size () * sizeof (tbf_le)) ||
			    !up (dTp.p, mi.tp.data (), mi.tp.size () * sizeof (tbf_le)) ||
			    !up (dXt.p, mi.xt.data (), mi.xt.size () * sizeof (tbf_le)) ||
			    !up (dTmOff.p, mi.tmOff.data (), mi.tmOff.size () * 4) ||
			    !up (dTpOff.p, mi.tpOff.data (), mi.tpOff.size () * 4) ||
			    !up (dXtOff.p, mi.xtOff.data (), mi.xtOff.size () * 4) || !up (dTaper.p, mi.taper, sizeof (mi.taper)) ||
			    !up (dFr.p, fr.data (), fr.size () * 8) || !up (dRa.p, ra.data (), ra.size () * 8)) {
				rc = fail (-5, "play matrix upload");
				break;
			}
			const tbf_tpl_mx mx = {dTm.p,    dTmOff.p,    dTp.p,       dTpOff.p,    dXt.p, dXtOff.p,
			                       dTaper.p, mi.wiringXT, mi.floor, mi.minLevel, mi.cap};
			hCnt.resize (nk);
			hOff.resize (nk + 1);
			if (tbf_tpl_matrix_launch (n, &mx, dFr.p, dRa.p, dStage.p, dCnt.p, dOff.p, dOut.p, s)) {
				rc = fail (-5, "play matrix kernels");
				break;
			}
			if (hipMemcpyAsync (hCnt.data (), dCnt.p, nk * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
			    hipMemcpyAsync (hOff.data (), dOff.p, (nk + 1) * 4, hipMemcpyDeviceToHost, s) != hipSuccess) {
				rc = fail (-5, "play matrix download");
				break;
			}
		}
		if (hipMemcpyAsync (hb.data (), dBank.p, sum * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
		    hipStreamSynchronize (s) != hipSuccess) {
			rc = fail (-5, "template download");
			break;
		}
		if (!hostMatrix) {
			for (size_t q = 0; q < nk; q++)
				if (hCnt[q] > mi.cap) {
					rc = fail (-5, "play matrix list longer than its staging");
					break;
				}
			if (rc)
				break;
			static_assert (sizeof (Contrib) == sizeof (tbf_contrib), "Contrib is tbf_contrib's layout");
			hOut.resize (hOff[nk]);
			if ((hOff[nk] && hipMemcpyAsync (hOut.data (), dOut.p, hOff[nk] * sizeof (Contrib), hipMemcpyDeviceToHost,
			                                 s) != hipSuccess) ||
			    hipStreamSynchronize (s) != hipSuccess) {
				rc = fail (-5, "play matrix download");
				break;
			}
		}
	} while (0);
	releaseAll ();
	if (rc)
		return rc;
	parallelFor (n, [&] (uint32_t t) {
		TgTemplate& T = *ts[t];
		if (!hostMatrix)
			for (int k = 0; k < 384; k++) {
				const size_t q = (size_t)t * 384 + k;
				T.keyContrib[k].assign (hOut.begin () + hOff[q], hOut.begin () + hOff[q + 1]);
			}
		T.bank.assign (hb.begin () + base[t], hb.begin () + base[t] + total[t]);
		GlibcRand rnd (seeds[t]);
		rnd.discard (T.total); /* the draws of the bank */
		T.finish (rnd);
	});
	for (uint32_t t = 0; t < n; t++) {
		ids[t] = (uint32_t)e->tpls.size ();
		e->tpls.push_back (std::move (ts[t]));
	}
	e->deviceReady = false;
	return 0;
}

int tbf_template_bank (tbf_engine* e, uint32_t tid, float* out, uint64_t cap, uint32_t* lens)
{
	if (!e || tid >= e->tpls.size ())
		return fail (-22, "bad template id");
	const TgTemplate& t = *e->tpls[tid];
	if (lens)
		for (int i = 1; i <= TBF_NW; i++)
			lens[i - 1] = t.len[i];
	if (out) {
		if (cap < t.bank.size ())
			return fail (-28, "buffer too small");
		memcpy (out, t.bank.data (), t.bank.size () * sizeof (float));
	}
	return (int)t.bank.size ();
}

/* the CLAP parameters' default values (clap_plugin_params get_info, src/clap.cpp:383-545;
 * the plugin's init copies them into its parameter array, 1062-1067) */
static void clapParamDefaults (double* params)
{
	static const float drawbar[9] = {7.0f, 8.0f, 8.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
	static const float top[9] = {1, 3, 1, 2, 3, 4, 5, 6, 8}, bottom[9] = {2, 2, 1, 1, 1, 1, 1, 1, 1};
	for (int i = 0; i < 64; i++)
		params[i] = 0.0;
	for (int i = 0; i < 9; i++) {
		params[TBF_P_DRAWBAR_MIN + i] = drawbar[i];
		params[20 + i]                = top[i];    /* P_RATIO_TOP_MIN */
		params[29 + i]                = bottom[i]; /* P_RATIO_BOTTOM_MIN */
	}
	params[TBF_P_DRUM]   = 1.0f;
	params[TBF_P_HORN]   = 1.0f;
	params[TBF_P_REVERB] = 0.1f;
}

int tbf_instances_add (tbf_engine* e, uint32_t n, const uint32_t* tpl_ids, const uint32_t* seeds, uint32_t* first)
{
	if (!e || (n && (!tpl_ids || !seeds)))
		return fail (-22, "null argument");
	const double sr = e->cfg.sample_rate;
	if (first)
		*first = (uint32_t)e->inst.size ();
	for (uint32_t q = 0; q < n; q++) {
		if (tpl_ids[q] >= e->tpls.size ())
			return fail (-22, "bad template id");
		e->inst.emplace_back ();
		Instance& in = e->inst.back ();
		in.tpl       = tpl_ids[q];
		in.ctlRand   = GlibcRand (seeds[q] ^ 0x5bd1e995u);
		memset (&in.k, 0, sizeof (in.k));
		memset (&in.s0, 0, sizeof (in.s0));
		memset (&in.ctl, 0, sizeof (in.ctl));
		clapParamDefaults (in.params);
		in.k.tpl = in.tpl;
		/* allocSynth order: allocReverb (rand x16 vib phases, fpdL, fpdR), allocWhirl,
		 * allocTonegen, allocPreamp (rand fpd)  -- b_synth/lv2.cpp:336-353 */
		GlibcRand rnd (seeds[q]);
		for (int c = 0; c < 2; c++)
			for (int l = 0; l < 8; l++)
				in.s0.rv.ch[c].vib[l] = rnd.next () - 2147483647 / 2;
		uint32_t f = 1;
		while (f < 16386)
			f = (uint32_t)rnd.next () * 0xFFFFFFFFu;
		in.s0.rv.fpdL = f;
		f          = 1;
		while (f < 16386)
			f = (uint32_t)rnd.next () * 0xFFFFFFFFu;
		in.s0.rv.fpdR = f;
		in.s0.rv.fpdL2 = in.s0.rv.fpdL;
		in.s0.rv.fpdR2 = in.s0.rv.fpdR;
		f          = 1;
		while (f < 16386)
			f = (uint32_t)rnd.next () * 0xFFFFFFFFu;
		in.s0.mo.odFpd  = f;
		in.s0.mo.fpFlip = 1;
		in.s0.rv.pdAge = 0; /* countM = 1 and zeroed rings: the first delayM outputs are 0 */
		in.s0.rv.pdPos = 0;
		for (int c = 0; c < 2; c++)
			for (int l = 0; l < 12; l++)
				in.s0.rv.ch[c].count[l] = 1;
		reverbConsts (in.k, sr, 1.0f, 0.2f, 0.0f, 0.0f, 0.4f, 0.8f);
		if (in.k.delay[12] < 0 || in.k.delay[12] >= TBF_PD_HIST) /* 560 at the fixed settings */
			return fail (-22, "predelay longer than its history");
		whirlConsts (in.k, e->wt, e->conf);
		in.whr.init (e->wt.sr, e->conf); /* the runtime whirl parameters, as the cfg left them */
		in.s0.wh.prm = in.whr.cur;
		in.rvG      = e->conf.reverbMix;  /* reverbConfig: setReverbMix */
		in.whBypass = e->conf.bypass;     /* whirlConfig: whirl.bypass */
		/* initWhirl -> computeRotationSpeeds -> setRevSelect(revSelect) ->
		 * useRevOption(revselects[revSelect]), revselects = {4, 0, 8} (src/whirl.cpp:226-293) */
		static const int revselects[3] = {4, 0, 8};
		const int        rs            = revselects[((e->conf.revSelect % 3) + 3) % 3];
		in.revSelect                   = ((e->conf.revSelect % 3) + 3) % 3;
		tbf_wh_state& w  = in.s0.wh;
		w.hornTarget     = e->wt.revHorn[rs];
		w.drumTarget     = e->wt.revDrum[rs];
		w.hornAcDc       = w.hornIncr < w.hornTarget ? 1 : (w.hornTarget < w.hornIncr ? -1 : 0);
		w.drumAcDc       = w.drumIncr < w.drumTarget ? 1 : (w.drumTarget < w.drumIncr ? -1 : 0);
		/* tonegen + vibrato runtime state (initToneGenerator, reset_vibrato) */
		in.s0.mo.keyCompLevel = 1.0f;
		in.s0.mo.percEnvGain  = 0.0f;
		in.s0.tg.outPos       = 1023 / 2;
		in.tg.init (e->tpls[in.tpl].get (), e->conf);
		if (e->slabLen == 0) {
			e->slabLen  = in.k.slabLen;
			e->rvLdsFit = tbf_rv_lds_fits (&in.k) != 0; /* same geometry for every instance */
		} else if (e->slabLen != in.k.slabLen)
			return fail (-22, "inconsistent reverb geometry");
	}
	e->deviceReady = false;
	e->actAll      = true;
	return 0;
}

uint32_t tbf_instance_count (const tbf_engine* e) { return e ? (uint32_t)e->inst.size () : 0; }

int tbf_instance_retune (tbf_engine* e, uint32_t i, uint32_t tpl_id)
{
	if (!e || i >= e->inst.size ())
		return fail (-22, "bad instance");
	if (tpl_id >= e->tpls.size ())
		return fail (-22, "bad template id");
	Instance&          in         = e->inst[i];
	const unsigned int newRouting = in.tg.newRouting;
	/* reinitToneGen (src/clap.cpp:129-157): allocTonegen + initToneGenerator + init_vibrato
	 * on the new tables ... */
	in.tpl   = tpl_id;
	in.k.tpl = tpl_id;
	in.tg.init (e->tpls[tpl_id].get (), e->conf);
	/* ... setToneGenParam (108-121) for the drawbars, vibrato switch and type from the
	 * parameter values (float) ... */
	for (int b = 0; b < 9; b++)
		in.tg.setDrawBar (b, (unsigned)rintf ((float)in.params[TBF_P_DRAWBAR_MIN + b]));
	in.tg.setVibratoUpper ((int)rintf ((float)in.params[TBF_P_VIBRATO]));
	in.tg.setVibratoFromInt ((int)floorf ((float)in.params[TBF_P_VIBRATO_TYPE]));
	/* ... and the routing word kept */
	in.tg.newRouting = newRouting;
	/* the device side: the instance's tone-generator + scanner state (wheel positions, key
	 * compression, percussion envelope and high-pass, stator, scanner ring) starts fresh
	 * at the next block; the preamp fields of tbf_mo_state, reverb and whirl go on */
	tbf_tg_state& g = in.s0.tg;
	memset (&g, 0, sizeof (g));
	g.outPos                = 1023 / 2;
	in.s0.mo.keyCompLevel = 1.0f;
	in.s0.mo.percEnvGain  = 0.0f;
	if (std::find (e->retuned.begin (), e->retuned.end (), i) == e->retuned.end ())
		e->retuned.push_back (i);
	in.progDirty = in.ctlDirty = true;
	markActive (e, i);
	return 0;
}

int tbf_note (tbf_engine* e, uint32_t i, int32_t key, int32_t on)
{
	if (!e || i >= e->inst.size ())
		return fail (-22, "bad instance");
	if (key < 0 || key >= 384)
		return 0; /* oscKeyOn/Off ignore keys >= MAX_KEYS */
	if (on)
		e->inst[i].tg.keyOn (key);
	else
		e->inst[i].tg.keyOff (key);
	markActive (e, i);
	return 0;
}

int tbf_set_param (tbf_engine* e, uint32_t i, int32_t index, double v)
{
	if (!e || i >= e->inst.size ())
		return fail (-22, "bad instance");
	Instance& in    = e->inst[i];
	float     value = (float)v;
	markActive (e, i);
	if (index >= 0 && index < 64)
		in.params[index] = value;
	/* src/clap.cpp:108-121 setToneGenParam + 162-207 setParam */
	if (index >= TBF_P_DRAWBAR_MIN && index <= TBF_P_DRAWBAR_MAX)
		in.tg.setDrawBar (index, (unsigned)rint (value));
	else if (index == TBF_P_VIBRATO)
		in.tg.setVibratoUpper ((int)rint (value));
	else if (index == TBF_P_VIBRATO_TYPE)
		in.tg.setVibratoFromInt ((int)floor (value));
	else if (index == TBF_P_DRUM || index == TBF_P_HORN)
		in.revOpt = (int)(floor (in.params[TBF_P_DRUM]) + 3 * floor (in.params[TBF_P_HORN]));
	else if (index == TBF_P_OVERDRIVE)
		in.odClean = (int)rint (1.0f - value);
	else if (index == TBF_P_CHARACTER) {
		setCharacter (in, value);
	} else if (index == TBF_P_REVERB)
		in.rvG = value;
	else if (index == TBF_P_PERCUSSION)
		in.tg.setPercEnabled ((int)rint (value));
	else if (index == TBF_P_PERCUSSION_VOLUME)
		in.tg.setPercVolume ((int)(1 - rint (value)));
	else if (index == TBF_P_PERCUSSION_DECAY)
		in.tg.setPercFast ((int)rint (value));
	else if (index == TBF_P_PERCUSSION_HARMONIC)
		in.tg.setPercFirst ((int)rint (value));
	else if (index >= TBF_P_BUS_DRAWBAR_BASE && index < TBF_P_BUS_DRAWBAR_BASE + 27)
		in.tg.setDrawBar (index - TBF_P_BUS_DRAWBAR_BASE, (unsigned)rint (value));
	else if (index == TBF_P_VIBRATO_LOWER)
		in.tg.setVibratoLower ((int)rint (value));
	else if (index == TBF_P_SWELL) {
		unsigned char u      = (unsigned char)rint (value * 127.0);
		in.tg.swellPedalGain = (float)((in.tg.outputLevelTrim * ((double)u)) / 127.0);
	} else if (index == TBF_P_WHIRL_BYPASS)
		in.whBypass = (int)rint (value);
	else if (!(index >= 0 && index < 64))
		return fail (-22, "unknown parameter id");
	in.ctlDirty = true;
	return 0;
}

int tbf_config_set (tbf_engine* e, const char* key, const char* value)
{
	if (!e || !key || !value)
		return fail (-22, "null argument");
	Config c     = e->conf;
	int    scope = 0;
	int    rc    = configSet (c, key, value, &scope);
	if (rc == -1)
		return fail (-22, std::string ("bad value for ") + key + ": " + value);
	if (rc == 0)
		return 1; /* not a key of the hot path: ignored, as the reference ignores it */
	if ((scope & CFG_SHARED) && !e->inst.empty ())
		return fail (-16, std::string (key) + " shapes the engine-wide tables: set it before tbf_instances_add");
	const Config old = e->conf;
	e->conf          = c;
	if (scope & CFG_SHARED) {
		if (int r = buildShared (e)) {
			e->conf = old;
			(void)buildShared (e);
			return r;
		}
		e->deviceReady = false;
	}
	return 0;
}

int tbf_config_parse (tbf_engine* e, const char* text)
{
	if (!e || !text)
		return fail (-22, "null argument");
	/* parseConfigurationLine (src/cfgParser.cpp:94-160): `name = value`, '#' comments,
	 * surrounding blanks trimmed.  All or nothing: every line is validated into a copy of
	 * the configuration first, and the copy replaces the engine's only when all pass, so
	 * a caller that gets an error knows that no key took effect. */
	Config      c       = e->conf;
	int         applied = 0, line = 0, scope = 0;
	std::string sharedKey;
	const char* p = text;
	while (*p) {
		const char* q = p;
		while (*q && *q != '\n')
			q++;
		std::string ln (p, q);
		p = *q ? q + 1 : q;
		line++;
		const size_t h = ln.find ('#');
		if (h != std::string::npos)
			ln.resize (h);
		const size_t eq = ln.find ('=');
		auto trim = [] (std::string s) {
			const size_t a = s.find_first_not_of (" \t\r"), b = s.find_last_not_of (" \t\r");
			return a == std::string::npos ? std::string () : s.substr (a, b - a + 1);
		};
		if (trim (ln).empty ())
			continue;
		if (eq == std::string::npos)
			return fail (-22, "line " + std::to_string (line) + ": expected name=value (nothing applied)");
		const std::string k = trim (ln.substr (0, eq)), v = trim (ln.substr (eq + 1));
		int               sc = 0;
		const int         rc = configSet (c, k.c_str (), v.c_str (), &sc);
		if (rc == -1)
			return fail (-22, "line " + std::to_string (line) + ": bad value for " + k + ": " + v + " (nothing applied)");
		if (rc == 0)
			continue; /* not a key of the hot path: ignored, as the reference ignores it */
		if ((sc & CFG_SHARED) && sharedKey.empty ())
			sharedKey = k;
		scope |= sc;
		applied++;
	}
	if ((scope & CFG_SHARED) && !e->inst.empty ())
		return fail (-16, sharedKey + " shapes the engine-wide tables: set it before tbf_instances_add (nothing applied)");
	const Config old = e->conf;
	e->conf          = c;
	if (scope & CFG_SHARED) {
		if (int r = buildShared (e)) {
			e->conf = old;
			(void)buildShared (e);
			return r;
		}
		e->deviceReady = false;
	}
	return applied;
}

} /* extern "C" */

/* ------------------------------------------------------------------ device setup */
/* wait for all pipelined stage work (before the host touches device buffers) */
static int drainStages (tbf_engine* e)
{
	if (!e->stagesBusy)
		return 0;
	for (hipStream_t q : e->gs)
		if (q)
			HIPCHK (hipStreamSynchronize (q));
	e->stagesBusy = false;
	return 0;
}

/* make stream s wait for every pipelined stage launch so far */
static int joinStages (tbf_engine* e, hipStream_t s)
{
	if (!e->stagesBusy)
		return 0;
	for (hipStream_t q : e->gs) {
		if (!q)
			continue;
		HIPCHK (hipEventRecord (e->sjoin, q));
		HIPCHK (hipStreamWaitEvent (s, e->sjoin, 0));
	}
	e->stagesBusy = false;
	return 0;
}

/* the device program pool with room for `entries`; the persistent slots of the first
 * `keep` instances are carried over */
static int growProg (tbf_engine* e, size_t entries, uint32_t keep)
{
	if (entries <= e->prog.cap)
		return 0;
	if (e->prog.p) /* rare: let every launch that may read the old pool finish */
		HIPCHK (hipDeviceSynchronize ());
	e->stagesBusy = false;
	DevBuf<tbf_prog_entry> np;
	if (np.ensure (entries + entries / 4))
		return fail (-12, "out of device memory (programs)");
	if (keep && e->prog.p)
		HIPCHK (hipMemcpy (np.p, e->prog.p, PERSIST (keep) * sizeof (tbf_prog_entry), hipMemcpyDeviceToDevice));
	e->prog.release ();
	e->prog = std::move (np);
	return 0;
}

static int ensureDevice (tbf_engine* e)
{
	if (e->deviceReady)
		return 0;
	if (e->cfg.device < 0)
		return fail (-19, "host-only engine (device -1) cannot render");
	HIPCHK (hipSetDevice (e->cfg.device));
	HIPCHK (hipStreamSynchronize (e->stream));
	if (int rc = drainStages (e))
		return rc;
	const uint32_t n = (uint32_t)e->inst.size ();
	/* wave banks + template descriptors.  On the device each wheel's wave is followed by
	 * its first TBF_BLK samples again, so a block's 128 samples from any position < len
	 * are contiguous (the interpreter's wrap split, src/tonegen.cpp:3376-3402, becomes
	 * plain indexing: len >= 384 > 128, so a block wraps at most once) */
	size_t total = 0;
	for (auto& t : e->tpls)
		for (int w = 1; w <= TBF_NW; w++)
			total += t->len[w] + (t->len[w] ? TBF_BLK : 0);
	if (e->bank.ensure (total) || e->tplDesc.ensure (e->tpls.size ()))
		return fail (-12, "out of device memory (bank)");
	std::vector<tbf_tpl_desc> desc (e->tpls.size ());
	std::vector<float>        ext (total);
	size_t                    o = 0;
	for (size_t q = 0; q < e->tpls.size (); q++) {
		const TgTemplate& t = *e->tpls[q];
		memset (desc[q].off, 0, sizeof (desc[q].off));
		memset (desc[q].len, 0, sizeof (desc[q].len));
		for (int w = 1; w <= TBF_NW; w++) {
			const uint32_t L = t.len[w];
			desc[q].off[w]   = (uint32_t)o;
			desc[q].len[w]   = L;
			if (!L)
				continue;
			const float* src = t.bank.data () + t.off[w];
			std::copy (src, src + L, ext.begin () + o);
			for (uint32_t k = 0; k < TBF_BLK; k++)
				ext[o + L + k] = src[k % L];
			o += L + TBF_BLK;
		}
		memcpy (desc[q].attackEnv, t.attackEnv, sizeof (desc[q].attackEnv));
		memcpy (desc[q].releaseEnv, t.releaseEnv, sizeof (desc[q].releaseEnv));
	}
	HIPCHK (hipMemcpy (e->bank.p, ext.data (), total * sizeof (float), hipMemcpyHostToDevice));
	HIPCHK (hipMemcpy (e->tplDesc.p, desc.data (), desc.size () * sizeof (tbf_tpl_desc), hipMemcpyHostToDevice));
	if (e->devCtl) { /* the templates' play matrices (keyContrib) for k_tgctl */
		std::vector<uint32_t>    off (e->tpls.size () * 385);
		std::vector<tbf_contrib> ent;
		for (size_t q = 0; q < e->tpls.size (); q++)
			for (int k = 0; k <= 384; k++) {
				off[q * 385 + k] = (uint32_t)ent.size ();
				if (k < 384)
					for (const Contrib& c : e->tpls[q]->keyContrib[k])
						ent.push_back ({(uint16_t)c.wheel, (uint16_t)c.bus, c.level});
			}
		e->ctlNw = 1;
		for (const tbf_contrib& c : ent)
			e->ctlNw = std::max<uint32_t> (e->ctlNw, (uint32_t)c.wheel + 1u);
		std::vector<float> kc (e->tpls.size () * 128);
		for (size_t q = 0; q < e->tpls.size (); q++)
			memcpy (kc.data () + q * 128, e->tpls[q]->keyCompTable, 128 * sizeof (float));
		if (e->dkeyComp.ensure (std::max<size_t> (kc.size (), 1)))
			return fail (-12, "out of device memory (key compression tables)");
		if (!kc.empty ())
			HIPCHK (hipMemcpy (e->dkeyComp.p, kc.data (), kc.size () * sizeof (float), hipMemcpyHostToDevice));
		if (e->coff.ensure (off.size ()) || e->contrib.ensure (std::max<size_t> (ent.size (), 1)))
			return fail (-12, "out of device memory (play matrices)");
		HIPCHK (hipMemcpy (e->coff.p, off.data (), off.size () * 4, hipMemcpyHostToDevice));
		if (!ent.empty ())
			HIPCHK (hipMemcpy (e->contrib.p, ent.data (), ent.size () * sizeof (tbf_contrib), hipMemcpyHostToDevice));
	}
	/* shared tables */
	const bool errNew = e->err.p == nullptr; /* the path flags are cumulative from the first allocation */
	if (e->vib.ensure (e->vibTab.size ()) || e->whTab.ensure (4 * (size_t)TBF_WH_TSTRIDE) || e->whBw.ensure (e->wt.bw.size ()) ||
	    e->err.ensure (4))
		return fail (-12, "out of device memory (tables)");
	HIPCHK (hipMemcpy (e->vib.p, e->vibTab.data (), e->vibTab.size () * 4, hipMemcpyHostToDevice));
	{
		/* xorshift32 (src/overdrive.cpp:158-160, src/reverb.cpp:775-783) is linear over
		 * GF(2): state after k steps = XOR over the set bits j of the state of
		 * xorshift^k (1 << j).  Column k of row j holds that image, k = 0 .. 128. */
		std::vector<uint32_t> J (32 * TBF_XS_JUMP + 128 * TBF_XS_JUMP);
		xs_jump_table (J.data (), TBF_XS_JUMP);
		/* followed by its nibble-sliced form [8][16][TBF_XS_JUMP] (xs_nib_table) */
		xs_nib_table (J.data () + 32 * TBF_XS_JUMP, J.data (), TBF_XS_JUMP);
		if (e->xsj.ensure (J.size ()))
			return fail (-12, "out of device memory (tables)");
		HIPCHK (hipMemcpy (e->xsj.p, J.data (), J.size () * 4, hipMemcpyHostToDevice));
	}
	{ /* each displacement table followed by its entry 0, so the kernel reads an entry and
	   * its successor (wrapping at 16384) as one pair */
		std::vector<float> padded (4 * (size_t)TBF_WH_TSTRIDE, 0.0f);
		for (int t = 0; t < 4; t++) {
			std::copy (e->wt.displ.begin () + (size_t)t * 16384, e->wt.displ.begin () + (size_t)(t + 1) * 16384,
			           padded.begin () + (size_t)t * TBF_WH_TSTRIDE);
			padded[(size_t)t * TBF_WH_TSTRIDE + 16384] = e->wt.displ[(size_t)t * 16384];
		}
		HIPCHK (hipMemcpy (e->whTab.p, padded.data (), padded.size () * 4, hipMemcpyHostToDevice));
	}
	HIPCHK (hipMemcpy (e->whBw.p, e->wt.bw.data (), e->wt.bw.size () * 4, hipMemcpyHostToDevice));
	if (errNew)
		HIPCHK (hipMemset (e->err.p, 0, 16));
	/* per-instance buffers: new instances start from their initial state, existing
	 * instances keep their device state */
	const uint32_t old = e->devInst;
	if (n > old) {
		DevBuf<tbf_inst_state> nst;
		DevBuf<float>          nwr;
		DevBuf<double>         nsl;
		if (nst.ensure (n) || nwr.ensure ((size_t)n * 4 * e->wringLen) || nsl.ensure ((size_t)n * e->slabLen))
			return fail (-12, "out of device memory (instances)");
		if (old) {
			HIPCHK (hipMemcpy (nst.p, e->st.p, old * sizeof (tbf_inst_state), hipMemcpyDeviceToDevice));
			HIPCHK (hipMemcpy (nwr.p, e->wring.p, (size_t)old * 4 * e->wringLen * 4, hipMemcpyDeviceToDevice));
			HIPCHK (hipMemcpy (nsl.p, e->rslab.p, (size_t)old * e->slabLen * 8, hipMemcpyDeviceToDevice));
		}
		std::vector<tbf_inst_state> s0 (n - old);
		for (uint32_t i = old; i < n; i++)
			s0[i - old] = e->inst[i].s0;
		HIPCHK (hipMemcpy (nst.p + old, s0.data (), (n - old) * sizeof (tbf_inst_state), hipMemcpyHostToDevice));
		HIPCHK (hipMemset (nwr.p + (size_t)old * 4 * e->wringLen, 0, (size_t)(n - old) * 4 * e->wringLen * 4));
		HIPCHK (hipMemset (nsl.p + (size_t)old * e->slabLen, 0, (size_t)(n - old) * e->slabLen * 8));
		e->st.release ();
		e->wring.release ();
		e->rslab.release ();
		e->st    = std::move (nst);
		e->wring = std::move (nwr);
		e->rslab = std::move (nsl);
		std::vector<tbf_inst_const> k (n);
		for (uint32_t i = 0; i < n; i++)
			k[i] = e->inst[i].k;
		if (e->cst.ensure (n) || e->ctl.ensure (2 * CTL_REGION (n)) || e->ctlIdx.ensure (2 * (size_t)n * TBF_CHUNK))
			return fail (-12, "out of device memory (control)");
		e->ctlVer++; /* both regions' persistent entries need the new pool */
		/* program pool: the existing instances' persistent programs move along (the device
		 * control path keeps them only there); new instances start with empty ones */
		if (int rc = growProg (e, PERSIST (n) + (e->devCtl ? PERSIST (n) : DPROG_CAP (n)), old))
			return rc;
		HIPCHK (hipMemset (e->prog.p + PERSIST (old), 0, (PERSIST (n) - PERSIST (old)) * sizeof (tbf_prog_entry)));
		if (e->devCtl) {
			DevBuf<tbf_tgc_state> ng;
			if (ng.ensure (n))
				return fail (-12, "out of device memory (control state)");
			if (old)
				HIPCHK (hipMemcpy (ng.p, e->tgc.p, old * sizeof (tbf_tgc_state), hipMemcpyDeviceToDevice));
			HIPCHK (hipMemset (ng.p + old, 0, (n - old) * sizeof (tbf_tgc_state)));
			e->tgc.release ();
			e->tgc = std::move (ng);
		}
		e->persistStale = true;
		HIPCHK (hipMemcpy (e->cst.p, k.data (), n * sizeof (tbf_inst_const), hipMemcpyHostToDevice));
		e->hCtl.resize (n);
		e->hProg.resize (PERSIST (n));
		e->pslot.resize (n, 0);
		for (uint32_t i = old; i < n; i++) {
			e->hCtl[i].prog_off = (uint32_t)(PSLOTS * i * SLOT);
			e->hProg[PSLOTS * i * SLOT].wheel = 0xFFFF; /* empty program header */
		}
		e->devInst = n;
	}
	e->deviceReady = true;
	return 0;
}

int tbf::controlById (Instance& in, int id, int value);

/* a scheduled event (tbf_render_events) at its block boundary */
static int applyEvent (tbf_engine* e, const tbf_event& ev)
{
	if (ev.inst >= e->inst.size ())
		return fail (-22, "event for a bad instance");
	switch (ev.kind) {
		case TBF_EV_NOTE: return tbf_note (e, ev.inst, ev.id, ev.value != 0.0);
		case TBF_EV_PARAM: return tbf_set_param (e, ev.inst, ev.id, ev.value);
		case TBF_EV_CONTROL:
			if (controlById (e->inst[ev.inst], ev.id, (int)ev.value) < 0)
				return fail (-22, "bad control function id");
			return 0;
		case TBF_EV_PROGRAM: return tbf_program_install (e, ev.inst, (uint32_t)ev.id);
		default: return fail (-22, "bad event kind");
	}
}

/* one block of host control for instance i (the message-queue / active-list / routing
 * part of oscGenerateFragment and the effect setters' per-block constants).  Updates
 * the instance's current control e->hCtl[i] / program e->hProg; returns true when the
 * control the next block renders with changed. */
static bool stepControl (tbf_engine* e, uint32_t i, bool& progChanged, tbf_tgc_rec* rec = nullptr,
                         std::vector<uint16_t>* msgOut = nullptr, std::vector<float>* gainOut = nullptr,
                         std::vector<tbf_wh_params>* whOut = nullptr)
{
	Instance&    in      = e->inst[i];
	tbf_seg_ctl& c       = e->hCtl[i];
	progChanged          = false;
	const bool   tgDirty = in.tg.dirty ();
	if (!tgDirty && !in.progDirty && !in.ctlDirty && in.revOpt < 0)
		return false;
	if (tgDirty && rec) {
		/* device control: the front end here, the per-wheel part in k_tgctl */
		const size_t k  = in.tg.msg.size ();
		const size_t kg = 2 * (size_t)in.tg.gainPairs (); /* the changed drawbar gains: (bus, gain) pairs */
		if (msgOut) { /* a host worker's own message and gain lists (renderImpl merges them) */
			const uint32_t at = (uint32_t)msgOut->size (), ag = (uint32_t)gainOut->size ();
			msgOut->resize (at + k);
			gainOut->resize (ag + kg);
			in.tg.stepFront (msgOut->data () + at, at, gainOut->data () + ag, ag, *rec, c);
		} else {
			const uint32_t at = (uint32_t)e->hMsg.size (), ag = (uint32_t)e->hGain.size ();
			e->hMsg.resize (at + k);
			e->hGain.resize (ag + kg);
			in.tg.stepFront (e->hMsg.data () + at, at, e->hGain.data () + ag, ag, *rec, c);
		}
		in.progDirty = false;
		in.ctlDirty  = true;
		progChanged  = true;
	} else if (tgDirty) {
		in.tg.step (in.prog, c);
		in.progDirty = true;
		in.ctlDirty  = true;
	}
	if (rec)
		in.progDirty = false; /* device control: programs come from k_tgctl only */
	if (in.progDirty) {
		/* host control: the program in the instance's first slot, behind its header */
		const size_t    np   = std::min (in.prog.size (), SLOT - 1);
		tbf_prog_entry* slot = e->hProg.data () + PSLOTS * i * SLOT;
		slot[0]              = tbf_prog_entry {};
		slot[0].wheel        = 0xFFFF;
		slot[0].pad          = (uint32_t)np;
		std::copy (in.prog.begin (), in.prog.begin () + (long)np, slot + 1);
		c.prog_off   = (uint32_t)(PSLOTS * i * SLOT);
		c.prog_len   = (uint32_t)np;
		in.progDirty = false;
		progChanged  = true;
	}
	if (!tgDirty) {
		/* mixdown fields that setters can change without a tonegen step */
		c.swellPedalGain   = in.tg.swellPedalGain;
		c.outputGain       = in.tg.swellPedalGain * in.tg.percDrawbarGain;
		c.percEnvGainDecay = in.tg.percEnvGainDecay;
		c.percEnvGainReset = in.tg.percEnvGainReset;
		c.vibTable         = in.tg.vibTable;
		c.vibMixed         = in.tg.vibMixed;
	}
	odCtl (in, e->cfg.sample_rate, c);
	c.rvWet       = in.rvG;
	c.whBypass    = (uint32_t)in.whBypass;
	c.whRevOption = in.revOpt; /* a one-shot: the next block gets a fresh entry without it */
	in.revOpt     = -1;
	c.whSet       = 0;         /* a one-shot too: the whirl keeps a set until the next one */
	if (in.whDirty) {
		const tbf_wh_params& p = in.whr.cur;
		if (whOut) { /* a host worker's own list (worker-local index, renderImpl rebases it) */
			whOut->push_back (p);
			c.whSet = (uint32_t)whOut->size ();
		} else {
			e->hWh.push_back (p);
			c.whSet = (uint32_t)e->hWh.size ();
		}
		in.whDirty = false;
	}
	in.ctlDirty = (c.whRevOption >= 0) || c.whSet;
	return true;
}

/* Device control: one chunk's host control (events + front-end steps) on host worker
 * threads, one contiguous instance range each.  Instances are independent and each keeps
 * its own events' order, so this equals the serial loop; only where the deltas sit in the
 * pool differs: worker t writes its k-th delta to position (first instance of its range) *
 * want + k of the staging (a range of m instances has at most m * want deltas), so nothing
 * is moved afterwards and the kernels reach the deltas through hIdx; dSeg lists the filled
 * segments for the uploads.  Events are [evBeg, evEnd) of ev (block < b0 + want; programme
 * changes excluded by the caller: randomizeDrawbars writes the shared programme table).
 * Fills what the serial loop fills: dCtl, hRec, hMsg, hCtlInst, stepped, hIdx (every row),
 * curIdx, chg, actList. */
static int stepChunkParallel (tbf_engine* e, uint32_t n, uint32_t want, uint32_t b0, const tbf_event* ev,
                              uint32_t evBeg, uint32_t evEnd, int rp, bool& delta)
{
	const unsigned T   = std::max (1u, std::min<unsigned> (hostThreads (), (n + 255) / 256));
	const uint32_t per = (n + T - 1) / T;
	auto&          out = e->parStep;
	out.resize (T);
	for (auto& o : out) {
		o.msgs.clear ();
		o.gains.clear ();
		o.whs.clear ();
		o.act.clear ();
		o.ctlInst.clear ();
		o.evs.clear ();
		o.dInst.clear ();
		o.fulls.clear ();
		o.nd = 0;
		o.rc = 0;
		o.err.clear ();
	}
	for (uint32_t a : e->actList) /* the active list by range, in order */
		out[a / per].act.push_back (a);
	/* the events by instance range, in order: a parallel counting partition over T segments
	 * of the event list (a serial pass cost ~2 ms at 524k events) */
	{
		const uint32_t        nev = evEnd - evBeg, seg = (nev + T - 1) / T;
		std::vector<uint32_t> cnt ((size_t)T * T, 0);
		parallelFor (T, [&] (uint32_t sgm) {
			const uint32_t k0 = evBeg + std::min (nev, sgm * seg), k1 = evBeg + std::min (nev, (sgm + 1) * seg);
			for (uint32_t k = k0; k < k1; k++)
				cnt[(size_t)sgm * T + ev[k].inst / per]++;
		});
		for (unsigned t = 0; t < T; t++) {
			uint32_t tot = 0;
			for (unsigned sgm = 0; sgm < T; sgm++) {
				const uint32_t c                = cnt[(size_t)sgm * T + t];
				cnt[(size_t)sgm * T + t] = tot; /* the segment's first slot in worker t's list */
				tot += c;
			}
			out[t].evs.resize (tot);
		}
		parallelFor (T, [&] (uint32_t sgm) {
			const uint32_t k0 = evBeg + std::min (nev, sgm * seg), k1 = evBeg + std::min (nev, (sgm + 1) * seg);
			uint32_t*      at = cnt.data () + (size_t)sgm * T;
			for (uint32_t k = k0; k < k1; k++) {
				const uint32_t t = ev[k].inst / per;
				out[t].evs[at[t]++] = k;
			}
		});
	}
	e->hRec.resize ((size_t)n * want);
	e->lastEmit.resize (n);
	e->lastProg.resize (n);
	e->dseen.assign (n, 0);
	std::vector<uint32_t>& cur = e->curIdx;
	const auto             ph0 = std::chrono::steady_clock::now ();
	std::vector<uint64_t>  thNs (T);
	parallelFor (T, [&] (uint32_t t) {
		const auto           th0  = std::chrono::steady_clock::now ();
		tbf_engine::ParStep& o    = out[t];
		const uint32_t       i0   = t * per, i1 = std::min (n, i0 + per);
		const uint32_t       base = i0 * want;
		tbf_tgc_rec*         Rr   = e->hRec.data () + base; /* the worker's part of the staging */
		tlAct                     = &o.act; /* (markActive's pushes; o.act is rebuilt below) */
		/* instance-major: an instance's blocks one after another, so its host state stays in
		 * the core's L1 over the chunk (block-major passes over the range missed it on every
		 * block).  Instances are independent; each keeps its events in order (a stable
		 * counting sort of the range's events by instance). */
		std::vector<uint32_t>& eo = o.eoff;
		std::vector<uint32_t>& es = o.esort;
		eo.assign ((size_t)(i1 - i0) + 1, 0);
		for (uint32_t k : o.evs)
			eo[ev[k].inst - i0 + 1]++;
		for (uint32_t i = i0; i < i1; i++)
			eo[i - i0 + 1] += eo[i - i0];
		es.resize (o.evs.size ());
		{
			std::vector<uint32_t>& fill = o.efill;
			fill.assign (eo.begin (), eo.end () - 1);
			for (uint32_t k : o.evs)
				es[fill[ev[k].inst - i0]++] = k;
		}
		for (uint32_t i = i0; i < i1 && !o.rc; i++) {
			uint32_t ci = i; /* the instance's pool entry at the current block */
			uint32_t k = eo[i - i0], kEnd = eo[i - i0 + 1];
			for (uint32_t len = 0; len < want; len++) {
				for (; k < kEnd && ev[es[k]].block <= b0 + len; k++) {
					if ((o.rc = applyEvent (e, ev[es[k]]))) {
						o.err = g_err;
						break;
					}
					markActive (e, i);
				}
				if (o.rc)
					break;
				if (e->inAct[i]) {
					bool         pc;
					tbf_tgc_rec& rec = Rr[o.nd];
					if (!e->dseen[i]) { /* the entry the device holds for i at the chunk start */
						e->dseen[i]    = 1;
						e->lastEmit[i] = e->hCtl[i];
					}
					if (stepControl (e, i, pc, &rec, &o.msgs, &o.gains, &o.whs)) {
						const uint32_t d = base + o.nd++;
						tbf_seg_ctl    c = e->hCtl[i];
						if (pc) {
							c.prog_off = (uint32_t)(PERSIST (n) + ((size_t)rp * n * TBF_CHUNK + d) * SLOT);
							if (!e->stepped[i]) {
								e->stepped[i] = 1;
								o.ctlInst.push_back (i);
							}
						} else {
							memset (&rec, 0, sizeof (rec));
							if (ci >= n)
								c.prog_off = e->lastProg[i];
						}
						e->lastProg[i] = c.prog_off;
						if (!e->dhas[i]) {
							e->dhas[i] = 1;
							o.dInst.push_back (i);
						}
						/* a delta that changes only what a key / drawbar step changes travels as
						 * its record (k_tgctl rebuilds the entry); any other change as a full entry */
						tbf_seg_ctl& le = e->lastEmit[i];
						tbf_seg_ctl  tc = le;
						tc.prog_off       = c.prog_off;
						tc.keyCompTarget  = c.keyCompTarget;
						tc.resetPercAtEnd = c.resetPercAtEnd;
						tc.routing        = c.routing;
						if (memcmp (&tc, &c, sizeof (c)) != 0) {
							o.fulls.push_back (c);
							rec.full = (uint32_t)o.fulls.size ();
							le       = c;
						}
						rec.keyCompTarget = c.keyCompTarget;
						rec.flags         = (uint8_t)((rec.flags & ~8u) | (c.resetPercAtEnd ? 8u : 0u));
						rec.oldRouting    = (uint8_t)c.routing;
						ci                = n + d;
						e->chg[i]         = 1;
					} else
						e->inAct[i] = 0;
				}
				e->hIdx[(size_t)len * n + i] = ci;
			}
			cur[i] = ci;
		}
		o.act.clear (); /* the range's instances still active, in order */
		for (uint32_t i = i0; i < i1; i++)
			if (e->inAct[i])
				o.act.push_back (i);
		tlAct = nullptr;
		thNs[t] = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds> (std::chrono::steady_clock::now () - th0).count ();
	});
	const auto ph1 = std::chrono::steady_clock::now ();
	std::vector<size_t> mb (T), gb (T), wb (T), fb (T);
	size_t              nm = 0, ng = 0, nw = 0, nf = 0;
	e->dSeg.clear ();
	for (unsigned t = 0; t < T; t++) {
		if (out[t].rc)
			return fail (out[t].rc, out[t].err); /* on the calling thread */
		mb[t] = nm;
		nm += out[t].msgs.size ();
		gb[t] = ng;
		ng += out[t].gains.size ();
		wb[t] = nw;
		nw += out[t].whs.size ();
		fb[t] = nf;
		nf += out[t].fulls.size ();
		if (out[t].nd) {
			e->dSeg.push_back ({t * per * want, out[t].nd});
			delta = true;
		}
	}
	if (e->dSeg.empty ())
		e->dSeg.push_back ({0, 0});
	e->hMsg.resize (nm);
	e->hGain.resize (ng);
	e->hWh.resize (nw);
	e->hFull.resize (nf);
	if (nm || ng || nw || nf)
		parallelFor (T, [&] (uint32_t t) { /* message, gain, full entry and whirl set offsets: worker-local -> chunk */
			tbf_engine::ParStep& o    = out[t];
			const size_t         base = (size_t)t * per * want;
			for (size_t d = base; d < base + o.nd; d++) {
				tbf_tgc_rec& r = e->hRec[d];
				if (r.flags & 0x80)
					r.msgOff += (uint32_t)mb[t];
				if (r.flags & 4)
					r.gainOff += (uint32_t)gb[t];
				if (r.full)
					r.full += (uint32_t)fb[t];
			}
			for (tbf_seg_ctl& f : o.fulls)
				if (f.whSet)
					f.whSet += (uint32_t)wb[t];
			if (!o.fulls.empty ())
				memcpy ((void*)(e->hFull.data () + fb[t]), o.fulls.data (), o.fulls.size () * sizeof (tbf_seg_ctl));
			if (!o.whs.empty ())
				memcpy ((void*)(e->hWh.data () + wb[t]), o.whs.data (), o.whs.size () * sizeof (tbf_wh_params));
			if (!o.msgs.empty ())
				memcpy (e->hMsg.data () + mb[t], o.msgs.data (), o.msgs.size () * sizeof (uint16_t));
			if (!o.gains.empty ())
				memcpy (e->hGain.data () + gb[t], o.gains.data (), o.gains.size () * sizeof (float));
		});
	e->actList.clear ();
	for (unsigned t = 0; t < T; t++) {
		e->actList.insert (e->actList.end (), out[t].act.begin (), out[t].act.end ());
		for (uint32_t i : out[t].ctlInst)
			e->hCtlInst.push_back (i);
		for (uint32_t i : out[t].dInst)
			e->hDInst.push_back (i);
	}
	if (getenv ("TBF_DEBUG_HOST_PHASES")) {
		const auto ph2 = std::chrono::steady_clock::now ();
		auto       ms  = [] (auto a, auto b) { return std::chrono::duration<double, std::milli> (b - a).count (); };
		uint64_t   mx = 0, sum = 0;
		for (uint64_t v : thNs) {
			mx = std::max (mx, v);
			sum += v;
		}
		fprintf (stderr, "stepChunkParallel T=%u: step %.3f ms (thread max %.3f, mean %.3f) merge %.3f ms\n", T,
		         ms (ph0, ph1), mx / 1e6, sum / 1e6 / T, ms (ph1, ph2));
	}
	return 0;
}

/* Device front end: a chunk whose events are all notes or front-end parameters (drawbars,
 * the vibrato and percussion switches: frontParam), over instances whose control is
 * otherwise settled (no other parameter, programme, rotor or whirl change pending, no
 * drawbar or routing step), is stepped by k_front on the device (csrc/tbf_ctl.hip): the
 * messages, the stepped blocks, the control records and the index table come from the
 * instances' front-end state at the chunk start and their events.  The host only
 * partitions the events by instance and applies them to its own mirror state (the truth
 * for any later host-stepped chunk): no records, no index table. */
static bool frontClean (const Instance& in)
{
	const TgControl& t = in.tg;
	return !in.ctlDirty && !in.progDirty && in.revOpt < 0 && !in.whDirty && t.msg.empty () && !t.drawBarChange &&
	       t.oldRouting == t.newRouting && t.gainsSent && t.gainMask == 0 &&
	       /* the rotary option a drum / horn event derives stays an exact small integer */
	       fabs (in.params[TBF_P_DRUM]) < 1e6 && fabs (in.params[TBF_P_HORN]) < 1e6;
}

/* a parameter event the device front end steps, as a TBF_FEV_* word without the block; 0
 * for any other.  Drawbars and the vibrato and percussion switches change what a control
 * record carries; the effect setters (rotary speed, overdrive on / character, reverb mix,
 * percussion volume / decay, swell, whirl bypass, vibrato type: src/clap.cpp:162-207) the
 * entry's effect fields (TBF_FEV_EFFECT, their values in fevVal).  Values the setters take
 * outside their sane range (a character outside [0, 1], a swell outside [0, 2], huge or
 * non-finite numbers) leave the chunk to the host front end. */
static uint32_t frontParam (int32_t idx, float v)
{
	auto fx = [] (uint32_t k) { return TBF_FEV_PARAM | (TBF_FEV_EFFECT << 12) | k; };
	const bool small = fabsf (v) < 1e6f; /* false for NaN too */
	switch (idx) {
		case TBF_P_DRUM:
		case TBF_P_HORN: return small ? fx (TBF_FX_ROTOR) : 0;
		case TBF_P_OVERDRIVE: return small ? fx (TBF_FX_CLEAN) : 0;
		case TBF_P_CHARACTER: return v >= 0.0f && v <= 1.0f ? fx (TBF_FX_CHARACTER) : 0;
		case TBF_P_REVERB: return std::isfinite (v) ? fx (TBF_FX_REVERB) : 0;
		case TBF_P_PERCUSSION_VOLUME: return small ? fx (TBF_FX_PERC_SOFT) : 0;
		case TBF_P_PERCUSSION_DECAY: return small ? fx (TBF_FX_PERC_FAST) : 0;
		case TBF_P_SWELL: return v >= 0.0f && v <= 2.0f ? fx (TBF_FX_SWELL) : 0;
		case TBF_P_WHIRL_BYPASS: return small ? fx (TBF_FX_BYPASS) : 0;
		case TBF_P_VIBRATO_TYPE: return small ? fx (TBF_FX_VIBTYPE) : 0;
		default: break;
	}
	int bus = -1;
	if (idx >= TBF_P_DRAWBAR_MIN && idx <= TBF_P_DRAWBAR_MAX)
		bus = idx;
	else if (idx >= TBF_P_BUS_DRAWBAR_BASE && idx < TBF_P_BUS_DRAWBAR_BASE + 27)
		bus = idx - TBF_P_BUS_DRAWBAR_BASE;
	if (bus >= 0) {
		const unsigned st = (unsigned)rint (v); /* as tbf_set_param hands it to setDrawBar */
		return TBF_FEV_PARAM | (TBF_FEV_DRAWBAR << 12) | ((st > 8 ? 15u : st) << 5) | (uint32_t)bus;
	}
	const uint32_t fl = (int)rint (v) != 0 ? 1u : 0u;
	switch (idx) {
		case TBF_P_VIBRATO: return TBF_FEV_PARAM | (TBF_FEV_VIB_UPPER << 12) | (fl << 9);
		case TBF_P_VIBRATO_LOWER: return TBF_FEV_PARAM | (TBF_FEV_VIB_LOWER << 12) | (fl << 9);
		case TBF_P_PERCUSSION: return TBF_FEV_PARAM | (TBF_FEV_PERC << 12) | (fl << 9);
		case TBF_P_PERCUSSION_HARMONIC: return TBF_FEV_PARAM | (TBF_FEV_PERC_FIRST << 12) | (fl << 9);
		default: return 0;
	}
}
static uint32_t frontParam (const tbf_event& E) { return frontParam (E.id, (float)E.value); }

/* the instances' front-end cleanliness (e->fclean), once per chunk; false when an active
 * instance is not clean (its pending step is the host's) */
static bool frontCleanAll (tbf_engine* e)
{
	const uint32_t        n  = (uint32_t)e->inst.size ();
	std::vector<uint8_t>& cl = e->fclean;
	cl.resize (n);
	const unsigned T   = std::max (1u, std::min<unsigned> (hostThreads (), (n + 255) / 256));
	const uint32_t per = (n + T - 1) / T;
	parallelFor (T, [&] (uint32_t t) {
		for (uint32_t i = t * per; i < std::min (n, (t + 1) * per); i++)
			cl[i] = frontClean (e->inst[i]) ? 1 : 0;
	});
	for (uint32_t i : e->actList)
		if (!cl[i])
			return false;
	return true;
}

/* One parallel pass over a chunk's events (sorted by block): a programme event among them,
 * an event for a bad instance, and -- with cl, the instances' cleanliness -- whether the
 * device front end takes them all (notes and frontParam kinds on clean instances), with
 * the events as compact records bucketed by (segment, instance range) for stepChunkFront.
 * (Three passes over the 24-B events used to do this: ~0.2 ms each at 524 k events; then a
 * scan, a partition and a gather by instance, ~0.3 ms each.) */
static void scanChunk (uint32_t n, uint32_t b0, const tbf_event* ev, uint32_t evBeg, uint32_t evEnd, const uint8_t* cl,
                       bool& progEv, bool& bad, bool& front, ChunkScan& cs)
{
	const uint32_t nev = evEnd - evBeg;
	cs.T   = std::max (1u, std::min<unsigned> (hostThreads (), (n + 255) / 256));
	assert (cs.T <= TBF_MAX_HOST_THREADS);
	cs.per = (n + cs.T - 1) / cs.T;
	cs.Te  = std::max (1u, std::min (hostThreads (), (nev + 32767) / 32768));
	cs.seg = (nev + cs.Te - 1) / cs.Te;
	if (cl) {
		cs.rec.resize (std::max<uint32_t> (nev, 1));
		cs.boff.resize ((size_t)cs.Te * (cs.T + 1));
	}
	std::vector<char> pe (cs.Te, 0), bd (cs.Te, 0), fr (cs.Te, 0);
	parallelFor (cs.Te, [&] (uint32_t sgm) {
		const uint32_t k0 = evBeg + std::min (nev, sgm * cs.seg), k1 = evBeg + std::min (nev, (sgm + 1) * cs.seg);
		bool           p = false, b = false, f = cl != nullptr; /* locals: the flags share a cache line */
		uint32_t       c[TBF_MAX_HOST_THREADS + 1] = {};         /* events per instance range (T <= TBF_MAX_HOST_THREADS) */
		for (uint32_t k = k0; k < k1; k++) {
			const tbf_event& E = ev[k];
			p                  = p || E.kind == TBF_EV_PROGRAM;
			if (E.inst >= n) {
				b = true;
				f = false;
				continue;
			}
			if (f) {
				f = (E.kind == TBF_EV_NOTE || (E.kind == TBF_EV_PARAM && frontParam (E))) && cl[E.inst];
				c[E.inst / cs.per]++;
			}
		}
		if (f) { /* the records, by range, into this segment's own part of rec (no shared lines) */
			uint32_t* bo = cs.boff.data () + (size_t)sgm * (cs.T + 1);
			uint32_t  at[TBF_MAX_HOST_THREADS];
			bo[0] = k0 - evBeg;
			for (unsigned t = 0; t < cs.T; t++) {
				at[t]     = bo[t];
				bo[t + 1] = bo[t] + c[t];
			}
			ChunkScan::Rec* rec = cs.rec.data ();
			for (uint32_t k = k0; k < k1; k++) {
				const tbf_event& E = ev[k];
				rec[at[E.inst / cs.per]++] = {E.inst, (E.block - b0) << 2 | (E.kind == TBF_EV_PARAM ? 1u : 0u) |
				                                          (E.value != 0.0 ? 2u : 0u),
				                              E.id, (float)E.value};
			}
		}
		pe[sgm] = p;
		bd[sgm] = b;
		fr[sgm] = f;
	});
	progEv = bad = false;
	front        = cl != nullptr;
	for (unsigned t = 0; t < cs.Te; t++) {
		progEv = progEv || pe[t];
		bad    = bad || bd[t];
		front  = front && fr[t];
	}
}

static int stepChunkFront (tbf_engine* e, uint32_t n, uint32_t want, uint32_t b0, const tbf_event* ev, uint32_t evBeg,
                           uint32_t evEnd, ChunkScan& cs, bool& delta)
{
	const unsigned T   = cs.T;
	const uint32_t per = cs.per;
	auto&          out = e->parStep;
	const auto     f0  = std::chrono::steady_clock::now ();
	out.resize (T);
	for (auto& o : out) {
		o.act.clear ();
		o.ctlInst.clear ();
		o.evs.clear ();
		o.gainLocal = 0;
		o.fx        = false;
	}
	/* the events by instance range come from scanChunk's buckets, in event order */
	const auto            f1 = std::chrono::steady_clock::now ();
	std::vector<uint32_t> wbase (T + 1, 0);
	auto seg = [&] (unsigned sgm, unsigned t) { return cs.boff.data () + (size_t)sgm * (T + 1) + t; };
	for (unsigned t = 0; t < T; t++) {
		size_t c = 0;
		for (unsigned sgm = 0; sgm < cs.Te; sgm++)
			c += seg (sgm, t)[1] - seg (sgm, t)[0];
		wbase[t + 1] = wbase[t] + (uint32_t)c;
	}
	e->hFevOff.resize (n + 1);
	e->hFev.resize (std::max<uint32_t> (wbase[T], 1));
	e->hFevVal.resize (std::max<uint32_t> (wbase[T], 1));
	e->hFront.resize (n);
	const bool          dbgPh = getenv ("TBF_DEBUG_HOST_PHASES") != nullptr;
	std::vector<double> thMs (dbgPh ? 3 * T : 0);
	parallelFor (T, [&] (uint32_t t) {
		const auto             g0 = std::chrono::steady_clock::now ();
		tbf_engine::ParStep&   o  = out[t];
		const uint32_t         i0 = t * per, i1 = std::min (n, i0 + per);
		std::vector<uint32_t>& eo = o.eoff;
		auto&                  es = o.erec;
		eo.assign ((size_t)(i1 > i0 ? i1 - i0 : 0) + 1, 0);
		for (unsigned sgm = 0; sgm < cs.Te; sgm++)
			for (uint32_t k = seg (sgm, t)[0]; k < seg (sgm, t)[1]; k++)
				eo[cs.rec[k].inst - i0 + 1]++;
		for (uint32_t i = i0; i < i1; i++)
			eo[i - i0 + 1] += eo[i - i0];
		es.resize (wbase[t + 1] - wbase[t]);
		{ /* the range's events by instance (a stable counting sort of its buckets, read in
		   * order, so the per-instance pass below reads them sequentially) */
			std::vector<uint32_t>& fill = o.efill;
			fill.assign (eo.begin (), eo.end () - 1);
			for (unsigned sgm = 0; sgm < cs.Te; sgm++)
				for (uint32_t k = seg (sgm, t)[0]; k < seg (sgm, t)[1]; k++) {
					const ChunkScan::Rec& r = cs.rec[k];
					es[fill[r.inst - i0]++] = {r.bf >> 2, r.id, r.v, r.bf & 3u};
				}
		}
		const auto g1 = std::chrono::steady_clock::now ();
		for (uint32_t i = i0; i < i1; i++) {
			Instance&        in = e->inst[i];
			TgControl&       tg = in.tg;
			tbf_front_state& F  = e->hFront[i];
			memset (&F, 0, sizeof (F));
			static_assert (sizeof (F.keys) == sizeof (tg.keyBits), "384 key bits");
			memcpy (F.keys, tg.keyBits, sizeof (F.keys));
			F.keyDown         = tg.keyDownCount;
			F.upperDown       = (int32_t)tg.upperKeyCount;
			F.pending         = tg.steadyPending ? 1u : 0u;
			F.percSendBus     = tg.percSendBus;
			F.routing         = tg.oldRouting;
			F.percEnabled     = tg.percEnabled ? 1 : 0;
			F.percTrigRestore = tg.percTrigRestore;
			F.percTriggerBus  = tg.percTriggerBus;
			F.percSendBusA    = tg.percSendBusA;
			F.percSendBusB    = tg.percSendBusB;
			F.gainOff         = o.gainLocal; /* + the thread's base, below */
			F.percReset[0]    = tg.percEnvScaling * tg.percEnvGainResetNorm; /* as setPercVolume */
			F.percReset[1]    = tg.percEnvScaling * tg.percEnvGainResetSoft;
			F.percDrawbar[0]  = tg.percDrawbarNormalGain;
			F.percDrawbar[1]  = tg.percDrawbarSoftGain;
			F.percDecay[0]    = tg.percEnvGainDecaySlowNorm;
			F.percDecay[1]    = tg.percEnvGainDecaySlowSoft;
			F.percDecay[2]    = tg.percEnvGainDecayFastNorm;
			F.percDecay[3]    = tg.percEnvGainDecayFastSoft;
			F.percSoft        = tg.percIsSoft != 0;
			F.percFast        = tg.percIsFast != 0;
			F.swell           = tg.swellPedalGain;
			e->hFevOff[i]     = wbase[t] + eo[i - i0];
			/* the host's front state takes the events too (it stays the truth for any later
			 * host-stepped chunk): the same setters, block by block, and the same steps as
			 * the device -- a block with inputs steps, and so does the one after it */
			bool     stepped = F.pending != 0, pend = F.pending != 0, fxd = false;
			uint32_t oldR = tg.oldRouting, ng = 0, msgsB = 0;
			int      curB = -1;
			auto     closeBlock = [&] () {
                const bool rcp = tg.newRouting != oldR, in = msgsB > 0 || tg.drawBarChange || rcp;
                ng += (uint32_t)__builtin_popcount (tg.gainMask);
                stepped = stepped || in;
                pend    = in;
                oldR    = tg.newRouting;
                tg.drawBarChange = 0;
                tg.gainMask      = 0;
                msgsB            = 0;
			};
			for (uint32_t j = eo[i - i0]; j < eo[i - i0 + 1]; j++) {
				const auto&    E   = es[j];
				const uint32_t blk = E.blk;
				if ((int)blk != curB) {
					if (curB >= 0)
						closeBlock ();
					if (curB >= 0 ? blk > (uint32_t)curB + 1 : blk > 0)
						pend = false; /* blocks without events between: the pending step is done */
					curB = (int)blk;
				}
				if (E.flag & 1u) {
					const float    v = E.v;
					const uint32_t w = frontParam (E.id, v);
					e->hFev[wbase[t] + j] = w | (blk << 16);
					if (E.id >= 0 && E.id < 64)
						in.params[E.id] = v;
					const uint32_t op = (w >> 12) & 7u;
					if (op == TBF_FEV_EFFECT) {
						/* tbf_set_param's setter on the mirror, and the value k_front applies */
						float x = 0.0f;
						switch (w & 31u) {
							case TBF_FX_ROTOR:
								x = (float)(int)(floor (in.params[TBF_P_DRUM]) + 3 * floor (in.params[TBF_P_HORN]));
								break;
							case TBF_FX_CLEAN:
								in.odClean = (int)rint (1.0f - v);
								x          = (float)in.odClean;
								break;
							case TBF_FX_CHARACTER:
								setCharacter (in, v);
								x = v;
								break;
							case TBF_FX_REVERB:
								in.rvG = v;
								x      = v;
								break;
							case TBF_FX_PERC_SOFT: {
								const int soft = (int)(1 - rint (v));
								tg.setPercVolume (soft);
								x = soft != 0 ? 1.0f : 0.0f;
								break;
							}
							case TBF_FX_PERC_FAST: {
								const int fast = (int)rint (v);
								tg.setPercFast (fast);
								x = fast != 0 ? 1.0f : 0.0f;
								break;
							}
							case TBF_FX_SWELL: {
								unsigned char u   = (unsigned char)rint (v * 127.0);
								tg.swellPedalGain = (float)((tg.outputLevelTrim * ((double)u)) / 127.0);
								x                 = tg.swellPedalGain;
								break;
							}
							case TBF_FX_BYPASS:
								in.whBypass = (int)rint (v);
								x           = (float)in.whBypass;
								break;
							case TBF_FX_VIBTYPE: {
								const int p = (int)floor (v);
								tg.setVibratoFromInt (p);
								x = (float)p;
								break;
							}
						}
						e->hFevVal[wbase[t] + j] = x;
						fxd                      = true;
						continue;
					}
					if (op == TBF_FEV_DRAWBAR)
						tg.setDrawBar ((int)(w & 31u), (unsigned)rint (v));
					else if (op == TBF_FEV_VIB_UPPER)
						tg.setVibratoUpper ((int)rint (v));
					else if (op == TBF_FEV_VIB_LOWER)
						tg.setVibratoLower ((int)rint (v));
					else if (op == TBF_FEV_PERC)
						tg.setPercEnabled ((int)rint (v));
					else
						tg.setPercFirst ((int)rint (v));
					continue;
				}
				const bool on = (E.flag & 2u) != 0;
				const bool ok = E.id >= 0 && E.id < 384; /* oscKeyOn/Off ignore keys >= MAX_KEYS */
				e->hFev[wbase[t] + j] = (ok ? (uint32_t)E.id : 0x0fffu) | (on ? 1u << 12 : 0u) | (blk << 16);
				msgsB += ok ? (uint32_t)tg.noteCount (E.id, on) : 0u;
			}
			if (curB >= 0) {
				closeBlock ();
				if ((uint32_t)curB + 1 < want)
					pend = false;
			} else
				pend = false; /* no events: block 0 takes the pending step */
			o.gainLocal += 2 * ng;
			tg.oldRouting = tg.newRouting;
			if (fxd) {
				/* effect setters: the control entry the instance ends the chunk with (the
				 * device wrote the chunk's own entries); the rotary option was a one-shot */
				tbf_seg_ctl& c     = e->hCtl[i];
				odCtl (in, e->cfg.sample_rate, c);
				c.rvWet            = in.rvG;
				c.whBypass         = (uint32_t)in.whBypass;
				c.swellPedalGain   = tg.swellPedalGain;
				c.outputGain       = tg.swellPedalGain * tg.percDrawbarGain;
				c.percEnvGainDecay = tg.percEnvGainDecay;
				c.percEnvGainReset = tg.percEnvGainReset;
				c.vibTable         = tg.vibTable;
				c.vibMixed         = tg.vibMixed;
				c.whRevOption      = -1;
				c.whSet            = 0;
				in.revOpt          = -1;
				in.ctlDirty        = false;
				e->chg[i]          = 1;
				o.fx               = true;
			}
			if (stepped) { /* stepped blocks: control deltas */
				e->stepped[i] = 1;
				o.ctlInst.push_back (i);
				e->chg[i] = 1;
				const int kd = tg.keyDownCount;
				e->hCtl[i].keyCompTarget  = tg.tpl->keyCompTable[kd < 0 ? 0 : (kd > 127 ? 127 : kd)];
				e->hCtl[i].resetPercAtEnd = tg.upperKeyCount == 0;
				e->hCtl[i].routing        = tg.oldRouting;
			}
			const bool last = pend;
			tg.steadyPending = last;
			e->inAct[i]      = tg.steadyPending ? 1 : 0;
			if (e->inAct[i])
				o.act.push_back (i);
		}
		if (dbgPh) {
			const auto g2 = std::chrono::steady_clock::now ();
			thMs[3 * t]     = std::chrono::duration<double, std::milli> (g0 - f1).count (); /* start delay */
			thMs[3 * t + 1] = std::chrono::duration<double, std::milli> (g1 - g0).count (); /* sort */
			thMs[3 * t + 2] = std::chrono::duration<double, std::milli> (g2 - g1).count (); /* mirror */
		}
	});
	e->hFevOff[n] = wbase[T];
	{ /* the gain-pair slots: each range's base */
		std::vector<uint32_t> gb (T + 1, 0);
		for (unsigned t = 0; t < T; t++)
			gb[t + 1] = gb[t] + out[t].gainLocal;
		e->frontGain = gb[T];
		parallelFor (T, [&] (uint32_t t) {
			for (uint32_t i = t * per; i < std::min (n, (t + 1) * per); i++)
				e->hFront[i].gainOff += gb[t];
		});
	}
	e->actList.clear ();
	for (unsigned t = 0; t < T; t++) {
		e->actList.insert (e->actList.end (), out[t].act.begin (), out[t].act.end ());
		for (uint32_t i : out[t].ctlInst)
			e->hCtlInst.push_back (i);
	}
	delta = !e->hCtlInst.empty ();
	for (unsigned t = 0; t < T; t++)
		delta = delta || out[t].fx;
	if (getenv ("TBF_DEBUG_HOST_PHASES")) {
		auto ms = [] (auto a, auto b) { return std::chrono::duration<double, std::milli> (b - a).count (); };
		fprintf (stderr, "stepChunkFront T=%u: partition %.3f ms, instances %.3f ms\n", T, ms (f0, f1),
		         ms (f1, std::chrono::steady_clock::now ()));
		double mx[3] = {0, 0, 0}, sm[3] = {0, 0, 0};
		for (unsigned t = 0; t < T; t++)
			for (int q = 0; q < 3; q++) {
				mx[q] = std::max (mx[q], thMs[3 * t + q]);
				sm[q] += thMs[3 * t + q] / T;
			}
		fprintf (stderr, "  threads (mean / max ms): start %.3f / %.3f, sort %.3f / %.3f, mirror %.3f / %.3f\n", sm[0], mx[0],
		         sm[1], mx[1], sm[2], mx[2]);
	}
	return 0;
}

/* The inter-stage buffers for a call of nblocks blocks: each holds, per instance, one
 * chunk of stageBlocks blocks -- a power of two from TBF_CHUNK up to steadyChunk, just
 * enough for the longest chunk this call can make, so a caller that renders 64 blocks at a
 * time never pays for longer chunks (n x blocks x 128 x 56 B at the default stage
 * groups: 15 GB at 4096 instances and the default 512-block chunks, 60 GB at 2048, 1.9 GB
 * at 64).  They only grow (a
 * different stride under chunks still in flight would be wrong), after every launch that
 * may read them has finished.  When the device cannot hold them, the chunk halves down to
 * TBF_CHUNK before the call fails, and steadyChunk stays at what fitted.  A buffer whose
 * producer and every reader run on one stage-group stream is single: the next chunk's
 * producer is ordered behind this chunk's readers by the stream (default groups {0,0,1,1,1,2}:
 * mid0, rvA and rvB single; mid1, mid2 by chunk parity). */
/* bytes of the stage buffers at n instances and chunks of `blocks` blocks (mid0 8 B, mid1 /
 * mid2 4 B, rvA / rvB 16 B per sample, each doubled when it alternates by chunk parity) */
static size_t stageFootprint (const tbf_engine* e, size_t n, uint32_t blocks)
{
	static const int prod[5] = {0, 1, 2, 3, 4}, rd[5][2] = {{1, -1}, {2, 4}, {3, -1}, {4, -1}, {5, -1}};
	static const size_t per[5] = {8, 4, 16, 16, 4};
	const bool rv = e->cfg.chain_mode != TBF_CHAIN_TONEGEN && e->cfg.chain_mode != TBF_CHAIN_TAP_PREAMP;
	size_t sum = 0;
	for (int b = 0; b < 5; b++) {
		if (b > 0 && !rv)
			break;
		bool dbl = false;
		for (int r : rd[b])
			dbl = dbl || (r >= 0 && e->grp[r] != e->grp[prod[b]]);
		sum += (dbl ? 2 : 1) * per[b];
	}
	return sum * n * blocks * TBF_BLK;
}

static int stageBuffers (tbf_engine* e, uint32_t n, uint32_t nblocks, hipStream_t s)
{
	uint32_t want = TBF_CHUNK;
	while (want < nblocks && want < e->steadyChunk)
		want *= 2;
	want = std::min (want, std::max (e->steadyChunk, (uint32_t)TBF_CHUNK));
	if (e->stageN == n && e->stageBlocks >= want && e->mid0.p)
		return 0;
	/* every launch that may read the old buffers: pipelined stages and the caller's stream
	 * (the engine's own streams and s; no device-wide synchronization, which would also
	 * wait for a caller's unrelated work on other streams) */
	if (int rc = drainStages (e))
		return rc;
	HIPCHK (hipStreamSynchronize (s));
	/* producer stage -> reader stages of mid0, mid1, rvA, rvB, mid2 */
	static const int prod[5] = {0, 1, 2, 3, 4}, rd[5][2] = {{1, -1}, {2, 4}, {3, -1}, {4, -1}, {5, -1}};
	for (int b = 0; b < 5; b++) {
		bool dbl = false;
		for (int r : rd[b])
			dbl = dbl || (r >= 0 && e->grp[r] != e->grp[prod[b]]);
		e->stageDbl[b] = dbl;
	}
	const bool rv = e->cfg.chain_mode != TBF_CHAIN_TONEGEN && e->cfg.chain_mode != TBF_CHAIN_TAP_PREAMP;
	auto       k  = [&] (int b) { return (size_t)(e->stageDbl[b] ? 2 : 1); };
	for (uint32_t blocks = want;;) {
		e->mid0.release (), e->mid1.release (), e->mid2.release (), e->rvA.release (), e->rvB.release ();
		const size_t need = (size_t)n * blocks * TBF_BLK;
		const bool   ok   = !e->mid0.ensure (k (0) * 2 * need) &&
		                (!rv || (!e->mid1.ensure (k (1) * need) && !e->mid2.ensure (k (4) * need) &&
		                         !e->rvA.ensure (k (2) * 2 * need) && !e->rvB.ensure (k (3) * 2 * need)));
		if (ok) {
			e->stageBlocks = blocks;
			e->stageN      = n;
			if (blocks < want) /* the device could not hold longer chunks */
				e->steadyChunk = blocks;
			return 0;
		}
		(void)hipGetLastError (); /* the failed hipMalloc's error */
		if (blocks <= TBF_CHUNK) {
			e->mid0.release (), e->mid1.release (), e->mid2.release (), e->rvA.release (), e->rvB.release ();
			e->stageBlocks = e->stageN = 0;
			return fail (-12, "out of device memory (stage buffers)");
		}
		blocks = std::max (blocks / 2, (uint32_t)TBF_CHUNK);
	}
}

static int renderImpl (tbf_engine* e, uint32_t nblocks, float* dL, float* dR, uint64_t stride, hipStream_t s,
                       const tbf_event* ev = nullptr, uint32_t nev = 0)
{
	int rc = ensureDevice (e);
	if (rc)
		return rc;
	const uint32_t n = (uint32_t)e->inst.size ();
	if (n == 0 || nblocks == 0)
		return 0;
	if (!e->retuned.empty ()) {
		/* retuned instances (tbf_instance_retune): fresh tone-generator state and the new
		 * template id, after every launch so far, before this call's first block */
		if ((rc = joinStages (e, s)))
			return rc;
		for (uint32_t i : e->retuned) {
			HIPCHK (hipMemcpyAsync (&e->st.p[i].mo, &e->inst[i].s0.mo, offsetof (tbf_mo_state, iirA),
			                        hipMemcpyHostToDevice, s));
			HIPCHK (hipMemcpyAsync (&e->st.p[i].tg, &e->inst[i].s0.tg, sizeof (tbf_tg_state),
			                        hipMemcpyHostToDevice, s));
			HIPCHK (hipMemcpyAsync (&e->cst.p[i].tpl, &e->inst[i].k.tpl, sizeof (uint32_t), hipMemcpyHostToDevice, s));
			if (e->devCtl) { /* a fresh per-wheel control state and an empty program */
				HIPCHK (hipMemsetAsync (e->tgc.p + i, 0, sizeof (tbf_tgc_state), s));
				HIPCHK (hipMemsetAsync (e->prog.p + PSLOTS * i * SLOT, 0, PSLOTS * SLOT * sizeof (tbf_prog_entry), s));
				e->pslot[i]         = 0;
				e->hCtl[i].prog_off = (uint32_t)(PSLOTS * i * SLOT);
				e->persistStale     = true;
			}
		}
		HIPCHK (hipStreamSynchronize (s));
		e->retuned.clear ();
	}
	if (stride < (uint64_t)nblocks * TBF_BLK)
		return fail (-22, "stride smaller than nblocks*128");
	if (e->actAll || e->inAct.size () != n) { /* new instances: step every one */
		e->inAct.assign (n, 1);
		e->actList.resize (n);
		for (uint32_t i = 0; i < n; i++)
			e->actList[i] = i;
		e->actAll = false;
	}
	tbf_launch P;
	memset (&P, 0, sizeof (P));
	P.bank      = e->bank.p;
	P.tpls      = e->tplDesc.p;
	P.cst       = e->cst.p;
	P.st        = e->st.p;
	P.wring     = e->wring.p;
	P.rslab     = e->rslab.p;
	P.ctl       = e->ctl.p;
	P.vibTab    = e->vib.p;
	P.xsJump    = e->xsj.p;
	P.whTab     = e->whTab.p;
	P.whBw      = e->whBw.p;
	P.outL      = dL;
	P.outR      = dR;
	P.outStride = stride;
	P.nInst     = n;
	P.wringLen  = e->wringLen;
	P.statorInc = e->statorInc;
	P.chain     = e->cfg.chain_mode;
	P.slabLen   = e->slabLen;
	P.errFlags  = e->err.p;
	P.dbg       = e->cfg.debug_flags;
	/* k_whirl_split where it keeps more waves per SIMD than k_whirl (tbf_render.hip) */
	P.whSplit = e->whSplit >= 0 ? (uint32_t)e->whSplit : (e->wringLen > 512 || n <= e->nCU) ? 1u : 0u;
	P.rvLds     = e->rvLdsOn && e->rvLdsFit;
	P.rvGrid    = e->rvGrid;
	P.rvWork    = e->rvWork.p;
	if (e->cfg.chain_mode == TBF_CHAIN_TONEGEN && e->mixFixed.ensure (n))
		return fail (-12, "out of device memory");
	P.mixFixed = e->mixFixed.p;
	/* inter-stage buffers for the longest chunk this call makes (stageBuffers): single, or
	 * two sets by chunk parity (see the pipelining below) */
	if ((rc = stageBuffers (e, n, nblocks, s)))
		return rc;
	const size_t   need     = (size_t)n * e->stageBlocks * TBF_BLK;
	const uint32_t maxChunk = std::min (e->steadyChunk, e->stageBlocks);
	P.midStride             = (uint64_t)e->stageBlocks * TBF_BLK;
	/* Cross-chunk pipelining.  Every stage is causal and keeps its own state, so stage k
	 * of chunk c depends only on stage k-1 of chunk c and on stage k of chunk c-1, which
	 * runs on the same stage-group stream; the stage buffers alternate by chunk parity.
	 * Used for the full chain; tonegen only, tap modes and a host-control chunk's uploads run on the
	 * caller's stream after joining.  With tbf_debug_kernel_times on, each launch is
	 * bracketed by events on its own stream (durations then include the overlap with the
	 * other streams' kernels). */
	const bool   pipe  = e->pipeline && e->cfg.chain_mode == TBF_CHAIN_FULL && !e->timeSerial;
	bool         outWait = false; /* the output stage has waited for the caller's stream */
	const size_t dprogCap = DPROG_CAP (n);
	e->chg.assign (n, 0);
	/* after a chunk with control deltas: the instances' final entries become their current
	 * (pool 0..n-1) control for the next chunk (one-shots cleared).  Device control: k_tgctl
	 * left each stepped instance's last program in its other persistent slot; the regions'
	 * persistent entries refresh at the start of the chunks that use them.  Host control:
	 * uploaded now, and the staging is reused, so it synchronizes. */
	auto endDelta = [&] () -> int {
		uint32_t lo = n, hi = 0;
		for (uint32_t i = 0; i < n; i++)
			if (e->chg[i]) {
				e->hCtl[i].whRevOption = -1;
				e->hCtl[i].whSet       = 0;
				/* a one-shot in the chunk's last block left the instance dirty only so that the
				 * next block clears it: the entry it ends with is cleared here already */
				Instance& in = e->inst[i];
				if (in.ctlDirty && !in.progDirty && in.revOpt < 0 && !in.whDirty)
					in.ctlDirty = false;
				lo                     = std::min (lo, i);
				hi                     = std::max (hi, i + 1);
				e->chg[i]              = 0;
			}
		if (e->devCtl) {
			for (uint32_t i : e->hCtlInst) {
				e->pslot[i]         = (uint8_t)((e->pslot[i] + 1) % PSLOTS);
				e->hCtl[i].prog_off = (uint32_t)((PSLOTS * i + e->pslot[i]) * SLOT);
			}
			e->ctlVer++;
			return 0;
		}
		HIPCHK (hipMemcpyAsync (e->ctl.p, e->hCtl.data (), n * sizeof (tbf_seg_ctl), hipMemcpyHostToDevice, s));
		if (hi > lo)
			HIPCHK (hipMemcpyAsync (e->prog.p + lo * PSLOTS * SLOT, e->hProg.data () + lo * PSLOTS * SLOT,
			                        (size_t)(hi - lo) * PSLOTS * SLOT * sizeof (tbf_prog_entry), hipMemcpyHostToDevice, s));
		HIPCHK (hipStreamSynchronize (s));
		return 0;
	};
	uint32_t b0 = 0, evi = 0;
	while (b0 < nblocks) {
		/* host control for the chunk, block by block: entry indices per (block, instance),
		 * new pool entries only where an instance's control changes */
		uint32_t want = std::min<uint32_t> (TBF_CHUNK, nblocks - b0);
		if (nblocks - b0 > TBF_CHUNK && maxChunk > TBF_CHUNK && e->actList.empty () && !e->persistStale) {
			/* no instance's control can change before the next event: a chunk without deltas,
			 * up to steadyChunk blocks (as far as the stage buffers reach), ending at the next
			 * event's block */
			uint32_t w = std::min (maxChunk, nblocks - b0);
			if (evi < nev)
				w = std::min (w, ev[evi].block > b0 ? ev[evi].block - b0 : 0u);
			if (w > TBF_CHUNK)
				want = w;
		}
		const uint64_t cix  = e->chunkSeq++;
		const bool     par  = (cix & 1) != 0;
		const uint32_t bset = (uint32_t)(cix & 1); /* stage-buffer set of this chunk */
		const int      rp   = e->devCtl ? (int)par : 0; /* control region of this chunk */
		/* device control, stage-group pipelining: a delta chunk pipelines like any other; its
		 * uploads and k_tgctl go on the first stage group's stream after the chunk before
		 * last (the previous user of this control region) has finished every stage */
		const bool     dpipe = e->devCtl && pipe;
		hipStream_t    us    = dpipe ? e->gs[0] : s;
		bool           usWaited = false;
		auto           usWait   = [&] () -> int {
            if (usWaited || !dpipe)
                return 0;
            usWaited = true;
            if (!e->stagesBusy) { /* after the caller's stream (earlier non-pipelined work) */
                HIPCHK (hipEventRecord (e->sjoin, s));
                HIPCHK (hipStreamWaitEvent (us, e->sjoin, 0));
            }
            HIPCHK (hipStreamWaitEvent (us, e->pev[(cix + 2) & 3][tbf_chain_stages (P.chain) - 1], 0));
            return 0;
		};
		if (e->devCtl && e->persistStale) {
			e->ctlVer++; /* the regions refresh below */
			e->persistStale = false;
		}
		if (e->persistStale) {
			/* the persistent pool (entry i = instance i's current control and programme) as
			 * of the START of this chunk: an instance without a delta at some block renders
			 * that block with entry i, so it must not yet hold a later block's events.
			 * Rare (after instances are added), so it syncs. */
			if ((rc = joinStages (e, s)))
				return rc;
			HIPCHK (hipMemcpyAsync (e->ctl.p, e->hCtl.data (), n * sizeof (tbf_seg_ctl), hipMemcpyHostToDevice, s));
			if (!e->devCtl) /* device control keeps the persistent programs on the device */
				HIPCHK (hipMemcpyAsync (e->prog.p, e->hProg.data (), PERSIST (n) * sizeof (tbf_prog_entry),
				                        hipMemcpyHostToDevice, s));
			HIPCHK (hipStreamSynchronize (s));
			e->persistStale = false;
		}
		if (e->devCtl) {
			/* staging of the chunk before last (its uploads are done once its event is) */
			e->dCtl.swap (e->dCtlB);
			e->hRec.swap (e->hRecB);
			e->hMsg.swap (e->hMsgB);
			e->hGain.swap (e->hGainB);
			e->hWh.swap (e->hWhB);
			e->hCtlInst.swap (e->hCtlInstB);
			e->hDInst.swap (e->hDInstB);
			e->hFull.swap (e->hFullB);
			e->hFront.swap (e->hFrontB);
			e->hFev.swap (e->hFevB);
			e->hFevVal.swap (e->hFevValB);
			e->hFevOff.swap (e->hFevOffB);
			e->hIdx.swap (e->hIdxB);
			e->hCtlPin.swap (e->hCtlPinB);
			std::swap (e->upEv, e->upEvB);
			const auto w0 = std::chrono::steady_clock::now ();
			HIPCHK (hipEventSynchronize (e->upEv));
			if (getenv ("TBF_DEBUG_HOST_PHASES"))
				fprintf (stderr, "chunk %llu: staging wait %.3f ms\n", (unsigned long long)e->chunkSeq,
				         std::chrono::duration<double, std::milli> (std::chrono::steady_clock::now () - w0).count ());
		}
		if (e->devCtl && e->regionVer[rp] != e->ctlVer) {
			/* this region's persistent entries: the control as of the START of this chunk (an
			 * instance renders its blocks before its first delta with entry i) */
			if (!dpipe && (rc = joinStages (e, s)))
				return rc;
			if ((rc = usWait ()))
				return rc;
			e->hCtlPin.resize (n);
			memcpy ((void*)e->hCtlPin.data (), e->hCtl.data (), n * sizeof (tbf_seg_ctl));
			HIPCHK (hipMemcpyAsync (e->ctl.p + rp * CTL_REGION (n), e->hCtlPin.data (), n * sizeof (tbf_seg_ctl),
			                        hipMemcpyHostToDevice, us));
			e->regionVer[rp] = e->ctlVer;
		}
		e->dCtl.clear ();
		e->dSeg.clear ();
		e->dProg.clear ();
		e->hRec.clear ();
		e->hMsg.clear ();
		e->hGain.clear ();
		e->hWh.clear ();
		e->hCtlInst.clear ();
		e->hDInst.clear ();
		e->hFull.clear ();
		e->stepped.assign (n, 0);
		e->dhas.assign (n, 0);
		e->hIdx.resize ((size_t)want * n);
		std::vector<uint32_t>& cur = e->curIdx;
		cur.resize (n);
		for (uint32_t i = 0; i < n; i++)
			cur[i] = i;
		bool       delta = false;
		uint32_t   len   = 0;
		const auto hc0   = std::chrono::steady_clock::now ();
		/* device control with many active instances: the chunk's host control on worker
		 * threads (serial when a programme change is among the events) */
		/* the chunk's events (sorted by block: a binary search), checked in parallel (a serial
		 * pass cost ~0.5 ms at 524k events) */
		uint32_t evEnd = evi;
		{
			uint32_t lo = evi, hi = nev;
			while (lo < hi) {
				const uint32_t mid = lo + (hi - lo) / 2;
				if (ev[mid].block < b0 + want)
					lo = mid + 1;
				else
					hi = mid;
			}
			evEnd = lo;
		}
		/* a chunk of note, drawbar and switch events only (frontParam) on clean instances: the
		 * device front end */
		bool       progEv = false, badEv = false, front = false;
		const bool frontCand = e->devCtl && dpipe && e->frontOn && evEnd - evi >= e->frontMin && frontCleanAll (e);
		ChunkScan& cs        = e->scan;
		const auto sc0       = std::chrono::steady_clock::now ();
		scanChunk (n, b0, ev, evi, evEnd, frontCand ? e->fclean.data () : nullptr, progEv, badEv, front, cs);
		if (getenv ("TBF_DEBUG_HOST_PHASES"))
			fprintf (stderr, "chunk %llu: clean %.3f ms, scan %.3f ms (%u events)\n", (unsigned long long)e->chunkSeq,
			         std::chrono::duration<double, std::milli> (sc0 - hc0).count (),
			         std::chrono::duration<double, std::milli> (std::chrono::steady_clock::now () - sc0).count (), evEnd - evi);
		if (badEv)
			return fail (-22, "event for a bad instance");
		bool dfront = false;
		if (frontCand && front && !progEv) {
			if ((rc = stepChunkFront (e, n, want, b0, ev, evi, evEnd, cs, delta)))
				return rc;
			evi    = evEnd;
			len    = want;
			dfront = true;
			e->frontChunks[0]++;
			if (getenv ("TBF_DEBUG_HOST_PHASES"))
				fprintf (stderr, "chunk %llu: device front end, %u note events\n", (unsigned long long)e->chunkSeq,
				         e->hFevOff[n]);
		}
		else {
			if (evEnd > evi)
				e->frontChunks[1]++;
			/* many instances to step: active now, or touched by this chunk's events */
			if (e->devCtl && !progEv && e->parCtl && e->actList.size () + (evEnd - evi) >= 1024) {
				if ((rc = stepChunkParallel (e, n, want, b0, ev, evi, evEnd, rp, delta)))
					return rc;
				evi = evEnd;
				len = want;
			}
		}
		for (; len < want; len++) {
			if (!e->devCtl && e->dProg.size () + (size_t)n * SLOT > dprogCap && len > 0)
				break; /* delta program pool full: end the chunk here */
			if (delta && len >= TBF_CHUNK)
				break; /* a chunk with deltas ends at TBF_CHUNK blocks, before the next block's events */
			for (; evi < nev && ev[evi].block <= b0 + len; evi++) {
				rc = applyEvent (e, ev[evi]);
				if (rc)
					return rc;
				markActive (e, ev[evi].inst);
			}
			/* only the instances whose control may still change are stepped: one that
			 * steps to no change stays unchanged until an event touches it */
			const bool hadDelta = delta;
			size_t     keep     = 0;
			for (size_t a = 0; a < e->actList.size (); a++) {
				const uint32_t i = e->actList[a];
				bool           pc;
				tbf_tgc_rec    rec;
				if (stepControl (e, i, pc, e->devCtl ? &rec : nullptr)) {
					tbf_seg_ctl c = e->hCtl[i];
					if (e->devCtl) {
						/* a stepped delta gets its own program slot, which k_tgctl fills; the
						 * others play the program before them */
						if (pc) {
							c.prog_off = (uint32_t)(PERSIST (n) + ((size_t)rp * n * TBF_CHUNK + e->dCtl.size ()) * SLOT);
							if (!e->stepped[i]) {
								e->stepped[i] = 1;
								e->hCtlInst.push_back (i);
							}
						} else {
							memset (&rec, 0, sizeof (rec));
							if (cur[i] >= n)
								c.prog_off = e->dCtl[cur[i] - n].prog_off;
						}
						if (!e->dhas[i]) {
							e->dhas[i] = 1;
							e->hDInst.push_back (i);
						}
						e->hFull.push_back (c); /* every delta a full entry on this path */
						rec.full = (uint32_t)e->hFull.size ();
						e->hRec.push_back (rec);
					} else if (pc) {
						c.prog_off = (uint32_t)(PERSIST (n) + e->dProg.size ());
						e->dProg.insert (e->dProg.end (), e->hProg.begin () + PSLOTS * i * SLOT,
						                 e->hProg.begin () + PSLOTS * i * SLOT + 1 + c.prog_len);
					} else if (cur[i] >= n)
						c.prog_off = e->dCtl[cur[i] - n].prog_off; /* program of the previous delta */
					cur[i] = n + (uint32_t)e->dCtl.size ();
					e->dCtl.push_back (c);
					e->chg[i] = 1;
					delta     = true;
					e->actList[keep++] = i;
				} else
					e->inAct[i] = 0;
			}
			e->actList.resize (keep);
			/* entry index table: written only once the chunk has a delta (before that
			 * every row is the identity) */
			if (delta) {
				if (!hadDelta)
					for (uint32_t r = 0; r < len; r++)
						for (uint32_t i = 0; i < n; i++)
							e->hIdx[(size_t)r * n + i] = i;
				std::copy (cur.begin (), cur.end (), e->hIdx.begin () + (size_t)len * n);
			}
		}
		e->hostCtlNs += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds> (
		                    std::chrono::steady_clock::now () - hc0)
		                    .count ();
		e->hostCtlBlocks += len;
		if (delta && len > TBF_CHUNK)
			return fail (-5, "internal: a chunk with control deltas longer than 64 blocks");
		const bool     piped   = pipe && (!delta || dpipe);
		auto at = [&] (int b) { return e->stageDbl[b] ? (size_t)bset * need : (size_t)0; };
		P.mid0 = e->mid0.p + 2 * at (0);
		P.mid1 = e->mid1.p ? e->mid1.p + at (1) : nullptr;
		P.mid2 = e->mid2.p ? e->mid2.p + at (4) : nullptr;
		P.rvA  = e->rvA.p ? e->rvA.p + 2 * at (2) : nullptr;
		P.rvB  = e->rvB.p ? e->rvB.p + 2 * at (3) : nullptr;
		if (!piped && (rc = joinStages (e, s)))
			return rc;
		if (delta) {
			/* device control: both regions' delta slots, sized once for a delta per
			 * instance and block (growProg synchronizes the device when it grows) */
			if (e->devCtl && (rc = growProg (e, PERSIST (n) + 2 * (size_t)n * TBF_CHUNK * SLOT, n)))
				return rc;
			if ((rc = usWait ()))
				return rc;
			if (!e->devCtl) /* device control: k_tgctl writes the deltas' entries (records + full entries) */
				HIPCHK (hipMemcpyAsync (e->ctl.p + rp * CTL_REGION (n) + n, e->dCtl.data (),
				                        e->dCtl.size () * sizeof (tbf_seg_ctl), hipMemcpyHostToDevice, us));
			if (!e->dProg.empty ())
				HIPCHK (hipMemcpyAsync (e->prog.p + PERSIST (n), e->dProg.data (),
				                        e->dProg.size () * sizeof (tbf_prog_entry), hipMemcpyHostToDevice, us));
			if (!dfront) /* (k_front writes the index table) */
				HIPCHK (hipMemcpyAsync (e->ctlIdx.p + (size_t)rp * n * TBF_CHUNK, e->hIdx.data (),
				                        (size_t)len * n * sizeof (uint32_t), hipMemcpyHostToDevice, us));
		}
		P.whSets = nullptr;
		if (delta && !e->hWh.empty ()) {
			/* the whirl parameter sets of the chunk's deltas, by region parity like the records */
			DevBuf<tbf_wh_params>& dw = rp ? e->dwhB : e->dwh;
			if (dw.cap < e->hWh.size ())
				HIPCHK (hipDeviceSynchronize ()); /* growing: nothing may still read the old buffer */
			if (dw.ensure (std::max<size_t> (e->hWh.size (), 64)))
				return fail (-12, "out of device memory (whirl parameter sets)");
			HIPCHK (hipMemcpyAsync (dw.p, e->hWh.data (), e->hWh.size () * sizeof (tbf_wh_params), hipMemcpyHostToDevice, us));
			P.whSets = dw.p;
		}
		P.prog      = e->prog.p;
		P.ctl       = e->ctl.p + rp * CTL_REGION (n);
		P.ctlIdx    = delta ? e->ctlIdx.p + (size_t)rp * n * TBF_CHUNK : nullptr;
		P.nBlocks   = len;
		/* k_tonegen block ranges (chunks without deltas) for small batches: about 2048 waves,
		 * ranges of >= 4 blocks (each range after the first renders one warm-up block).  At
		 * 4096 instances a split measured no gain (0.73 ms alone either way: the kernel is
		 * bound by its bank gathers and VALU, not by waves in flight). */
		P.tgSplit = e->tgSplit >= 0 ? (uint32_t)std::max (e->tgSplit, 1)
		                            : std::max (1u, std::min ({8u, 2048u / std::max (n, 1u), len / 4}));
		P.tgSplit = std::min (P.tgSplit, std::max (len, 1u));
		P.outOffset = (uint64_t)b0 * TBF_BLK;
		P.nCtlInst  = 0;
		if (e->devCtl && (dfront ? delta : !e->hDInst.empty ())) {
			/* k_tgctl: the stepped blocks' programs, ahead of k_tonegen on this stream */
			/* records per region parity: k_tgctl of the chunk before last (same stream, or
			 * the caller's stream when not pipelined) read the other set */
			DevBuf<tbf_tgc_rec>& drec = rp ? e->drecB : e->drec;
			DevBuf<uint16_t>&    dmsg = rp ? e->dmsgB : e->dmsg;
			DevBuf<float>&       dgn  = rp ? e->dgainB : e->dgain;
			DevBuf<uint32_t>&    dci  = rp ? e->dctlInstB : e->dctlInst;
			DevBuf<tbf_seg_ctl>& dfl  = rp ? e->dfullB : e->dfull;
			const size_t nRec  = dfront ? (size_t)n * len : e->hRec.size ();
			const size_t nMsg  = dfront ? 2 * (size_t)e->hFevOff[n] : e->hMsg.size ();
			const size_t nGain = dfront ? (size_t)e->frontGain : e->hGain.size ();
			if (drec.cap < nRec || dmsg.cap < nMsg || dci.cap < e->hDInst.size () || dgn.cap < nGain ||
			    dfl.cap < (dfront ? (size_t)n * len : e->hFull.size ()))
			{
				if (getenv ("TBF_DEBUG_HOST_PHASES"))
					fprintf (stderr, "chunk %llu: control record buffers grow (device sync)\n", (unsigned long long)e->chunkSeq);
				HIPCHK (hipDeviceSynchronize ()); /* growing: nothing may still read the old buffers */
			}
			const size_t nFull = dfront ? (size_t)n * len : e->hFull.size (); /* k_front writes its effect entries */
			if (drec.ensure (std::max<size_t> (nRec, 1)) || dmsg.ensure (std::max<size_t> (nMsg, 1)) ||
			    dgn.ensure (std::max<size_t> (nGain, 27)) ||
			    dci.ensure (e->hDInst.size ()) || dfl.ensure (std::max<size_t> (nFull, 1)))
				return fail (-12, "out of device memory (control records)");
			if (dfront) {
				/* k_front: the records, messages and index table from the key states and events */
				DevBuf<tbf_front_state>& dfs = rp ? e->dfrontB : e->dfront;
				DevBuf<uint32_t>&        dfe = rp ? e->dfevB : e->dfev;
				DevBuf<uint32_t>&        dfo = rp ? e->dfoffB : e->dfoff;
				DevBuf<float>&           dfv = rp ? e->dfvalB : e->dfval;
				if (dfs.cap < n || dfe.cap < e->hFev.size () || dfv.cap < e->hFev.size () || dfo.cap < (size_t)n + 1 ||
				    e->dident.cap < n)
					HIPCHK (hipDeviceSynchronize ()); /* growing: nothing may still read the old buffers */
				if (dfs.ensure (n) || dfe.ensure (e->hFev.size ()) || dfv.ensure (e->hFev.size ()) ||
				    dfo.ensure ((size_t)n + 1) || e->dident.ensure (n))
					return fail (-12, "out of device memory (front end)");
				if (e->hIdent.size () != n) {
					e->hIdent.resize (n);
					for (uint32_t i = 0; i < n; i++)
						e->hIdent[i] = i;
					HIPCHK (hipMemcpy (e->dident.p, e->hIdent.data (), (size_t)n * 4, hipMemcpyHostToDevice));
				}
				HIPCHK (hipMemcpyAsync (dfs.p, e->hFront.data (), (size_t)n * sizeof (tbf_front_state), hipMemcpyHostToDevice, us));
				HIPCHK (hipMemcpyAsync (dfe.p, e->hFev.data (), e->hFev.size () * 4, hipMemcpyHostToDevice, us));
				HIPCHK (hipMemcpyAsync (dfo.p, e->hFevOff.data (), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, us));
				HIPCHK (hipMemcpyAsync (dfv.p, e->hFevVal.data (), e->hFev.size () * 4, hipMemcpyHostToDevice, us));
				P.front   = dfs.p;
				P.fev     = dfe.p;
				P.fevVal  = dfv.p;
				P.fulls   = dfl.p;
				P.fevOff  = dfo.p;
				P.keyComp = e->dkeyComp.p;
				P.rec     = drec.p;
				P.msgs    = dmsg.p;
				P.gains   = dgn.p;
				if ((rc = tbf_launch_front (&P, us)))
					return fail (rc, std::string ("k_front launch failed: ") + hipGetErrorString (hipGetLastError ()));
			}
			if (!dfront && e->dSeg.empty ())
				HIPCHK (hipMemcpyAsync (drec.p, e->hRec.data (), e->hRec.size () * sizeof (tbf_tgc_rec),
				                        hipMemcpyHostToDevice, us));
			for (const auto& g : e->dSeg)
				if (!dfront && g.second)
					HIPCHK (hipMemcpyAsync (drec.p + g.first, e->hRec.data () + g.first,
					                        g.second * sizeof (tbf_tgc_rec), hipMemcpyHostToDevice, us));
			if (!dfront && !e->hMsg.empty ())
				HIPCHK (hipMemcpyAsync (dmsg.p, e->hMsg.data (), e->hMsg.size () * sizeof (uint16_t),
				                        hipMemcpyHostToDevice, us));
			if (!dfront && !e->hGain.empty ())
				HIPCHK (hipMemcpyAsync (dgn.p, e->hGain.data (), e->hGain.size () * sizeof (float),
				                        hipMemcpyHostToDevice, us));
			if (!dfront && !e->hFull.empty ())
				HIPCHK (hipMemcpyAsync (dfl.p, e->hFull.data (), e->hFull.size () * sizeof (tbf_seg_ctl),
				                        hipMemcpyHostToDevice, us));
			if (!dfront)
				HIPCHK (hipMemcpyAsync (dci.p, e->hDInst.data (), e->hDInst.size () * 4, hipMemcpyHostToDevice, us));
			P.tgc      = e->tgc.p;
			P.rec      = drec.p;
			P.msgs     = dmsg.p;
			P.gains    = dgn.p;
			P.ctlInst  = dfront ? e->dident.p : dci.p;
			P.nCtlInst = dfront ? n : (uint32_t)e->hDInst.size ();
			P.fulls    = dfl.p;
			P.progBase = (uint32_t)(PERSIST (n) + (size_t)rp * n * TBF_CHUNK * SLOT);
			P.coff     = e->coff.p;
			P.contrib  = e->contrib.p;
			P.ctlNw    = e->ctlNw;
			if ((rc = tbf_launch_tgctl (&P, us)))
				return fail (rc, std::string ("k_tgctl launch failed: ") + hipGetErrorString (hipGetLastError ()));
		}
		if (e->devCtl)
			HIPCHK (hipEventRecord (e->upEv, us)); /* this parity's staging is free after it */
		if (usWaited && piped) /* the stage streams now follow the uploads on us */
			e->stagesBusy = true;
		const int nst = tbf_chain_stages (P.chain);
		if (piped) {
			/* stage-group streams: every chunk's stage k on stream gs[grp[k]], so a stage runs
			 * as soon as this chunk's previous stage and the previous chunk's same stage are
			 * done, whatever the later stages of the previous chunk are doing.  Buffer parity
			 * par was last read by the chunk before last: wait for those readers (stage k's
			 * output mid0 is read by k_mixpre, mid1 by k_rv_pre and k_rv_post, rvA by
			 * k_rv_core, rvB by k_rv_post, mid2 by k_whirl) when they run on another stream. */
			static const int readers[TBF_NSTAGES][2] = {{1, -1}, {2, 4}, {3, -1}, {4, -1}, {5, -1}, {-1, -1}};
			auto strm = [&] (int k) { return e->gs[e->grp[k]]; };
			for (int k = 0; k < nst; k++) {
				hipStream_t sk = strm (k);
				if (k == 0 && !e->stagesBusy) { /* after the caller's stream (uploads, earlier chunks) */
					HIPCHK (hipEventRecord (e->sjoin, s));
					HIPCHK (hipStreamWaitEvent (sk, e->sjoin, 0));
				}
				if (k == nst - 1 && !outWait) { /* the output stage writes the caller's buffers */
					HIPCHK (hipEventRecord (e->sjoin, s));
					HIPCHK (hipStreamWaitEvent (sk, e->sjoin, 0));
					outWait = true;
				}
				if (k > 0 && strm (k - 1) != sk)
					HIPCHK (hipStreamWaitEvent (sk, e->sdone[k - 1], 0));
				for (int r : readers[k])
					if (r >= 0 && r < nst && strm (r) != sk)
						HIPCHK (hipStreamWaitEvent (sk, e->pev[(cix + 2) & 3][r], 0));
				hipEvent_t e0 = nullptr, e1 = nullptr;
				if (e->timeOn) {
					HIPCHK (hipEventCreate (&e0));
					HIPCHK (hipEventCreate (&e1));
					HIPCHK (hipEventRecord (e0, sk));
				}
				rc = tbf_launch_stage (&P, k, sk);
				if (rc)
					return fail (rc, std::string ("kernel launch failed: ") + hipGetErrorString (hipGetLastError ()));
				if (e->timeOn) {
					HIPCHK (hipEventRecord (e1, sk));
					e->tev.push_back ({k, {e0, e1}});
				}
				HIPCHK (hipEventRecord (e->sdone[k], sk));
				HIPCHK (hipEventRecord (e->pev[cix & 3][k], sk));
			}
			e->stagesBusy = true;
			if (delta && (rc = endDelta ()))
				return rc;
			b0 += len;
			continue;
		}
		for (int k = 0; k < nst; k++) {
			hipEvent_t e0 = nullptr, e1 = nullptr;
			if (e->timeOn) {
				HIPCHK (hipEventCreate (&e0));
				HIPCHK (hipEventCreate (&e1));
				HIPCHK (hipEventRecord (e0, s));
			}
			rc = tbf_launch_stage (&P, k, s);
			if (rc)
				return fail (rc, std::string ("kernel launch failed: ") + hipGetErrorString (hipGetLastError ()));
			if (e->timeOn) {
				HIPCHK (hipEventRecord (e1, s));
				e->tev.push_back ({k, {e0, e1}});
			}
		}
		if (delta && (rc = endDelta ()))
			return rc;
		b0 += len;
	}
	for (; evi < nev; evi++) { /* events at or after the last block apply to the next render */
		rc = applyEvent (e, ev[evi]);
		if (rc)
			return rc;
	}
	if (e->stagesBusy) {
		/* the caller's stream waits for the last chunk's output stage (which follows
		 * every earlier stage launch); later chunks keep overlapping from the streams */
		HIPCHK (hipStreamWaitEvent (s, e->sdone[tbf_chain_stages (P.chain) - 1], 0));
	}
	return 0;
}

extern "C" {

int tbf_render_device (tbf_engine* e, uint32_t nblocks, float* dL, float* dR, uint64_t stride, void* stream)
{
	if (!e || !dL || !dR)
		return fail (-22, "null argument");
	if (e->cfg.device < 0)
		return fail (-19, "host-only engine (device -1) cannot render");
	HIPCHK (hipSetDevice (e->cfg.device));
	return renderImpl (e, nblocks, dL, dR, stride, stream ? (hipStream_t)stream : e->stream);
}

int tbf_render_events (tbf_engine* e, uint32_t nblocks, const tbf_event* ev, uint32_t nev, float* dL, float* dR,
                       uint64_t stride, void* stream)
{
	if (!e || !dL || !dR || (nev && !ev))
		return fail (-22, "null argument");
	if (e->cfg.device < 0)
		return fail (-19, "host-only engine (device -1) cannot render");
	{ /* sorted by block (in parallel: large event lists) */
		const unsigned    T  = std::max (1u, std::min (hostThreads (), (nev + 32767) / 32768));
		const uint32_t    sg = (nev + T - 1) / T;
		std::vector<char> bad (T, 0);
		parallelFor (T, [&] (uint32_t t) {
			const uint32_t k0 = std::max (1u, std::min (nev, t * sg)), k1 = std::min (nev, (t + 1) * sg);
			for (uint32_t k = k0; k < k1; k++)
				if (ev[k].block < ev[k - 1].block) {
					bad[t] = 1;
					return;
				}
		});
		for (char b : bad)
			if (b)
				return fail (-22, "events must be sorted by block");
	}
	HIPCHK (hipSetDevice (e->cfg.device));
	return renderImpl (e, nblocks, dL, dR, stride, stream ? (hipStream_t)stream : e->stream, ev, nev);
}

int tbf_render (tbf_engine* e, uint32_t nblocks, float* outL, float* outR, uint64_t stride)
{
	if (!e || !outL || !outR)
		return fail (-22, "null argument");
	if (e->cfg.device < 0)
		return fail (-19, "host-only engine (device -1) cannot render");
	HIPCHK (hipSetDevice (e->cfg.device));
	const uint32_t n   = (uint32_t)e->inst.size ();
	const size_t   per = (size_t)nblocks * TBF_BLK;
	if (stride < per)
		return fail (-22, "stride smaller than nblocks*128");
	if (e->outL.ensure ((size_t)n * per) || e->outR.ensure ((size_t)n * per))
		return fail (-12, "out of device memory (outputs)");
	int rc = renderImpl (e, nblocks, e->outL.p, e->outR.p, per, e->stream);
	if (rc)
		return rc;
	HIPCHK (hipMemcpy2DAsync (outL, stride * 4, e->outL.p, per * 4, per * 4, n, hipMemcpyDeviceToHost, e->stream));
	HIPCHK (hipMemcpy2DAsync (outR, stride * 4, e->outR.p, per * 4, per * 4, n, hipMemcpyDeviceToHost, e->stream));
	HIPCHK (hipStreamSynchronize (e->stream));
	return 0;
}

int tbf_synth_sound (tbf_engine* e, uint32_t nframes, float* outL, float* outR, uint64_t stride)
{
	if (!e || !outL || !outR)
		return fail (-22, "null argument");
	if (stride < nframes)
		return fail (-22, "stride smaller than nframes");
	const uint32_t n = (uint32_t)e->inst.size ();
	if (n != e->fifoN) {
		/* instances added since the FIFO was filled: they join at the next block (zeros
		 * for the rest of the current one); the others keep their buffered samples */
		std::vector<float> L ((size_t)n * e->fifoLen, 0.f), R ((size_t)n * e->fifoLen, 0.f);
		for (uint32_t i = 0; i < std::min (n, e->fifoN); i++) {
			std::copy_n (e->fifoL.begin () + (size_t)i * e->fifoLen, e->fifoLen, L.begin () + (size_t)i * e->fifoLen);
			std::copy_n (e->fifoR.begin () + (size_t)i * e->fifoLen, e->fifoLen, R.begin () + (size_t)i * e->fifoLen);
		}
		e->fifoL.swap (L);
		e->fifoR.swap (R);
		e->fifoN = n;
	}
	uint32_t written = 0;
	while (written < nframes) {
		if (e->boffset >= e->fifoLen) {
			/* the 128-sample FIFO of synthSound (b_synth/lv2.cpp:1270-1287, src/clap.cpp
			 * PluginRenderAudio) ran dry: render every block this call still needs in one
			 * launch (no event can land between them, so the samples are those of
			 * block-by-block rendering) */
			const uint32_t m = std::min<uint32_t> ((nframes - written + TBF_BLK - 1) / TBF_BLK, 64);
			e->fifoLen       = m * TBF_BLK;
			e->fifoL.resize ((size_t)n * e->fifoLen);
			e->fifoR.resize ((size_t)n * e->fifoLen);
			e->boffset = 0;
			int rc     = tbf_render (e, m, e->fifoL.data (), e->fifoR.data (), e->fifoLen);
			if (rc)
				return rc;
		}
		const uint32_t nread = std::min (nframes - written, e->fifoLen - e->boffset);
		for (uint32_t i = 0; i < n; i++) {
			memcpy (outL + (size_t)i * stride + written, e->fifoL.data () + (size_t)i * e->fifoLen + e->boffset, nread * 4);
			memcpy (outR + (size_t)i * stride + written, e->fifoR.data () + (size_t)i * e->fifoLen + e->boffset, nread * 4);
		}
		written += nread;
		e->boffset += nread;
	}
	return 0;
}

int tbf_synchronize (tbf_engine* e)
{
	if (!e)
		return fail (-22, "null argument");
	if (e->cfg.device < 0)
		return 0;
	HIPCHK (hipSetDevice (e->cfg.device));
	HIPCHK (hipStreamSynchronize (e->stream));
	return drainStages (e);
}

int tbf_error_flags (tbf_engine* e, uint32_t* flags)
{
	if (!e || !flags)
		return fail (-22, "null argument");
	*flags = 0;
	if (!e->err.p)
		return 0;
	HIPCHK (hipSetDevice (e->cfg.device));
	if (int rc = drainStages (e))
		return rc;
	/* the engine stream carries the non-pipelined chunks: read after them, on it */
	HIPCHK (hipMemcpyAsync (flags, e->err.p, 4, hipMemcpyDeviceToHost, e->stream));
	HIPCHK (hipStreamSynchronize (e->stream));
	return 0;
}

int tbf_debug_contrib (tbf_engine* e, uint32_t tid, int32_t key, int16_t* wheel, int16_t* bus, float* level,
                       uint32_t cap)
{
	if (!e || tid >= e->tpls.size () || key < 0 || key >= 384)
		return fail (-22, "bad argument");
	const auto& v = e->tpls[tid]->keyContrib[key];
	for (uint32_t i = 0; i < v.size () && i < cap; i++) {
		wheel[i] = v[i].wheel;
		bus[i]   = v[i].bus;
		level[i] = v[i].level;
	}
	return (int)v.size ();
}

int tbf_debug_tables (tbf_engine* e, uint32_t tid, float* attack, float* release, float* keycomp)
{
	if (!e || tid >= e->tpls.size ())
		return fail (-22, "bad argument");
	const TgTemplate& t = *e->tpls[tid];
	if (attack) memcpy (attack, t.attackEnv, sizeof (t.attackEnv));
	if (release) memcpy (release, t.releaseEnv, sizeof (t.releaseEnv));
	if (keycomp) memcpy (keycomp, t.keyCompTable, sizeof (t.keyCompTable));
	return 0;
}

int tbf_debug_device_program (tbf_engine* e, uint32_t i, float* out, uint32_t cap)
{
	if (!e || i >= e->inst.size () || e->cfg.device < 0 || i >= e->hCtl.size ())
		return fail (-22, "bad instance");
	HIPCHK (hipSetDevice (e->cfg.device));
	if (int rc = drainStages (e))
		return rc;
	HIPCHK (hipStreamSynchronize (e->stream));
	HIPCHK (hipDeviceSynchronize ());
	std::vector<tbf_prog_entry> v (SLOT);
	HIPCHK (hipMemcpy (v.data (), e->prog.p + e->hCtl[i].prog_off, SLOT * sizeof (tbf_prog_entry), hipMemcpyDeviceToHost));
	const uint32_t np = std::min<uint32_t> (v[0].pad, (uint32_t)SLOT - 1);
	for (uint32_t q = 0; q < np && q < cap; q++) {
		const tbf_prog_entry& p = v[1 + q];
		float*                o = out + 9 * q;
		o[0] = p.wheel; o[1] = p.env; o[2] = p.row;
		o[3] = p.sg; o[4] = p.pg; o[5] = p.vg; o[6] = p.nsg; o[7] = p.npg; o[8] = p.nvg;
	}
	return (int)np;
}

int tbf_debug_pool_check (uint32_t jobs)
{
	std::vector<std::atomic<int>> hits (64);
	int                           bad = 0;
	for (uint32_t it = 0; it < jobs; it++) {
		const uint32_t n = 1 + (it * 7919u) % 40;
		for (auto& h : hits)
			h.store (0);
		parallelFor (n, [&] (uint32_t t) {
			hits[t].fetch_add (1);
			if ((t & 7) == 0)
				std::this_thread::yield ();
		});
		bool ok = true;
		for (uint32_t i = 0; i < 64; i++)
			ok = ok && hits[i].load () == (i < n ? 1 : 0);
		bad += ok ? 0 : 1;
	}
	return bad;
}

int tbf_debug_host_time (tbf_engine* e, int32_t reset, double* ms, uint64_t* blocks)
{
	if (!e)
		return fail (-22, "null argument");
	if (ms) *ms = (double)e->hostCtlNs * 1e-6;
	if (blocks) *blocks = e->hostCtlBlocks;
	if (reset)
		e->hostCtlNs = e->hostCtlBlocks = 0;
	return 0;
}

int tbf_debug_layout (const tbf_engine* e, uint32_t* wring_len, float* max_ahead, uint32_t* slab_len)
{
	if (!e)
		return fail (-22, "null argument");
	if (wring_len) *wring_len = e->wringLen;
	if (max_ahead) *max_ahead = e->wt.maxAhead;
	if (slab_len) *slab_len = e->slabLen;
	return 0;
}

int tbf_debug_chunks (const tbf_engine* e, uint32_t* delta_blocks, uint32_t* steady_blocks)
{
	if (!e)
		return fail (-22, "null argument");
	if (delta_blocks) *delta_blocks = TBF_CHUNK;
	if (steady_blocks) *steady_blocks = e->steadyChunk;
	return 0;
}

int tbf_debug_front_chunks (const tbf_engine* e, uint64_t* device_chunks, uint64_t* host_chunks)
{
	if (!e)
		return fail (-22, "null argument");
	if (device_chunks) *device_chunks = e->frontChunks[0];
	if (host_chunks) *host_chunks = e->frontChunks[1];
	return 0;
}

int tbf_set_steady_chunk (tbf_engine* e, uint32_t blocks)
{
	if (!e)
		return fail (-22, "null argument");
	e->steadyChunk = std::min (std::max (blocks, (uint32_t)TBF_CHUNK), (uint32_t)TBF_STEADY_MAX);
	/* clamped here to what the device can hold for the current instances (the stage
	 * buffers' footprint against the free memory plus the buffers held now), so the value
	 * returned is the one renders use; stageBuffers still halves it on an allocation failure */
	const size_t n = e->inst.size ();
	if (e->cfg.device >= 0 && n) {
		size_t freeB = 0, totalB = 0;
		if (hipSetDevice (e->cfg.device) == hipSuccess && hipMemGetInfo (&freeB, &totalB) == hipSuccess) {
			const size_t held = (e->mid0.cap + e->mid1.cap + e->mid2.cap) * sizeof (float) + (e->rvA.cap + e->rvB.cap) * sizeof (double);
			while (e->steadyChunk > TBF_CHUNK && stageFootprint (e, n, e->steadyChunk) > freeB + held)
				e->steadyChunk /= 2;
		} else
			(void)hipGetLastError ();
	}
	if (e->stageBlocks > e->steadyChunk)
		e->stageN = 0; /* reallocated (smaller) at the next render */
	return (int)e->steadyChunk;
}

int tbf_debug_reverb_phase (tbf_engine* e, uint32_t i, int32_t ch, int32_t line, double value)
{
	if (!e || i >= e->inst.size () || ch < 0 || ch > 1 || line < 0 || line > 7)
		return fail (-22, "bad arguments");
	e->inst[i].s0.rv.ch[ch].vib[line] = value; /* an instance not on the device yet takes it at upload */
	if (e->deviceReady && i < e->devInst) {
		HIPCHK (hipSetDevice (e->cfg.device));
		if (int rc = drainStages (e))
			return rc;
		HIPCHK (hipStreamSynchronize (e->stream));
		HIPCHK (hipMemcpy (&e->st.p[i].rv.ch[ch].vib[line], &value, sizeof (double), hipMemcpyHostToDevice));
	}
	return 0;
}

int tbf_debug_step (tbf_engine* e, uint32_t i, float* out, uint32_t cap)
{
	if (!e || i >= e->inst.size ())
		return fail (-22, "bad instance");
	if (e->devCtl)
		return fail (-95, "host programs: the per-wheel control runs on the device (TBF_HOST_CONTROL=1 for the host path)");
	Instance& in = e->inst[i];
	tbf_seg_ctl c;
	memset (&c, 0, sizeof (c));
	in.tg.step (in.prog, c);
	in.progDirty = in.ctlDirty = true;
	markActive (e, i);
	for (uint32_t q = 0; q < in.prog.size () && q < cap; q++) {
		const tbf_prog_entry& p = in.prog[q];
		float*                o = out + 9 * q;
		o[0] = p.wheel; o[1] = p.env; o[2] = p.row;
		o[3] = p.sg; o[4] = p.pg; o[5] = p.vg; o[6] = p.nsg; o[7] = p.npg; o[8] = p.nvg;
	}
	return (int)in.prog.size ();
}

int tbf_debug_render_program (tbf_engine* e, uint32_t i, float* out, uint32_t cap)
{
	if (!e || i >= e->inst.size ())
		return fail (-22, "bad instance");
	if (e->devCtl)
		return fail (-95, "host programs: the per-wheel control runs on the device (TBF_HOST_CONTROL=1 for the host path)");
	const size_t n = e->inst.size ();
	if (e->hCtl.size () < n) { /* a host-only engine never sized the pool */
		e->hCtl.resize (n);
		e->hProg.resize (PERSIST (n));
	}
	bool pc;
	(void)stepControl (e, i, pc); /* exactly the per-block step renderImpl makes */
	const std::vector<tbf_prog_entry>& prog = e->inst[i].prog;
	for (uint32_t q = 0; q < prog.size () && q < cap; q++) {
		const tbf_prog_entry& p = prog[q];
		float*                o = out + 9 * q;
		o[0] = p.wheel; o[1] = p.env; o[2] = p.row;
		o[3] = p.sg; o[4] = p.pg; o[5] = p.vg; o[6] = p.nsg; o[7] = p.npg; o[8] = p.nvg;
	}
	return (int)prog.size ();
}

int tbf_debug_exact (int32_t op, const double* in, double* out, uint32_t n)
{
	if (!in || !out || op < 0 || op > 5)
		return fail (-22, "bad arguments");
	static std::vector<uint32_t> J;
	if (op == 3 && J.empty ()) { /* the device layout: bit rows, then the nibble-sliced rows */
		J.resize (32 * TBF_XS_JUMP + 128 * TBF_XS_JUMP);
		xs_jump_table (J.data (), TBF_XS_JUMP);
		xs_nib_table (J.data () + 32 * TBF_XS_JUMP, J.data (), TBF_XS_JUMP);
	}
	for (uint32_t i = 0; i < n; i++) {
		const double* a = in + 3 * i;
		double*       o = out + 2 * i;
		o[0] = o[1] = 0.0;
		if (op == 0) {
			double D = 0.0;
			o[0]     = phase_run (a[0], a[1], (int)a[2], D) ? 1.0 : 0.0;
			o[1]     = D;
		} else if (op == 1) {
			o[0] = cnt_adv ((int)a[0], (int)a[1], (int)a[2]);
		} else if (op == 2) {
			o[0] = wrap1 (a[0]);
		} else if (op == 5) {
			GlibcRand j ((unsigned)a[0]), l ((unsigned)a[0]);
			j.discard ((uint64_t)a[1]);
			for (uint64_t q = 0; q < (uint64_t)a[1]; q++)
				l.next ();
			o[0] = j.next ();
			o[1] = l.next ();
		} else if (op == 4) {
			/* op 4: phase_run_cached along a run of 4096 sub-blocks of m steps from v0
			 * (advancing like the kernel) vs phase_run: out = mismatches, cache hits */
			double   v = a[0], cD = 0, cLo = 0, cHi = 0;
			const int m = (int)a[2];
			uint32_t bad = 0, hits = 0;
			for (int s = 0; s < 4096; s++) {
				double    D1 = 0, D2 = 0;
				const double pD = cD;
				const bool ok1 = phase_run (v, a[1], m, D1);
				const bool ok2 = phase_run_cached (v, a[1], m, D2, cD, cLo, cHi);
				hits += (pD > 0 && cD == pD && ok2) ? 1 : 0;
				if (ok1 != ok2 || (ok1 && D1 != D2))
					bad++;
				if (ok1)
					v = v + (double)m * D1;
				else
					for (int q = 0; q < m; q++)
						v += a[1];
			}
			o[0] = bad;
			o[1] = hits;
		} else {
			/* op 3: xorshift jump as the kernels take it (nibble-sliced table, which must
			 * agree with the bit-row form) vs k literal steps from x0 */
			const uint32_t x0 = (uint32_t)a[0];
			const int      k  = (int)a[1];
			if (k < 0 || k >= TBF_XS_JUMP)
				return fail (-22, "jump length out of range");
			uint32_t x = x0;
			for (int q = 0; q < k; q++)
				x = xs_step (x);
			const uint32_t* N = J.data () + 32 * TBF_XS_JUMP;
			uint32_t        r = 0;
			for (int q = 0; q < 8; q++)
				r ^= N[(q * 16 + ((x0 >> (4 * q)) & 15u)) * TBF_XS_JUMP + k];
			if (r != xs_jump_ref (J.data (), TBF_XS_JUMP, x0, k))
				return fail (-5, "nibble-sliced jump differs from the bit-row jump");
			o[0] = r;
			o[1] = x;
		}
	}
	return 0;
}

int tbf_debug_calibrate (int32_t op, void* buf, uint64_t n, void* stream)
{
	if (!buf || op < 0 || op > 12 || n < 16)
		return fail (-22, "bad arguments");
	int rc = tbf_launch_calibrate (op, buf, n, (hipStream_t)stream);
	return rc ? fail (rc, "calibration launch failed") : 0;
}

int tbf_debug_kernel_times (tbf_engine* e, int32_t enable, double* ms6, uint32_t* count6)
{
	if (!e)
		return fail (-22, "null engine");
	if (enable == 1 || enable == 2 || enable == -1) {
		e->timeOn     = enable >= 1;
		e->timeSerial = enable == 2;
		return 0;
	}
	if (e->cfg.device >= 0)
		HIPCHK (hipSetDevice (e->cfg.device));
	double   ms[TBF_NSTAGES] = {0};
	uint32_t cnt[TBF_NSTAGES] = {0};
	for (auto& t : e->tev) {
		HIPCHK (hipEventSynchronize (t.second.second));
		float v = 0.f;
		HIPCHK (hipEventElapsedTime (&v, t.second.first, t.second.second));
		ms[t.first] += v;
		cnt[t.first]++;
		(void)hipEventDestroy (t.second.first);
		(void)hipEventDestroy (t.second.second);
	}
	e->tev.clear ();
	for (int k = 0; k < TBF_NSTAGES; k++) {
		if (ms6) ms6[k] = ms[k];
		if (count6) count6[k] = cnt[k];
	}
	return 0;
}

} /* extern "C" */
