/*
 * tbf_engine_impl.h -- private engine state shared by the C-ABI translation units
 * (tbf_engine.cpp: construction, device setup, rendering; tbf_control.cpp: MIDI control
 * functions and programmes).  Not part of the ABI.
 */
#ifndef TBF_ENGINE_IMPL_H
#define TBF_ENGINE_IMPL_H

#include <hip/hip_runtime.h>

#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <utility>
#include <algorithm>
#include <vector>

#include "../../include/tbf.h"
#include "tbf_host.h"
#include "tbf_types.h"

namespace tbf {

/* one programme of the .pgm table (struct _programme, src/program.h:104-140; the
 * fields the engine applies) */
struct Programme {
	uint32_t flags = 0;
	char     name[32] = {0};
	unsigned drawbars[9] = {0}, lowerDrawbars[9] = {0}, pedalDrawbars[9] = {0};
	uint32_t scanner = 0;
	int      percussionEnabled = 0, percussionVolume = 0, percussionSpeed = 0, percussionHarmonic = 0;
	int      overdriveSelect = 0;
	int      rotarySpeedSelect = 0;
	float    reverbMix = 0.f;
	int      keyboardSplitLower = 0, keyboardSplitPedals = 0;
	int      transpose[7] = {0};
};

int  fail (int code, const std::string& msg);
int  controlById (struct Instance& in, int id, int value); /* tbf_control.cpp */
void setCharacter (struct Instance& in, float v);

} // namespace tbf

namespace tbf {

struct Instance {
	uint32_t       tpl = 0;
	TgControl      tg;
	tbf_inst_const k;
	tbf_inst_state s0;
	tbf_seg_ctl    ctl;
	double         params[64];
	/* preamp (struct b_preamp) */
	int            odClean = 1;
	float          odA = 0.0f, odB = 0.0f, odC = 1.0f, odD = 0.5f;
	struct OdCache { /* the preamp's control fields for these parameters (odCtl) */
		float       A = 0.f, B = 0.f, C = 0.f, D = 0.f;
		int         clean = 0;
		bool        valid = false;
		tbf_seg_ctl ctl;
	} odc;
	/* reverb mix */
	float          rvG = 0.1f;
	int            whBypass = 0;
	int            revOpt = -1;   /* useRevOption (n) pending for the next block */
	int            revSelect = 0; /* whirl revSelect: WHIRL_SLOW after initWhirl (src/whirl.cpp:1131) */
	WhirlRt        whr;           /* the whirl's MIDI-settable fields ... */
	bool           whDirty = false; /* ... changed since the last block's parameter set */
	GlibcRand      ctlRand{1};    /* control-plane rand() stream (randomizeDrawbars) */
	bool           ctlDirty = true;
	bool           progDirty = true;
	std::vector<tbf_prog_entry> prog;
};

/* host staging in pinned memory (pageable memory if no device: host-only engines), so
 * uploads from it are truly asynchronous; the renderer double-buffers these by chunk */
template <typename T>
struct PinnedVec {
	T*     p      = nullptr;
	size_t n      = 0, cap = 0;
	bool   pinned = false;
	PinnedVec ()  = default;
	PinnedVec (const PinnedVec&) = delete;
	PinnedVec& operator= (const PinnedVec&) = delete;
	~PinnedVec () { release (); }
	void release ()
	{
		if (p && pinned)
			(void)hipHostFree (p);
		else
			free (p);
		p   = nullptr;
		n   = cap = 0;
	}
	void reserve (size_t c)
	{
		if (c <= cap)
			return;
		const size_t nc = std::max<size_t> (std::max<size_t> (c, 2 * cap), 1024);
		T*           q  = nullptr;
		bool         pq = hipHostMalloc ((void**)&q, nc * sizeof (T), 0) == hipSuccess;
		if (!pq)
			q = (T*)malloc (nc * sizeof (T));
		if (n)
			memcpy ((void*)q, (const void*)p, n * sizeof (T));
		const size_t keep = n;
		release ();
		p      = q;
		n      = keep;
		cap    = nc;
		pinned = pq;
	}
	void   push_back (const T& v)
	{
		if (n == cap)
			reserve (n + 1);
		p[n++] = v;
	}
	void   resize (size_t m)
	{
		reserve (m);
		n = m;
	}
	void   clear () { n = 0; }
	size_t size () const { return n; }
	bool   empty () const { return n == 0; }
	T*     data () { return p; }
	T*     begin () { return p; }
	T*     end () { return p + n; }
	T&     operator[] (size_t i) { return p[i]; }
	void   swap (PinnedVec& o)
	{
		std::swap (p, o.p);
		std::swap (n, o.n);
		std::swap (cap, o.cap);
		std::swap (pinned, o.pinned);
	}
};

/* a chunk's event scan (scanChunk, csrc/tbf_engine.cpp): instance ranges and event
 * segments of the device front end's partition, with the per-segment counts */
struct ChunkScan {
	unsigned              T = 1, Te = 1; /* instance ranges, event segments */
	uint32_t              per = 1, seg = 0;
	/* the events of segment s for instance range t, in order, as compact records (written by
	 * the scan itself, so the front end never reads the 24-B events again): rec[boff[s (T +
	 * 1) + t] .. boff[s (T + 1) + t + 1]), inside segment s's own part of rec */
	struct Rec {
		uint32_t inst;
		uint32_t bf; /* block in the chunk << 2 | 1: parameter event | 2: value != 0 */
		int32_t  id;
		float    v;
	};
	std::vector<Rec>      rec;
	std::vector<uint32_t> boff;
};

template <typename T>
struct DevBuf {
	T*     p   = nullptr;
	size_t cap = 0;
	DevBuf ()                         = default;
	DevBuf (const DevBuf&)            = delete; /* one owner: the destructor frees */
	DevBuf& operator= (const DevBuf&) = delete;
	DevBuf& operator= (DevBuf&& o) noexcept /* takes o's buffer (frees its own) */
	{
		if (this != &o) {
			release ();
			p     = o.p;
			cap   = o.cap;
			o.p   = nullptr;
			o.cap = 0;
		}
		return *this;
	}
	~DevBuf () { release (); }
	int    ensure (size_t n)
	{
		if (n <= cap)
			return 0;
		if (p)
			(void)hipFree (p);
		p   = nullptr;
		cap = 0;
		if (hipMalloc ((void**)&p, std::max<size_t> (n, 1) * sizeof (T)) != hipSuccess)
			return -12;
		cap = n;
		return 0;
	}
	void release ()
	{
		if (p)
			(void)hipFree (p);
		p   = nullptr;
		cap = 0;
	}
};

} // namespace tbf

using namespace tbf; /* private header: the engine's own translation units only */

#define TBF_NSTAGES 6 /* k_tonegen, k_mixpre, k_rv_pre, k_rv_core, k_rv_post, k_whirl */

struct tbf_engine {
	tbf_engine_config                       cfg;
	Config                                  conf; /* cfg keys (tbf_config_set) for tables built from now on */
	hipStream_t                             stream = nullptr;
	WhirlTables                             wt;
	std::vector<uint32_t>                   vibTab;
	uint32_t                                statorInc = 0;
	uint32_t                                wringLen  = 512;
	std::vector<std::unique_ptr<TgTemplate>> tpls;
	std::vector<Instance>                   inst;
	std::vector<uint32_t>                   retuned; /* tbf_instance_retune: device state to reset */
	uint64_t                                hostCtlNs = 0, hostCtlBlocks = 0; /* tbf_debug_host_time */
	/* reverb ring layout (identical for all instances: A..F are fixed) */
	uint32_t                                slabLen = 0;
	/* device side */
	bool                                    deviceReady = false;
	uint32_t                                devInst     = 0;
	DevBuf<float>                           bank;
	DevBuf<tbf_tpl_desc>                    tplDesc;
	DevBuf<tbf_inst_const>                  cst;
	DevBuf<tbf_inst_state>                  st;
	DevBuf<float>                           wring;
	DevBuf<double>                          rslab;
	DevBuf<tbf_seg_ctl>                     ctl;
	DevBuf<tbf_prog_entry>                  prog;
	/* device-side tone-generator control (k_tgctl, tbf_ctl.hip) */
	bool                                    devCtl = false;
	DevBuf<tbf_tgc_state>                   tgc;
	DevBuf<tbf_tgc_rec>                     drec;
	DevBuf<uint16_t>                        dmsg;
	DevBuf<uint32_t>                        dctlInst;
	DevBuf<uint32_t>                        coff;
	uint32_t                                ctlNw = 1; /* k_tgctl's staged wheels (largest wheel in coff/contrib + 1) */
	DevBuf<tbf_contrib>                     contrib;
	PinnedVec<tbf_tgc_rec>                  hRec;     /* per delta of the chunk */
	PinnedVec<uint16_t>                     hMsg;     /* the chunk's key messages */
	PinnedVec<float>                        hGain;    /* the chunk's changed drawbar gains: (bus, gain) pairs */
	PinnedVec<float>                        hGainB;
	DevBuf<float>                           dgain, dgainB;
	PinnedVec<tbf_wh_params>                hWh, hWhB; /* the chunk's whirl parameter sets (tbf_seg_ctl.whSet) */
	DevBuf<tbf_wh_params>                   dwh, dwhB;
	PinnedVec<uint32_t>                     hCtlInst; /* instances with a stepped delta */
	PinnedVec<uint32_t>                     hDInst, hDInstB; /* instances with any delta: k_tgctl's grid */
	PinnedVec<tbf_seg_ctl>                  hFull, hFullB;   /* the chunk's full control entries (tbf_tgc_rec.full) */
	DevBuf<tbf_seg_ctl>                     dfull, dfullB;
	std::vector<tbf_seg_ctl>                lastEmit; /* per instance: the last full entry the device holds (parallel front end) */
	std::vector<uint8_t>                    dseen, dhas; /* per chunk: lastEmit taken / in hDInst */
	std::vector<uint32_t>                   lastProg;    /* per instance: the last delta's prog_off */
	/* device front end (k_front) for note-only chunks: per instance key state at the chunk
	 * start, the instances' note events by instance, their offsets; by chunk parity */
	bool                                    frontOn = true; /* TBF_DEVICE_FRONT=0 disables */
	uint32_t                                frontGain = 0;  /* device front end: the chunk's gain-pair floats */
	PinnedVec<tbf_front_state>              hFront, hFrontB;
	PinnedVec<uint32_t>                     hFev, hFevB, hFevOff, hFevOffB;
	PinnedVec<float>                        hFevVal, hFevValB; /* TBF_FEV_EFFECT events' values */
	DevBuf<tbf_front_state>                 dfront, dfrontB;
	DevBuf<uint32_t>                        dfev, dfevB, dfoff, dfoffB;
	DevBuf<float>                           dfval, dfvalB;
	DevBuf<float>                           dkeyComp;   /* [tpl][128] keyCompTable */
	DevBuf<uint32_t>                        dident;     /* 0 .. n-1: k_tgctl's grid over every instance */
	std::vector<uint32_t>                   hIdent;
	std::vector<uint8_t>                    fclean; /* per instance: no control change pending but notes */
	ChunkScan                               scan;   /* the chunk's event scan (scanChunk) */
	/* the other parity of the chunk staging (the previous chunk's, in flight), and the
	 * events after each parity's uploads */
	PinnedVec<tbf_seg_ctl>                  dCtlB, hCtlPin, hCtlPinB;
	PinnedVec<tbf_tgc_rec>                  hRecB;
	PinnedVec<uint16_t>                     hMsgB;
	PinnedVec<uint32_t>                     hCtlInstB, hIdxB;
	hipEvent_t                              upEv = nullptr, upEvB = nullptr;
	std::vector<uint8_t>                    stepped;  /* membership of hCtlInst */
	std::vector<uint8_t>                    pslot;    /* persistent program slot (0..TBF_PROG_PSLOTS-1) per instance */
	/* device control, pipelined delta chunks: the control pool (persistent entries +
	 * deltas), the index table and the control records come in two regions by chunk
	 * parity; region p's persistent entries are refreshed from hCtl when they are older
	 * than its version (ctlVer counts the changes of hCtl) */
	uint64_t                                ctlVer = 1, regionVer[2] = {0, 0};
	int                                     whSplit = -1; /* k_whirl_split: -1 at rings > 512 or <= 1 instance per CU, 0 / 1 (TBF_WHIRL_SPLIT) */
	uint32_t                                nCU     = 256; /* the device's CUs */
	uint32_t                                frontMin = 64; /* events a chunk needs for the device front end (TBF_FRONT_MIN; 64: profiles/r05/s23) */
	bool                                    parCtl = true; /* TBF_HOST_SERIAL=1 steps serially */
	/* threaded host control (stepChunkParallel): per worker, kept between chunks so the
	 * buffers stay allocated; worker t writes its deltas straight into the staging at pool
	 * position base_t = (first instance of its range) * blocks, and dSeg lists the filled
	 * segments {base_t, count_t} that are uploaded (empty: the pool is [0, dCtl.size ())) */
	struct alignas (128) ParStep { /* own cache lines: workers bump these per delta */
		std::vector<uint16_t> msgs;
		std::vector<float>    gains;
		std::vector<tbf_wh_params> whs;
		std::vector<uint32_t> act, ctlInst, evs, dInst, eoff, esort, efill;
		/* a front-end chunk's events of the range, by instance: what the mirror pass reads */
		struct FrontRec {
			uint32_t blk;  /* block in the chunk */
			int32_t  id;   /* key / parameter index */
			float    v;    /* (float) value */
			uint32_t flag; /* 1: parameter event, 2: value != 0 */
		};
		std::vector<FrontRec> erec;
		std::vector<tbf_seg_ctl> fulls;
		uint32_t              nd = 0;
		uint32_t              gainLocal = 0; /* device front end: the range's gain-pair floats */
		bool                  fx = false;    /* ... and whether an effect setter stepped an entry */
		int                   rc = 0;
		std::string           err; /* the worker's tbf_last_error text (it is thread-local) */
	};
	std::vector<ParStep>                    parStep;
	std::vector<std::pair<uint32_t, uint32_t>> dSeg;
	DevBuf<tbf_tgc_rec>                     drecB;
	DevBuf<uint16_t>                        dmsgB;
	DevBuf<uint32_t>                        dctlInstB;
	DevBuf<uint32_t>                        vib;
	DevBuf<uint32_t>                        xsj; /* xorshift32 jump table */
	DevBuf<float>                           whTab, whBw;
	DevBuf<uint32_t>                        err;
	/* tbf_debug_kernel_times: HIP events around every stage launch */
	bool                                    timeOn = false;
	bool                                    timeSerial = false; /* time with pipelining off */
	std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> tev;
	DevBuf<float>                           outL, outR;
	DevBuf<float>                           mid0, mid1, mid2; /* inter-stage blocks of one launch chunk */
	DevBuf<double>                          rvA, rvB;   /* reverb inter-kernel streams (FP64) */
	std::vector<tbf_seg_ctl>                hCtl;  /* current control per instance (pool entries 0..n-1) */
	std::vector<tbf_prog_entry>             hProg; /* current program per instance (slots i * PROG_CAP) */
	/* per-chunk control deltas (tbf_render_events / renderImpl) */
	PinnedVec<tbf_seg_ctl>                  dCtl;
	std::vector<tbf_prog_entry>             dProg;
	PinnedVec<uint32_t>                     hIdx;
	std::vector<uint8_t>                    chg;
	/* instances whose control may change at the next block (renderImpl steps only
	 * these): every entry point that changes an instance marks it (markActive) */
	std::vector<uint32_t>                   actList;
	std::vector<uint8_t>                    inAct;   /* membership of actList */
	bool                                    actAll = true; /* instances added: step all */
	std::vector<uint32_t>                   curIdx;  /* pool entry per instance, current block */
	DevBuf<uint32_t>                        ctlIdx;
	bool                                    persistStale = true; /* device pool entries 0..n-1 need upload */
	/* cross-chunk pipelining (renderImpl): stage k of every chunk runs on the stream of its
	 * stage group grp[k] (so the stage's own state is ordered by its stream), the stages of
	 * one chunk are chained by events, and a stage that overwrites a stage buffer of parity
	 * c % 2 waits for chunk c - 2's readers of it on other streams.  A stage therefore starts
	 * as soon as its inputs are ready, whatever the later stages of earlier chunks do.
	 * Three groups: the device exposes few hardware queues per process (GPU_MAX_HW_QUEUES 4)
	 * and streams sharing one serialize. */
	hipStream_t                             gs[TBF_NSTAGES] = {};     /* groups 0 .. grp[TBF_NSTAGES - 1] */
	hipEvent_t                              sdone[TBF_NSTAGES] = {};  /* the last launched chunk's stage k */
	hipEvent_t                              pev[4][TBF_NSTAGES] = {}; /* chunk c's stage k, ring by c mod 4 */
	hipEvent_t                              sjoin = nullptr;
	uint64_t                                chunkSeq = 0;
	bool                                    stagesBusy = false; /* pipelined work may be outstanding */
	bool                                    pipeline = true;    /* TBF_PIPELINE=0 disables */
	/* stage k's stream (TBF_PIPE_GROUPS): k_tonegen + k_mixpre | k_rv_pre + k_rv_core + k_rv_post |
	 * k_whirl.  Against {0,0,1,1,2,2}: rvB single (its producer and reader share a stream),
	 * mid2 by parity, 56 instead of 68 B per stereo sample, and the step 131.7 -> 128.3 ms
	 * (profiles/r05/s20_groups) */
	int                                     grp[TBF_NSTAGES] = {0, 0, 1, 1, 1, 2};
	bool                                    rvLdsOn  = true;  /* k_rv_core_lds when the rings fit (TBF_RV_LDS=0: k_rv_core) */
	bool                                    rvLdsFit = false; /* the instances' rings fit k_rv_core_lds */
	uint32_t                                rvGrid   = 0;     /* k_rv_core_lds persistent workgroups (TBF_RV_PERSIST=0: one per pair) */
	DevBuf<uint32_t>                        rvWork;           /* its work counter */
	DevBuf<uint8_t>                         mixFixed;         /* tonegen only: k_tonegen wrote the output (tbf_launch.mixFixed) */
	int                                     tgSplit  = -1;    /* k_tonegen block ranges (TBF_TG_SPLIT; -1: by batch size) */
	uint32_t                                steadyChunk = TBF_STEADY_DEFAULT; /* blocks per chunk without control deltas (TBF_STEADY_CHUNK,
	                                                                           * tbf_set_steady_chunk) */
	/* the stage buffers as allocated (stageBuffers): blocks per chunk they hold (a power of two
	 * from TBF_CHUNK up to steadyChunk, grown to the longest chunk a call can make, never past
	 * what the device could allocate), for stageN instances; a buffer whose producer and
	 * readers share a stage-group stream is single (dbl[] false), the others alternate by
	 * chunk parity */
	uint32_t                                stageBlocks = 0, stageN = 0;
	uint64_t                                frontChunks[2] = {0, 0}; /* chunks with events: device, host front end */
	bool                                    stageDbl[5] = {true, true, true, true, true}; /* mid0 mid1 rvA rvB mid2 */
	/* programme table (.pgm), src/program.h:26 MAXPROGS; pgm.controller.offset */
	std::vector<Programme>                  progs = std::vector<Programme> (129);
	int                                     pgmOffset = 1;
	/* synth_sound FIFO */
	std::vector<float>                      fifoL, fifoR;
	uint32_t                                boffset = TBF_BLK; /* read position in the FIFO ... */
	uint32_t                                fifoLen = TBF_BLK; /* ... of fifoLen samples per instance ... */
	uint32_t                                fifoN   = 0;       /* ... for fifoN instances */
};

namespace tbf {
/* the calling thread's active list while renderImpl steps an instance range on a host
 * worker thread (nullptr: the engine's own list) */
extern thread_local std::vector<uint32_t>* tlAct;
inline void markActive (tbf_engine* e, uint32_t i)
{
	if (i < e->inAct.size () && !e->inAct[i]) {
		e->inAct[i] = 1;
		(tlAct ? *tlAct : e->actList).push_back (i);
	}
}
} // namespace tbf

#endif
