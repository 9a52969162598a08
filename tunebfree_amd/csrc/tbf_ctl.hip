/*
 * tbf_ctl.hip -- k_tgctl: the tone generator's per-wheel control on the device
 * (SURVEY.md §8(f) row 1).
 *
 * oscGenerateFragment (src/tonegen.cpp:3218-3594) starts each block with control work:
 * the message queue's key events update the activated-oscillator table (per wheel: a
 * level per bus, a reference count) and the active list (3257-3327); the active-list
 * loop recomputes the routed sums of the wheels a key or drawbar touched and emits one
 * core-program instruction per active wheel (3333-3566); released wheels leave the list
 * (3576-3594).  With dense events that work, done on the host for thousands of
 * instances, outweighs the render by two orders of magnitude (profiles/r02/
 * dense_events_*.json), so it runs here: the host keeps the front end (which keys are
 * down, drawbar gains, the routing word: tbf_init.cpp TgControl::stepFront) and hands
 * each stepped block a tbf_tgc_rec; this kernel owns the per-wheel state
 * (tbf_tgc_state, HBM) and writes the block's program where k_tonegen reads it.
 *
 * One wave per instance with stepped blocks in the chunk, blocks in order; the instance's
 * routed sums, reference counts, list and flags staged in LDS for the launch, its bus
 * levels read and written in place in HBM (at 184 wheels they would take 20 KB of LDS a
 * workgroup: four rounds of workgroups at 4096 instances instead of one):
 *   messages   in queue order; the key's keyContrib list (sorted by wheel, then bus) is
 *              spread over the lanes, four passes of 64 entries loaded together a message
 *              ahead.  Each (wheel, bus) appears once per key, so the bus-level adds are
 *              lane-parallel (one read batch per group) and keep the reference's
 *              per-(wheel, bus) order; a wheel's reference-count / flag update is made once per wheel group
 *              by its first lane, which gives what the reference's per-element sequence
 *              gives (first element sees the old count, the rest see it > 0); newly
 *              activated wheels join the list in element order (ballot ranks).
 *   active loop lane = list position: the routed sums (the reference's 9-term sums in
 *              order), the instruction, the flags cleared; removals are applied after,
 *              serially, in list order (swap-with-last, as the reference).
 * Strict float: -ffp-contract=off (Makefile), every sum in the reference's order.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tbf.h"
#include "tbf_types.h"

#define NL 64
#define NW TBF_NW

/* the per-wheel arrays, staged in dynamic LDS for the launch's wheel count P.ctlNw (the
 * largest wheel any play matrix names, + 1: 184 for the tonewheel organ with its
 * crosstalk wheels, 35 B a wheel, so ~6.4 KB + CtlLds: 16 workgroups per CU, and the
 * bench's 4096 instances in one round).  The bus levels ([nw][27] floats, 20 KB at 184
 * wheels: 5 workgroups per CU, four rounds, when they were staged here too) stay in the
 * instance's tbf_tgc_state in HBM, read and written in place (ctl_bl_load). */
struct CtlW {
	float*    sums;    /* [nw][6]  routed sums */
	int32_t*  ref;     /* [nw] */
	uint16_t* list;    /* [nw] activeOscList */
	int16_t*  acl1;    /* [nw] */
	uint16_t* removed; /* [nw] */
	uint8_t*  rf;      /* [nw] */
};
#define CTL_MSGCAP 256 /* a launch's messages prefetched into LDS (more: read per block) */
#ifndef CTL_ABL
#define CTL_ABL 0 /* timing experiments (wrong output): 1 no bus-level loads or stores in the messages, 2 none in ctl_block */
#endif
#define FR_CAP 8192    /* k_front: a wave's (64 instances') events staged in LDS (more: read from HBM) */

struct CtlLds {
	float    dbg[27];
	uint32_t mc0[CTL_MSGCAP], mc1[CTL_MSGCAP]; /* each message's keyContrib range */
	uint16_t msg[CTL_MSGCAP];
};

__host__ __device__ constexpr size_t ctl_wbytes (uint32_t nw)
{
	return (size_t)nw * (6 * 4 + 4 + 2 + 2 + 2 + 1);
}

__device__ __forceinline__ CtlW ctl_carve (uint8_t* p, uint32_t nw)
{
	CtlW w;
	w.sums    = (float*)p;
	w.ref     = (int32_t*)(w.sums + (size_t)nw * 6);
	w.list    = (uint16_t*)(w.ref + nw);
	w.acl1    = (int16_t*)(w.list + nw);
	w.removed = (uint16_t*)(w.acl1 + nw);
	w.rf      = (uint8_t*)(w.removed + nw);
	return w;
}

__device__ __forceinline__ uint64_t lanemask_lt () { return (1ull << threadIdx.x) - 1ull; }

/* TBF_CTL_PROF (A/B builds only): shader-clock cycles per k_tgctl phase, printed by a few
 * workgroups */
#ifdef TBF_CTL_PROF
#define CTL_T(v) const uint64_t v = __builtin_amdgcn_s_memtime ()
#define CTL_ACC(acc, t0) acc += __builtin_amdgcn_s_memtime () - (t0)
#define CTL_PARAM , uint64_t (&pt)[4]
#define CTL_ARG , pt
#else
#define CTL_T(v)
#define CTL_ACC(acc, t0)
#define CTL_PARAM
#define CTL_ARG
#endif

/* the workgroup is one wave: LDS accesses of a wave execute in issue order, so a read
 * after a write sees it; only the compiler must not move LDS accesses across this point
 * (a __syncthreads also waited for every outstanding global store: the program stores) */
__device__ __forceinline__ void wave_sync ()
{
	__builtin_amdgcn_fence (__ATOMIC_ACQ_REL, "wavefront");
	__builtin_amdgcn_wave_barrier ();
}

/* the same for LDS accesses whose data flow stays within a lane or goes through wave-uniform
 * registers: only the compiler's order matters */
__device__ __forceinline__ void lds_order () { __asm__ __volatile__ ("" ::: "memory"); }

/* A bus level, read at the device's coherence point (L2, not the CU's L1), since another
 * lane of the wave may have written it in an earlier message.
 * HARDWARE ASSUMPTION (not a promise of the AMDGPU memory model, which treats the lanes as
 * separate threads): a wave's vector memory instructions leave the CU in issue order, and
 * requests to one address go to one L2 channel, which serves them in arrival order; so a
 * load issued after a store to the same address (any lane) reads the stored value.  Between
 * the messages of a block nothing else orders them (a vmcnt(0) wait per message would also
 * wait out the next message's contribution loads, issued a message ahead); ctl_block, once
 * per block, waits for the block's stores first (ctl_store_fence).  Pinned by
 * test_gpu_device_control_large_clusters (~1500 messages a launch, every bus level read back
 * after another lane's store) and the dense device-front-end tests, bit for bit. */
__device__ __forceinline__ float ctl_bl_load (const float* p)
{
	return __hip_atomic_load (p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

/* every vector memory operation of the wave so far complete (s_waitcnt vmcnt(0): on gfx9
 * it counts stores too, so the bus levels the messages stored have reached L2) */
__device__ __forceinline__ void ctl_store_fence () { __builtin_amdgcn_s_waitcnt (0x0F70); }

/* 16 B of a wheel's bus-level row the same way: a buffer load with the sc1 policy (bit 4 of
 * the cache-policy operand on gfx950), through the instance's rows as a buffer resource */
typedef unsigned int v4u __attribute__ ((ext_vector_type (4)));
__device__ __forceinline__ v4u ctl_row_load (__amdgpu_buffer_rsrc_t r, uint32_t w, int q)
{
	return __builtin_amdgcn_raw_buffer_load_b128 (r, (int)(w * TBF_BL_ROW * 4u + 16u * (uint32_t)q), 0, 16);
}

/* One pass of a key message (src/tonegen.cpp:3270-3322): the entries base + lane of the
 * key's keyContrib range [c0, c1), packed as wheel | bus << 16 | lead << 24 with the level;
 * a message's first CTL_PG passes are loaded together, a message ahead of their use, so
 * the contribution table's load latency hides behind the message before. */
#define CTL_PG 4 /* passes per load group: keyContrib lists of up to 256 entries in one */

struct CtlGroup {
	uint32_t wb[CTL_PG]; /* the entry's wheel | bus << 16 (lanes past the range: entry 0's or the last's) */
	uint32_t pw[CTL_PG]; /* the wheel of the entry before it */
	float    lev[CTL_PG];
};

__device__ __forceinline__ CtlGroup ctl_group_load (const tbf_contrib* __restrict__ kc, uint32_t c0, uint32_t c1,
                                                    uint32_t g0)
{
	/* every lane loads (an index clamped into the range, or entry 0), so the group's loads
	 * issue back to back without exec-mask branches */
	/* nothing here consumes the loaded data: the loads stay in flight until the group is
	 * applied, after the wait for the bus levels of the message before */
	CtlGroup g;
#pragma unroll
	for (int q = 0; q < CTL_PG; q++) {
		const uint32_t    e  = g0 + (uint32_t)(q * NL) + threadIdx.x;
		const uint32_t    ec = e < c1 ? e : (c1 > c0 ? c1 - 1 : 0u); /* contrib holds >= 1 entry */
		const tbf_contrib c  = kc[ec];
		g.wb[q]              = (uint32_t)c.wheel | ((uint32_t)c.bus << 16);
		g.lev[q]             = c.level;
		g.pw[q]              = kc[ec > c0 ? ec - 1 : ec].wheel;
	}
	return g;
}

/* A wheel group's part in a pass runs from its first lane to the next group's first lane
 * (or the pass end); lane 0 continues a group begun in the previous pass.  The owner's
 * reference count, flags and list position are read in one batch, then written; L (the
 * list end) is wave-uniform in a scalar register.  b: the entry's bus level as loaded. */
__device__ __forceinline__ void ctl_pass_apply (const CtlW& W, float* __restrict__ gbl, uint32_t wb, uint32_t pw, float lev,
                                                float b, uint32_t e, uint32_t c0, uint32_t nval, bool on, uint32_t& L)
{
	const int      lane  = threadIdx.x;
	const uint32_t w     = wb & 0xFFFFu, bus = wb >> 16;
	const bool     valid = (uint32_t)lane < nval;
	const bool     lead  = valid && (e == c0 || pw != w);
	const uint64_t ld    = __ballot (lead);
	const uint64_t after = (lane + 1 < NL) ? (ld >> (lane + 1)) : 0ull;
	const uint32_t next  = after ? (uint32_t)(lane + 1 + __builtin_ctzll (after)) : nval;
	const bool     owner = valid && (lead || lane == 0);
	const int      part  = (int)(next - (uint32_t)lane);
	const uint32_t wr    = valid ? w : 0u; /* the reads unconditional, from a valid index */
	const int      r0    = W.ref[wr];
	const uint32_t f0    = W.rf[wr];
	const int      a0    = W.acl1[wr];
#if CTL_ABL != 1
	if (valid)
		gbl[w * TBF_BL_ROW + bus] = on ? b + lev : b - lev;
#endif
	bool join = false;
	if (owner) {
		int      r1;
		uint32_t f1;
		if (on) {
			r1 = r0 + part;
			if (lead && r0 == 0) {
				f1   = 0x0006;
				join = a0 == 0;
			} else
				f1 = f0 | 0x0004;
		} else {
			r1 = r0 - part;
			f1 = r1 == 0 ? 0x0005 : (f0 | 0x0004);
		}
		W.ref[w] = r1;
		W.rf[w]  = (uint8_t)f1;
	}
	const uint64_t jb = __ballot (join);
	if (join) {
		const uint32_t pos = L + (uint32_t)__builtin_popcountll (jb & lanemask_lt ());
		W.list[pos]        = (uint16_t)w;
		W.acl1[w]          = (int16_t)(pos + 1);
	}
	L += (uint32_t)__builtin_popcountll (jb);
	lds_order ();
}

/* one key message whose first load group g is loaded: per group, the bus levels of all its
 * entries are read together (each (wheel, bus) appears once in a key's list), then the
 * passes applied in order */
__device__ __forceinline__ void ctl_message (const CtlW& W, float* __restrict__ gbl, const tbf_contrib* __restrict__ kc,
                                             uint32_t c0, uint32_t c1, bool on, CtlGroup g, uint32_t& L)
{
	for (uint32_t g0 = c0; g0 < c1; g0 += CTL_PG * NL) {
		if (g0 != c0)
			g = ctl_group_load (kc, c0, c1, g0);
		float b[CTL_PG];
#pragma unroll
		for (int q = 0; q < CTL_PG; q++) /* every lane: lanes past the range read a valid entry's level */
#if CTL_ABL == 1
			b[q] = 0.f;
#else
			b[q] = ctl_bl_load (gbl + (g.wb[q] & 0xFFFFu) * TBF_BL_ROW + (g.wb[q] >> 16));
#endif
#pragma unroll
		for (int q = 0; q < CTL_PG; q++) {
			const uint32_t base = g0 + (uint32_t)(q * NL);
			if (base < c1)
				ctl_pass_apply (W, gbl, g.wb[q], g.pw[q], g.lev[q], b[q], base + threadIdx.x, c0,
				                c1 - base < (uint32_t)NL ? c1 - base : (uint32_t)NL, on, L);
		}
	}
}

/* the active-list loop and the removals of one block (src/tonegen.cpp:3333-3594); writes
 * the program (header + one entry per active wheel) at out */
__device__ void ctl_block (CtlLds& sm, const CtlW& W, const float* __restrict__ gbl, uint32_t flags, uint32_t routing,
                           uint32_t percSendBus, tbf_prog_entry* __restrict__ out, uint32_t& L CTL_PARAM)
{
	CTL_T (q0);
	const int      lane      = threadIdx.x;
	const uint32_t L0        = L;
	/* the instance's bus-level rows as a buffer resource (dword 3: gfx950's raw 32-bit format) */
	const __amdgpu_buffer_rsrc_t blr =
		__builtin_amdgcn_make_buffer_rsrc ((void*)gbl, (short)0, (int)((TBF_NW + 1) * TBF_BL_ROW * 4), 0x00020000);
	const bool     dbChange  = (flags & 1) != 0;
	const bool     recompute = (flags & 2) != 0;
	ctl_store_fence (); /* the messages' bus-level stores before the row loads below */
	uint32_t       nrem      = 0;
	uint64_t       rb0       = 0; /* the first pass's removals */
	uint32_t       on0       = 0; /* and its lanes' wheels */
	for (uint32_t base = 0; base < L0; base += NL) {
		const uint32_t i     = base + lane;
		const bool     valid = i < L0;
		bool           rem   = false;
		uint32_t       on    = 0;
		if (valid) {
			on                = W.list[i];
			const uint32_t rf = W.rf[on];
			float*         S  = W.sums + on * 6;
			tbf_prog_entry E;
			E.wheel = (uint16_t)on;
			E.env = 0;
			E.row = 0;
			E.nsg = E.npg = E.nvg = 0.0f;
			E.pad = 0;
			if (rf & 0x0001) {
				rem   = true;
				E.env = 2;
				E.row = (uint8_t)(i & 7);
				E.sg  = S[4];
				E.pg  = S[3];
				E.vg  = S[5];
			} else {
				float sumUpper = S[0], sumLower = S[1], sumPedal = S[2];
				float sumPercn = S[3], sumSwell = S[4], sumScanr = S[5];
				if (rf & 0x0002) {
					E.sg = E.pg = E.vg = 0.0f;
				} else {
					E.sg = sumSwell;
					E.pg = sumPercn;
					E.vg = sumScanr;
				}
				bool reroute = false;
				if ((rf & 0x0004) || dbChange) {
					float bl[TBF_BL_ROW];
#pragma unroll
					for (int q = 0; q < TBF_BL_ROW / 4; q++) {
#if CTL_ABL == 2
						const v4u v = {(unsigned)q, (unsigned)q, (unsigned)q, (unsigned)q};
#else
						const v4u v = ctl_row_load (blr, on, q);
#endif
						bl[4 * q]     = __uint_as_float (v.x);
						bl[4 * q + 1] = __uint_as_float (v.y);
						bl[4 * q + 2] = __uint_as_float (v.z);
						bl[4 * q + 3] = __uint_as_float (v.w);
					}
					float sum = 0.0f;
					for (int d = 0; d < 9; d++)
						sum += bl[d] * sm.dbg[d];
					sumUpper = sum;
					sum      = 0.0f;
					for (int d = 9; d < 18; d++)
						sum += bl[d] * sm.dbg[d];
					sumLower = sum;
					sum      = 0.0f;
					for (int d = 18; d < 27; d++)
						sum += bl[d] * sm.dbg[d];
					sumPedal = sum;
					reroute  = true;
				}
				if (reroute || recompute) {
					sumPercn = (routing & 0x0C) ? ctl_bl_load (gbl + on * TBF_BL_ROW + percSendBus) : 0.0f;
					sumScanr = 0.0f;
					sumSwell = sumPedal;
					if (routing & 0x02)
						sumScanr += sumUpper;
					else
						sumSwell += sumUpper;
					if (routing & 0x01)
						sumScanr += sumLower;
					else
						sumSwell += sumLower;
					S[0] = sumUpper;
					S[1] = sumLower;
					S[2] = sumPedal;
					S[3] = sumPercn;
					S[4] = sumSwell;
					S[5] = sumScanr;
				}
				if (rf & 0x0006) {
					E.env = 1;
					E.row = (uint8_t)(i & 7);
					E.nsg = sumSwell;
					E.npg = sumPercn;
					E.nvg = sumScanr;
				}
			}
			W.rf[on]   = 0;
			out[1 + i] = E;
		}
		const uint64_t rb = __ballot (rem);
		if (base == 0) {
			rb0 = rb;
			on0 = on;
		} else if (rem)
			W.removed[nrem - (uint32_t)__builtin_popcountll (rb0) + (uint32_t)__builtin_popcountll (rb & lanemask_lt ())] =
				(uint16_t)on;
		nrem += (uint32_t)__builtin_popcountll (rb);
	}
	CTL_ACC (pt[0], q0);
	CTL_T (q1);
	if (lane == 0) {
		tbf_prog_entry H = {};
		H.wheel          = 0xFFFF;
		H.pad            = L0;
		out[0]           = H;
	}
	/* the removals (3576-3594): in order, each swapped with the list's last entry, by lane 0
	 * (a register-held list with readlane / lane-select swaps measured slower, 500 k against
	 * 330 k cycles a wave under dense events); the first pass's victims come from their
	 * lanes' registers, later passes' (lists over 64 wheels) through LDS.  The list and
	 * positions go through LDS in issue order: one read batch per removal. */
	lds_order ();
	const uint32_t n0 = (uint32_t)__builtin_popcountll (rb0);
	uint32_t       Lr = L0;
	for (uint64_t m = rb0; m; m &= m - 1) {
		const uint32_t vic = (uint32_t)__builtin_amdgcn_readlane ((int)on0, __builtin_ctzll (m));
		Lr--;
		if (lane == 0) {
			const int      act = W.acl1[vic] - 1;
			const uint32_t mov = W.list[Lr];
			W.acl1[vic]        = 0;
			if (0 < Lr && mov != vic) {
				W.list[act] = (uint16_t)mov;
				W.acl1[mov] = (int16_t)(act + 1);
			}
		}
		lds_order ();
	}
	if (lane == 0)
		for (uint32_t r = 0; r < nrem - n0; r++) {
			const uint32_t vic = W.removed[r];
			const int      act = W.acl1[vic] - 1;
			W.acl1[vic]        = 0;
			Lr--;
			if (0 < Lr) {
				const uint32_t mov = W.list[Lr];
				if (mov != vic) {
					W.list[act] = (uint16_t)mov;
					W.acl1[mov] = (int16_t)(act + 1);
				}
			}
		}
	L = L0 - nrem;
	lds_order ();
	CTL_ACC (pt[1], q1);
}

/* One wave per instance with control deltas in the chunk.  The chunk's per-block inputs
 * are read lane-parallel up front (lane b = block b: its pool index and record), and the
 * messages of the launch with their keyContrib ranges into LDS, so a block's work waits on
 * no chain of dependent global loads (index -> record -> message -> range, one after the
 * other per block before).
 * First every delta's control entry is written to the pool: a full entry as the host sent
 * it (fulls), a patched one from the instance's entry before it -- the last full delta
 * before it, else the persistent entry -- with the record's key-compression target,
 * percussion reset and routing, and the program of the last stepped delta at or before it
 * (else the persistent program).  Then the stepped blocks' per-wheel control in order. */
__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL))) k_tgctl (const tbf_launch P)
{
	__shared__ CtlLds         sm;
	extern __shared__ uint8_t wdyn[];
	const int                 lane = threadIdx.x;
#ifdef TBF_CTL_PROF
	const uint64_t pr_rt0 = __builtin_amdgcn_s_memrealtime ();
	CTL_T (pr_c0);
#endif
	const uint32_t            nw   = P.ctlNw;
	const CtlW                W    = ctl_carve (wdyn, nw);
	const uint32_t            inst = P.ctlInst[blockIdx.x];
	tbf_tgc_state*            G    = P.tgc + inst;
	const uint32_t            tpl  = P.cst[inst].tpl;
	const uint32_t*           coff = P.coff + (size_t)tpl * 385;
	const uint32_t            n    = P.nInst;
	/* lane b: block b's pool index; a block starts a delta when its index differs from the
	 * block before's (block 0: from the instance's persistent entry) */
	const uint32_t nb    = P.nBlocks;
	const uint32_t idx   = (uint32_t)lane < nb ? P.ctlIdx[(size_t)lane * n + inst] : inst;
	const uint32_t pidx  = lane == 0 ? inst : (uint32_t)__shfl_up ((int)idx, 1);
	const bool     isNew = (uint32_t)lane < nb && idx >= n && idx != pidx;
	tbf_tgc_rec    R     = {};
	if (isNew)
		R = P.rec[idx - n];
	{
		const uint64_t le = lane == NL - 1 ? ~0ull : ((2ull << lane) - 1ull); /* lanes <= this one */
		const uint64_t fm = __ballot (isNew && R.full != 0) & le, km = __ballot (isNew && (R.flags & 0x80)) & le;
		const int      lf = fm ? 63 - __builtin_clzll (fm) : 0, ls = km ? 63 - __builtin_clzll (km) : 0;
		const uint32_t ff = (uint32_t)__shfl ((int)R.full, lf), ki = (uint32_t)__shfl ((int)idx, ls);
		if (isNew) {
			/* word by word (a struct copy with patched fields went through scratch) */
			const uint32_t* src = (const uint32_t*)(fm ? P.fulls + (ff - 1) : P.ctl + inst);
			uint32_t*       dst = (uint32_t*)((tbf_seg_ctl*)P.ctl + idx);
			const uint32_t  pp  = km ? P.progBase + (ki - n) * (uint32_t)TBF_PROG_SLOT : P.ctl[inst].prog_off;
			const bool      pat = R.full == 0 || (R.flags & 0x10); /* 0x10: k_front's effect entry */
			constexpr int NWD = (int)(sizeof (tbf_seg_ctl) / 4);
			uint32_t      wd[NWD]; /* all loads before the stores (src and dst share the pool) */
#pragma unroll
			for (int k = 0; k < NWD; k++)
				wd[k] = src[k];
#pragma unroll
			for (int k = 0; k < NWD; k++) {
				uint32_t v = wd[k];
				if (pat) {
					if (k == (int)(offsetof (tbf_seg_ctl, prog_off) / 4))
						v = pp;
					else if (k == (int)(offsetof (tbf_seg_ctl, keyCompTarget) / 4))
						v = __float_as_uint (R.keyCompTarget);
					else if (k == (int)(offsetof (tbf_seg_ctl, resetPercAtEnd) / 4))
						v = (R.flags >> 3) & 1u;
					else if (k == (int)(offsetof (tbf_seg_ctl, routing) / 4))
						v = R.oldRouting;
				}
				dst[k] = v;
			}
		}
	}
#ifdef TBF_CTL_PROF
	uint64_t pr_stage = 0, pr_msg = 0, pr_blk = 0, pr_end = 0, pt[4] = {0, 0, 0, 0};
	CTL_T (pr_k0);
#endif
	const uint32_t poff = P.progBase + (idx - n) * (uint32_t)TBF_PROG_SLOT; /* a stepped delta's program */
	const bool     stepped = isNew && (R.flags & 0x80);
	const uint64_t todo0   = __ballot (stepped);
	if (todo0 == 0)
		return; /* control deltas without a tone-generator step */
	/* the messages: lane b's R.nMsg at an exclusive prefix offset */
	uint32_t nm = stepped ? R.nMsg : 0, mpos = nm;
	for (int d = 1; d < NL; d <<= 1) {
		const uint32_t v = (uint32_t)__shfl_up ((int)mpos, d);
		if (lane >= d)
			mpos += v;
	}
	const uint32_t M  = (uint32_t)__shfl ((int)mpos, NL - 1);
	mpos -= nm;
	const bool     pre = M <= CTL_MSGCAP;
	for (size_t i = lane; i < (size_t)nw * 6; i += NL)
		W.sums[i] = (&G->sums[0][0])[i];
	for (uint32_t w = lane; w < nw; w += NL) {
		W.ref[w]  = G->refCount[w];
		W.list[w] = G->list[w];
		W.acl1[w] = G->aclPos1[w];
		W.rf[w]   = G->rflags[w];
	}
	uint32_t L = __builtin_amdgcn_readfirstlane (G->listEnd); /* activeOscLEnd, wave-uniform */
	if (lane < 27)
		sm.dbg[lane] = G->gain[lane];
	if (pre)
		for (uint32_t m = 0; m < nm; m++)
			sm.msg[mpos + m] = P.msgs[R.msgOff + m];
	wave_sync ();
	if (pre) {
		for (uint32_t j = lane; j < M; j += NL) {
			const uint32_t kn = sm.msg[j] & 0x0fffu;
			sm.mc0[j]         = kn < 384 ? coff[kn] : 0u;
			sm.mc1[j]         = kn < 384 ? coff[kn + 1] : 0u;
		}
		wave_sync ();
	}
	/* the first pass of the next message (in launch order: blocks ascending, each block's
	 * messages at its prefix offset), loaded one message ahead */
	float* const gbl = &G->busLevel[0][0];
	CtlGroup     pf  = {};
	if (pre && M > 0)
		pf = ctl_group_load (P.contrib, sm.mc0[0], sm.mc1[0], sm.mc0[0]);
	CTL_ACC (pr_stage, pr_k0);
	int64_t  last = -1; /* prog_off of the last program written */
	uint64_t todo = todo0;
	while (todo) {
		const int b = __builtin_ctzll (todo);
		todo &= todo - 1;
		const uint32_t flags = (uint32_t)__builtin_amdgcn_readlane ((int)R.flags, b);
		if (flags & 4) {
			const uint32_t go = (uint32_t)__builtin_amdgcn_readlane ((int)R.gainOff, b);
			const uint32_t ng = (uint32_t)__builtin_amdgcn_readlane ((int)R.pad, b);
			if ((uint32_t)lane < ng) {
				const uint32_t bus = __float_as_uint (P.gains[go + 2 * lane]);
				sm.dbg[bus < 27 ? bus : 0] = P.gains[go + 2 * lane + 1];
			}
			wave_sync ();
		}
		CTL_T (pr_m0);
		const uint32_t bm = (uint32_t)__builtin_amdgcn_readlane ((int)nm, b);
		const uint32_t bp = (uint32_t)__builtin_amdgcn_readlane ((int)mpos, b);
		const uint32_t bo = (uint32_t)__builtin_amdgcn_readlane ((int)R.msgOff, b);
		for (uint32_t m = 0; m < bm; m++) {
			if (pre) {
				const uint32_t j   = bp + m;
				const uint32_t msg = sm.msg[j], c0 = sm.mc0[j], c1 = sm.mc1[j];
				const CtlGroup cur = pf;
				if (j + 1 < M)
					pf = ctl_group_load (P.contrib, sm.mc0[j + 1], sm.mc1[j + 1], sm.mc0[j + 1]);
				/* keys outside [0, 384) have the empty range */
				ctl_message (W, gbl, P.contrib, c0, c1, (msg & 0xf000u) == 0x1000u, cur, L);
			} else {
				const uint32_t msg = P.msgs[bo + m], kn0 = msg & 0x0fffu;
				if (kn0 >= 384)
					continue;
				const uint32_t c0 = coff[kn0], c1 = coff[kn0 + 1];
				ctl_message (W, gbl, P.contrib, c0, c1, (msg & 0xf000u) == 0x1000u, ctl_group_load (P.contrib, c0, c1, c0),
				             L);
			}
		}
		CTL_ACC (pr_msg, pr_m0);
		CTL_T (pr_b0);
		const uint32_t off = (uint32_t)__builtin_amdgcn_readlane ((int)poff, b);
		ctl_block (sm, W, gbl, flags, (uint32_t)__builtin_amdgcn_readlane ((int)R.oldRouting, b),
		           (uint32_t)__builtin_amdgcn_readlane ((int)R.percSendBus, b), (tbf_prog_entry*)P.prog + off, L CTL_ARG);
		last = off;
		CTL_ACC (pr_blk, pr_b0);
	}
	CTL_T (pr_e0);
	/* the instance's last program becomes its persistent one, in the slot after the current
	 * persistent entry's (mod TBF_PROG_PSLOTS; the host advances its entry the same way
	 * after the chunk) */
	if (last >= 0) {
		const uint32_t cur   = P.ctl[inst].prog_off;
		const uint32_t slot0 = (uint32_t)TBF_PROG_PSLOTS * inst * TBF_PROG_SLOT;
		const uint32_t nxt   = ((cur - slot0) / TBF_PROG_SLOT + 1) % TBF_PROG_PSLOTS;
		const uint32_t dst   = slot0 + nxt * TBF_PROG_SLOT;
		const tbf_prog_entry* src = P.prog + last;
		tbf_prog_entry*       d   = (tbf_prog_entry*)P.prog + dst;
		const uint32_t        cnt = src[0].pad + 1;
		for (uint32_t k = lane; k < cnt; k += NL)
			d[k] = src[k];
	}
	wave_sync ();
	for (size_t i = lane; i < (size_t)nw * 6; i += NL)
		(&G->sums[0][0])[i] = W.sums[i];
	for (uint32_t w = lane; w < nw; w += NL) {
		G->refCount[w] = W.ref[w];
		G->list[w]     = W.list[w];
		G->aclPos1[w]  = W.acl1[w];
		G->rflags[w]   = W.rf[w];
	}
	if (lane == 0)
		G->listEnd = L;
	if (lane < 27)
		G->gain[lane] = sm.dbg[lane];
#ifdef TBF_CTL_PROF
	CTL_ACC (pr_end, pr_e0);
	if (lane == 0 && (blockIdx.x & 255) == 0)
		printf ("ctlprof wg %u blocks %d L %u pre %lu stage %lu msg %lu blk %lu (pass %lu rem %lu) end %lu total %lu rt0 %lu rt1 %lu\n",
		        blockIdx.x, __builtin_popcountll (todo0), L, pr_k0 - pr_c0, pr_stage, pr_msg, pr_blk, pt[0], pt[1], pr_end,
		        __builtin_amdgcn_s_memtime () - pr_c0, pr_rt0, __builtin_amdgcn_s_memrealtime ());
#endif
}

/* The device front end of a chunk whose events are notes, drawbar moves and the vibrato
 * and percussion switches (src/tonegen.cpp:3096-3166 oscKeyOn / oscKeyOff, 2738-2756
 * setDrawBar, 1678-1765 setPercEnabled / setPercFirst, src/vibrato.cpp routing; the
 * per-block step of TgControl::stepFront / mixCtl): one lane per instance, 64 instances a
 * wave, each lane walking its instance's events in order from its front state at the chunk
 * start (one wave per instance with lane 0 walking, before: 4096 single-wave workgroups
 * that waited for free wave slots behind the render stages).  A key event
 * updates activeKeys and the key counts and queues its messages; a drawbar or percussion
 * event updates the drawbar gains (the changed buses' (bus, gain) pairs go out with the
 * block's record) and the drawbar-change flag; a switch updates the routing word.  A block
 * with inputs (messages, a drawbar change or a routing change), or right after one
 * (steadyPending), is stepped: it gets a control delta (pool index nInst + inst * nBlocks
 * + k) whose record k_tgctl turns into the entry (the persistent entry with this block's
 * keyCompTarget, percussion reset and routing) and the program.  Writes the records, the
 * messages, the gain pairs and the chunk's index table. */
__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL))) k_front (const tbf_launch P)
{
	/* per lane (instance) i: activeKeys keys[w][i], the drawBarGain of the buses changed
	 * since the last step gl[bus][i]; the wave's events (instances i0 .. i0 + 63 are
	 * contiguous in fev, their first FR_CAP staged) and the first instance's template's
	 * key-compression table, read lane-parallel up front so the walks wait on LDS, not on
	 * one dependent global load per event */
	__shared__ uint32_t keys[12][NL];
	__shared__ float    gl[27][NL];
	__shared__ uint32_t fevs[FR_CAP];
	__shared__ float    kcs[128];
	const int             lane = threadIdx.x;
	const uint32_t        n = P.nInst, nb = P.nBlocks;
	const uint32_t        i0 = blockIdx.x * NL, iN = i0 + NL < n ? i0 + NL : n;
	const uint32_t        inst = i0 + (uint32_t)lane;
	const bool            act  = inst < n;
	const tbf_front_state& F   = P.front[act ? inst : iN - 1];
	const uint32_t        w0 = P.fevOff[i0], w1 = P.fevOff[iN];
	const uint32_t        e0 = P.fevOff[act ? inst : iN - 1], eEnd = act ? P.fevOff[inst + 1] : e0;
	const uint32_t        tpl0 = P.cst[i0].tpl;
#pragma unroll
	for (int w = 0; w < 12; w++)
		keys[w][lane] = F.keys[w];
	{
		const float* kt = P.keyComp + (size_t)tpl0 * 128;
		kcs[lane]       = kt[lane];
		kcs[lane + NL]  = kt[lane + NL];
		const uint32_t ne = w1 - w0 < FR_CAP ? w1 - w0 : FR_CAP;
		for (uint32_t i = lane; i < ne; i += NL)
			fevs[i] = P.fev[w0 + i];
	}
	wave_sync ();
	if (!act)
		return;
	auto fev = [&] (uint32_t e) { return e - w0 < FR_CAP ? fevs[e - w0] : P.fev[e]; };
	const uint32_t tpl = P.cst[inst].tpl;
	const float*   kct = P.keyComp + (size_t)tpl * 128;
	auto kcomp = [&] (int i) { return tpl == tpl0 ? kcs[i] : kct[i]; };
	uint32_t*      ctlIdx = (uint32_t*)P.ctlIdx;
	uint16_t*      msgs   = (uint16_t*)P.msgs;
	tbf_tgc_rec*   rec    = (tbf_tgc_rec*)P.rec;
	float*         gains  = (float*)P.gains;
	int            kdc = F.keyDown, ukc = F.upperDown;
	bool           pending = F.pending != 0;
	uint32_t       r = F.routing, oldR = F.routing, psb = F.percSendBus;
	int            pe = F.percEnabled, restore = F.percTrigRestore;
	const int      ptb = F.percTriggerBus;
	uint32_t       gm = 0, dbc = 0, go = F.gainOff;
	uint32_t       e = e0;
	uint32_t       mo = 2 * e; /* the instance's message slots: at most two per event */
	uint32_t       idx = inst, k = 0;
	/* the effect setters' fields: the instance's entry at the chunk start, changed in
	 * registers; a block whose fields changed gets a full entry of its own */
	tbf_seg_ctl    E = P.ctl[inst];
	tbf_seg_ctl*   fulls = (tbf_seg_ctl*)P.fulls;
	int            soft = F.percSoft != 0, fast = F.percFast != 0;
	float          swell = F.swell;
	bool           fx = false, revClear = false;
	int            revPend = -1;
	/* drawBarLevel[bus][s] = (float)((float)s / 8.0) on every bus (TgControl::init) */
	auto level = [] (uint32_t s) { return (float)((double)(float)s / 8.0); };
	for (uint32_t b = 0; b < nb; b++) {
		const uint32_t m0 = mo;
		for (; e < eEnd && (fev (e) >> 16) == b; e++) {
			const uint32_t v = fev (e);
			if (v & TBF_FEV_PARAM) {
				const uint32_t op = (v >> 12) & 7u, bus = v & 31u, set = (v >> 5) & 15u;
				const bool     fl = (v >> 9) & 1u;
				if (op == TBF_FEV_EFFECT) {
					/* the CLAP setParam effect setters (src/clap.cpp:162-207), as tbf_set_param and
					 * stepControl apply them to the instance's control entry */
					/* a known setter marks the entry full (fx); an unknown bus is skipped and leaves
					 * fx as an earlier event of the block set it (frontParam emits none today) */
					const float x  = P.fevVal[e];
					const bool  kn = bus <= TBF_FX_VIBTYPE; /* TBF_FX_ROTOR .. TBF_FX_VIBTYPE (tbf_types.h) */
					fx = fx || kn;
					switch (bus) {
						case TBF_FX_ROTOR: revPend = (int)x; break; /* used by this block only */
						case TBF_FX_CLEAN: E.odClean = (uint32_t)(int)x; break;
						case TBF_FX_CHARACTER: {
							/* fsetCharacter's output level C (linseg in float), then the preamp's
							 * per-block constants (src/overdrive.cpp:60-140; odCtlCompute) */
							/* the reference's double tables, narrowed to float as tbf::setCharacter does */
							const float Av[5] = {(float)0.0, (float)0.25, (float)0.50, (float)0.75, (float)1.00};
							const float Cv[5] = {(float)1.0, (float)0.70, (float)0.25, (float)0.15, (float)0.13};
							for (int q = 0; q < 4; q++)
								if (x <= Av[q + 1]) {
									const float a = Av[q], bb = Av[q + 1], p = Cv[q], qq = Cv[q + 1];
									E.odOutput    = (double)(p + (x - a) * (qq - p) / (bb - a));
									break;
								}
							double density = x * 4.0, out = fabs (density);
							density        = density * fabs (density);
							double count   = density;
							int    iter    = 0;
							while (count > 1.0 && iter < 64) { /* the host admits A in [0, 1]: <= 15 */
								iter++;
								count = count - 1.0;
							}
							while (out > 1.0)
								out = out - 1.0;
							E.odIter       = iter;
							E.odOut        = out;
							E.odDensityPos = density > 0 ? 1u : 0u;
							break;
						}
						case TBF_FX_REVERB: E.rvWet = (double)x; break;
						case TBF_FX_PERC_SOFT:
						case TBF_FX_PERC_FAST:
							if (bus == TBF_FX_PERC_SOFT) {
								soft               = (int)x != 0;
								E.percEnvGainReset = F.percReset[soft];
								E.outputGain       = swell * F.percDrawbar[soft];
							} else
								fast = (int)x != 0;
							E.percEnvGainDecay = F.percDecay[fast * 2 + soft];
							break;
						case TBF_FX_SWELL:
							swell            = x;
							E.swellPedalGain = swell;
							E.outputGain     = swell * F.percDrawbar[soft];
							break;
						case TBF_FX_BYPASS: E.whBypass = (uint32_t)(int)x; break;
						case TBF_FX_VIBTYPE: {
							const int q = (int)x;
							if (q >= 0 && q <= 5) {
								E.vibTable = (uint32_t)(q / 2);
								E.vibMixed = (uint32_t)(q & 1);
							}
							break;
						}
						default: break;
					}
					continue;
				}
				if (op == TBF_FEV_DRAWBAR) {
					if (set > 8)
						continue; /* setDrawBar ignores settings > 8 */
					dbc = 1;
					if ((int)bus == ptb) {
						restore = (int)set;
						if (pe)
							continue;
					}
					gl[bus][lane] = level (set);
					gm |= 1u << bus;
				} else if (op == TBF_FEV_VIB_UPPER) {
					r = fl ? (r | 0x02u) : (r & ~0x02u);
				} else if (op == TBF_FEV_VIB_LOWER) {
					r = fl ? (r | 0x01u) : (r & ~0x01u);
				} else if (op == TBF_FEV_PERC) {
					r = fl ? (r | 0x0Cu) : (r & ~0x0Cu);
					if (-1 < ptb) {
						gl[ptb][lane] = fl ? 0.0f : level ((uint32_t)restore);
						gm |= 1u << ptb;
						dbc = 1;
					}
					pe = fl;
				} else if (op == TBF_FEV_PERC_FIRST) {
					psb = fl ? F.percSendBusA : F.percSendBusB;
				}
				continue;
			}
			const uint32_t key = v & 0x0fffu;
			const bool     on  = (v >> 12) & 1u;
			if (key >= 384) /* the host packs keys outside [0, MAX_KEYS) as 0x0fff: ignored (3098) */
				continue;
			const uint32_t w = key >> 5, bit = 1u << (key & 31);
			if (keys[w][lane] & bit) { /* keyOff, or keyOn's release of a held key first */
				keys[w][lane] &= ~bit;
				if (key < 128)
					ukc--;
				kdc--;
				msgs[mo++] = (uint16_t)key;
			}
			if (on) {
				keys[w][lane] |= bit;
				if (key < 128)
					ukc++;
				kdc++;
				msgs[mo++] = (uint16_t)(0x1000u | key);
			}
		}
		const uint32_t nm   = mo - m0;
		const bool     rcp  = r != oldR;
		const bool     tgs  = nm > 0 || dbc || rcp || pending; /* a tone-generator step */
		const bool     fxE  = fx || revPend >= 0 || revClear;  /* an entry with new effect fields */
		if (tgs || fxE) {
			const uint32_t d  = inst * nb + k++;
			const uint32_t ng = (uint32_t)__builtin_popcount (gm);
			tbf_tgc_rec    R;
			R.msgOff        = m0;
			R.nMsg          = nm;
			R.gainOff       = ng ? go : 0;
			R.full          = 0;
			R.keyCompTarget = kcomp (kdc < 0 ? 0 : (kdc > 127 ? 127 : kdc));
			R.flags         = (uint8_t)((tgs ? 0x80u | dbc | (rcp ? 2u : 0u) | (ng ? 4u : 0u) : 0u) | (ukc == 0 ? 8u : 0u));
			R.oldRouting    = (uint8_t)r;
			R.percSendBus   = (uint8_t)psb;
			R.pad           = (uint8_t)ng;
			for (uint32_t m = gm; m; m &= m - 1) { /* the changed buses in bus order */
				const uint32_t bus = (uint32_t)__builtin_ctz (m);
				gains[go++]        = __uint_as_float (bus);
				gains[go++]        = gl[bus][lane];
			}
			if (fxE) {
				/* a full entry with this block's effect fields; k_tgctl patches its key fields
				 * and program from the record (flag 0x10) and every later delta of the chunk
				 * starts from it.  A rotary selection is used by this block only: the next
				 * block gets an entry without it. */
				E.whRevOption = revPend;
				E.whSet       = 0;
				fulls[d]      = E;
				R.full        = d + 1;
				R.flags |= 0x10u;
				revClear = revPend >= 0;
				revPend  = -1;
				fx       = false;
			}
			rec[d] = R;
			idx    = n + d;
			if (tgs) {
				pending = nm > 0 || dbc || rcp;
				oldR    = r;
				gm = dbc = 0;
			}
		}
		ctlIdx[(size_t)b * n + inst] = idx;
	}
}

extern "C" int tbf_launch_front (const tbf_launch* P, hipStream_t stream)
{
	if (P->nInst == 0 || P->nBlocks > NL || P->instBase != 0)
		return -22;
	hipLaunchKernelGGL (k_front, dim3 ((P->nInst + NL - 1) / NL), dim3 (NL), 0, stream, *P);
	return hipGetLastError () == hipSuccess ? 0 : -5;
}

extern "C" int tbf_launch_tgctl (const tbf_launch* P, hipStream_t stream)
{
	if (P->nCtlInst == 0)
		return 0;
	if (P->ctlNw == 0 || P->ctlNw > TBF_NW + 1 || P->nBlocks > NL)
		return -22; /* the wheel count the play matrices name; one lane per block */
	hipLaunchKernelGGL (k_tgctl, dim3 (P->nCtlInst), dim3 (NL), ctl_wbytes (P->ctlNw), stream, *P);
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
