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
 * One wave per instance with stepped blocks in the chunk, blocks in order, the instance's
 * bus levels and routed sums staged in LDS for the launch (their read-modify-writes were
 * global round trips, one per message and list pass):
 *   messages   in queue order; the key's keyContrib list (sorted by wheel, then bus) is
 *              spread over the lanes.  Each (wheel, bus) appears once per key, so the
 *              bus-level adds are lane-parallel and keep the reference's per-(wheel, bus)
 *              order; a wheel's reference-count / flag update is made once per wheel group
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

struct CtlLds {
	float    bl[NW + 1][27]; /* the instance's bus levels and routed sums, staged for the launch */
	float    sums[NW + 1][6];
	int32_t  ref[NW + 1];
	uint16_t list[NW + 1];
	int16_t  acl1[NW + 1];
	uint16_t removed[NW + 1];
	uint8_t  rf[NW + 1];
	float    dbg[27];
	uint32_t L;
	uint32_t nrem;
};

__device__ __forceinline__ uint64_t lanemask_lt () { return (1ull << threadIdx.x) - 1ull; }

/* one key message (src/tonegen.cpp:3270-3322) */
__device__ void ctl_message (CtlLds& sm, const tbf_contrib* __restrict__ kc, uint32_t c0, uint32_t c1, bool on)
{
	const int lane = threadIdx.x;
	for (uint32_t base = c0; base < c1; base += NL) {
		const uint32_t e     = base + lane;
		const bool     valid = e < c1;
		uint32_t       w = 0, bus = 0;
		float          lev  = 0.f;
		bool           lead = false;
		if (valid) {
			const tbf_contrib c = kc[e];
			w                   = c.wheel;
			bus                 = c.bus;
			lev                 = c.level;
			lead                = (e == c0) || kc[e - 1].wheel != w;
		}
		/* a wheel group's part in this pass: from its first lane to the next group's first
		 * lane (or the pass end); lane 0 continues a group begun in the previous pass */
		const uint64_t ld    = __ballot (lead);
		const uint32_t nval  = c1 - base < (uint32_t)NL ? c1 - base : (uint32_t)NL;
		const uint64_t after = (lane + 1 < NL) ? (ld >> (lane + 1)) : 0ull;
		const uint32_t next  = after ? (uint32_t)(lane + 1 + __builtin_ctzll (after)) : nval;
		const bool     owner = valid && (lead || lane == 0);
		const int      part  = (int)(next - (uint32_t)lane);
		bool           join  = false;
		if (valid) {
			float* bl = &sm.bl[w][bus];
			*bl       = on ? *bl + lev : *bl - lev;
		}
		if (owner) {
			const int r0 = sm.ref[w];
			if (on) {
				if (lead && r0 == 0) {
					sm.rf[w] = 0x0006;
					join     = sm.acl1[w] == 0;
				} else {
					sm.rf[w] |= 0x0004;
				}
				sm.ref[w] = r0 + part;
			} else {
				const int r1 = r0 - part;
				sm.ref[w]    = r1;
				sm.rf[w]     = r1 == 0 ? 0x0005 : (sm.rf[w] | 0x0004);
			}
		}
		const uint64_t jb = __ballot (join);
		if (join) {
			const uint32_t pos = sm.L + (uint32_t)__builtin_popcountll (jb & lanemask_lt ());
			sm.list[pos]       = (uint16_t)w;
			sm.acl1[w]         = (int16_t)(pos + 1);
		}
		__syncthreads ();
		if (lane == 0)
			sm.L += (uint32_t)__builtin_popcountll (jb);
		__threadfence_block ();
		__syncthreads ();
	}
}

/* the active-list loop and the removals of one block (src/tonegen.cpp:3333-3594); writes
 * the program (header + one entry per active wheel) at out */
__device__ void ctl_block (CtlLds& sm, const tbf_tgc_rec& R, tbf_prog_entry* __restrict__ out)
{
	const int      lane        = threadIdx.x;
	const uint32_t L0          = sm.L;
	const bool     dbChange    = (R.flags & 1) != 0;
	const bool     recompute   = (R.flags & 2) != 0;
	const uint32_t routing     = R.oldRouting;
	const uint32_t percSendBus = R.percSendBus;
	if (lane == 0)
		sm.nrem = 0;
	__syncthreads ();
	for (uint32_t base = 0; base < L0; base += NL) {
		const uint32_t i     = base + lane;
		const bool     valid = i < L0;
		bool           rem   = false;
		uint32_t       on    = 0;
		if (valid) {
			on                = sm.list[i];
			const uint32_t rf = sm.rf[on];
			float*         S  = sm.sums[on];
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
					const float* bl  = sm.bl[on];
					float        sum = 0.0f;
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
					sumPercn = (routing & 0x0C) ? sm.bl[on][percSendBus] : 0.0f;
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
			sm.rf[on]  = 0;
			out[1 + i] = E;
		}
		const uint64_t rb = __ballot (rem);
		if (rem)
			sm.removed[sm.nrem + (uint32_t)__builtin_popcountll (rb & lanemask_lt ())] = (uint16_t)on;
		__syncthreads ();
		if (lane == 0)
			sm.nrem += (uint32_t)__builtin_popcountll (rb);
		__syncthreads ();
	}
	if (lane == 0) {
		tbf_prog_entry H = {};
		H.wheel          = 0xFFFF;
		H.pad            = L0;
		out[0]           = H;
		/* removal list, in order (3576-3594) */
		uint32_t L = L0;
		for (uint32_t r = 0; r < sm.nrem; r++) {
			const uint32_t vic = sm.removed[r];
			const int      act = sm.acl1[vic] - 1;
			sm.acl1[vic]       = 0;
			L--;
			if (0 < L) {
				const uint32_t mov = sm.list[L];
				if (mov != vic) {
					sm.list[act]  = (uint16_t)mov;
					sm.acl1[mov] = (int16_t)(act + 1);
				}
			}
		}
		sm.L = L;
	}
	__threadfence_block ();
	__syncthreads ();
}

__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL))) k_tgctl (const tbf_launch P)
{
	__shared__ CtlLds sm;
	const int         lane = threadIdx.x;
	const uint32_t    inst = P.ctlInst[blockIdx.x];
	tbf_tgc_state*    G    = P.tgc + inst;
	const uint32_t    tpl  = P.cst[inst].tpl;
	const uint32_t*   coff = P.coff + (size_t)tpl * 385;
	for (int i = lane; i < (NW + 1) * 27; i += NL)
		(&sm.bl[0][0])[i] = (&G->busLevel[0][0])[i];
	for (int i = lane; i < (NW + 1) * 6; i += NL)
		(&sm.sums[0][0])[i] = (&G->sums[0][0])[i];
	for (int w = lane; w <= NW; w += NL) {
		sm.ref[w]  = G->refCount[w];
		sm.list[w] = G->list[w];
		sm.acl1[w] = G->aclPos1[w];
		sm.rf[w]   = G->rflags[w];
	}
	if (lane == 0)
		sm.L = G->listEnd;
	if (lane < 27)
		sm.dbg[lane] = G->gain[lane];
	__syncthreads ();
	const uint32_t n    = P.nInst;
	uint32_t       prev = inst;
	int64_t        last = -1; /* prog_off of the last program written */
	for (uint32_t b = 0; b < P.nBlocks; b++) {
		const uint32_t idx = P.ctlIdx[(size_t)b * n + inst];
		if (idx == prev || idx < n)
			continue;
		prev                 = idx;
		const tbf_tgc_rec& R = P.rec[idx - n];
		if (!(R.flags & 0x80))
			continue; /* a control change without a tone-generator step */
		if ((R.flags & 4) && lane < 27)
			sm.dbg[lane] = P.gains[R.gainOff + lane];
		__syncthreads ();
		for (uint32_t m = 0; m < R.nMsg; m++) {
			const uint32_t msg = P.msgs[R.msgOff + m];
			const uint32_t kn  = msg & 0x0fffu;
			if (kn >= 384)
				continue;
			ctl_message (sm, P.contrib, coff[kn], coff[kn + 1], (msg & 0xf000u) == 0x1000u);
		}
		const uint32_t off = P.ctl[idx].prog_off;
		ctl_block (sm, R, (tbf_prog_entry*)P.prog + off);
		last = off;
	}
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
	__syncthreads ();
	for (int i = lane; i < (NW + 1) * 27; i += NL)
		(&G->busLevel[0][0])[i] = (&sm.bl[0][0])[i];
	for (int i = lane; i < (NW + 1) * 6; i += NL)
		(&G->sums[0][0])[i] = (&sm.sums[0][0])[i];
	for (int w = lane; w <= NW; w += NL) {
		G->refCount[w] = sm.ref[w];
		G->list[w]     = sm.list[w];
		G->aclPos1[w]  = sm.acl1[w];
		G->rflags[w]   = sm.rf[w];
	}
	if (lane == 0)
		G->listEnd = sm.L;
	if (lane < 27)
		G->gain[lane] = sm.dbg[lane];
}

extern "C" int tbf_launch_tgctl (const tbf_launch* P, hipStream_t stream)
{
	if (P->nCtlInst == 0)
		return 0;
	hipLaunchKernelGGL (k_tgctl, dim3 (P->nCtlInst), dim3 (NL), 0, stream, *P);
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
