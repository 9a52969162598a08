/*
 * tbf_render.hip -- gfx950 render kernels for the tuneBfree block quartet
 *   oscGenerateFragment -> preamp -> b_reverb::reverb -> whirlProc3
 * (src/tonegen.cpp:3218, src/overdrive.cpp:329, src/reverb.cpp:274, src/whirl.cpp:1653).
 *
 * Three kernels per launch chunk, each one wave64 per organ instance looping over the
 * chunk's 128-sample blocks with that stage's state resident in LDS:
 *   k_tonegen  tonegen + vibrato + mixdown + overdrive   -> mid1 [inst][block*128]
 *   k_reverb   MatrixVerb (FP64)                         -> mid2
 *   k_whirl    horn/drum rotors + mic mix                -> outL / outR
 * Every stage is causal, so running all blocks of stage k before stage k+1 is exact.
 * Splitting the stages gives each kernel its own register and LDS budget (occupancy
 * 3-4 waves/SIMD instead of 2 for the fused kernel); mid1/mid2 add 16 B per stereo
 * sample of HBM traffic against the reverb's 416 B.
 *
 * Inside a stage: lane = sample (tonegen: 2 samples/lane; reverb/whirl: 64-sample
 * sub-blocks).  Every ring read of a sub-block happens before its ring writes, which is
 * exact because every ring delay exceeds the sub-block (reverb >= 560, whirl >= 79
 * samples ahead).  Per-sample IIR/phase recurrences run on single lanes in the
 * reference's literal operation order.
 * Float discipline: compiled with -ffp-contract=off, no fast-math, denormals kept;
 * every expression follows the reference's evaluation order so results are
 * bit-identical to the strict-IEEE oracle except for FP64 libm (sin/asin) ulps.
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/tbf.h"
#include "tbf_types.h"
#include "tbf_exact.h"
#include "tbf_sin.h"

#define NL 64

/* occupancy targets (waves per SIMD); LDS and VGPR budgets are sized for them */
#define TG_WAVES 4
#define TG_SPLIT_MAX 8 /* k_tonegen block ranges (waves) per instance */
#ifndef TG_CACHE
#define TG_CACHE 1 /* steady chunks: the program's wheels, lengths and offsets held in the lanes */
#endif
#ifndef TG_LDS_ALL
#define TG_LDS_ALL 1 /* entries staged in LDS for steady chunks too (their per-block scalar loads: 21.8 -> 18.8 ms with TG_CACHE) */
#endif
#ifndef TG_ABL
#define TG_ABL 0 /* timing experiments (wrong output): 1 bank reads from one row, 2 no scanner */
#endif
#define TG_PCAP 128    /* a delta chunk's program entries staged in LDS per block (longer: read from HBM) */
#ifndef TG_GRFL
#define TG_GRFL 0 /* 1: the entries' gains moved to scalar registers (v_readfirstlane) after their LDS reads */
#endif
#ifndef TG_LCACHE
#define TG_LCACHE 1 /* TG_CACHE's per-entry bank position, end and length in LDS, not in the lanes */
#endif
#define RV_WAVES 3
/* k_whirl: 4 waves per SIMD (128 VGPRs, 9.8 KB of LDS: 16 instances per CU, so 4096 run
 * at once on 256 CUs), motions and ring adds in 2 groups of 2 rings (4 rings per group
 * need 168 VGPRs) */
#ifndef WH_WAVES
#define WH_WAVES 4
#endif
#ifndef WH_RG
#define WH_RG 2 /* k_whirl rings per motion group (4 or 2) */
#endif
#ifndef WH_SERIAL_PIPE
#define WH_SERIAL_PIPE 1 /* k_whirl serial passes: next group's reads ahead of this group's chain */
#endif
#ifndef WH_PAD
/* floats after each LDS ring / horn-A row: the rows of one serial pass 16-B aligned (its
 * 4-sample reads and writes) and each lane's 16 B on banks of its own */
#define WH_PAD 4
#endif
/* wave priority raised (s_setprio 1) while a wave runs a serial chain, so the SIMD issues
 * the chain's dependent instructions ahead of other waves' lane-parallel work */
#define PRIO_UP() __builtin_amdgcn_s_setprio (1)
#define PRIO_DOWN() __builtin_amdgcn_s_setprio (0)

template <bool B> struct BoolC {
	static constexpr bool value = B;
};
template <int K> struct IntC {
	static constexpr int value = K;
};

/* ------------------------------------------------------------------ LDS layouts */
struct TgLds {
	tbf_tg_state st;
#if TG_LCACHE
	/* TG_CACHE, entry e < 2 NL: bank index of the wheel's current sample, and the wave's end
	 * and length in the bank (a block advances the index by TBF_BLK, less the length past
	 * the end) */
	uint32_t     cbase[2 * NL], cend[2 * NL], clen[2 * NL];
#endif
	float        swl[TBF_BLK];
	float        vin[TBF_BLK];
	float        prc[TBF_BLK];
	union {
		struct { /* core-program entries resolved by the interpreter prologue */
			uint32_t base[TBF_NW + 8]; /* bank index of the wheel's current sample (the device
			                            * bank repeats each wave's first 128 samples after it) */
			float4   g[TG_PCAP];       /* {sg, pg, vg, nsg} of a program of <= TG_PCAP entries ... */
			float2   h[TG_PCAP];       /* ... {npg, nvg} */
			uint32_t er[TG_PCAP];      /* ... env | row << 8 */
		} ent;
		struct { /* vibrato */
			float   vout[TBF_BLK];
			float   va[TBF_BLK];
			float   vg[TBF_BLK];
			int32_t vh[TBF_BLK];
		} v;
	} u;
};


template <int W>
struct WhLds {
	tbf_wh_state st;
	alignas (16) float wring[4][W + WH_PAD]; /* rows padded: the serial lanes 2, 3 read rings 2, 3 at the same index */
	float        xf[TBF_SUB + 4];
	float        x1[TBF_SUB + 4];
	float        x2[TBF_SUB + 4];
	/* horn A rows by parity ap: ab[ap] takes the next sub-block's input and horn A filters
	 * it in place (A runs one sub-block ahead), ab[ap ^ 1] holds A's output of this
	 * sub-block, horn B's input */
	alignas (16) float ab[2][TBF_SUB + WH_PAD];
	int          brake;
	int          aReady; /* ab[ap ^ 1] holds this sub-block's horn A output */
	int          ap;
};

/* the control entry of instance `inst` for block `blk` of the chunk: events land at
 * block boundaries, so the host records a new pool entry only where one changes */
__device__ __forceinline__ const tbf_seg_ctl& ctl_of (const tbf_launch& P, const tbf_seg_ctl* __restrict__ ctl,
                                                      uint32_t blk, uint32_t inst)
{
	return ctl[P.ctlIdx ? P.ctlIdx[(size_t)blk * P.nInst + inst] : inst];
}

/* copy a state sub-struct between HBM and LDS, one dword per lane (of the calling wave) */
template <typename T>
__device__ __forceinline__ void copy_words (T* dst, const T* src)
{
	static_assert (sizeof (T) % 4 == 0, "state structs are dword-sized");
	const uint32_t* s = (const uint32_t*)src;
	uint32_t*       d = (uint32_t*)dst;
	for (uint32_t i = threadIdx.x & (NL - 1); i < sizeof (T) / 4; i += NL)
		d[i] = s[i];
}

__device__ __forceinline__ uint32_t xorshift (uint32_t s)
{
	s ^= s << 13;
	s ^= s >> 17;
	s ^= s << 5;
	return s;
}

/* xorshift32 state after a per-lane k steps from a uniform x0, from the nibble-sliced table
 * (xs_nib_table): one coalesced row load per nibble of x0, 8 in flight together */
__device__ __forceinline__ uint32_t xs_jump_n (const uint32_t* __restrict__ J, uint32_t x0, int k)
{
	const uint32_t* N = J + 32 * TBF_XS_JUMP;
	x0                = __builtin_amdgcn_readfirstlane (x0);
	uint32_t v[8];
#pragma unroll
	for (int i = 0; i < 8; i++)
		v[i] = N[(i * 16 + ((x0 >> (4 * i)) & 15u)) * TBF_XS_JUMP + k];
	return ((v[0] ^ v[1]) ^ (v[2] ^ v[3])) ^ ((v[4] ^ v[5]) ^ (v[6] ^ v[7]));
}

/* lane l's value, wave-uniform (l uniform) */
__device__ __forceinline__ int rl (int v, int l) { return __builtin_amdgcn_readlane (v, l); }

__device__ __forceinline__ double rld (double v, int l)
{
	const unsigned long long u = __double_as_longlong (v);
	const unsigned lo = __builtin_amdgcn_readlane ((unsigned)u, l), hi = __builtin_amdgcn_readlane ((unsigned)(u >> 32), l);
	return __longlong_as_double ((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ int wave_min (int v)
{
	for (int o = 32; o > 0; o >>= 1)
		v = min (v, __shfl_xor (v, o));
	return v;
}

__device__ __forceinline__ int wave_max (int v)
{
	for (int o = 32; o > 0; o >>= 1)
		v = max (v, __shfl_xor (v, o));
	return v;
}

/* LDS ordering between the lanes of a one-wave workgroup: a wave's LDS instructions
 * execute in issue order, so a read after a write sees it without a wait; only the
 * compiler must not move LDS accesses across this point (s_barrier and its lgkmcnt(0)
 * drain would expose the LDS latency at every sync) */
__device__ __forceinline__ void wave_sync ()
{
	__builtin_amdgcn_fence (__ATOMIC_ACQ_REL, "wavefront");
	__builtin_amdgcn_wave_barrier ();
}

/* Whole-wave lane shifts by DPP (wave_shr:1 / wave_shl:1, GFX9 DPP controls 0x138 /
 * 0x130): lane i receives lane i-1 (shr) or i+1 (shl); the lane with no source gets 0
 * (bound_ctrl; callers mask it), so the shift is one v_mov_b32_dpp into a fresh register
 * (keeping the old value needed a copy first).  VALU-only, unlike __shfl_up/down
 * (ds_bpermute). */
__device__ __forceinline__ int lane_shr1 (int v) { return __builtin_amdgcn_mov_dpp (v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int lane_shl1 (int v) { return __builtin_amdgcn_mov_dpp (v, 0x130, 0xF, 0xF, true); }
__device__ __forceinline__ float lane_shr1 (float v) { return __int_as_float (lane_shr1 (__float_as_int (v))); }
__device__ __forceinline__ float lane_shl1 (float v) { return __int_as_float (lane_shl1 (__float_as_int (v))); }
/* lane n receives lane n-1's v, lane 0 receives first: one DPP move with the old value
 * (bound_ctrl off), so there is no select on the lane index -- a select lets the compiler
 * put the DPP move under a branch that disables lane 0, and a DPP move reading a disabled
 * lane gets 0 */
__device__ __forceinline__ float lane_shr1_or (float v, float first)
{
	return __int_as_float (__builtin_amdgcn_update_dpp (__float_as_int (first), __float_as_int (v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ double lane_shr1 (double v)
{
	const unsigned long long u = __double_as_longlong (v);
	const unsigned long long lo = (unsigned)lane_shr1 ((int)(unsigned)u), hi = (unsigned)lane_shr1 ((int)(unsigned)(u >> 32));
	return __longlong_as_double ((long long)((hi << 32) | lo));
}

/* Airwindows 32-bit dither term, src/overdrive.cpp:153-159 / src/reverb.cpp:775-783.
 * The reference multiplies by a long double literal; FP64 here (the
 * difference reaches the float output with probability ~1e-17 per sample). */
__device__ __forceinline__ double dither_add (double v, uint32_t fpd)
{
	int expon;
	frexpf ((float)v, &expon);
	double t = ((double)fpd - 2147483647.0) * 5.5e-36;
	t        = t * ldexp (1.0, expon + 62);
	return v + t;
}

/* a lane's two samples (n, n + 64) of a 128-sample block: packed FP32 math */
typedef float f2v __attribute__ ((ext_vector_type (2)));
/* 4-byte-aligned float pairs / quads: one global load for consecutive table entries */
typedef float f2u __attribute__ ((ext_vector_type (2), aligned (4)));
typedef float f4u __attribute__ ((ext_vector_type (4), aligned (4)));

/* fmodf (x, 1.f) of a motion's table position (src/whirl.cpp:1436, 1458): the argument is
 * angle * 16384 + phase with the rotor angle in [0, 1) (every update is an fmod (., 1) or
 * a brake target fmod (., 1.0)), the mic offsets fwAng = micAngle / 4 in [0, 0.25] and
 * bwAng = 1 - micAngle / 4 in [0.75, 1] (micAngle = 1 - deg / 180, deg in [0, 180],
 * src/whirl.cpp:1139, 1380-1381) and phases below 16384: so 0 <= x < 2^24, where fmodf
 * (x, 1) is x - floorf (x) exactly (the fractional bits).  NaN stays NaN either way. */
__device__ __forceinline__ float frac1 (float x) { return x - floorf (x); }

/* RBJ biquad, Direct Form II in float (EQ_IIR, src/whirl.cpp:1479-1485); coefficients
 * a1 a2 b0 b1 b2 in registers */
__device__ __forceinline__ float eq_iir (float c0, float c1, float c2, float c3, float c4, float& z0, float& z1,
                                         float x)
{
	float temp = x - (c0 * z0) - (c1 * z1);
	float y    = (temp * c2) + (c3 * z0) + (c4 * z1);
	z1         = z0;
	z0         = temp;
	return y;
}

/* One motion's ordered adds into a ring for a 64-sample sub-block (HN_MOTION /
 * DR_MOTION, src/whirl.cpp:1432-1469): sample n adds a_n into slot U_n and b_n into
 * slot U_n + 1, in sample order.  With U non-decreasing, the samples sharing a slot
 * value form a group G(u) and slot t receives, in order, b of G(t-1) then a of G(t).
 * Groups have at most 2 samples (checked by the caller), so the first lane of each
 * group owns slot t = U (and slot t + 1 when no group sits at t + 1) and finds its
 * neighbours' terms with lane shifts; owners never share a slot. */
/* the owner lanes' slots and ordered sums of one motion (see motion_add) */
struct MotionOwn {
	bool     first, own2, pair, lead, lead2;
	uint32_t t;
	float    a, an, b, bn, bp1, bp2;
};

__device__ __forceinline__ MotionOwn motion_own (int U, float a, float b, int lane)
{
	MotionOwn m;
	const int Up  = lane_shr1 (U);
	const int Up2 = lane_shr1 (Up);
	const int Un  = lane_shl1 (U);
	const int Un2 = lane_shl1 (Un);
	m.bp1         = lane_shr1 (b);
	m.bp2         = lane_shr1 (m.bp1);
	m.an          = lane_shl1 (a);
	m.bn          = lane_shl1 (b);
	m.a           = a;
	m.b           = b;
	m.t           = (uint32_t)U;
	m.first       = lane == 0 || U != Up;
	m.pair        = lane < NL - 1 && Un == U;
	m.lead        = lane > 0 && Up == U - 1;
	m.lead2       = lane > 1 && Up2 == Up;
	const bool nextExists = m.pair ? lane < NL - 2 : lane < NL - 1;
	const int  Unx        = m.pair ? Un2 : Un;
	m.own2                = !nextExists || Unx != U + 1;
	return m;
}

/* slot t: b of the group at t-1 (<= 2 samples, in order), then a of the group at t.  A
 * skipped add keeps v (v + 0 is not v for v = -0), so each optional add is a select of the
 * sum, not a branch: the passes stay branch-free */
__device__ __forceinline__ float motion_sum_t (const MotionOwn& m, float v)
{
	float t = v + m.bp2;
	v       = (m.lead && m.lead2) ? t : v;
	t       = v + m.bp1;
	v       = m.lead ? t : v;
	v += m.a;
	t = v + m.an;
	return m.pair ? t : v;
}

/* slot t + 1 when no group sits there: b of this group */
__device__ __forceinline__ float motion_sum_t1 (const MotionOwn& m, float w)
{
	w += m.b;
	const float t = w + m.bn;
	return m.pair ? t : w;
}

template <int W>
__device__ __forceinline__ void motion_add (float* ring, int U, float a, float b, int lane)
{
	const uint32_t  WM = (uint32_t)W - 1u;
	const MotionOwn m  = motion_own (U, a, b, lane);
	if (m.first) {
		/* both slots read before either is written (one LDS round trip): an owner's
		 * slot t+1 is read but left alone when another group owns it */
		const uint32_t i0 = m.t & WM, i1 = (m.t + 1) & WM;
		const float    v = ring[i0], w = ring[i1];
		ring[i0]         = motion_sum_t (m, v);
		if (m.own2)
			ring[i1] = motion_sum_t1 (m, w);
	}
}

/* ================================================================== k_tonegen */

/* A chunk without control deltas plays one program on every block: its entries' wheels,
 * wave lengths and bank offsets are loaded once per launch into the lanes (entry lane and
 * lane + 64), and each block only advances the wheel positions in registers -- the per-block
 * prologue's chain of dependent loads (entry -> wheel position -> length and offset) is gone.
 * The positions go back to the state after the launch (tg_cache_store). */
struct TgCache {
	bool     on;
	int      np;
	bool     anyEnv;
#if !TG_LCACHE
	uint32_t w[2], len[2], off[2], pos[2];
#endif
};

#if TG_LCACHE
/* The positions live in LDS (sm.cbase / cend / clen): held in the lanes, they were spilled
 * around the interpreter, and each block's reload from scratch waited (vmcnt) for the
 * previous block's output stores too. */
__device__ __forceinline__ void tg_cache_load (TgCache& c, const tbf_launch& P, TgLds& sm, const tbf_seg_ctl& G,
                                               const tbf_tpl_desc* T)
{
	const int             lane = threadIdx.x & (NL - 1);
	const tbf_prog_entry* prog = P.prog + G.prog_off + 1;
	c.np                       = (int)P.prog[G.prog_off].pad;
	c.on                       = c.np <= 2 * NL;
	int env                    = 0;
#pragma unroll
	for (int k = 0; k < 2; k++) {
		const int e = lane + k * NL;
		if (c.on && e < c.np) {
			const uint32_t w = prog[e].wheel, len = T->len[w], off = T->off[w];
			sm.cbase[e]      = off + sm.st.pos[w];
			sm.cend[e]       = off + len;
			sm.clen[e]       = len;
			env |= prog[e].env != 0;
		}
	}
	c.anyEnv = __any (env);
}

__device__ __forceinline__ void tg_cache_store (const TgCache& c, TgLds& sm, const tbf_launch& P, const tbf_seg_ctl& G,
                                                const tbf_tpl_desc* T)
{
	const int             lane = threadIdx.x & (NL - 1);
	const tbf_prog_entry* prog = P.prog + G.prog_off + 1;
	if (!c.on)
		return;
#pragma unroll
	for (int k = 0; k < 2; k++) {
		const int e = lane + k * NL;
		if (e < c.np) {
			const uint32_t w = prog[e].wheel;
			sm.st.pos[w]     = sm.cbase[e] - T->off[w];
		}
	}
}
#else
__device__ __forceinline__ void tg_cache_load (TgCache& c, const tbf_launch& P, const TgLds& sm, const tbf_seg_ctl& G,
                                               const tbf_tpl_desc* T)
{
	const int             lane = threadIdx.x & (NL - 1);
	const tbf_prog_entry* prog = P.prog + G.prog_off + 1;
	c.np                       = (int)P.prog[G.prog_off].pad;
	c.on                       = c.np <= 2 * NL;
	int env                    = 0;
#pragma unroll
	for (int k = 0; k < 2; k++) {
		const int e = lane + k * NL;
		c.w[k] = c.len[k] = c.off[k] = c.pos[k] = 0;
		if (c.on && e < c.np) {
			const uint32_t w = prog[e].wheel;
			c.w[k]           = w;
			c.len[k]         = T->len[w];
			c.off[k]         = T->off[w];
			c.pos[k]         = sm.st.pos[w];
			env |= prog[e].env != 0;
		}
	}
	c.anyEnv = __any (env);
}

__device__ __forceinline__ void tg_cache_store (const TgCache& c, TgLds& sm)
{
	const int lane = threadIdx.x & (NL - 1);
	if (!c.on)
		return;
#pragma unroll
	for (int k = 0; k < 2; k++)
		if (lane + k * NL < c.np)
			sm.st.pos[c.w[k]] = c.pos[k];
}
#endif

/* oscGenerateFragment core interpreter + vibratoProc + mixdown, src/tonegen.cpp:3607-3777 */
__device__ __forceinline__ void stage_tonegen (const tbf_launch& P, TgLds& sm, const tbf_seg_ctl& G, const tbf_tpl_desc* T,
                              float2* __restrict__ out, float* __restrict__ oL = nullptr, float* __restrict__ oR = nullptr,
                              float kc = 0.f, float pe = 0.f, TgCache* tc = nullptr)
{
	const int             lane = threadIdx.x & (NL - 1);
	tbf_tg_state&         st   = sm.st;
	/* the program slot: header (entry count) then the entries */
	const tbf_prog_entry* __restrict__ prog = P.prog + G.prog_off + 1;
	const int             np   = (int)P.prog[G.prog_off].pad;

	/* core interpreter.  Prologue, lane per entry: resolve the wheel's bank position and
	 * advance st.pos (each wheel appears once per program).  The device bank repeats each
	 * wave's first 128 samples after its end, so the reference's wrap split
	 * (src/tonegen.cpp:3376-3402) is plain indexing from base. */
	/* A delta chunk (P.ctlIdx) plays a program k_tgctl has just written, a new one on every
	 * block under dense events: its entries are read once, lane-parallel, into LDS here, for
	 * the main loop's broadcast reads (the main loop's scalar loads of them missed the
	 * scalar cache four entries at a time).  A chunk without deltas replays one program,
	 * whose entries stay in the scalar cache. */
	const bool lp      = (P.ctlIdx != nullptr || TG_LDS_ALL) && np <= TG_PCAP;
	bool       anyEnv;
	if (tc && tc->on) {
		/* the launch's program, entries held in the lanes (TgCache) */
#pragma unroll
		for (int k = 0; k < 2; k++) {
			const int e = lane + k * NL;
			if (e < np) {
#if TG_LCACHE
				const uint32_t b = sm.cbase[e], nb = b + TBF_BLK; /* off + pos, off + pos + TBF_BLK */
				sm.u.ent.base[e] = b;
				sm.cbase[e]      = (sm.cend[e] < nb) ? nb - sm.clen[e] : nb; /* (len < pos + TBF_BLK) as below */
#else
				const uint32_t pos = tc->pos[k], len = tc->len[k];
				sm.u.ent.base[e] = tc->off[k] + pos;
				tc->pos[k]       = (len < pos + TBF_BLK) ? pos + TBF_BLK - len : pos + TBF_BLK;
#endif
				if (lp) { /* the gains through LDS too (the scanner's rows overwrite them each block) */
					const uint4 a = ((const uint4*)(prog + e))[0], b = ((const uint4*)(prog + e))[1];
					sm.u.ent.g[e] = make_float4 (__uint_as_float (a.y), __uint_as_float (a.z), __uint_as_float (a.w), __uint_as_float (b.x));
					sm.u.ent.h[e] = make_float2 (__uint_as_float (b.y), __uint_as_float (b.z));
					sm.u.ent.er[e] = a.x >> 16;
				}
			}
		}
		anyEnv = tc->anyEnv;
	} else {
		int envHere = 0;
		for (int e = lane; e < np; e += NL) {
			const uint32_t w   = prog[e].wheel;
			const uint32_t pos = st.pos[w];
			const uint32_t len = T->len[w];
			sm.u.ent.base[e]   = T->off[w] + pos;
			st.pos[w]          = (len < pos + TBF_BLK) ? pos + TBF_BLK - len : pos + TBF_BLK;
			envHere |= prog[e].env != 0;
			if (lp) {
				const uint4 a = ((const uint4*)(prog + e))[0], b = ((const uint4*)(prog + e))[1];
				sm.u.ent.g[e] = make_float4 (__uint_as_float (a.y), __uint_as_float (a.z), __uint_as_float (a.w), __uint_as_float (b.x));
				sm.u.ent.h[e] = make_float2 (__uint_as_float (b.y), __uint_as_float (b.z));
				sm.u.ent.er[e] = a.x >> 16; /* env | row << 8 */
			}
		}
		anyEnv = __any (envHere);
	}
	wave_sync ();
	/* main loop in program order (the adds keep the reference's order); a lane holds
	 * samples lane and lane + 64 as a pair, so each bus costs one packed multiply and one
	 * packed add (v_pk_mul_f32 / v_pk_add_f32: two IEEE float ops, no contraction).  The
	 * loops have no data-dependent branch, so the unrolled entries' loads are in flight
	 * together.  The sums start at -0.f: -0 + a == a for every a, so the first entry's add
	 * equals the reference's copy (CR_CPY). */
	f2v  sw = {-0.f, -0.f}, vb = {-0.f, -0.f}, pc = {-0.f, -0.f};
	auto loops = [&] (auto LP) {
		constexpr bool L = decltype (LP)::value;
		/* entry e's gains {sg, pg, vg, nsg, npg, nvg} and env | row << 8 */
		auto ent = [&] (int e, float (&g)[6], uint32_t& er) {
			if constexpr (L) {
				/* broadcast reads made wave-uniform (readfirstlane): the envelope branch below
				 * is then a scalar branch, so a steady entry skips the envelope arithmetic */
				const float4 a = sm.u.ent.g[e];
				const float2 b = sm.u.ent.h[e];
#if TG_GRFL
				auto rfl = [] (float v) { return __int_as_float (__builtin_amdgcn_readfirstlane (__float_as_int (v))); };
				g[0] = rfl (a.x); g[1] = rfl (a.y); g[2] = rfl (a.z); g[3] = rfl (a.w); g[4] = rfl (b.x); g[5] = rfl (b.y);
#else
				/* the gains stay in the lanes (every lane read the same LDS word): only the
				 * envelope word needs to be scalar, for the branch */
				g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w; g[4] = b.x; g[5] = b.y;
#endif
				er = (uint32_t)__builtin_amdgcn_readfirstlane ((int)sm.u.ent.er[e]);
			} else {
				const tbf_prog_entry& E = prog[e];
				g[0] = E.sg; g[1] = E.pg; g[2] = E.vg; g[3] = E.nsg; g[4] = E.npg; g[5] = E.nvg;
				er = (uint32_t)E.env | ((uint32_t)E.row << 8);
			}
		};
		/* groups of four entries: every load of a group (bank samples, envelope rows) is
		 * issued before its arithmetic, and the next group's loads before this group's
		 * arithmetic (two register sets, A and B, alternating: a copy from one set to the
		 * other at the loop's back edge would wait for the loads); the remainder one entry
		 * at a time */
		constexpr int K = 4;
		struct Grp {
			f2v xs[K], evs[K];
		};
		auto load = [&] (Grp& G, int e, auto EC) {
			constexpr bool EN = decltype (EC)::value; /* the block has envelope entries */
#pragma unroll
			for (int k = 0; k < K; k++) {
#if TG_ABL == 1 /* timing experiment only (wrong output): every entry reads the bank's first row */
				const float* __restrict__ bp = P.bank + (sm.u.ent.base[e + k] & 63u);
#else
				const float* __restrict__ bp = P.bank + sm.u.ent.base[e + k];
#endif
				G.xs[k]                      = f2v {bp[lane], bp[lane + NL]};
				if constexpr (EN) { /* (a steady entry loads row 0 of the attack table: an L1 hit) */
					float    gg[6];
					uint32_t er;
					ent (e + k, gg, er);
					const uint32_t env = er & 0xffu, row = (er >> 8) & 7u;
					const float*   ep  = (env == 2 ? T->releaseEnv[row] : T->attackEnv[row]);
					G.evs[k]           = f2v {ep[lane], ep[lane + NL]};
				}
			}
		};
		auto compute = [&] (const Grp& G, int e, auto EC) {
			constexpr bool EN = decltype (EC)::value;
#pragma unroll
			for (int k = 0; k < K; k++) {
				float    g[6];
				uint32_t er;
				ent (e + k, g, er);
				if (EN && (er & 0xffu)) {
					/* envelope entry x * (g + e (ng - g)) (src/tonegen.cpp:3640-3662) */
					sw = sw + G.xs[k] * (g[0] + (G.evs[k] * (g[3] - g[0])));
					vb = vb + G.xs[k] * (g[2] + (G.evs[k] * (g[5] - g[2])));
					pc = pc + G.xs[k] * (g[1] + (G.evs[k] * (g[4] - g[1])));
				} else { /* x * g (3667-3685) */
					sw = sw + G.xs[k] * g[0];
					vb = vb + G.xs[k] * g[2];
					pc = pc + G.xs[k] * g[1];
				}
			}
		};
		/* one entry: the remainder */
		auto single = [&] (int e, auto EC) {
			constexpr bool EN = decltype (EC)::value;
			float          g[6];
			uint32_t       er;
			ent (e, g, er);
			const float* __restrict__ bp = P.bank + sm.u.ent.base[e];
			const f2v x                  = f2v {bp[lane], bp[lane + NL]};
			if (EN && (er & 0xffu)) {
				const uint32_t env = er & 0xffu, row = (er >> 8) & 7u;
				const float*   ep  = (env == 2 ? T->releaseEnv[row] : T->attackEnv[row]);
				const f2v      ev  = f2v {ep[lane], ep[lane + NL]};
				sw                 = sw + x * (g[0] + (ev * (g[3] - g[0])));
				vb                 = vb + x * (g[2] + (ev * (g[5] - g[2])));
				pc                 = pc + x * (g[1] + (ev * (g[4] - g[1])));
			} else {
				sw = sw + x * g[0];
				vb = vb + x * g[2];
				pc = pc + x * g[1];
			}
		};
		auto run = [&] (auto EC) {
			const int nG = np / K;
			Grp       A, B;
			int       gi = 0;
			if (nG > 0)
				load (A, 0, EC);
			for (; gi + 2 <= nG; gi += 2) {
				load (B, K * (gi + 1), EC);
				compute (A, K * gi, EC);
				if (gi + 2 < nG)
					load (A, K * (gi + 2), EC);
				compute (B, K * (gi + 1), EC);
			}
			if (gi < nG)
				compute (A, K * gi, EC);
			for (int e = K * nG; e < np; e++)
				single (e, EC);
		};
		if (anyEnv)
			run (BoolC<true> {});
		else
			run (BoolC<false> {});
	};
	if (lp)
		loops (BoolC<true> {});
	else
		loops (BoolC<false> {});
	if (np == 0) /* no program: the buses stay cleared (+0) */
		sw = vb = pc = f2v{0.f, 0.f};
	wave_sync (); /* the entry table is overwritten below */
	sm.swl[lane] = sw.x; sm.swl[lane + NL] = sw.y;
	sm.vin[lane] = vb.x; sm.vin[lane + NL] = vb.y;
	sm.prc[lane] = pc.x; sm.prc[lane + NL] = pc.y;
	wave_sync ();

	const uint32_t routing = G.routing;
	/* vibrato scanner, src/vibrato.cpp:365-411 */
#if TG_ABL == 2 /* timing experiment only (wrong output): no scanner */
	if (false) {
#else
	if (routing & 0x03) {
#endif
		const uint32_t* otab  = P.vibTab + 2048u * G.vibTable;
		const uint32_t  out0  = st.outPos;
		const uint32_t  stat0 = st.stator;
		const float     fnorm = (float)(1.0 / 65536.0);
		for (int k = 0; k < 2; k++) {
			const int      n  = lane + k * NL;
			const uint32_t op = (out0 + n) & 0x3FFu;
			const uint32_t sn = (stat0 + (uint32_t)n * P.statorInc) & 0x07ffffffu;
			const uint32_t j  = ((op << 16) + otab[sn >> 16]) & 0x03FFFFFFu;
			const int      h  = (int)(j >> 16);
			const float    f  = fnorm * ((float)(j & 0xFFFF));
			const float    x  = sm.vin[n];
			const float    g  = f * x;
			sm.u.v.va[n] = x - g;
			sm.u.v.vg[n] = g;
			sm.u.v.vh[n] = n + (int)(((uint32_t)h - op) & 0x3FFu); /* slot offset from out0 */
		}
		wave_sync ();
		/* The scatter as two passes of ordered adds (motion_add, the whirl rings' owner
		 * scheme): sample m adds x - g into slot out0 + vh[m] and g into the slot after, in
		 * sample order; for non-decreasing slots with groups of <= 2 equal slots in a pass,
		 * the first lane of each group owns its slot (and the next when no group sits
		 * there) and takes its neighbours' terms by DPP, and the second pass (samples
		 * 64..127) reads what the first wrote.  Then every output slot is read and cleared:
		 * all writes land >= 1 slot ahead of the writing sample's own output slot, so an
		 * output read after all of them sees exactly the earlier samples' (src/vibrato.cpp:
		 * 380-409).  Preconditions (wave votes): 1 <= vh[m] - m <= 31 and the slots
		 * non-decreasing over the block, no three equal in a row; lane 0 replays serially
		 * otherwise.  (The ordered gather before this looped over each slot's candidate
		 * samples: 30 % of the kernel's cycles, tools/phase_prof.py.) */
		const int U0 = sm.u.v.vh[lane], U1 = sm.u.v.vh[lane + NL];
		const float a0 = sm.u.v.va[lane], b0 = sm.u.v.vg[lane], a1 = sm.u.v.va[lane + NL], b1 = sm.u.v.vg[lane + NL];
		int bad = (U0 - lane < 1 || U0 - lane > 31 || U1 - (lane + NL) < 1 || U1 - (lane + NL) > 31) ? 1 : 0;
		{
			const int      P0 = lane_shr1 (U0), P1 = lane_shr1 (U1), L63 = rl (U0, NL - 1);
			const int      Pr1 = lane == 0 ? L63 : P1; /* sample lane + 63 */
			const uint64_t e0  = __ballot (lane > 0 && U0 == P0), e1 = __ballot (U1 == Pr1 && lane > 0);
			bad = bad || (lane > 0 && U0 < P0) || U1 < Pr1;
			/* three equal in a row inside a pass: two consecutive eq bits */
			bad = __any (bad) || (e0 & (e0 >> 1)) != 0 || (e1 & (e1 >> 1)) != 0 || (P.dbg & TBF_DEBUG_FORCE_SERIAL);
		}
		if (!bad) {
			motion_add<TBF_VRING> (st.vring, (int)out0 + U0, a0, b0, lane);
			wave_sync ();
			motion_add<TBF_VRING> (st.vring, (int)out0 + U1, a1, b1, lane);
			wave_sync ();
			for (int k = 0; k < 2; k++) {
				const int      wo   = lane + k * NL;
				const uint32_t slot = (out0 + wo) & (TBF_VRING - 1);
				const float    v    = st.vring[slot];
				const float    x    = sm.vin[wo];
				sm.u.v.vout[wo]     = G.vibMixed ? (x + v) * (float)0.7071067811865475 : v;
				st.vring[slot]      = 0.f;
			}
		} else {
			if (lane == 0) {
				atomicOr (P.errFlags, (uint32_t)TBF_PATH_VIB_SERIAL);
				for (int n = 0; n < TBF_BLK; n++) {
					const uint32_t op = (out0 + n) & 0x3FFu;
					const int      h  = (int)((op + (uint32_t)(sm.u.v.vh[n] - n)) & 0x3FFu);
					const int      k2 = (h + 1) & 0x3FF;
					st.vring[h & (TBF_VRING - 1)] += sm.u.v.va[n];
					st.vring[k2 & (TBF_VRING - 1)] += sm.u.v.vg[n];
					const float x = sm.vin[n];
					const float v = st.vring[op & (TBF_VRING - 1)];
					sm.u.v.vout[n] = G.vibMixed ? (x + v) * (float)0.7071067811865475 : v;
					st.vring[op & (TBF_VRING - 1)] = 0.f;
				}
			}
		}
		wave_sync ();
		if (lane == 0) {
			st.outPos = (out0 + TBF_BLK) & 0x3FFu;
			st.stator = (stat0 + (uint32_t)TBF_BLK * P.statorInc) & 0x07ffffffu;
		}
	}

	/* the mixdown's per-sample terms (src/tonegen.cpp:3712-3777) without its two gain chases
	 * (keyCompLevel += delta, percEnvGain *= decay), which k_mixpre runs with one chain per
	 * lane: s = the swell bus, plus the scanner output when the vibrato is routed in; p =
	 * HIPASS_PERCUSSION's first difference of the percussion bus (3719-3731) */
	for (int k = 0; k < 2; k++) {
		const int   n = lane + k * NL;
		const float x = sm.swl[n];
		const float s = (routing & 0x03) ? (x + sm.u.v.vout[n]) : x;
		const float p = (routing & 0x0C) ? ((n == 0 ? st.pz : sm.prc[n - 1]) - sm.prc[n]) : 0.f;
		if (oL) { /* the products with fixed-point gain chases (k_tonegen, tonegen only) */
			const float y = (routing & 0x0C) ? (G.outputGain * kc * (s + (p * pe))) : (G.swellPedalGain * kc * s);
			oL[n] = y;
			oR[n] = y;
		} else if (out)
			out[n] = make_float2 (s, p);
	}
	wave_sync (); /* every lane has read st.pz */
	if (lane == 0 && (routing & 0x0C))
		st.pz = sm.prc[TBF_BLK - 1];
	wave_sync ();
}

/* whether the mixdown's two gain chases (k_mixpre's v = v m + a) sit at a fixed point under
 * control G: then they keep v, bit for bit, for every block with that control */
__device__ __forceinline__ bool mix_fixed (const tbf_seg_ctl& G, const tbf_mo_state& M)
{
	const float kc = M.keyCompLevel, pe = M.percEnvGain;
	const bool  perc = (G.routing & 0x0C) != 0;
	const float kc1  = (kc * 1.f) + ((G.keyCompTarget - kc) / (float)TBF_BLK);
	const float pe1  = (pe * (perc ? G.percEnvGainDecay : 1.f)) + 0.f;
	return __float_as_uint (kc1) == __float_as_uint (kc) && __float_as_uint (pe1) == __float_as_uint (pe) &&
	       !(G.resetPercAtEnd && __float_as_uint (G.percEnvGainReset) != __float_as_uint (pe));
}

/* One workgroup per instance, one wave per block range.  A chunk whose blocks all play
 * the instance's current program (no control delta: ctlIdx == NULL) may split its blocks
 * into P.tgSplit ranges, one wave each, for more waves in flight.  A range after the first
 * starts one block early from the chunk-start state advanced in closed form: wheel
 * positions (pos + 128 b) mod len for the program's wheels (a block advances them by 128,
 * mod len >= 384; pos = len and pos = 0 read the same samples, the bank repeating each
 * wave's first 128), the scanner's stator and output position; then the warm-up block,
 * whose output is dropped, rebuilds what a block carries into the next: the scanner
 * ring's next 31 slots hold only the previous block's contributions (every slot is
 * cleared when read, and a block's scatter reaches at most 31 slots past its end), and pz
 * is that block's last percussion sample.  The ranges of an instance share a workgroup, so
 * every wave has read the chunk-start state (the barrier below) before the last range
 * writes the state back; separate workgroups could start in any order. */
__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL * TG_SPLIT_MAX), amdgpu_waves_per_eu (TG_WAVES)))
k_tonegen (const tbf_launch P, const tbf_seg_ctl* __restrict__ ctl, const tbf_tpl_desc* __restrict__ tpls,
           const tbf_inst_const* __restrict__ cst)
{
	extern __shared__ TgLds smv[]; /* one per wave */
	const uint32_t ns   = blockDim.x / NL;
	const uint32_t part = __builtin_amdgcn_readfirstlane (threadIdx.x / NL);
	const int      lane = threadIdx.x & (NL - 1);
	const uint32_t inst = blockIdx.x + P.instBase;
	if (inst >= P.nInst)
		return;
	TgLds&              sm = smv[part];
	const tbf_tpl_desc* T  = tpls + cst[inst].tpl;
	tbf_tg_state*       S  = &P.st[inst].tg;
	float2*             o  = (float2*)P.mid0 + (size_t)inst * P.midStride;
	const uint32_t      b0 = (P.nBlocks * part) / ns, b1 = (P.nBlocks * (part + 1)) / ns;
	/* tonegen only, no control delta in the chunk (every block has the instance's current
	 * control) and the gain chases at a fixed point: the products are computed here and
	 * written as the output, and k_mixpre skips the instance (mixFixed).  The chain runs
	 * its stages in order, so the preamp state read here is the previous chunk's final one. */
	bool        fixed = false;
	const float kcF = P.st[inst].mo.keyCompLevel, peF = P.st[inst].mo.percEnvGain;
	if (P.chain == TBF_CHAIN_TONEGEN) {
		fixed = !P.ctlIdx && mix_fixed (ctl_of (P, ctl, 0, inst), P.st[inst].mo);
		if (threadIdx.x == 0)
			P.mixFixed[inst] = fixed ? 1 : 0;
	}
	{
		const uint32_t* src = (const uint32_t*)S;
		uint32_t*       dst = (uint32_t*)&sm.st;
		for (uint32_t i = lane; i < sizeof (tbf_tg_state) / 4; i += NL)
			dst[i] = src[i];
	}
	__syncthreads (); /* every range has read the chunk-start state */
	if (part > 0) {
		const tbf_seg_ctl&    G    = ctl_of (P, ctl, 0, inst);
		const tbf_prog_entry* prog = P.prog + G.prog_off + 1;
		const int             np   = (int)P.prog[G.prog_off].pad;
		const uint32_t        adv  = (uint32_t)TBF_BLK * (b0 - 1); /* samples before the warm-up block */
		for (int e = lane; e < np; e += NL) {
			const uint32_t w = prog[e].wheel;
			sm.st.pos[w]     = (sm.st.pos[w] + adv) % T->len[w];
		}
		for (int i = lane; i < TBF_VRING; i += NL)
			sm.st.vring[i] = 0.f;
		if (lane == 0) {
			sm.st.outPos = (sm.st.outPos + adv) & 0x3FFu;
			sm.st.stator = (sm.st.stator + adv * P.statorInc) & 0x07ffffffu;
		}
		wave_sync ();
	}
	/* a chunk without deltas plays the instance's current program on every block */
	TgCache tc;
	tc.on = false;
	if (!P.ctlIdx && TG_CACHE)
		tg_cache_load (tc, P, sm, ctl_of (P, ctl, 0, inst), T);
	if (part > 0)
		stage_tonegen (P, sm, ctl_of (P, ctl, 0, inst), T, nullptr, nullptr, nullptr, 0.f, 0.f, &tc);
	for (uint32_t blk = b0; blk < b1; blk++) {
		const size_t so = P.outOffset + (size_t)blk * TBF_BLK;
		if (fixed)
			stage_tonegen (P, sm, ctl_of (P, ctl, blk, inst), T, nullptr, P.outL + (size_t)inst * P.outStride + so,
			               P.outR + (size_t)inst * P.outStride + so, kcF, peF, &tc);
		else
			stage_tonegen (P, sm, ctl_of (P, ctl, blk, inst), T, o + (size_t)blk * TBF_BLK, nullptr, nullptr, 0.f, 0.f, &tc);
	}
	if (part == ns - 1) {
#if TG_LCACHE
		tg_cache_store (tc, sm, P, ctl_of (P, ctl, 0, inst), T);
#else
		tg_cache_store (tc, sm);
#endif
		wave_sync ();
		const uint32_t* src = (const uint32_t*)&sm.st;
		uint32_t*       dst = (uint32_t*)S;
		for (uint32_t i = lane; i < sizeof (tbf_tg_state) / 4; i += NL)
			dst[i] = src[i];
	}
}

/* ================================================================== k_mixpre
 * The mixdown's two gain chases (src/tonegen.cpp:3734-3777: keyCompLevel += delta and
 * percEnvGain *= decay, once per sample) and the preamp (preamp / airwindows_density,
 * src/overdrive.cpp:60-170, FP64) as a chain block: MP_CB instances per workgroup, in tiles of
 * MP_T samples staged in LDS:
 *   wave 0     the serial recurrences, one chain per lane: lane 2j runs instance j's
 *              keyCompLevel chase and the preamp high-pass's iirSampleA chain, lane 2j + 1 its
 *              percEnvGain chase and iirSampleB (fpFlip hands the two high-pass chains
 *              alternate samples, so each covers half a tile).  One FP64 instruction stream
 *              advances 64 chains; a wave per instance served 2.
 *   wave 1     the preamp's xorshift dither stream (fpd), lane j = instance j
 *   waves 2..  lane-parallel work, one instance per task and wave (MP_WIDE: 64-sample tiles;
 *              else two instances per task, a half-wave each, 32-sample tiles): the gain
 *              products, the denormal guard, the waveshaper, blend and dither, the stores
 * Iteration it: the chases of tile it, the products of tile it - 1, the high-pass of tile
 * it - 2, the waveshaper of tile it - 3; one barrier per iteration.  Every chain runs the
 * reference's operations in its order.  Tonegen-only chains (configs[1]) stop after the
 * products, which are then the output. */
#ifndef MP_CB
/* instances per workgroup: 28 with 14 helper waves (16 waves, 147 workgroups at 4096
 * instances) hide more of the waveshaper's FP64 latency than 32 with 8 (10 waves, 128):
 * alone 6.72 -> 5.23 ms per 512 blocks, the step 115.5 -> 113.7 ms (profiles/r06/s19) */
#define MP_CB 28
#endif
#ifndef MP_PROF
#define MP_PROF 0 /* profiling variant: s_memtime per role and section (tools/mp_prof.py) */
#endif
#ifndef MP_ABL
#define MP_ABL 0 /* timing experiments (wrong output): 1 no waveshaper, 2 no serial chains, 3 no dither */
#endif
#ifndef MP_SIN_PAIRS
#define MP_SIN_PAIRS 0 /* the density sines in pairs (tbf_sin2) instead of one vote for all tasks */
#endif
#ifndef MP_PRIO
#define MP_PRIO 2 /* the helpers raise their priority at the waveshaper's start and drop it after density
                   * step MP_PRIO - 1, so the two helpers of a SIMD progress together instead of in age order */
#endif
#ifndef MP_WIDE
#define MP_WIDE 1 /* tiles of 64 samples, a helper task = one instance (0: 32, an instance pair) */
#endif
#if MP_WIDE
/* a tile is a whole wave of samples: each iteration gives a CU 2048 samples of waveshaper
 * work (four density sines each, chains of dependent FP64 operations), eight chains per
 * SIMD instead of four, which the 32-sample tiles left latency-bound (tools/mp_prof.py) */
#define MP_T 64
#define MP_NTK (MP_CB / MP_H)     /* helper tasks (instances) per tile */
#define MP_XR 3                   /* preamp-input rows by tile mod 3 (tiles it-1 .. it-3 alive) */
#define MP_CR 4                   /* control slots by block mod 4 (two tiles per block) */
#else
#define MP_T 32                   /* samples per tile: one per lane of a half-wave */
#define MP_NTK (MP_CB / 2 / MP_H) /* helper tasks (instance pairs) per tile */
#define MP_XR 4
#define MP_CR 2
#endif
#define MP_S (MP_T + 1)           /* row stride of the per-sample rows (odd: conflict-free columns) */
#define MP_HS (MP_T / 2 + 1)      /* row stride of the high-pass rows (a chain's MP_T / 2 samples) */
#ifndef MP_H
#define MP_H 14                   /* helper waves */
#endif
#define MP_THREADS (NL * (2 + MP_H))
#define MP_TPB (TBF_BLK / MP_T)   /* tiles per block */
static_assert (2 * MP_CB <= NL && (MP_WIDE ? MP_T == NL && MP_CB % MP_H == 0 : 2 * MP_T == NL && MP_CB % (2 * MP_H) == 0),
               "k_mixpre geometry");
#define MP_ROWS (2 * MP_CB + (2 * MP_CB < NL)) /* chain rows, + one that idle chain lanes write */

/* one block's control of an instance as k_mixpre uses it, staged in LDS by the dither wave
 * a block ahead (so no global load sits on an iteration's path) */
struct MpCtl {
	float    gain;    /* percussion routed ? outputGain : swellPedalGain */
	float    keyCompTarget, decay, reset;
	uint32_t flags;   /* MPF_* */
	int32_t  iter;    /* odIter */
	double   iir, out, output, wet, dry;
};
#define MPF_PERC 1u  /* percussion routed (routing & 0x0C) */
#define MPF_CLEAN 2u /* preamp off */
#define MPF_DPOS 4u  /* density > 0 */
#define MPF_RST 8u   /* percEnvGain resets at the block end */

__device__ __forceinline__ MpCtl mp_ctl (const tbf_seg_ctl& G)
{
	MpCtl c;
	const bool perc = (G.routing & 0x0C) != 0;
	c.gain          = perc ? G.outputGain : G.swellPedalGain;
	c.keyCompTarget = G.keyCompTarget;
	c.decay         = G.percEnvGainDecay;
	c.reset         = G.percEnvGainReset;
	c.flags = (perc ? MPF_PERC : 0u) | (G.odClean ? MPF_CLEAN : 0u) | (G.odDensityPos ? MPF_DPOS : 0u) | (G.resetPercAtEnd ? MPF_RST : 0u);
	c.iter   = G.odIter;
	c.iir    = G.odIir;
	c.out    = G.odOut;
	c.output = G.odOutput;
	c.wet    = G.odWet;
	c.dry    = G.odDry;
	return c;
}

struct MixPreLds {
	float    g[2][MP_ROWS][MP_S];    /* chase values before each sample, by tile parity: row 2j
	                                  * keyCompLevel, 2j + 1 percEnvGain of instance j */
	double   x[MP_XR][MP_ROWS][MP_HS]; /* preamp input (guarded), by tile mod MP_XR: row 2j + q holds the
	                                    * samples of instance j's high-pass chain q */
	double   h[2][MP_ROWS][MP_HS];   /* high-pass output, same rows, by tile parity */
	uint32_t f[4][MP_CB][MP_S];      /* fpd before each sample (entry MP_T: after the tile), by tile mod 4 */
	MpCtl    c[MP_CR][MP_CB];        /* the control of block b in slot b mod MP_CR */
};

/* the preamp after its high-pass (src/overdrive.cpp:117-168): density waveshaper, output
 * level, dry/wet blend, dither (f1 = the stream after this sample's step) */
__device__ __forceinline__ float preamp_shape (double x, double dry, const MpCtl& C, uint32_t f1)
{
	double br;
	for (int c = 0; c < C.iter; c++) {
		br = fabs (x) * 1.57079633;
		if (br > 1.57079633)
			br = 1.57079633;
		br = tbf_sin (br);
		x  = (x > 0.0) ? br : -br;
	}
	br = fabs (x) * 1.57079633;
	if (br > 1.57079633)
		br = 1.57079633;
	br = (C.flags & MPF_DPOS) ? tbf_sin (br) : 1 - cos (br);
	if (x > 0)
		x = (x * (1 - C.out)) + (br * C.out);
	else
		x = (x * (1 - C.out)) - (br * C.out);
	if (C.output < 1.0)
		x *= C.output;
	if (C.wet < 1.0)
		x = (dry * C.dry) + (x * C.wet);
	return (float)dither_add (x, f1);
}

/* preamp_shape of a helper's NT tasks at once: the density loops run side by side (to the
 * largest iteration count of the wave; a task past its own count keeps its value) with the
 * sines of a step under one wave vote (tbf_sin_n), so the tasks' FP64 dependency chains
 * interleave: a lone density loop is four sines in a row, ~1.2 k cycles each at two waves
 * per SIMD, latency-bound.  The same operations per task as preamp_shape. */
template <int NT>
__device__ __forceinline__ void preamp_shape_n (const double (&x0)[NT], const double (&dry)[NT], const MpCtl* const (&C)[NT],
                                                const uint32_t (&f1)[NT], float (&y)[NT])
{
	double x[NT];
	int    itm = 0;
	bool   dpos = true;
#pragma unroll
	for (int t = 0; t < NT; t++) {
		x[t] = x0[t];
		itm  = max (itm, C[t]->iter);
		dpos = dpos && (C[t]->flags & MPF_DPOS);
	}
	const int itw = wave_max (itm);
#if MP_PRIO
	__builtin_amdgcn_s_setprio (1);
#endif
	for (int c = 0; c < itw; c++) {
#if MP_PRIO
		if (c == MP_PRIO)
			__builtin_amdgcn_s_setprio (0);
#endif
		double br[NT];
#pragma unroll
		for (int t = 0; t < NT; t++) {
			br[t] = fabs (x[t]) * 1.57079633;
			if (br[t] > 1.57079633)
				br[t] = 1.57079633;
		}
#if MP_SIN_PAIRS
#pragma unroll
		for (int t = 0; t < NT; t += 2)
			tbf_sin2 (br[t], br[t + 1], br[t], br[t + 1]);
#else
		tbf_sin_n<NT> (br);
#endif
#pragma unroll
		for (int t = 0; t < NT; t++)
			if (c < C[t]->iter)
				x[t] = (x[t] > 0.0) ? br[t] : -br[t];
	}
#if MP_PRIO
	__builtin_amdgcn_s_setprio (0);
#endif
	double br[NT];
#pragma unroll
	for (int t = 0; t < NT; t++) {
		br[t] = fabs (x[t]) * 1.57079633;
		if (br[t] > 1.57079633)
			br[t] = 1.57079633;
	}
	if (__all (dpos)) {
		tbf_sin_n<NT> (br);
	} else {
#pragma unroll
		for (int t = 0; t < NT; t++)
			br[t] = (C[t]->flags & MPF_DPOS) ? tbf_sin (br[t]) : 1 - cos (br[t]);
	}
#pragma unroll
	for (int t = 0; t < NT; t++) {
		const MpCtl& K = *C[t];
		double       v = x[t];
		if (v > 0)
			v = (v * (1 - K.out)) + (br[t] * K.out);
		else
			v = (v * (1 - K.out)) - (br[t] * K.out);
		if (K.output < 1.0)
			v *= K.output;
		if (K.wet < 1.0)
			v = (dry[t] * K.dry) + (v * K.wet);
		y[t] = (float)dither_add (v, f1[t]);
	}
}

__global__ void __launch_bounds__ (MP_THREADS)
k_mixpre (const tbf_launch P, const tbf_seg_ctl* __restrict__ ctl)
{
	__shared__ MixPreLds sm;
	const int      w = __builtin_amdgcn_readfirstlane (threadIdx.x >> 6), lane = threadIdx.x & (NL - 1);
	const uint32_t inst0 = P.instBase + blockIdx.x * MP_CB;
	if (inst0 >= P.nInst)
		return;
	const int  nj  = (int)min ((uint32_t)MP_CB, P.nInst - inst0);
	const int  nT  = (int)P.nBlocks * MP_TPB;
	const int  nIt = nT + 3;
	const bool pre = P.chain != TBF_CHAIN_TONEGEN; /* tonegen only: no preamp */
	/* tonegen only: instances whose output k_tonegen wrote (fixed-point chases, mixFixed);
	 * a workgroup of only those has nothing to do (their state does not change) */
	if (!pre && __all (lane >= nj || P.mixFixed[inst0 + (lane < nj ? lane : 0)]))
		return;
	if (w == 0) {
		const int      cl = min (lane, MP_ROWS - 1); /* chain row (lanes past 2 MP_CB: the idle row) */
		const int      j = min (lane >> 1, MP_CB - 1), q = lane & 1;
		const bool     ok   = lane < 2 * MP_CB && j < nj;
		tbf_mo_state*  M    = &P.st[inst0 + (ok ? j : 0)].mo;
		float          v    = q ? M->percEnvGain : M->keyCompLevel;
		double         iir  = q ? M->iirB : M->iirA;
		/* chase step v = v m + a: keyCompLevel + delta is (v 1) + delta, percEnvGain * decay is
		 * (v decay) + 0 (or (v 1) + 0 without percussion), the same values (v >= +0) */
		float  m = 1.f, a = 0.f, rsv = 0.f;
		bool   rs = false, hp = false;
		double ia = 0.0;
		__syncthreads ();
#if MP_PROF
		unsigned long long sw0 = 0, sb0 = 0;
#endif
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
#if MP_PROF
			const unsigned long long _s0 = __builtin_amdgcn_s_memtime ();
#endif
			if (it < nT) {
				if (it % MP_TPB == 0) {
					const MpCtl& C = sm.c[(it / MP_TPB) % MP_CR][j];
					m   = q ? ((C.flags & MPF_PERC) ? C.decay : 1.f) : 1.f;
					a   = q ? 0.f : (C.keyCompTarget - v) / (float)TBF_BLK; /* keyCompDelta at the block start */
					rs  = q && (C.flags & MPF_RST);
					rsv = C.reset;
				}
				float* row = sm.g[it & 1][cl];
#if MP_ABL == 2 /* timing experiment only (wrong output): no serial chase or high-pass */
				if (true) {
#else
				if (__all ((v * m) + a == v)) { /* a fixed point on every lane (no percussion, the key
				                                  * compression settled): the whole tile is v */
#endif
#pragma unroll 8
					for (int k = 0; k < MP_T; k++)
						row[k] = v;
				} else {
					PRIO_UP ();
					for (int i0 = 0; i0 < MP_T; i0 += 8) {
						float o[8];
#pragma unroll
						for (int k = 0; k < 8; k++) {
							o[k] = v;
							v    = (v * m) + a;
						}
#pragma unroll
						for (int k = 0; k < 8; k++)
							row[i0 + k] = o[k];
					}
					PRIO_DOWN ();
				}
				if (it % MP_TPB == MP_TPB - 1 && rs)
					v = rsv;
			}
			const int th = it - 2; /* the high-pass (src/overdrive.cpp:104-115) of tile th */
			if (pre && th >= 0 && th < nT) {
				if (th % MP_TPB == 0) {
					const MpCtl& C = sm.c[(th / MP_TPB) % MP_CR][j];
					hp             = !(C.flags & MPF_CLEAN);
					ia             = C.iir;
				}
#if MP_ABL == 2
				if (false) {
#else
				if (hp) {
#endif
					const double* xr = sm.x[th % MP_XR][cl];
					double*       hr = sm.h[th & 1][cl];
					const double  om = 1.0 - ia;
					PRIO_UP ();
#pragma unroll
					for (int i0 = 0; i0 < MP_T / 2; i0 += 8) {
						double xv[8];
#pragma unroll
						for (int k = 0; k < 8; k++)
							xv[k] = xr[i0 + k];
#pragma unroll
						for (int k = 0; k < 8; k++) {
							iir        = (iir * om) + (xv[k] * ia);
							hr[i0 + k] = xv[k] - iir;
						}
					}
					PRIO_DOWN ();
				}
			}
#if MP_PROF
			const unsigned long long _s1 = __builtin_amdgcn_s_memtime ();
			sw0 += _s1 - _s0;
#endif
			__syncthreads ();
#if MP_PROF
			sb0 += __builtin_amdgcn_s_memtime () - _s1;
#endif
		}
#if MP_PROF
		if (blockIdx.x == 0 && lane == 0) {
			P.outL[P.outOffset + 8] = (float)(sw0 * 1e-3);
			P.outL[P.outOffset + 9] = (float)(sb0 * 1e-3);
			P.outL[P.outOffset + 10] = (float)((__builtin_amdgcn_s_getreg ((31 << 11) | 4) >> 4) & 3);
		}
#endif
		if (ok) {
			if (q) {
				M->percEnvGain = v;
				M->iirB        = iir;
			} else {
				M->keyCompLevel = v;
				M->iirA         = iir;
			}
		}
		return;
	}
	if (w == 1) {
		/* the control staging (block b into slot b mod MP_CR at iteration MP_TPB b - 1, from
		 * registers loaded a block earlier) and the dither stream: it advances once per sample of every
		 * block the preamp runs (src/overdrive.cpp:153-159), f[n] = the state before sample
		 * n's step */
		const bool     ok   = lane < nj;
		const uint32_t inst = inst0 + (ok ? lane : 0);
		tbf_mo_state*  M    = &P.st[inst].mo;
		uint32_t       fs   = M->odFpd;
		const int      nB   = (int)P.nBlocks;
		MpCtl          nxt;
		if (lane < MP_CB) {
			sm.c[0][lane] = mp_ctl (ctl_of (P, ctl, 0, inst));
			nxt           = mp_ctl (ctl_of (P, ctl, (uint32_t)min (1, nB - 1), inst));
		}
		bool adv = false;
		__syncthreads ();
#if MP_PROF
		unsigned long long dw0 = 0, db0 = 0;
#endif
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
#if MP_PROF
			const unsigned long long _d0 = __builtin_amdgcn_s_memtime ();
#endif
			if (lane < MP_CB) {
#if MP_ABL == 3 /* timing experiment only (wrong output): no dither stream */
				if (false) {
#else
				if (pre && it < nT) {
#endif
					if (it % MP_TPB == 0)
						adv =!(sm.c[(it / MP_TPB) % MP_CR][lane].flags & MPF_CLEAN);
					uint32_t* f = sm.f[it & 3][lane];
#pragma unroll 8
					for (int n = 0; n < MP_T; n++) {
						f[n] = fs;
						fs   = adv ? xs_step (fs) : fs;
					}
					f[MP_T] = fs;
				}
				const int b = (it + 1) / MP_TPB; /* the block starting at the next iteration */
				if ((it + 1) % MP_TPB == 0 && b < nB) {
					sm.c[b % MP_CR][lane] = nxt;
					nxt               = mp_ctl (ctl_of (P, ctl, (uint32_t)min (b + 1, nB - 1), inst));
				}
			}
#if MP_PROF
			const unsigned long long _d1 = __builtin_amdgcn_s_memtime ();
			dw0 += _d1 - _d0;
#endif
			__syncthreads ();
#if MP_PROF
			db0 += __builtin_amdgcn_s_memtime () - _d1;
#endif
		}
#if MP_PROF
		if (blockIdx.x == 0 && lane == 0) {
			P.outL[P.outOffset + 16] = (float)(dw0 * 1e-3);
			P.outL[P.outOffset + 17] = (float)(db0 * 1e-3);
			P.outL[P.outOffset + 18] = (float)((__builtin_amdgcn_s_getreg ((31 << 11) | 4) >> 4) & 3);
		}
#endif
		if (ok && pre && lane < MP_CB)
			M->odFpd = fs;
		return;
	}
	/* helpers: task t = instance h + MP_H t, lane n = sample n of the tile (MP_WIDE; else
	 * instances 2 (h + MP_H t) + {0, 1}, half-wave hj each, lane n of the half-wave = sample n).
	 * The (s, p) input is read two iterations before its use, into two register sets
	 * alternating by iteration parity (the loop is unrolled by two, so the sets stay static) */
	const int     h = w - 2, hj = MP_WIDE ? 0 : lane >> 5, n = lane & (MP_T - 1);
	const float2* in[MP_NTK];
	float*        o1[MP_NTK];
	float*        oL[MP_NTK];
	float*        oR[MP_NTK];
	int           jT[MP_NTK], rT[MP_NTK];
	bool          okT[MP_NTK];
	float2        pS[2][MP_NTK];
#pragma unroll
	for (int t = 0; t < MP_NTK; t++) {
		const int j       = MP_WIDE ? h + MP_H * t : 2 * (h + MP_H * t) + hj;
		okT[t]            = j < nj;
		jT[t]             = okT[t] ? j : nj - 1;
		const uint32_t is = inst0 + jT[t];
		in[t]             = (const float2*)P.mid0 + (size_t)is * P.midStride + n;
		o1[t]             = P.mid1 ? P.mid1 + (size_t)is * P.midStride + n : nullptr;
		oL[t]             = P.outL + (size_t)is * P.outStride + P.outOffset + n;
		oR[t]             = P.outR + (size_t)is * P.outStride + P.outOffset + n;
		/* sample n's high-pass chain: iirSampleA takes the samples of parity 0 when fpFlip
		 * is set at the block start (128 samples leave it unchanged), else parity 1 */
		const int q0      = P.st[is].mo.fpFlip ? 0 : 1;
		rT[t]             = 2 * jT[t] + ((n & 1) ^ q0);
		pS[0][t]          = in[t][0];
		pS[1][t]          = in[t][(size_t)min (1, nT - 1) * MP_T];
	}
	const bool tap = P.chain == TBF_CHAIN_TAP_PREAMP;
#if MP_PROF /* profiling variant only: s_memtime per helper section, written over instance 0's output */
	unsigned long long pf[3] = {0, 0, 0};
#define MP_T0() const unsigned long long _t0 = __builtin_amdgcn_s_memtime ()
#define MP_TS(i, a) { asm volatile ("" ::: "memory"); const unsigned long long _t = __builtin_amdgcn_s_memtime (); pf[i] += _t - (a); }
#else
#define MP_T0()
#define MP_TS(i, a)
#endif
	__syncthreads ();
	auto step = [&] (const int it, float2 (&qS)[MP_NTK]) {
		MP_T0 ();
		/* the waveshaper of tile it - 3: high-pass output, dry input, the dither state after
		 * the sample's step */
		const int kw = it - 3;
		if (pre && kw >= 0 && kw < nT) {
			const size_t so = (size_t)kw * MP_T;
#if MP_NTK > 1
			/* the tasks' waveshapers side by side (preamp_shape_n) */
			float ys[MP_NTK];
			{
				const MpCtl* Cp[MP_NTK];
				double       xd[MP_NTK], xh[MP_NTK];
				uint32_t     f1[MP_NTK];
				bool         cl[MP_NTK];
				bool         allCl = true;
#pragma unroll
				for (int t = 0; t < MP_NTK; t++) {
					Cp[t] = &sm.c[(kw / MP_TPB) % MP_CR][jT[t]];
					xd[t] = sm.x[kw % MP_XR][rT[t]][n >> 1];
					xh[t] = sm.h[kw & 1][rT[t]][n >> 1];
					f1[t] = sm.f[kw & 3][jT[t]][n + 1];
#if MP_ABL == 1 /* timing experiment only (wrong output): helpers without the waveshaper */
					cl[t] = true;
#else
					cl[t] = (Cp[t]->flags & MPF_CLEAN) != 0;
#endif
					allCl = allCl && cl[t];
				}
				if (!__all (allCl))
					preamp_shape_n<MP_NTK> (xh, xd, Cp, f1, ys);
#pragma unroll
				for (int t = 0; t < MP_NTK; t++)
					if (cl[t])
						ys[t] = (float)xd[t];
			}
#endif
#pragma unroll
			for (int t = 0; t < MP_NTK; t++) {
#if MP_NTK > 1
				const float y = ys[t];
#else
				const MpCtl& C  = sm.c[(kw / MP_TPB) % MP_CR][jT[t]];
				const double xd = sm.x[kw % MP_XR][rT[t]][n >> 1];
				float        y;
				if (C.flags & MPF_CLEAN)
					y = (float)xd;
				else
					y = preamp_shape (sm.h[kw & 1][rT[t]][n >> 1], xd, C, sm.f[kw & 3][jT[t]][n + 1]);
#endif
				if (okT[t]) {
					if (tap) {
						oL[t][so] = y;
						oR[t][so] = y;
					} else
						o1[t][so] = y;
				}
			}
		}
#if MP_PROF
		const unsigned long long _t1 = __builtin_amdgcn_s_memtime ();
		pf[0] += _t1 - _t0;
#endif
		/* the products of tile it - 1 (src/tonegen.cpp:3734-3777) and the preamp input:
		 * denormal guard with the dither state before the sample (src/overdrive.cpp:95-100) */
		const int kp = it - 1;
		if (kp >= 0 && kp < nT) {
#pragma unroll
			for (int t = 0; t < MP_NTK; t++) {
				const MpCtl& C  = sm.c[(kp / MP_TPB) % MP_CR][jT[t]];
				const float  kc = sm.g[kp & 1][2 * jT[t]][n];
				const float  pe = sm.g[kp & 1][2 * jT[t] + 1][n];
				const float2 sp = qS[t];
				const float  y  = (C.flags & MPF_PERC) ? (C.gain * kc * (sp.x + (sp.y * pe))) : (C.gain * kc * sp.x);
				if (!pre) {
					if (okT[t] && !P.mixFixed[inst0 + jT[t]]) {
						oL[t][(size_t)kp * MP_T] = y;
						oR[t][(size_t)kp * MP_T] = y;
					}
				} else {
					double x = (double)y;
					if (!(C.flags & MPF_CLEAN) && fabs (x) < 1.18e-23)
						x = sm.f[kp & 3][jT[t]][n] * 1.18e-17;
					sm.x[kp % MP_XR][rT[t]][n >> 1] = x;
				}
			}
		}
		/* the input of tile it + 1 into the set just consumed (clamped past the last tile: a
		 * harmless re-read, so the loads need no branch) */
		const int tl = min (it + 1, nT - 1);
#pragma unroll
		for (int t = 0; t < MP_NTK; t++)
			qS[t] = in[t][(size_t)tl * MP_T];
#if MP_PROF
		const unsigned long long _t2 = __builtin_amdgcn_s_memtime ();
		pf[1] += _t2 - _t1;
#endif
		__syncthreads ();
		MP_TS (2, _t2);
	};
#pragma unroll 1
	for (int it = 0; it < nIt; it += 2) {
		step (it, pS[1]);
		if (it + 1 < nIt)
			step (it + 1, pS[0]);
	}
#if MP_PROF
	if (blockIdx.x == 0 && h == 0 && lane == 0)
		for (int i = 0; i < 3; i++)
			P.outL[P.outOffset + i] = (float)(pf[i] * 1e-3);
	if (blockIdx.x == 0 && lane == 0) { /* every helper: its sections and its SIMD (HW_ID bits 5:4) */
		for (int i = 0; i < 3; i++)
			P.outL[P.outOffset + 32 + 4 * h + i] = (float)(pf[i] * 1e-3);
		P.outL[P.outOffset + 32 + 4 * h + 3] = (float)((__builtin_amdgcn_s_getreg ((31 << 11) | 4) >> 4) & 3);
	}
#endif
#undef MP_T0
#undef MP_TS
}

/* ================================================================== reverb */
/* b_reverb::reverb (src/reverb.cpp:274-794) as three kernels.  The MatrixVerb's serial
 * FP64 biquads sit outside its feedback network: biquadA filters the predelayed input
 * before the allpasses (src/reverb.cpp:361-375), biquadB -> asin -> biquadC filter the
 * tap mix on its way out (733-764).  So:
 *   k_rv_pre   predelay, biquadA, sin(x * wet)                 -> rvA [inst][c][n] (FP64)
 *   k_rv_core  allpasses, 16 modulated taps, Householder feedback, ring writes
 *                                                               -> tap mix rvB (FP64)
 *   k_rv_post  biquadB, clamp + asin, biquadC, dry mix, dither, (L+R)/sqrt2 -> mid2
 * k_rv_core has no serial recurrence besides the one-sample feedback shift, so it runs
 * lane-parallel (one workgroup per instance and channel); the two chain kernels run the
 * serial biquads with one chain per lane (chain blocks, below).  The xorshift dither
 * streams (fpdL/fpdR advance once per sample regardless of the signal,
 * src/reverb.cpp:775-783) are carried by both chain kernels. */

#define RV_WIN 72 /* tap window per line: 64 samples + max offset 2 * vibDepth (5.4) + 2 */

/* sin (v0 + (n+1) D) by angle addition from the start phase's S = sin v0, C = cos v0 and the
 * step rows sd = sin ((n+1) D), cm = 2 sin^2 ((n+1) D / 2): S + (C sd - S cm).  Not libm's
 * bits either way (FP64 sines only need a few ulps; the float outputs
 * are bit-identical); RVL_SINFMA forms C sd - S cm with one fma (3 FP64 instructions for 4:
 * k_rv_core_lds 9.48 -> 9.42 ms alone per 512 blocks, profiles/r06/s2).  Every network
 * kernel and path uses this one expression, so they agree however a render is split. */
#ifndef RVL_SINFMA
#define RVL_SINFMA 1
#endif
__device__ __forceinline__ double rv_sin_add (double S, double C, double sd, double cm)
{
#if RVL_SINFMA
	return S + __builtin_fma (C, sd, -(S * cm));
#else
	return S + ((C * sd) - (S * cm));
#endif
}

struct RvCoreLds {
	tbf_rv_chan st;
	double      win[8][RV_WIN];  /* tap windows of the sub-block: slots count+1 .. count+72 */
	double      sd[8][TBF_SUB];  /* sin ((n+1) D) of each line's closed-form step D ... */
	double      cm[8][TBF_SUB];  /* ... and 1 - cos ((n+1) D) = 2 sin^2 ((n+1) D / 2) */
	double      tabD[8];         /* the D the rows above hold (-1: none yet) */
};

/* FP64 stage buffers of one chunk: [inst][c][midStride] */
__device__ __forceinline__ double* rv_buf (double* base, const tbf_launch& P, uint32_t inst, int c)
{
	return base + ((size_t)inst * 2 + c) * P.midStride;
}

/* One channel of the feedback network, 64-sample sub-blocks: allpasses I..L (lines
 * 8-11), delay lines A..H (0-7) with vibrato-modulated two-tap reads, crossmod and
 * Householder feedback (src/reverb.cpp:381-730).  The two channels never mix inside the
 * network, so each is its own wave.  Every read of a channel's rings precedes every
 * write (all ring delays >= 560 > 64), and a sub-block's reads never touch the slots
 * the previous sub-block writes (they lie >= 65 slots ahead of them), so the kernel is
 * software-pipelined: the reads of sub-block k+1 are issued before the writes of
 * sub-block k, and their latency overlaps k+1's phase/sin work.  The tap reads of a
 * sub-block fall in slots count+1 .. count+64+7 of each line; those windows are
 * fetched into registers and the modulated taps come from cross-lane permutes.
 * Per-line scalars (counter, delay, ring offset) live one per lane in a VGPR and are
 * read out with v_readlane where a line needs them. */
struct RvFetch {
	double wlo[8]; /* line l, slot count+1+lane */
	double whi;    /* lane 8l+j: line l, slot count+65+j */
	double apOld[4]; /* allpass reads at count+1+lane */
	double a0;       /* network input (k_rv_pre output) */
};


__device__ __forceinline__ int wrap_slot (int s, int d) { return s - ((s > d) ? d + 1 : 0); }

/* issue every global read of a sub-block whose ring counters are lane-held in cntv.
 * full: the whole tap windows, slots count+1 .. count+72 (wlo: +1..+64, whi: +65..+72);
 * carry: only slots count+9 .. count+72 (into wlo), since slots +1..+8 are the previous
 * sub-block's +65..+72, still in its window and not written since (the sub-block in
 * between writes slots count-64 .. count-1) */
template <typename T> __device__ __forceinline__ T rv_ld (const T* p) { return *p; }
/* ring and tap-mix stores are nontemporal (2.94 -> 2.90 ms; nontemporal loads: 4.23 ms) */
template <typename T> __device__ __forceinline__ void rv_st (T* p, T v) { __builtin_nontemporal_store (v, p); }

__device__ __forceinline__ void rv_core_fetch (const double* slab, int cntv, int dlyv, int roffv,
                                               const double* __restrict__ a0s, size_t o, RvFetch& f, bool carry)
{
	const int lane = threadIdx.x;
#pragma unroll
	for (int l = 8; l < 12; l++) {
		const int d    = rl (dlyv, l);
		f.apOld[l - 8] = rv_ld (&slab[rl (roffv, l) + wrap_slot (rl (cntv, l) + lane + 1, d)]);
	}
	const int k0 = carry ? 9 : 1;
#pragma unroll
	for (int l = 0; l < 8; l++) {
		const int d = rl (dlyv, l);
		f.wlo[l]    = rv_ld (&slab[rl (roffv, l) + wrap_slot (rl (cntv, l) + k0 + lane, d)]);
	}
	if (!carry) {
		const int l = lane >> 3, j = lane & 7;
		const int d = __shfl (dlyv, l), cl = __shfl (cntv, l), ro = __shfl (roffv, l);
		f.whi       = rv_ld (&slab[ro + wrap_slot (cl + 1 + NL + j, d)]);
	}
	f.a0 = rv_ld (&a0s[o]);
}

/* Vibrato phases (src/reverb.cpp:479-496) and tap offsets (sin (v) + 1) * vibDepth.
 * When a line's phase run has the exact closed form v_n = v0 + (n+1) D (phase_run),
 * sin (v_n) = S + (C sd_n - S cm_n) with S, C = sincos (v0) and sd_n = sin ((n+1) D),
 * cm_n = 2 sin^2 ((n+1) D / 2); the rows sd, cm are cached per D, which changes only
 * when the phase crosses a binade.  The correction term is < 0.013 in magnitude, so the
 * result carries the accuracy of S; its tap offset is identical to the literal sin's in
 * ~87 % of samples, against ~47 % for a 1-ulp change of sin, which SURVEY.md §0.9
 * measured to change no float output.  Otherwise the literal recurrence and sin.
 *
 * rv_core_lines: the per-line (wave-uniform) part for all 8 lines at once, line l on
 * lane l (lanes 8..63 duplicate): closed-form check, step D, sincos of the start phase;
 * the end phase of every closed-form line is stored. */
__device__ __forceinline__ uint64_t rv_core_lines (RvCoreLds& sm, double vdl, double& v0x, double& Sx, double& Cx, double& Dx,
                                                    bool force)
{
	const int    lane = threadIdx.x;
	const int    li   = lane & 7;
	tbf_rv_chan& st   = sm.st;
	const double v0   = st.vib[li];
	double       D = 0.0, cD = st.phD[li], cLo = st.phLo[li], cHi = st.phHi[li];
	const bool   ok = phase_run_cached (v0, vdl, TBF_SUB, D, cD, cLo, cHi) && !force;
	sincos (v0, &Sx, &Cx);
	v0x = v0;
	Dx  = D;
	__syncthreads (); /* every lane has read st */
	if (lane < 8) {
		st.phD[li]  = cD;
		st.phLo[li] = cLo;
		st.phHi[li] = cHi;
		if (ok)
			st.vib[li] = v0 + (double)TBF_SUB * D; /* exact, = lane 63's v_n */
	}
	return __ballot (ok) & 0xff;
}

/* the lane's tap offset on line l */
__device__ __forceinline__ double rv_core_tap (RvCoreLds& sm, const tbf_inst_const& K, int l, uint64_t okm, double v0x,
                                               double Sx, double Cx, double Dx)
{
	const int n = threadIdx.x;
	double    s;
	if ((okm >> l) & 1) {
		const double D  = rld (Dx, l);
		const double dn = (double)(n + 1) * D; /* exact */
		if (sm.tabD[l] != D) {                /* wave-uniform */
			const double h = sin (dn * 0.5);
			sm.sd[l][n]    = sin (dn);
			sm.cm[l][n]    = 2.0 * h * h;
			__syncthreads (); /* every lane has compared tabD[l] */
			if (n == 0)
				sm.tabD[l] = D;
		}
		const double S = rld (Sx, l), C = rld (Cx, l);
		s              = rv_sin_add (S, C, sm.sd[l][n], sm.cm[l][n]);
	} else {
		const double dl = K.vibDelta[l];
		double       v  = rld (v0x, l);
		for (int i = 0; i <= n; i++)
			v += dl;
		if (n == NL - 1)
			sm.st.vib[l] = v;
		s = sin (v);
	}
	return (s + 1.0) * K.vibDepth;
}

/* one wave per (instance, channel) */
__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL), amdgpu_waves_per_eu (RV_WAVES)))
k_rv_core (const tbf_launch P, const tbf_inst_const* __restrict__ cst)
{
	__shared__ RvCoreLds sm;
	const int      lane = threadIdx.x;
	const int      n    = lane;
	const uint32_t inst = (blockIdx.x >> 1) + P.instBase;
	const int      c    = blockIdx.x & 1;
	if (inst >= P.nInst)
		return;
	const tbf_inst_const& K    = cst[inst];
	tbf_rv_chan*          S    = &P.st[inst].rv.ch[c];
	double* slab = P.rslab + (size_t)inst * P.slabLen;
	const double*         a0s  = rv_buf (P.rvA, P, inst, c);
	double*               bout = rv_buf (P.rvB, P, inst, c);
	copy_words (&sm.st, S);
	if (lane < 8)
		sm.tabD[lane] = -1.0;
	__syncthreads ();
	/* lane l < 12: counter, delay and ring offset of line l; lane l < 8: the feedback
	 * of the channel's last sample on line l */
	const int    dlyv = lane < 12 ? K.delay[lane] : 0;
	const double vdl  = K.vibDelta[lane & 7];
	const int roffv = lane < 12 ? (int)K.ringOff[c * 13 + lane] : 0;
	/* counters in [0, d] from here on: an out-of-range counter steps exactly like d
	 * (`count++; if (count < 0 || count > d) count = 0`), so every later slot is
	 * wrap_slot (count + k, d) for k <= 72 < d + 1 (all delays >= 560) */
	int cntv = lane < 12 ? sm.st.count[lane] : 0;
	cntv     = (cntv < 0 || cntv > dlyv) ? dlyv : cntv;
	double    fbv   = lane < 8 ? sm.st.fb[lane] : 0.0;
	const uint32_t nSub = P.nBlocks * (TBF_BLK / TBF_SUB);
	RvFetch        f;
	if (nSub > 0)
		rv_core_fetch (slab, cntv, dlyv, roffv, a0s, lane, f, false);
#pragma unroll 1
	for (uint32_t s = 0; s < nSub; s++) {
		const size_t o = (size_t)s * TBF_SUB + lane;
		/* per-line phase analysis and sincos, lanes 0..7 in parallel */
		double         v0x, Sx, Cx, Dx;
		const uint64_t okm = rv_core_lines (sm, vdl, v0x, Sx, Cx, Dx, (P.dbg & TBF_DEBUG_FORCE_SERIAL) != 0);
		if (okm != 0xff && lane == 0)
			atomicOr (P.errFlags, (uint32_t)TBF_PATH_RV_PHASE);
		/* windows to LDS (the reads were issued one sub-block ago) */
		if (s == 0) {
#pragma unroll
			for (int l = 0; l < 8; l++)
				sm.win[l][lane] = f.wlo[l];
			sm.win[lane >> 3][NL + (lane & 7)] = f.whi;
		} else {
			/* carried slots +1..+8 = the last sub-block's +65..+72, then the fetched +9..+72 */
			const double tail = sm.win[lane >> 3][NL + (lane & 7)];
			__syncthreads (); /* every lane has read its tail slot */
			sm.win[lane >> 3][lane & 7] = tail;
#pragma unroll
			for (int l = 0; l < 8; l++)
				sm.win[l][8 + lane] = f.wlo[l];
		}
		__syncthreads ();
		/* two-tap interpolation and blend */
		double I[8];
#pragma unroll 2
		for (int l = 0; l < 8; l++) {
			const double off = rv_core_tap (sm, K, l, okm, v0x, Sx, Cx, Dx);
			const int    d   = rl (dlyv, l);
			const int    cn  = wrap_slot (rl (cntv, l) + n + 1, d);
			const int    wk  = (int)(cn + off);
			const int    rel = n + (wk - cn); /* window index of slot wk */
			const double fr  = off - floor (off);
			const bool   inw = rel >= 0 && rel + 1 < RV_WIN;
			const int    i0  = inw ? rel : 0;
			double       r0 = sm.win[l][i0], r1 = sm.win[l][i0 + 1];
			if (!inw) { /* outside the window (not reachable at the fixed vibDepth): ring reads */
				atomicOr (P.errFlags, (uint32_t)TBF_PATH_RV_WINDOW);
				const double* a = slab + rl (roffv, l);
				r0              = a[wrap_slot (wk, d)];
				r1              = a[wrap_slot (wk + 1, d)];
			}
			double x = (r0 * (1 - fr));
			x += (r1 * fr);
			I[l] = ((1.0 - K.blend) * x) + (r0 * K.blend);
		}
		I[0] = (I[0] * K.oneMinusAbsCm) + (I[4] * K.crossmod);
		I[4] = (I[4] * K.oneMinusAbsCm) + (I[0] * K.crossmod);
		double fb[8];
		fb[0] = (I[0] - (I[1] + I[2] + I[3])) * K.regen;
		fb[1] = (I[1] - (I[0] + I[2] + I[3])) * K.regen;
		fb[2] = (I[2] - (I[0] + I[1] + I[3])) * K.regen;
		fb[3] = (I[3] - (I[0] + I[1] + I[2])) * K.regen;
		fb[4] = (I[4] - (I[5] + I[6] + I[7])) * K.regen;
		fb[5] = (I[5] - (I[4] + I[6] + I[7])) * K.regen;
		fb[6] = (I[6] - (I[4] + I[5] + I[7])) * K.regen;
		fb[7] = (I[7] - (I[4] + I[5] + I[6])) * K.regen;
		const double mix = (I[0] + I[1] + I[2] + I[3] + I[4] + I[5] + I[6] + I[7]) / 8.0;
		/* allpass outputs (a = a0 - old/2 written at count; out = a/2 + old) */
		double apw[4], ap[4];
#pragma unroll
		for (int l = 0; l < 4; l++) {
			double a = f.a0;
			a -= f.apOld[l] * 0.5;
			apw[l] = a;
			a *= 0.5;
			a += f.apOld[l];
			ap[l] = a;
		}
		/* reads of the next sub-block, in flight before this one's writes */
		const int ncv = wrap_slot (cntv + TBF_SUB, dlyv);
		if (s + 1 < nSub)
			rv_core_fetch (slab, ncv, dlyv, roffv, a0s, o + TBF_SUB, f, true);
		rv_st (&bout[o], mix);
#pragma unroll
		for (int l = 8; l < 12; l++)
			rv_st (&slab[rl (roffv, l) + wrap_slot (rl (cntv, l) + n, rl (dlyv, l))], apw[l - 8]);
		/* delay-line writes: allpass output + the previous sample's feedback */
		const int srcAp[8] = {3, 2, 1, 0, 0, 1, 2, 3};
		double    fbn      = fbv;
#pragma unroll
		for (int l = 0; l < 8; l++) {
			const double up = lane_shr1 (fb[l]), carry = rld (fbv, l);
			const double prev = lane == 0 ? carry : up;
			rv_st (&slab[rl (roffv, l) + wrap_slot (rl (cntv, l) + n, rl (dlyv, l))], ap[srcAp[l]] + prev);
			const double last = rld (fb[l], NL - 1);
			fbn               = lane == l ? last : fbn;
		}
		fbv  = fbn;
		cntv = ncv;
	}
	if (lane < 12)
		sm.st.count[lane] = cntv;
	if (lane < 8)
		sm.st.fb[lane] = fbv;
	__syncthreads ();
	copy_words (S, &sm.st);
}

/* ------------------------------------------------------------------ k_rv_core_lds
 * The feedback network with the channel's 12 rings resident in LDS for the whole launch:
 * loaded once at the start, stored once at the end (2 x 129 KB per channel and chunk
 * instead of 16 B per line and sample streamed through HBM).  One workgroup of RVL_G
 * waves per (instance, channel), one workgroup per CU (the rings fill its LDS).
 *
 * Why RVL_G sub-blocks can run at once: a sample at time t reads, on a delay line of
 * delay d, the value written at time t + j - d: taps at slot count+1+j (j <= 71, the
 * window; off < 8 in fact), allpasses at count+1 (j = 0).  With 64 RVL_G <= d on the
 * allpass lines (d >= 756) and 64 RVL_G + 72 <= d on the tap lines (d >= 1146) at the
 * reference's fixed settings (the host checks both, tbf_rv_lds_fits), every read of a
 * group of RVL_G sub-blocks returns a value written before the group, and a write of
 * the group only ever replaces a value that the group's earlier samples read.  So all
 * reads of a group may precede all its writes, exactly as k_rv_core's reads of a
 * sub-block precede its writes; a worker's writes wait (barrier) for the reads of the
 * 72 samples before its first, which lie in the previous worker's sub-block.  The
 * one serial term, feedback(n - 1), crosses sub-blocks through LDS (carry) between the
 * read phase and the write phase.  Per sub-block the arithmetic is k_rv_core's: the
 * same phases (closed form v0 + (n+1) D with the same start phases, or the literal
 * recurrence), the same sine rows, taps, Householder mix and allpasses. */
#ifndef RVL_G
#define RVL_G 11 /* sub-blocks (worker waves) per group: 64 RVL_G <= the shortest allpass delay (756), 64 RVL_G + 72 <= the shortest tap-line delay (1146) */
#endif
/* the network's ring geometry at the reference's fixed settings (reverbConsts: size =
 * 0.4f^2 * 90 + 10, delay = (int)(dmul * size); lines 128-B aligned): compile-time constants, so
 * the ring addressing needs no per-line lane reads; tbf_rv_lds_fits checks an instance
 * against them */
constexpr int RVL_DLY[12] = {1927, 1781, 1732, 1634, 1488, 1439, 1293, 1146, 1049, 1000, 902, 756};
/* in HBM: each line's d + 1 slots rounded up to TBF_RING_ALIGN (reverbConsts) */
constexpr int rvl_hofs (int l) { return l == 0 ? 0 : rvl_hofs (l - 1) + ((RVL_DLY[l - 1] + TBF_RING_ALIGN) & ~(TBF_RING_ALIGN - 1)); }
constexpr int RVL_OFS[12] = {rvl_hofs (0), rvl_hofs (1), rvl_hofs (2), rvl_hofs (3), rvl_hofs (4),  rvl_hofs (5),
                             rvl_hofs (6), rvl_hofs (7), rvl_hofs (8), rvl_hofs (9), rvl_hofs (10), rvl_hofs (11)};
/* In LDS each line of delay d holds its d + 1 slots followed by a mirror of slots
 * 0 .. RVL_MIR - 1, so the reads of a sub-block (slots count + 1 .. count + 71 for the
 * taps, count + 1 .. count + 64 for the allpasses, with count in [0, d]) never wrap: a tap
 * pair is two adjacent doubles (one ds_read2_b64) at a plain index.  A write to a slot
 * below RVL_MIR also writes its mirror. */
#define RVL_MIR 72
constexpr int rvl_lofs (int l) { return l == 0 ? 0 : rvl_lofs (l - 1) + ((RVL_DLY[l - 1] + 1 + RVL_MIR + 1) & ~1); }
constexpr int RVL_LOFS[12] = {rvl_lofs (0), rvl_lofs (1), rvl_lofs (2),  rvl_lofs (3),  rvl_lofs (4),  rvl_lofs (5),
                              rvl_lofs (6), rvl_lofs (7), rvl_lofs (8), rvl_lofs (9), rvl_lofs (10), rvl_lofs (11)};
#define RVL_RING (rvl_lofs (12)) /* LDS ring doubles of a channel's lines 0..11 with their mirrors */
#define RVL_MIN_BLOCKS 8 /* shorter launches take the streaming k_rv_core */
#define RVL_THREADS (NL * (RVL_G + 1)) /* RVL_G worker waves + the planner wave */

struct RvLds {
	double      ring[RVL_RING];
	double2     sc[2][8][TBF_SUB];     /* sine rows of each line's closed-form step, by group parity:
	                                    * {sin ((n+1) D), 2 sin^2 ((n+1) D / 2)}, one 16-B read */
	double      tabD[2][8];            /* the step each row holds (-1: none) */
	double      v0[2][RVL_G][8];       /* group plan: phase of line l at the start of sub-block j ... */
	double2     SC[2][RVL_G][8];       /* ... and its {sine, cosine} (closed-form lines) */
	uint32_t    okm[2][RVL_G];         /* closed-form lines of sub-block j (the rows sc hold its step) ... */
	uint32_t    okx[2][RVL_G];         /* ... closed-form lines whose step Dx is not the rows' (a group
	                                    * crossing a binade: the rows are computed inline) */
	double      Dx[2][RVL_G][8];
	double      carry[2][RVL_G][8];    /* feedback of sub-block j's last sample */
	tbf_rv_chan st;
};
static_assert (sizeof (RvLds) <= 160 * 1024, "k_rv_core_lds: a channel's rings fill gfx950's 160 KB of LDS");

/* a ring write at slot i of a line of delay d, and at its mirror when i < RVL_MIR */
__device__ __forceinline__ void rvl_write (double* rg, int i, int d, double v)
{
	rg[i] = v;
	if (i < RVL_MIR)
		rg[i + d + 1] = v;
}

#ifndef RVL_FAST2
#define RVL_FAST2 1 /* tap index without the FP64 sum (a vote on the rare carry), allpass products as fmas (exact) */
#endif
#ifndef RVL_PRIO
#define RVL_PRIO 1 /* workers raise their priority at a phase start and drop it part-way, so the three workers
                    * of a SIMD progress together instead of in age order (1: drop after the tap reads, 2: after
                    * the Householder mix) */
#endif
#ifndef RVL_EXPECT
#define RVL_EXPECT 1 /* the ring wrap / mirror branches marked unlikely, so the common case falls through */
#endif
#if RVL_EXPECT
#define RVL_RARE(x) __builtin_expect (!!(x), 0)
#else
#define RVL_RARE(x) (x)
#endif
#ifndef RVL_SCAL
#define RVL_SCAL 1 /* the workers' line counters in scalar registers, wraps as scalar branches (below) */
#endif
/* lane n's slot c + n of a line of delay D, wrapped past D (wrap_slot), for a wave-uniform c
 * in [0, D + 1]: a sub-block wraps a line in about one of D / 64 groups, so the test is a
 * scalar branch around the lanes' correction and the common case is one add */
template <int D>
__device__ __forceinline__ int rvl_slot (int c, int n)
{
	int s = c + n;
	if (RVL_RARE (c > D - (NL - 1))) {
		/* opaque to the optimizer, so the branch stays a branch (if-converted, the lanes'
		 * compare and selects ran in every sub-block) */
		__asm__ __volatile__ ("" : "+v"(s));
		s -= (s > D) ? D + 1 : 0;
	}
	return s;
}

/* rvl_slot of tap line l (0..7) one past the worker's counter (the taps' count + 1) */
__device__ __forceinline__ int rvl_slot_l (int l, const int (&cs)[12], int n)
{
	switch (l) { /* l is a constant after unrolling: the delay a template argument */
		case 0: return rvl_slot<RVL_DLY[0]> (cs[0] + 1, n);
		case 1: return rvl_slot<RVL_DLY[1]> (cs[1] + 1, n);
		case 2: return rvl_slot<RVL_DLY[2]> (cs[2] + 1, n);
		case 3: return rvl_slot<RVL_DLY[3]> (cs[3] + 1, n);
		case 4: return rvl_slot<RVL_DLY[4]> (cs[4] + 1, n);
		case 5: return rvl_slot<RVL_DLY[5]> (cs[5] + 1, n);
		case 6: return rvl_slot<RVL_DLY[6]> (cs[6] + 1, n);
		default: return rvl_slot<RVL_DLY[7]> (cs[7] + 1, n);
	}
}

/* rvl_write at slot rvl_slot<D> (c, n): the mirror (slots below RVL_MIR) is possible only when
 * c < RVL_MIR or the sub-block wraps, again a scalar test */
template <int D>
__device__ __forceinline__ void rvl_write_s (double* rg, int c, int n, double v)
{
	if (!RVL_RARE (c < RVL_MIR || c > D - (NL - 1))) { /* the common case: no wrap, no mirror */
		rg[c + n] = v;
	} else {
		int i = c + n;
		__asm__ __volatile__ ("" : "+v"(i)); /* a branch, not selects (rvl_slot) */
		i -= (i > D) ? D + 1 : 0;
		rg[i] = v;
		if (i < RVL_MIR)
			rg[i + D + 1] = v;
	}
}

/* lane n receives lane n-1's v, lane 0 receives first (FP64 lane_shr1_or: the DPP moves keep
 * the old value in the lane with no source) */
__device__ __forceinline__ double lane_shr1_or (double v, double first)
{
	const unsigned long long u = __double_as_longlong (v), f = __double_as_longlong (first);
	const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp ((int)(unsigned)f, (int)(unsigned)u, 0x138, 0xF, 0xF, false);
	const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp ((int)(unsigned)(f >> 32), (int)(unsigned)(u >> 32), 0x138, 0xF, 0xF, false);
	return __longlong_as_double ((long long)(((unsigned long long)hi << 32) | lo));
}

/* the planner wave: the phase plan of group g into buffer b (start phases, closed-form
 * flags, sincos of the start phases, sine rows); st.vib advanced past the group.  It
 * depends only on the phases, so it runs while the workers process the group before. */
__device__ __forceinline__ void rvl_plan (RvLds& sm, double d, int nb, int b, bool force, uint32_t* errFlags)
{
	const int    lane = threadIdx.x & (NL - 1);
	const int    li   = lane & 7; /* every lane analyses line lane & 7; d = vibDelta[li] */
	const double v0   = sm.st.vib[li];
	double       D = 0.0, cD = sm.st.phD[li], cLo = sm.st.phLo[li], cHi = sm.st.phHi[li];
	/* the group's whole run closed-form: sub-block j starts at v0 + 64 j D exactly */
	const bool     ok  = phase_run_cached (v0, d, TBF_SUB * nb, D, cD, cLo, cHi) && !force;
	const uint64_t okb = __ballot (lane < 8 && ok);
#pragma unroll 1
	for (int l = 0; l < 8; l++) {
		if (!((okb >> l) & 1))
			continue;
		const double Dl = rld (D, l);
		if (sm.tabD[b][l] != Dl) { /* rare: a new step (binade) */
			const double dn  = (double)(lane + 1) * Dl; /* exact */
			const double h   = sin (dn * 0.5);
			sm.sc[b][l][lane] = double2 {sin (dn), 2.0 * h * h};
			__builtin_amdgcn_wave_barrier ();
			if (lane == 0)
				sm.tabD[b][l] = Dl;
		}
	}
	/* lane q = 8 j + l (and q + 64): sub-block j, line l */
	for (int q = lane; q < 8 * nb; q += NL) {
		const int j = q >> 3;
		if (ok) {
			const double v = v0 + (double)(TBF_SUB * j) * D; /* exact inside the binade */
			double       sv, cv;
			sincos (v, &sv, &cv);
			sm.v0[b][j][li] = v;
			sm.SC[b][j][li] = double2 {sv, cv};
		}
	}
	if (lane < RVL_G) {
		sm.okm[b][lane] = lane < nb ? (uint32_t)(okb & 0xff) : 0u;
		sm.okx[b][lane] = 0u;
	}
	__builtin_amdgcn_wave_barrier ();
	if (lane < 8) {
		sm.st.phD[li]  = cD;
		sm.st.phLo[li] = cLo;
		sm.st.phHi[li] = cHi;
		double v = v0;
		if (ok) {
			v = v0 + (double)(TBF_SUB * nb) * D;
		} else {
			/* rare (a binade crossing or a rounding tie in the group, or forced): walk the
			 * sub-blocks like k_rv_core: one is closed-form when its own run is (with the
			 * line's rows when they hold its step, else rows computed inline), else the
			 * literal recurrence (64 adds).  So the two network kernels agree however a
			 * render is split into launches and groups. */
			atomicOr (errFlags, (uint32_t)TBF_PATH_RV_PHASE);
			for (int j = 0; j < nb; j++) {
				sm.v0[b][j][li] = v;
				double     Dj = 0.0, c1 = cD, c2 = cLo, c3 = cHi;
				const bool oj = phase_run_cached (v, d, TBF_SUB, Dj, c1, c2, c3) && !force;
				if (oj) {
					double sv, cv;
					sincos (v, &sv, &cv);
					sm.SC[b][j][li] = double2 {sv, cv};
					if (Dj == sm.tabD[b][li])
						atomicOr (&sm.okm[b][j], 1u << li);
					else {
						sm.Dx[b][j][li] = Dj;
						atomicOr (&sm.okx[b][j], 1u << li);
					}
					v = v + (double)TBF_SUB * Dj;
				} else {
					for (int i = 0; i < TBF_SUB; i++)
						v += d;
				}
			}
		}
		sm.st.vib[li] = v;
	}
}

/* one (instance, channel) of a k_rv_core_lds launch */
__device__ __forceinline__ void rvl_pair (const tbf_launch& P, const tbf_inst_const* __restrict__ cst, RvLds& sm,
                                          const uint32_t inst, const int c)
{
	const int      tid  = threadIdx.x;
	const int      w    = tid >> 6; /* worker: the sub-block within a group; w == RVL_G: planner */
	const int      n    = tid & (NL - 1);
	const tbf_inst_const& K     = cst[inst];
	tbf_rv_chan*          S     = &P.st[inst].rv.ch[c];
	const uint32_t        rbase = K.ringOff[c * 13];
	double*               slab  = P.rslab + (size_t)inst * P.slabLen + rbase; /* lines 0..11 at RVL_OFS */
	const double*         a0s   = rv_buf (P.rvA, P, inst, c);
	double*               bout  = rv_buf (P.rvB, P, inst, c);
	/* lane l < 12: delay and counter of line l (the LDS ring offsets are RVL_LOFS) */
	const int dlyv = n < 12 ? K.delay[n] : 0;
	const double vdl = K.vibDelta[n & 7]; /* lane-held: no vector load of K inside the loop */
	const uint32_t nSub  = P.nBlocks * (TBF_BLK / TBF_SUB);
	const uint32_t nGrp  = (nSub + RVL_G - 1) / RVL_G;
	const bool     force = (P.dbg & TBF_DEBUG_FORCE_SERIAL) != 0;
	if (w < RVL_G) {
		/* the workers load the rings and fill the mirrors: every load in flight before the
		 * first LDS store (clamped indices keep the loads unconditional) */
		constexpr int WT = NL * RVL_G;
#pragma unroll
		for (int l0 = 0; l0 < 12; l0 += 6) { /* six lines' loads in flight at a time */
			double v[6][(RVL_DLY[0] + 1 + RVL_MIR + WT - 1) / WT];
#pragma unroll
			for (int l = l0; l < l0 + 6; l++)
#pragma unroll
				for (int k = 0; k * WT < RVL_DLY[l] + 1 + RVL_MIR; k++) {
					const int i = tid + k * WT; /* LDS slot: i <= d canonical, then the mirror */
					const int j = i <= RVL_DLY[l] ? i : (i - RVL_DLY[l] - 1 < RVL_MIR ? i - RVL_DLY[l] - 1 : 0);
					v[l - l0][k] = slab[RVL_OFS[l] + j];
				}
#pragma unroll
			for (int l = l0; l < l0 + 6; l++)
#pragma unroll
				for (int k = 0; k * WT < RVL_DLY[l] + 1 + RVL_MIR; k++) {
					const int i = tid + k * WT;
					if (i < RVL_DLY[l] + 1 + RVL_MIR)
						sm.ring[RVL_LOFS[l] + i] = v[l - l0][k];
				}
		}
	} else {
		/* meanwhile the planner loads the channel state and plans the first group, which
		 * reads no ring */
		const uint32_t* src = (const uint32_t*)S;
		uint32_t*       dst = (uint32_t*)&sm.st;
		for (uint32_t i = (uint32_t)n; i < sizeof (tbf_rv_chan) / 4; i += NL)
			dst[i] = src[i];
		if (n < 16)
			(&sm.tabD[0][0])[n] = -1.0;
		__builtin_amdgcn_fence (__ATOMIC_SEQ_CST, "wavefront");
		__builtin_amdgcn_wave_barrier ();
		if (n < 8)
			sm.carry[1][RVL_G - 1][n] = sm.st.fb[n]; /* as the "previous group's" last feedback */
		if (nGrp > 0)
			rvl_plan (sm, vdl, (int)min ((uint32_t)RVL_G, nSub), 0, force, P.errFlags);
	}
	__syncthreads ();
	int cntv = n < 12 ? sm.st.count[n] : 0;
	cntv     = (cntv < 0 || cntv > dlyv) ? dlyv : cntv; /* see k_rv_core */
	/* this worker's sub-block counter (64 RVL_G <= d: one wrap at most) */
	int cw = wrap_slot (cntv + TBF_SUB * (w < RVL_G ? w : 0), dlyv);
	const double oneMB = 1.0 - K.blend;
	/* the network input two groups ahead: a0 for this group, a0n for the next (an HBM
	 * load waited for in the same group's read phase would expose its latency) */
	double a0 = 0.0, a0n = 0.0;
	if (w < RVL_G && (uint32_t)w < nSub)
		a0 = a0s[(size_t)w * TBF_SUB + n];
	if (w < RVL_G && (uint32_t)(RVL_G + w) < nSub)
		a0n = a0s[(size_t)(RVL_G + w) * TBF_SUB + n];
	double pmix = 0.0; /* the previous group's tap mix, stored a group late */
	size_t po   = 0;
	bool   pst  = false;
	__syncthreads ();
	/* the workers and the planner run separate loops with the same two barriers per group, so
	 * the registers of one role are not held live across the other's code */
	if (w < RVL_G) {
#if RVL_SCAL
		/* this worker's first slot of each line in the group, wave-uniform (SGPRs) */
		int cs[12];
#pragma unroll
		for (int l = 0; l < 12; l++)
			cs[l] = rl (cw, l);
#define RVL_C(l) cs[l]
#else
#define RVL_C(l) rl (cw, l)
#endif
#pragma unroll 1
		for (uint32_t g = 0; g < nGrp; g++) {
			const int  nb  = (int)min ((uint32_t)RVL_G, nSub - g * RVL_G);
			const int  par = g & 1;
			const bool act = w < nb;
			/* ---- read phase (workers): taps, mix, allpass reads; nothing is written to the
			 * rings.  The planner plans the next group meanwhile. ---- */
			double       apw[4], ap[4], fb[8], mix;
			const size_t o = ((size_t)g * RVL_G + (uint32_t)w) * TBF_SUB + n;
			/* HBM traffic at the start of the group, a whole group ahead of any wait on it: the
			 * input two groups ahead (every wave, the index clamped, so that no branch joins
			 * the loaded register) and the previous group's tap mix.  Issued at the end of
			 * the write phase, the copy a0n <- load at the loop's back edge waited for the
			 * load, and for the store, right away. */
			const double nxt = a0s[(size_t)min ((g + 2) * RVL_G + (uint32_t)min (w, RVL_G - 1), nSub - 1) * TBF_SUB + n];
			if (pst)
				rv_st (&bout[po], pmix);
			if (act) {
#if RVL_PRIO
				__builtin_amdgcn_s_setprio (1);
#endif
				/* the lines' vibrato sines: closed form on every line (wave-uniform, the rule), or
				 * per line the closed form or the literal recurrence and sin */
				const uint32_t om = __builtin_amdgcn_readfirstlane (sm.okm[par][w]);
				double         sn[8];
				if (om == 0xffu) {
#pragma unroll
					for (int l = 0; l < 8; l++) {
						const double2 SC = sm.SC[par][w][l], q = sm.sc[par][l][n];
						sn[l]            = rv_sin_add (SC.x, SC.y, q.x, q.y);
					}
				} else {
					const uint32_t ox = __builtin_amdgcn_readfirstlane (sm.okx[par][w]);
#pragma unroll
					for (int l = 0; l < 8; l++) {
						if ((om >> l) & 1) {
							const double2 SC = sm.SC[par][w][l], q = sm.sc[par][l][n];
							sn[l]            = rv_sin_add (SC.x, SC.y, q.x, q.y);
						} else if ((ox >> l) & 1) { /* k_rv_core's rows for this step (rv_core_tap) */
							const double2 SC = sm.SC[par][w][l];
							const double  dn = (double)(n + 1) * sm.Dx[par][w][l]; /* exact */
							const double  hh = sin (dn * 0.5);
							const double  sd = sin (dn), cm = 2.0 * hh * hh;
							sn[l]            = rv_sin_add (SC.x, SC.y, sd, cm);
						} else {
							const double dl = rld (vdl, l);
							double       v  = sm.v0[par][w][l];
							for (int i = 0; i <= n; i++)
								v += dl;
							sn[l] = sin (v);
						}
					}
				}
				/* every line's tap address first, then all eight tap-pair reads in flight
				 * together, then the interpolations (a line's read was waited for before the
				 * next line's address was formed) */
				double I[8], fr[8], r0[8], r1[8];
				int    wk[8];
#if RVL_SCAL && RVL_FAST2
				double offv[8];
				int    cnv[8];
				bool   slow = false;
#endif
#pragma unroll
				for (int l = 0; l < 8; l++) {
					const double off = (sn[l] + 1.0) * K.vibDepth;
#if RVL_SCAL
					const int cn = rvl_slot_l (l, cs, n);
					/* off >= 0, so off - floor (off) is exact (or off < 0 tiny, |off| >= 2.7 2^-53: one
					 * rounding of off + 1, below 1): v_fract_f64's value */
					fr[l] = __builtin_amdgcn_fract (off);
#if RVL_FAST2
					/* (int)(cn + off) == cn + (int)off unless the sum's rounding (ulp <= 2^-42, the
					 * sum < 2048) carries the fraction to the next integer, or off < 0: both need
					 * fr >= 1 - 2^-21, i.e. fr's high word >= 0x3FEFFFFF (one integer compare);
					 * such a wave recomputes the reference's expression below */
					offv[l] = off;
					cnv[l]  = cn;
					wk[l]   = cn + (int)off;
					slow    = slow || (uint32_t)(__double_as_longlong (fr[l]) >> 32) >= 0x3FEFFFFFu;
#else
					wk[l] = (int)(cn + off); /* <= d + 5: the mirror covers wk + 1 */
#endif
#else
					const int    cn  = wrap_slot (rl (cw, l) + n + 1, RVL_DLY[l]);
					wk[l]            = (int)(cn + off); /* <= d + 5: the mirror covers wk + 1 */
					fr[l]            = off - floor (off);
#endif
				}
#if RVL_SCAL && RVL_FAST2
				if (__builtin_expect (__any (slow), 0)) {
#pragma unroll
					for (int l = 0; l < 8; l++)
						wk[l] = (int)(cnv[l] + offv[l]);
				}
#endif
#pragma unroll
				for (int l = 0; l < 8; l++) {
					const double* rg = sm.ring + RVL_LOFS[l];
					r0[l]            = rg[wk[l]];
					r1[l]            = rg[wk[l] + 1];
				}
#if RVL_PRIO == 1
				__builtin_amdgcn_s_setprio (0);
#endif
#pragma unroll
				for (int l = 0; l < 8; l++) {
					double x = (r0[l] * (1 - fr[l]));
					x += (r1[l] * fr[l]);
					I[l] = (oneMB * x) + (r0[l] * K.blend);
				}
				I[0]  = (I[0] * K.oneMinusAbsCm) + (I[4] * K.crossmod);
				I[4]  = (I[4] * K.oneMinusAbsCm) + (I[0] * K.crossmod);
				fb[0] = (I[0] - (I[1] + I[2] + I[3])) * K.regen;
				fb[1] = (I[1] - (I[0] + I[2] + I[3])) * K.regen;
				fb[2] = (I[2] - (I[0] + I[1] + I[3])) * K.regen;
				fb[3] = (I[3] - (I[0] + I[1] + I[2])) * K.regen;
				fb[4] = (I[4] - (I[5] + I[6] + I[7])) * K.regen;
				fb[5] = (I[5] - (I[4] + I[6] + I[7])) * K.regen;
				fb[6] = (I[6] - (I[4] + I[5] + I[7])) * K.regen;
				fb[7] = (I[7] - (I[4] + I[5] + I[6])) * K.regen;
				mix = (I[0] + I[1] + I[2] + I[3] + I[4] + I[5] + I[6] + I[7]) / 8.0;
#if RVL_PRIO == 2
				__builtin_amdgcn_s_setprio (0);
#endif
#pragma unroll
				for (int l = 8; l < 12; l++) {
					const double old = sm.ring[RVL_LOFS[l] + RVL_C (l) + n + 1]; /* <= d + 64: mirror */
#if RVL_FAST2
					/* a0 - old 0.5 then (.) 0.5 + old: both products by 0.5 are exact unless an
					 * operand is subnormal (< 2.2e-308; the input's denormal guard,
					 * src/reverb.cpp:343-346, keeps the network's values above ~1e-25), so one fma
					 * each gives the reference's values */
					const double a = __builtin_fma (old, -0.5, a0);
					apw[l - 8]     = a;
					ap[l - 8]      = __builtin_fma (a, 0.5, old);
#else
					double       a   = a0;
					a -= old * 0.5;
					apw[l - 8] = a;
					a *= 0.5;
					a += old;
					ap[l - 8] = a;
#endif
				}
				if (n == NL - 1) {
#pragma unroll
					for (int l = 0; l < 8; l++)
						sm.carry[par][w][l] = fb[l];
				}
			}
			__syncthreads ();
			/* ---- write phase ---- */
			if (act) {
#if RVL_PRIO
				__builtin_amdgcn_s_setprio (1);
#endif
				/* the previous sub-block's last feedback, all 8 lines read before any ring write */
				const double* cp = w == 0 ? sm.carry[par ^ 1][RVL_G - 1] : sm.carry[par][w - 1];
				double        cprv[8];
#pragma unroll
				for (int l = 0; l < 8; l++)
					cprv[l] = cp[l];
#if RVL_SCAL
				rvl_write_s<RVL_DLY[8]> (sm.ring + RVL_LOFS[8], cs[8], n, apw[0]);
				rvl_write_s<RVL_DLY[9]> (sm.ring + RVL_LOFS[9], cs[9], n, apw[1]);
				rvl_write_s<RVL_DLY[10]> (sm.ring + RVL_LOFS[10], cs[10], n, apw[2]);
				rvl_write_s<RVL_DLY[11]> (sm.ring + RVL_LOFS[11], cs[11], n, apw[3]);
				/* feedback (n - 1): lane 0 takes the previous sub-block's last, the DPP move's old value */
				rvl_write_s<RVL_DLY[0]> (sm.ring + RVL_LOFS[0], cs[0], n, ap[3] + lane_shr1_or (fb[0], cprv[0]));
				rvl_write_s<RVL_DLY[1]> (sm.ring + RVL_LOFS[1], cs[1], n, ap[2] + lane_shr1_or (fb[1], cprv[1]));
#if RVL_PRIO
				__builtin_amdgcn_s_setprio (0);
#endif
				rvl_write_s<RVL_DLY[2]> (sm.ring + RVL_LOFS[2], cs[2], n, ap[1] + lane_shr1_or (fb[2], cprv[2]));
				rvl_write_s<RVL_DLY[3]> (sm.ring + RVL_LOFS[3], cs[3], n, ap[0] + lane_shr1_or (fb[3], cprv[3]));
				rvl_write_s<RVL_DLY[4]> (sm.ring + RVL_LOFS[4], cs[4], n, ap[0] + lane_shr1_or (fb[4], cprv[4]));
				rvl_write_s<RVL_DLY[5]> (sm.ring + RVL_LOFS[5], cs[5], n, ap[1] + lane_shr1_or (fb[5], cprv[5]));
				rvl_write_s<RVL_DLY[6]> (sm.ring + RVL_LOFS[6], cs[6], n, ap[2] + lane_shr1_or (fb[6], cprv[6]));
				rvl_write_s<RVL_DLY[7]> (sm.ring + RVL_LOFS[7], cs[7], n, ap[3] + lane_shr1_or (fb[7], cprv[7]));
#else
#pragma unroll
				for (int l = 8; l < 12; l++)
					rvl_write (sm.ring + RVL_LOFS[l], wrap_slot (rl (cw, l) + n, RVL_DLY[l]), RVL_DLY[l], apw[l - 8]);
				const int srcAp[8] = {3, 2, 1, 0, 0, 1, 2, 3};
#pragma unroll
				for (int l = 0; l < 8; l++) {
					const double up   = lane_shr1 (fb[l]);
					const double prev = n == 0 ? cprv[l] : up;
					rvl_write (sm.ring + RVL_LOFS[l], wrap_slot (rl (cw, l) + n, RVL_DLY[l]), RVL_DLY[l], ap[srcAp[l]] + prev);
				}
#endif
				/* the tap mix, stored at the start of the next group (see above) */
				pmix = mix;
				po   = o;
			}
			pst = act;
			a0  = a0n;
			a0n = nxt;
			cw = wrap_slot (cw + TBF_SUB * RVL_G, dlyv);
#if RVL_SCAL
#pragma unroll
			for (int l = 0; l < 12; l++)
				cs[l] = wrap_slot (cs[l] + TBF_SUB * RVL_G, RVL_DLY[l]);
#endif
			__syncthreads ();
		}
#undef RVL_C
	} else {
#pragma unroll 1
		for (uint32_t g = 0; g < nGrp; g++) {
			if (g + 1 < nGrp) {
				/* the planner is the youngest wave of its SIMD: at equal priority the two
				 * workers beside it took the issue slots first and every worker waited for
				 * the plan at the barrier (tools/rvl_prof.py: 5.7k cycles per group against
				 * 3.3-4.8k for a worker's read phase) */
				__builtin_amdgcn_s_setprio (2);
				rvl_plan (sm, vdl, (int)min ((uint32_t)RVL_G, nSub - (g + 1) * RVL_G), (g & 1) ^ 1, force, P.errFlags);
				__builtin_amdgcn_s_setprio (0);
			}
			__syncthreads ();
			__syncthreads ();
		}
	}
	if (pst)
		rv_st (&bout[po], pmix);
	/* state: counters after nSub * 64 steps, the last sample's feedback */
	if (w == 0) {
		if (n < 12)
			sm.st.count[n] = (int)(((uint32_t)cntv + (uint64_t)nSub * TBF_SUB) % (uint32_t)(dlyv + 1));
		if (n < 8 && nGrp > 0)
			sm.st.fb[n] = sm.carry[(nGrp - 1) & 1][(nSub - 1) % RVL_G][n];
	}
	__syncthreads ();
#pragma unroll
	for (int l = 0; l < 12; l++) /* the canonical slots */
		for (int i = tid; i <= RVL_DLY[l]; i += RVL_THREADS)
			slab[RVL_OFS[l] + i] = sm.ring[RVL_LOFS[l] + i];
	if (w == 0)
		copy_words (S, &sm.st);
}

/* A workgroup needs a whole CU's LDS, so it can start only on a CU that has drained, while
 * the neighbouring chunks' kernels keep refilling freed CUs with small workgroups.  So the
 * grid is persistent (P.rvGrid workgroups, one per CU by default): each workgroup takes
 * (instance, channel) pairs from a work counter (P.rvWork, zeroed before the launch) until
 * none is left, and acquires its CU once per launch instead of once per pair.  Every wave of
 * a workgroup reads the same counter value, so all of them leave the loop together. */
__global__ void __attribute__ ((amdgpu_flat_work_group_size (RVL_THREADS, RVL_THREADS)))
k_rv_core_lds (const tbf_launch P, const tbf_inst_const* __restrict__ cst)
{
	__shared__ RvLds    sm;
	__shared__ uint32_t next;
	const uint32_t      nPair = 2 * (P.nInst - P.instBase);
	for (;;) {
		if (threadIdx.x == 0)
			next = atomicAdd (P.rvWork, 1u);
		__syncthreads (); /* also: the previous pair's ring and state stores have read the LDS */
		const uint32_t q = __builtin_amdgcn_readfirstlane (next);
		if (q >= nPair)
			break;
		rvl_pair (P, cst, sm, P.instBase + (q >> 1), (int)(q & 1)); /* its barriers order the next write of `next` */
	}
}

/* ------------------------------------------------------------------ chain blocks
 * The reverb's serial FP64 biquads with one chain per lane.  A workgroup serves RVC_CB
 * instances, i.e. RVC_NC = 2 RVC_CB chains (chain r = 2 j + c: instance j, channel c), in
 * tiles of RVC_T samples staged in LDS as [chain][sample] rows of odd stride RVC_S, so a
 * column (one sample of every chain) is one conflict-free ds_read_b64:
 *   wave 0     the serial recurrences, lane = chain: one FP64 instruction stream advances
 *              64 chains (one wave per instance would serve 2)
 *   wave 1     the chains' xorshift dither streams (fpdL/fpdR, src/reverb.cpp:775-783),
 *              lane = chain, written ahead as f[chain][n] = state before sample n
 *   waves 2..  lane-parallel work, one instance at a time (wave-uniform, so its constants
 *              come in as scalar loads): lane = (channel, sample of the tile); HBM loads
 *              one tile ahead, predelay ring, denormal guard, sin / asin, dry mix,
 *              dither, mono sum, stores
 * A tile's stages advance one per iteration, with one barrier per iteration.  Every
 * chain runs the reference's operations in its order, so the bits are the reference's. */
#ifndef RVC_CB
/* instances per workgroup: 28 with 14 helper waves (147 workgroups) against 32 with 8: k_rv_pre
 * alone 2.79 -> 2.37 ms per 512 blocks, the step 113.6 -> 113.2 ms (profiles/r06/s21) */
#define RVC_CB 28
#endif
#define RVC_NC (2 * RVC_CB)      /* chains per workgroup (<= 64: one per lane of wave 0) */
#define RVC_T 32                 /* samples per tile: one per lane of a half-wave */
#define RVC_S (RVC_T + 1)        /* LDS row stride (odd: conflict-free columns) */
#ifndef RVC_H
#define RVC_H 14 /* helper waves */
#endif
#define RVC_TASKS RVC_CB          /* helper tasks per tile: one instance each */
#define RVC_NTK (RVC_TASKS / RVC_H)
static_assert (RVC_TASKS % RVC_H == 0, "helper tasks split evenly");
#define RVC_THREADS (NL * (2 + RVC_H))
static_assert (RVC_NC <= NL && RVC_T * 2 == NL && TBF_BLK % RVC_T == 0, "chain-block geometry");
#define RVC_ROWS (RVC_NC + (RVC_NC < NL)) /* chain rows, + one that the serial and dither waves' idle lanes use */

/* one transposed-DF2 biquad step (biquadA/B/C, src/reverb.cpp:361-369, 733-741, 756-764) */
__device__ __forceinline__ double rvc_bq (double x, double c0, double c1, double c2, double c3, double c4, double& s7,
                                          double& s8)
{
	const double t = (x * c0) + s7;
	s7             = (x * c1) - (t * c3) + s8;
	s8             = (x * c2) - (t * c4);
	return t;
}

/* the xorshift states of one tile of every chain: f[n] = state before sample n (n = 0 ..
 * RVC_T; entry RVC_T = the state after the tile) */
__device__ __forceinline__ void rvc_dither_row (uint32_t* f, uint32_t& s)
{
#pragma unroll 8
	for (int n = 0; n < RVC_T; n++) {
		f[n] = s;
		s    = xs_step (s);
	}
	f[RVC_T] = s;
}

/* the predelay slot k samples after counter c in [0, d] (k <= d + 1): cnt_adv's steady state */
__device__ __forceinline__ int rvc_slot (int c, int d, int k)
{
	const int v = c + k;
	return v > d ? v - d - 1 : v;
}

/* a launch's per-block values sit one per lane: lane b = block b.  A launch of more than 64
 * blocks has no control deltas (every block plays the instance's current entry), so its
 * blocks past 63 read lane 63 */
__device__ __forceinline__ int blk_lane (int b) { return b < NL ? b : NL - 1; }

/* a helper task's per-block reverb wet level, lane b = block b of the launch */
__device__ __forceinline__ double rvc_wet_lanes (const tbf_launch& P, const tbf_seg_ctl* __restrict__ ctl, uint32_t inst)
{
	const uint32_t b = threadIdx.x & (NL - 1);
	return b < P.nBlocks ? ctl_of (P, ctl, b, inst).rvWet : 0.0;
}

/* the serial chains of one tile, in place: one biquad (q = 1) or two interleaved */
template <int Q>
__device__ __forceinline__ void rvc_serial (double* const (&row)[Q], const double (&c)[Q][5], double (&s)[Q][2])
{
	PRIO_UP ();
	for (int i0 = 0; i0 < RVC_T; i0 += 8) {
		double xv[Q][8];
#pragma unroll
		for (int k = 0; k < 8; k++)
#pragma unroll
			for (int q = 0; q < Q; q++)
				xv[q][k] = row[q][i0 + k];
#pragma unroll
		for (int k = 0; k < 8; k++)
#pragma unroll
			for (int q = 0; q < Q; q++)
				row[q][i0 + k] = rvc_bq (xv[q][k], c[q][0], c[q][1], c[q][2], c[q][3], c[q][4], s[q][0], s[q][1]);
	}
	PRIO_DOWN ();
}

/* One chain's biquad over a tile with its input products precomputed (src/reverb.cpp:733-741,
 * 756-764): p0 = x c0, p1 = x c1, p2 = x c2 are the reference's rounded products, so
 *   t = p0 + s7;  s7 = (p1 - t c3) + s8;  s8 = p2 - t c4
 * is its recurrence bit for bit, six FP64 operations a step where rvc_bq has nine (the
 * chain wave is issue-bound: tools/rvp_prof.py, profiles/r06/s5).  t goes over p0.  Groups
 * of eight, the next group's products read while this group's steps run. */
__device__ __forceinline__ void rvc_serial_p (double* r0, const double* r1, const double* r2, double c3, double c4, double& s7,
                                              double& s8)
{
	PRIO_UP ();
	double a0[8], a1[8], a2[8], b0[8], b1[8], b2[8];
	auto ld = [&] (double (&x0)[8], double (&x1)[8], double (&x2)[8], int i0) {
#pragma unroll
		for (int k = 0; k < 8; k++) {
			x0[k] = r0[i0 + k];
			x1[k] = r1[i0 + k];
			x2[k] = r2[i0 + k];
		}
	};
	auto run = [&] (const double (&x0)[8], const double (&x1)[8], const double (&x2)[8], int i0) {
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const double t = x0[k] + s7;
			s7             = (x1[k] - (t * c3)) + s8;
			s8             = x2[k] - (t * c4);
			r0[i0 + k]     = t;
		}
	};
	ld (a0, a1, a2, 0);
#pragma unroll
	for (int i0 = 0; i0 < RVC_T; i0 += 16) {
		ld (b0, b1, b2, i0 + 8);
		run (a0, a1, a2, i0);
		if (i0 + 16 < RVC_T)
			ld (a0, a1, a2, i0 + 16);
		run (b0, b1, b2, i0 + 8);
	}
	PRIO_DOWN ();
}

struct RvPreLds {
	double   x[2][RVC_ROWS][RVC_S]; /* predelayed input -> biquadA output, in place */
	uint32_t f[2][RVC_ROWS][RVC_S]; /* fpdL / fpdR of the sample delayM back (the predelay's input guard) */
};

/* predelay, denormal guard, biquadA, sin (x * wet) (src/reverb.cpp:339-375) -> rvA.
 * The predelay ring slot read at sample m holds the input of sample m - delayM guarded
 * with that sample's dither state (or 0 while m < delayM), so the kernel reads the input
 * delayM samples back, from this chunk's mid1 or the history of earlier chunks
 * (TBF_PD_HIST), and the dither wave runs the stream delayM samples behind.
 * A tile is loaded at iteration k (its HBM reads issued at k - 2), filtered at k + 1 and
 * stored at k + 2.  Each role runs its own loop with the same barriers.  The HBM reads
 * are unconditional (indices clamped): a read under a branch joins its register with the
 * old value, and that copy waits for the read right away. */
__global__ void __launch_bounds__ (RVC_THREADS)
k_rv_pre (const tbf_launch P, const tbf_inst_const* __restrict__ cst, const tbf_seg_ctl* __restrict__ ctl)
{
	__shared__ RvPreLds sm;
	const int      w = __builtin_amdgcn_readfirstlane (threadIdx.x >> 6), lane = threadIdx.x & (NL - 1);
	const uint32_t inst0 = P.instBase + blockIdx.x * RVC_CB;
	if (inst0 >= P.nInst)
		return;
	const int nj  = (int)min ((uint32_t)RVC_CB, P.nInst - inst0);
	const int nT  = (int)P.nBlocks * (TBF_BLK / RVC_T);
	const int nIt = nT + 2;
	/* waves 0, 1: lane = chain 2 j + c */
	const int     cj = lane >> 1, cc = lane & 1;
	const bool    cok = cj < nj;
	const int     crow = lane < RVC_NC ? lane : RVC_NC; /* chain lanes past the block's chains: the idle row */
	tbf_rv_state* CS  = &P.st[inst0 + (cok ? cj : 0)].rv;
	if (w == 0) {
		const double* cf   = cst[inst0 + (cok ? cj : 0)].bq[0];
		const double  c[1][5] = {{cf[0], cf[1], cf[2], cf[3], cf[4]}};
		double        s[1][2] = {{CS->bq[0][2 * cc], CS->bq[0][2 * cc + 1]}};
		__syncthreads ();
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
			if (it >= 1 && it - 1 < nT) { /* biquadA of tile it - 1 */
				double* const row[1] = {sm.x[(it - 1) & 1][crow]};
				rvc_serial<1> (row, c, s);
			}
			__syncthreads ();
		}
		if (cok) {
			CS->bq[0][2 * cc]     = s[0][0];
			CS->bq[0][2 * cc + 1] = s[0][1];
		}
		return;
	}
	if (w == 1) {
		/* the dither stream delayM samples behind: it advances only over samples whose
		 * delayed input exists (instance age >= delayM) */
		const int d    = cst[inst0 + (cok ? cj : 0)].delay[12];
		const int age0 = min (max (CS->pdAge, 0), d);
		uint32_t  fs   = cc ? CS->fpdR : CS->fpdL;
		auto      row  = [&] (int k) {
            const int lead = min (max (d - age0 - k * RVC_T, 0), RVC_T); /* samples with no input yet */
            uint32_t* f    = sm.f[k & 1][crow];
#pragma unroll 8
            for (int n = 0; n < RVC_T; n++) {
                f[n] = fs;
                fs   = n >= lead ? xs_step (fs) : fs;
            }
		};
		if (nT > 0)
			row (0);
		__syncthreads ();
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
			if (it + 1 < nT)
				row (it + 1);
			__syncthreads ();
		}
		if (cok) {
			if (cc)
				CS->fpdR = fs;
			else
				CS->fpdL = fs;
		}
		return;
	}
	/* helpers: task t = instance h + RVC_H t (wave-uniform); lane = channel hc, sample n.
	 * HBM reads run two tiles ahead, into two register sets that alternate by iteration
	 * parity (the loop is unrolled by two, so the sets stay static) */
	const int    h = w - 2, hc = lane >> 5, n = lane & (RVC_T - 1);
	float        pIn[2][RVC_NTK];
	double       wetv[RVC_NTK];
	int          dM[RVC_NTK], age[RVC_NTK];
	uint32_t     pos[RVC_NTK];
	const float* in[RVC_NTK];
	float*       hst[RVC_NTK]; /* the predelay history */
	double*      ra[RVC_NTK];
	/* the input delayM samples before sample k of the chunk (lane n: k = 32 tile + n) */
	auto src = [&] (int t, int tile) {
		const int p = tile * RVC_T + n - dM[t];
		return p >= 0 ? in[t] + p : hst[t] + ((pos[t] + (uint32_t)p) & (TBF_PD_HIST - 1));
	};
#pragma unroll
	for (int t = 0; t < RVC_NTK; t++) {
		const int             j    = h + t * RVC_H;
		const uint32_t        inst = inst0 + (j < nj ? j : nj - 1);
		const tbf_inst_const& K    = cst[inst];
		const tbf_rv_state&   S    = P.st[inst].rv;
		hst[t]  = (float*)(P.rslab + (size_t)inst * P.slabLen + K.ringOff[12]);
		in[t]   = P.mid1 + (size_t)inst * P.midStride;
		ra[t]   = rv_buf (P.rvA, P, inst, hc) + n;
		dM[t]   = K.delay[12];
		age[t]  = min (max (S.pdAge, 0), dM[t]);
		pos[t]  = S.pdPos;
		wetv[t] = rvc_wet_lanes (P, ctl, inst);
		pIn[0][t] = *src (t, 0);
		pIn[1][t] = *src (t, min (1, nT - 1));
	}
	__syncthreads ();
	auto step = [&] (const int it, float (&qIn)[RVC_NTK]) {
		const int b = it & 1; /* tiles it and it - 2 share the buffer */
		double    sv[RVC_NTK];
		/* the filtered tile it - 2, read before tile it overwrites it */
#pragma unroll
		for (int t = 0; t < RVC_NTK; t++)
			sv[t] = sm.x[b][2 * (h + t * RVC_H) + hc][n];
		/* tile it: the predelayed samples (src/reverb.cpp:339-358): the input delayM back,
		 * guarded with its dither state, or the zeroed ring's 0 before the instance's
		 * first delayM samples */
		if (it < nT) {
#pragma unroll
			for (int t = 0; t < RVC_NTK; t++) {
				const int r = 2 * (h + t * RVC_H) + hc;
				double    x = (double)qIn[t];
				if (fabs (x) < 1.18e-23)
					x = sm.f[b][r][n] * 1.18e-17;
				const double xv = age[t] + it * RVC_T + n >= dM[t] ? x : 0.0;
				sm.x[b][r][n] = xv;
			}
		}
		/* HBM reads of tile it + 2 into the set just consumed (clamped past the last tile:
		 * a harmless re-read, so the loads need no branch) */
		const int tl = min (it + 2, nT - 1);
#pragma unroll
		for (int t = 0; t < RVC_NTK; t++)
			qIn[t] = *src (t, tl);
		/* sin (x * wet) of tile it - 2 */
		if (it >= 2) {
			const int k2 = it - 2;
			double    sx[RVC_NTK];
#pragma unroll
			for (int t = 0; t < RVC_NTK; t++)
				sx[t] = sv[t] * rld (wetv[t], blk_lane ((k2 * RVC_T) / TBF_BLK));
			/* the tasks' sines in pairs (tbf_sin2: their chains interleave) */
#pragma unroll
			for (int t = 0; t + 1 < RVC_NTK; t += 2) {
				tbf_sin2 (sx[t], sx[t + 1], sx[t], sx[t + 1]);
			}
			if (RVC_NTK & 1)
				sx[RVC_NTK - 1] = tbf_sin (sx[RVC_NTK - 1]);
#pragma unroll
			for (int t = 0; t < RVC_NTK; t++)
				if (h + t * RVC_H < nj)
					ra[t][(size_t)k2 * RVC_T] = sx[t];
		}
		__syncthreads ();
	};
#pragma unroll 1
	for (int it = 0; it < nIt; it += 2) {
		step (it, pIn[0]);
		if (it + 1 < nIt)
			step (it + 1, pIn[1]);
	}
	/* the chunk's last inputs into the history (after every read of it above, in this
	 * wave's program order), the position and the age */
	const int nS = nT * RVC_T;
#pragma unroll
	for (int t = 0; t < RVC_NTK; t++) {
		const int j = h + t * RVC_H;
		if (j >= nj)
			continue;
		for (int m = max (0, nS - TBF_PD_HIST) + lane; m < nS; m += NL)
			hst[t][(pos[t] + (uint32_t)m) & (TBF_PD_HIST - 1)] = in[t][m];
		if (lane == 0) {
			tbf_rv_state& S = P.st[inst0 + j].rv;
			S.pdPos         = (pos[t] + (uint32_t)nS) & (TBF_PD_HIST - 1);
			S.pdAge         = min (age[t] + nS, dM[t]);
		}
	}
}

/* k_rv_post's chain block: RVP_CB instances per workgroup (k_rv_pre keeps RVC_CB) */
#ifndef RVP_CB
#define RVP_CB 16 /* 256 workgroups: all CUs (32 per workgroup: step 129.7 -> 127.5 ms at 16, profiles/r05/s37) */
#endif
#ifndef RVP_PROF
#define RVP_PROF 0 /* profiling variant (never the product): s_memtime work / barrier clocks per role (tools/rvp_prof.py) */
#endif
#if RVP_PROF /* workgroup 0's serial, dither and first helper waves write k cycles over instance 0's first outputs (tap chain) */
#define RVP_PROF_DECL() unsigned long long pw_ = 0, pb_ = 0, pa_ = 0, pc_ = 0
#define RVP_T0() pa_ = __builtin_amdgcn_s_memtime ()
#define RVP_T1() { asm volatile ("" ::: "memory"); pc_ = __builtin_amdgcn_s_memtime (); pw_ += pc_ - pa_; }
#define RVP_T2() { asm volatile ("" ::: "memory"); pb_ += __builtin_amdgcn_s_memtime () - pc_; }
#define RVP_PROF_OUT(i) { if (blockIdx.x == 0 && lane == 0) { \
	if ((i) >= 0) { P.outL[P.outOffset + (i)] = (float)(pw_ * 1e-3); P.outL[P.outOffset + (i) + 1] = (float)(pb_ * 1e-3); } \
	P.outL[P.outOffset + 16 + 3 * w] = (float)(pw_ * 1e-3); P.outL[P.outOffset + 17 + 3 * w] = (float)(pb_ * 1e-3); \
	P.outL[P.outOffset + 18 + 3 * w] = (float)((__builtin_amdgcn_s_getreg ((31 << 11) | 4) >> 4) & 3); } }
#else
#define RVP_PROF_DECL()
#define RVP_T0()
#define RVP_T1()
#define RVP_T2()
#define RVP_PROF_OUT(i)
#endif
#ifndef RVP_H
#define RVP_H 8 /* helper waves */
#endif
#define RVP_NC (2 * RVP_CB)
#define RVP_ROWS (RVP_NC + (RVP_NC < NL)) /* chain rows, + one that the idle chain lanes use */
#define RVP_NTK (RVP_CB / RVP_H)
static_assert (RVP_CB % RVP_H == 0 && RVP_NC <= NL, "k_rv_post chain-block geometry");

#define RVP_SER 2                                   /* serial chain waves (biquadB, biquadC) */
#define RVP_THREADS (NL * (RVP_SER + 1 + RVP_H))    /* + the dither wave and the helpers */

struct RvPostLds {
	double   y[2][RVP_ROWS][RVC_S]; /* tap mix x c0 -> biquadB output, in place */
	double   z[2][RVP_ROWS][RVC_S]; /* asin output x c0 -> biquadC output, in place */
	double   y1[2][RVP_ROWS][RVC_S], y2[2][RVP_ROWS][RVC_S]; /* x c1, x c2 of the tap mix */
	double   z1[2][RVP_ROWS][RVC_S], z2[2][RVP_ROWS][RVC_S]; /* x c1, x c2 of the asin output */
	uint32_t f[2][RVP_ROWS][RVC_S]; /* fpdL / fpdR before each sample (entry RVC_T: after the tile) */
};

/* biquadB, clamp + asin, biquadC, dry mix, dither, (L + R) / sqrt 2 (src/reverb.cpp:733-787)
 * -> mid2.  A tile is loaded at iteration k (its HBM reads issued at k - 2), biquadB at
 * k + 1, asin at k + 2, biquadC at k + 3, output at k + 4.  Wave 0 runs the
 * biquadB chains, wave 1 the biquadC chains (one chain per lane each; one wave with both
 * interleaved was the kernel's bound, 4.2 k cycles an iteration against 1.4 k for the
 * helpers), wave 2 the dither streams, and the helpers write each input's three products. */
__global__ void __launch_bounds__ (RVP_THREADS)
k_rv_post (const tbf_launch P, const tbf_inst_const* __restrict__ cst, const tbf_seg_ctl* __restrict__ ctl)
{
	__shared__ RvPostLds sm;
	const int      w = __builtin_amdgcn_readfirstlane (threadIdx.x >> 6), lane = threadIdx.x & (NL - 1);
	const uint32_t inst0 = P.instBase + blockIdx.x * RVP_CB;
	if (inst0 >= P.nInst)
		return;
	const int     nj  = (int)min ((uint32_t)RVP_CB, P.nInst - inst0);
	const int     nT  = (int)P.nBlocks * (TBF_BLK / RVC_T);
	const int     nIt = nT + 4;
	const int     cj = lane >> 1, cc = lane & 1;
	const bool    cok = cj < nj;
	const int     crow = lane < RVP_NC ? lane : RVP_NC; /* chain lanes past the block's chains: the idle row */
	tbf_rv_state* CS  = &P.st[inst0 + (cok ? cj : 0)].rv;
	if (w < 2) {
		/* w 0: biquadB of tile it - 1 (rows y); w 1: biquadC of tile it - 3 (rows z) */
		const tbf_inst_const& K  = cst[inst0 + (cok ? cj : 0)];
		const int             q  = w + 1;
		const double          c3 = K.bq[q][3], c4 = K.bq[q][4];
		double                s7 = CS->bq[q][2 * cc], s8 = CS->bq[q][2 * cc + 1];
		__syncthreads ();
		RVP_PROF_DECL ();
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
			RVP_T0 ();
			const int tile = it - 1 - 2 * w;
			if (tile >= 0 && tile < nT) {
				const int pb = (it - 1) & 1;
				if (w == 0)
					rvc_serial_p (sm.y[pb][crow], sm.y1[pb][crow], sm.y2[pb][crow], c3, c4, s7, s8);
				else
					rvc_serial_p (sm.z[pb][crow], sm.z1[pb][crow], sm.z2[pb][crow], c3, c4, s7, s8);
			}
			RVP_T1 ();
			__syncthreads ();
			RVP_T2 ();
		}
		RVP_PROF_OUT (w == 0 ? 0 : -1);
		if (cok) {
			CS->bq[q][2 * cc]     = s7;
			CS->bq[q][2 * cc + 1] = s8;
		}
		return;
	}
	if (w == RVP_SER) {
		uint32_t fs = cc ? CS->fpdR2 : CS->fpdL2;
		__syncthreads ();
		RVP_PROF_DECL ();
#pragma unroll 1
		for (int it = 0; it < nIt; it++) {
			RVP_T0 ();
			if (it >= 3 && it - 3 < nT)
				rvc_dither_row (sm.f[(it - 3) & 1][crow], fs);
			RVP_T1 ();
			__syncthreads ();
			RVP_T2 ();
		}
		RVP_PROF_OUT (4);
		if (cok) {
			if (cc)
				CS->fpdR2 = fs;
			else
				CS->fpdL2 = fs;
		}
		return;
	}
	/* helpers: HBM reads two tiles ahead into two register sets alternating by iteration
	 * parity (see k_rv_pre) */
	const bool   tap = P.chain == TBF_CHAIN_TAP_REVERB;
	const int    h = w - RVP_SER - 1, hc = lane >> 5, n = lane & (RVC_T - 1);
	double       pB[2][RVP_NTK], wetv[RVP_NTK];
	float        pIn[2][RVP_NTK];
	const double* rb[RVP_NTK];
	const float*  in[RVP_NTK];
	float*        out[RVP_NTK];
	double       cB[RVP_NTK][3], cC[RVP_NTK][3]; /* the task's biquadB / biquadC input coefficients c0 c1 c2 */
#pragma unroll
	for (int t = 0; t < RVP_NTK; t++) {
		const int      j    = h + t * RVP_H;
		const uint32_t inst = inst0 + (j < nj ? j : nj - 1);
		rb[t]     = rv_buf (P.rvB, P, inst, hc) + n;
		in[t]     = P.mid1 + (size_t)inst * P.midStride + n;
		out[t]    = tap ? (hc ? P.outR : P.outL) + (size_t)inst * P.outStride + P.outOffset + n
		                : P.mid2 + (size_t)inst * P.midStride + n;
		wetv[t]   = rvc_wet_lanes (P, ctl, inst);
		pB[0][t]  = rb[t][0];
		pB[1][t]  = rb[t][(size_t)min (1, nT - 1) * RVC_T];
		pIn[0][t] = pIn[1][t] = 0.f;
		for (int k = 0; k < 3; k++) {
			cB[t][k] = cst[inst].bq[1][k];
			cC[t][k] = cst[inst].bq[2][k];
		}
	}
	__syncthreads ();
	RVP_PROF_DECL ();
	auto step = [&] (const int it, double (&qB)[RVP_NTK], float (&qIn)[RVP_NTK]) {
		RVP_T0 ();
		const int b = it & 1; /* tiles it, it - 2 and it - 4 share the buffers */
		/* output of tile it - 4: dry mix, dither, mono sum (src/reverb.cpp:766-787); the
		 * half-waves hold L and R, and 0.7071 (L + R) == 0.7071 (R + L) */
		float yv[RVP_NTK];
		if (it >= 4) {
			const int ob = blk_lane (((it - 4) * RVC_T) / TBF_BLK);
#pragma unroll
			for (int t = 0; t < RVP_NTK; t++) {
				const double wet = rld (wetv[t], ob);
				const int    r   = 2 * (h + t * RVP_H) + hc;
				double       x   = sm.z[b][r][n];
				if (wet != 1.0) {
					double dry = (double)qIn[t];
					if (fabs (dry) < 1.18e-23)
						dry = sm.f[b][r][n] * 1.18e-17;
					x += (dry * (1.0 - wet));
				}
				const double ov = dither_add (x, sm.f[b][r][n + 1]);
				const double ow = __shfl_xor (ov, 32);
				yv[t]           = (float)(0.7071067811865476 * (ov + ow));
			}
		}
		/* clamp + asin of tile it - 2 (src/reverb.cpp:743-751); the tap mix of tile it,
		 * which reuses the biquadB buffer, after the reads */
		double av[RVP_NTK];
#pragma unroll
		for (int t = 0; t < RVP_NTK; t++)
			av[t] = sm.y[b][2 * (h + t * RVP_H) + hc][n];
		if (it < nT) {
#pragma unroll
			for (int t = 0; t < RVP_NTK; t++) {
				const int r = 2 * (h + t * RVP_H) + hc;
				sm.y[b][r][n]  = qB[t] * cB[t][0];
				sm.y1[b][r][n] = qB[t] * cB[t][1];
				sm.y2[b][r][n] = qB[t] * cB[t][2];
			}
		}
		/* HBM reads into the set just consumed (indices clamped, so the loads need no
		 * branch): the tap mix of tile it + 2, the dry input of tile it - 2 (output at
		 * iteration it + 2) */
		const int tb = min (it + 2, nT - 1), ti = max (0, min (it - 2, nT - 1));
#pragma unroll
		for (int t = 0; t < RVP_NTK; t++) {
			qB[t]  = rb[t][(size_t)tb * RVC_T];
			qIn[t] = in[t][(size_t)ti * RVC_T];
		}
		if (it >= 2 && it - 2 < nT) {
			double y[RVP_NTK];
			bool   small = true;
#pragma unroll
			for (int t = 0; t < RVP_NTK; t++) {
				y[t] = av[t];
				if (y[t] > 1.0)
					y[t] = 1.0;
				if (y[t] < -1.0)
					y[t] = -1.0;
				small = small && fabs (y[t]) < 0.5;
			}
			/* every task's value inside OCML asin's polynomial branch (the tap mix is small):
			 * that branch alone, straight-line, so the tasks' chains interleave (tbf_sin.h) */
			double as[RVP_NTK];
			if (__all (small)) {
#pragma unroll
				for (int t = 0; t < RVP_NTK; t++)
					as[t] = tbf_asin_poly (y[t]);
			} else {
#pragma unroll
				for (int t = 0; t < RVP_NTK; t++)
					as[t] = asin (y[t]);
			}
#pragma unroll
			for (int t = 0; t < RVP_NTK; t++) {
				const int r = 2 * (h + t * RVP_H) + hc;
				sm.z[b][r][n]  = as[t] * cC[t][0];
				sm.z1[b][r][n] = as[t] * cC[t][1];
				sm.z2[b][r][n] = as[t] * cC[t][2];
			}
		}
		if (it >= 4) {
			const size_t so = (size_t)(it - 4) * RVC_T;
#pragma unroll
			for (int t = 0; t < RVP_NTK; t++)
				if (h + t * RVP_H < nj && (tap || hc == 0))
					out[t][so] = yv[t];
		}
		RVP_T1 ();
		__syncthreads ();
		RVP_T2 ();
	};
#pragma unroll 1
	for (int it = 0; it < nIt; it += 2) {
		step (it, pB[0], pIn[0]);
		if (it + 1 < nIt)
			step (it + 1, pB[1], pIn[1]);
	}
	RVP_PROF_OUT (h == 0 ? 8 : -1);
}

/* ================================================================== k_whirl */
#ifndef WH_EXPECT
#define WH_EXPECT 1 /* rare paths (bypass, horn A catching up, a wrapped drum window, the rotor-angle and
                     * motion replays, a new parameter set) marked unlikely: the common case falls through */
#endif
#if WH_EXPECT
#define WH_RARE(x) __builtin_expect (!!(x), 0)
#else
#define WH_RARE(x) (x)
#endif
__device__ void whirl_speed (tbf_wh_state& st, const tbf_inst_const& K, int revOpt, int& brake)
{
	/* the rotor state in registers: its LDS reads issued together, not one per branch */
	double hornAngle = st.hornAngle, drumAngle = st.drumAngle, hornIncr = st.hornIncr, drumIncr = st.drumIncr;
	double hornTarget = st.hornTarget, drumTarget = st.drumTarget;
	int    hornAcDc = st.hornAcDc, drumAcDc = st.drumAcDc;
	const double hnBrakePos = st.prm.hnBrakePos, drBrakePos = st.prm.drBrakePos;
	/* useRevOption (src/whirl.cpp:174-196) for an event landing before this block */
	if (revOpt >= 0) {
		const int i   = revOpt % 9;
		hornTarget = K.revHorn[i];
		drumTarget = K.revDrum[i];
		if (hornIncr < hornTarget)
			hornAcDc = 1;
		else if (hornTarget < hornIncr)
			hornAcDc = -1;
		if (drumIncr < drumTarget)
			drumAcDc = 1;
		else if (drumTarget < drumIncr)
			drumAcDc = -1;
	}
	/* src/whirl.cpp:1219-1374 */
	if (hornAcDc) {
		int flywheel = 0;
		if (hnBrakePos > 0 && hornTarget == 0 && hornIncr > 0 && hornIncr < K.hnHardstop) {
			const double targetPos = fmod (1.25 - hnBrakePos, 1.0);
			if (fabs (hornAngle - targetPos) < (2.0 / 16384)) {
				hornAngle = targetPos;
				hornIncr  = 0;
			} else {
				const float diffinc = (float)(fmod (1. + targetPos - hornAngle, 1.0) / (float)TBF_BLK);
				if (hornIncr > diffinc)
					hornIncr = diffinc;
				else if (hornIncr < K.minspeed)
					hornIncr = K.minspeed;
				flywheel = 1;
			}
		}
		if (!flywheel) {
			const double l = hornAcDc > 0 ? st.prm.lAcc[0] : st.prm.lAcc[1];
			hornIncr += (1 - l) * (hornTarget - hornIncr);
		}
		if (fabs (hornTarget - hornIncr) < K.deadzone) {
			hornAcDc = 0;
			hornIncr = hornTarget;
		}
	}
	if (drumAcDc) {
		int flywheel = 0;
		if (drBrakePos > 0 && drumTarget == 0 && drumIncr > 0 && drumIncr < K.drHardstop) {
			const double targetPos = fmod (drBrakePos + .75, 1.0);
			if (fabs (drumAngle - targetPos) < (2.0 / 16384)) {
				drumAngle = targetPos;
				drumIncr  = 0;
			} else {
				const float diffinc = (float)(fmod (1. + targetPos - drumAngle, 1.0) / (float)TBF_BLK);
				if (drumIncr > diffinc)
					drumIncr = diffinc;
				else if (drumIncr < K.minspeed)
					drumIncr = K.minspeed;
				flywheel = 1;
			}
		}
		if (!flywheel) {
			const double l = drumAcDc > 0 ? st.prm.lAcc[2] : st.prm.lAcc[3];
			drumIncr += (1 - l) * (drumTarget - drumIncr);
		}
		if (fabs (drumTarget - drumIncr) < K.deadzone) {
			drumAcDc = 0;
			drumIncr = drumTarget;
		}
	}
	brake = 0;
	if (hnBrakePos > 0) {
		const double targetPos = fmod (1.25 - hnBrakePos, 1.0);
		if (!hornAcDc && hornIncr == 0 && hornAngle != targetPos) {
			brake |= 1;
			if (fabs (hornAngle - targetPos) < (2.0 / 16384)) {
				hornAngle = targetPos;
			} else {
				hornIncr = fmod (1. + targetPos - hornAngle, 1.0) / (float)TBF_BLK;
				if (hornIncr > K.hnLimit)
					hornIncr = K.hnLimit;
			}
		}
	}
	if (drBrakePos > 0) {
		const double targetPos = fmod (drBrakePos + .75, 1.0);
		if (!drumAcDc && drumIncr == 0 && drumAngle != targetPos) {
			brake |= 2;
			if (fabs (drumAngle - targetPos) < (2.0 / 16384)) {
				drumAngle = targetPos;
			} else {
				drumIncr = fmod (1. + targetPos - drumAngle, 1.0) / (float)TBF_BLK;
				if (drumIncr > K.drLimit)
					drumIncr = K.drLimit;
			}
		}
	}
	st.hornAngle  = hornAngle;
	st.drumAngle  = drumAngle;
	st.hornIncr   = hornIncr;
	st.drumIncr   = drumIncr;
	st.hornTarget = hornTarget;
	st.drumTarget = drumTarget;
	st.hornAcDc   = hornAcDc;
	st.drumAcDc   = drumAcDc;
}

/* One pass of motion_add over a group of RG rings (motion q of each): every lane reads its
 * two slots of every ring, then the owners write them.  So the rings' reads go out
 * together and the pass costs one LDS round trip.  The owner and neighbour relations of
 * motion_own are lane masks here: the fast path's precondition vote already compared each
 * slot with the previous lane's, eqm (U_n == U_n-1) and s1m (U_n == U_n-1 + 1), and every
 * other relation is a shift of those (pair: eq of the next lane, lead2: eq of the previous
 * one, own2: s1 of the lane after the group), so they cost scalar instructions and the
 * selects take them as lane masks.  The same adds in the same order as motion_add. */
__device__ __forceinline__ bool lane_in (uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64 (m); }

template <int W, int RG>
__device__ __forceinline__ void motion_pass (float (*ring)[W + WH_PAD], const int (&mu)[RG][3], const float (&ma)[RG][3],
                                             const float (&mb)[RG][3], const uint64_t (&eqm)[RG][3],
                                             const uint64_t (&s1m)[RG][3], const int q)
{
	const uint32_t WM = (uint32_t)W - 1u;
	uint32_t       i0[RG], i1[RG];
	float          v[RG], w[RG];
#pragma unroll
	for (int gi = 0; gi < RG; gi++) {
		i0[gi] = (uint32_t)mu[gi][q] & WM;
		i1[gi] = ((uint32_t)mu[gi][q] + 1u) & WM;
		v[gi]  = ring[gi][i0[gi]];
		w[gi]  = ring[gi][i1[gi]];
	}
#pragma unroll
	for (int gi = 0; gi < RG; gi++) {
		const uint64_t eq = eqm[gi][q], s1 = s1m[gi][q];
		const uint64_t pair = eq >> 1, lead = s1, lead2 = eq << 1;
		const uint64_t own2 = ~((pair & (s1 >> 2)) | (~pair & (s1 >> 1)));
		const float    a = ma[gi][q], b = mb[gi][q];
		const float    bp1 = lane_shr1 (b), bp2 = lane_shr1 (bp1), an = lane_shl1 (a), bn = lane_shl1 (b);
		float          x  = v[gi] + bp2;
		float          nv = lane_in (lead & lead2) ? x : v[gi];
		x                 = nv + bp1;
		nv                = lane_in (lead) ? x : nv;
		nv += a;
		x  = nv + an;
		nv = lane_in (pair) ? x : nv;
		float nw = w[gi] + b;
		x        = nw + bn;
		nw       = lane_in (pair) ? x : nw;
		if (lane_in (~eq))
			ring[gi][i0[gi]] = nv;
		if (lane_in (~eq & own2))
			ring[gi][i1[gi]] = nw;
	}
}

/* one DF2 state recurrence (EQ_IIR, src/whirl.cpp:1479-1485) over a sub-block in one lane:
 * temp[i] = (x[i] - a1 temp[i-1]) - a2 temp[i-2], written over x[i].  Element i of the row
 * is r[i], or with WRAP r[(base + i) & m] (a ring window that wraps); read in groups of
 * eight before their temps are written.  The outputs y = (temp b0 + b1 temp[-1]) + b2
 * temp[-2] are lane-parallel afterwards (wh_outputs).  scrub applies the block-end NaN
 * scrub (src/whirl.cpp:1622-1630) to the incoming state first. */
template <bool WRAP>
__device__ __forceinline__ void wh_serial (float* r, uint32_t base, uint32_t m, float* fz, float a1, float a2, bool scrub)
{
	float z0 = fz[0], z1 = fz[1];
	if (scrub) {
		if (isnan (z0))
			z0 = 0.f;
		if (isnan (z1))
			z1 = 0.f;
	}
#if WH_SERIAL_PIPE
	/* two register sets of eight: the next group's reads are in flight while this group's
	 * recurrence runs (the groups' elements are distinct, so no read passes a write of its
	 * own element) */
	auto ld = [&] (float (&v)[8], int i0) {
#pragma unroll
		for (int k = 0; k < 8; k++)
			v[k] = WRAP ? r[(base + (uint32_t)(i0 + k)) & m] : r[i0 + k];
	};
	auto run = [&] (float (&v)[8], int i0) {
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const float t = v[k] - (a1 * z0) - (a2 * z1);
			z1            = z0;
			z0            = t;
			v[k]          = t;
		}
#pragma unroll
		for (int k = 0; k < 8; k++) {
			if (WRAP)
				r[(base + (uint32_t)(i0 + k)) & m] = v[k];
			else
				r[i0 + k] = v[k];
		}
	};
	float xa[8], xb[8];
	ld (xa, 0);
#pragma unroll
	for (int i0 = 0; i0 < TBF_SUB; i0 += 16) {
		ld (xb, i0 + 8);
		run (xa, i0);
		if (i0 + 16 < TBF_SUB)
			ld (xa, i0 + 16);
		run (xb, i0 + 8);
	}
#else
	for (int i0 = 0; i0 < TBF_SUB; i0 += 8) {
		float xv[8];
#pragma unroll
		for (int k = 0; k < 8; k++)
			xv[k] = WRAP ? r[(base + (uint32_t)(i0 + k)) & m] : r[i0 + k];
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const float t = xv[k] - (a1 * z0) - (a2 * z1);
			z1            = z0;
			z0            = t;
			xv[k]         = t;
		}
#pragma unroll
		for (int k = 0; k < 8; k++) {
			if (WRAP)
				r[(base + (uint32_t)(i0 + k)) & m] = xv[k];
			else
				r[i0 + k] = xv[k];
		}
	}
#endif
	fz[0] = z0;
	fz[1] = z1;
}

/* wh_serial<false> on a 16-B aligned row, 4 samples per LDS read / write (ds_read_b128 /
 * ds_write_b128: 32 LDS instructions per pass instead of 128); the same operations in the
 * same order, the next group of 8 read while this one's recurrence runs */
__device__ __forceinline__ void wh_serial_v (float* r, float* fz, float a1, float a2, bool scrub)
{
	float z0 = fz[0], z1 = fz[1];
	if (scrub) {
		if (isnan (z0))
			z0 = 0.f;
		if (isnan (z1))
			z1 = 0.f;
	}
	PRIO_UP ();
	float4* r4  = (float4*)r;
	auto    run = [&] (float4 (&v)[2], int g) {
		float x[8] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w};
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const float t = x[k] - (a1 * z0) - (a2 * z1);
			z1            = z0;
			z0            = t;
			x[k]          = t;
		}
		r4[2 * g]     = make_float4 (x[0], x[1], x[2], x[3]);
		r4[2 * g + 1] = make_float4 (x[4], x[5], x[6], x[7]);
	};
	float4 xa[2], xb[2];
	xa[0] = r4[0];
	xa[1] = r4[1];
#pragma unroll
	for (int g = 0; g < TBF_SUB / 8; g += 2) {
		xb[0] = r4[2 * g + 2];
		xb[1] = r4[2 * g + 3];
		run (xa, g);
		if (g + 2 < TBF_SUB / 8) {
			xa[0] = r4[2 * g + 4];
			xa[1] = r4[2 * g + 5];
		}
		run (xb, g + 1);
	}
	PRIO_DOWN ();
	fz[0] = z0;
	fz[1] = z1;
}

/* the filter outputs, lane n = sample n: t = temp[n], z0 / z1 = the state the pass started
 * from (temp[-1], temp[-2]); the neighbours' temps by DPP lane shifts */
__device__ __forceinline__ float wh_output (float t, float z0, float z1, const float* c)
{
	const float t1 = lane_shr1_or (t, z0);  /* temp[n-1] */
	const float t2 = lane_shr1_or (t1, z1); /* temp[n-2] */
	return (t * c[2]) + (c[3] * t1) + (c[4] * t2);
}

/* A sub-block's two output stores, held back until the next sub-block has issued its
 * motion-table loads: vmcnt retires in issue order, so a store issued before a load is
 * waited for with it, and every sub-block waits for its table loads (and every block for
 * its input) -- with the stores issued first, each of those waits also waited out the
 * previous stores' write latency. */
struct WhOut {
	float* l;
	float* r;
	float  vl, vr;
};

/* the held stores; unconditional (a store under a branch makes the wait counts after it
 * unknown, and the compiler then waits for everything) */
__device__ __forceinline__ void wh_flush (const WhOut& o)
{
	*o.l = o.vl;
	*o.r = o.vr;
}

/* whirlProc2 (src/whirl.cpp:1191-1638) + whirlProc3 mic mix (1653-1681).  in0 / in1: this
 * block's input (samples lane, lane + 64); the next block's is loaded from inNext into
 * nx0 / nx1 during the first sub-block (inNext may be this block's own input when there
 * is no next block: a harmless re-read) */
template <int W>
__device__ void stage_whirl (const tbf_launch& P, WhLds<W>& sm, const bool bypass, const int revOpt, const tbf_inst_const& K,
                             const float in0, const float in1, const float* __restrict__ inNext, float& nx0, float& nx1,
                             const bool hasNext, float* __restrict__ oL, float* __restrict__ oR, WhOut& pend)
{
	const int     lane  = threadIdx.x;
	tbf_wh_state& st    = sm.st;
	const float*  hnFwd = P.whTab;
	const float*  hnBwd = P.whTab + TBF_WH_TSTRIDE;
	const float*  drFwd = P.whTab + 2 * TBF_WH_TSTRIDE;
	const float*  drBwd = P.whTab + 3 * TBF_WH_TSTRIDE;
	const float*  bfw   = P.whBw;
	const float*  bbw   = P.whBw + 16384 * 5;

	if (WH_RARE (bypass)) {
		/* whirlProc2 bypass (src/whirl.cpp:1197-1215) + whirlProc3 mix */
		nx0 = inNext[lane];
		nx1 = inNext[lane + NL];
		wh_flush (pend);
		oL[lane] = in0 * K.mic[0] + in0 * K.mic[1] + 0.f * K.mic[2] + 0.f * K.mic[3];
		oR[lane] = in0 * K.mic[4] + in0 * K.mic[5] + 0.f * K.mic[6] + 0.f * K.mic[7];
		/* the second sub-block's outputs become the held stores, so that the held
		 * stores always carry the latest output of their lane (a later flush of an older
		 * one would overwrite a newer value) */
		pend.l  = oL + NL + lane;
		pend.r  = oR + NL + lane;
		pend.vl = in1 * K.mic[0] + in1 * K.mic[1] + 0.f * K.mic[2] + 0.f * K.mic[3];
		pend.vr = in1 * K.mic[4] + in1 * K.mic[5] + 0.f * K.mic[6] + 0.f * K.mic[7];
		return;
	}
	if (lane == 0) {
		int brake;
		/* a control entry carrying a rotary selection is used for exactly one block */
		whirl_speed (st, K, revOpt, brake);
		sm.brake = brake;
	}
	wave_sync ();
	const double   hornIncr = st.hornIncr, drumIncr = st.drumIncr;
	const uint32_t WM       = (uint32_t)W - 1u;
	/* the horn filters' coefficients of this block (the runtime set in the state); serial
	 * filter coefficients: lane 0 horn A, lane 1 horn B, lanes 2-3 drum shelf */
	float ha[5], hb[5];
#pragma unroll
	for (int j = 0; j < 5; j++) {
		ha[j] = st.prm.hafw[j];
		hb[j] = st.prm.hbfw[j];
	}
	/* a1, a2 of the serial lanes' recurrences: lane 0 horn A, lane 1 horn B, lanes 2-3 drum shelves */
	const float fa0 = lane == 0 ? ha[0] : (lane == 1 ? hb[0] : K.drf[0]);
	const float fa1 = lane == 0 ? ha[1] : (lane == 1 ? hb[1] : K.drf[1]);

	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const int      n      = lane;
		const uint32_t outpos = (st.outpos + (uint32_t)n) & 2047u;
		const int32_t  unwrap = (int32_t)(st.outpos + (uint32_t)n - outpos); /* 0 or 2048 */
		const float    xin    = (float)((double)(sb == 0 ? in0 : in1) + 1e-14);
		/* ring reads + clear at outpos: before this sub-block's writes, which land >= 79
		 * slots ahead (src/whirl.cpp:1585-1600); the drum rings' outputs are read by the
		 * shelves in place first */
		const uint32_t o   = outpos & WM;
		const float    hlv = sm.wring[0][o], hrv = sm.wring[1][o];
		sm.wring[0][o]     = 0.f;
		sm.wring[1][o]     = 0.f;
		if (lane < 4) {
			const int i = lane;
			sm.xf[i] = st.adx[0][(st.adi[0] + 3 - i) & 7];
			sm.x1[i] = st.adx[1][(st.adi[1] + 3 - i) & 7];
			sm.x2[i] = st.adx[2][(st.adi[2] + 3 - i) & 7];
		}
		/* DF2 biquads: horn B runs on horn A's output, so A runs one sub-block ahead and
		 * one serial pass advances A over the next sub-block (lane 0), B over this one into
		 * xf (lane 1) and the drum shelves over this one's ring outputs, in place (lanes 2,
		 * 3).  A's own pass over this sub-block runs only when it is not ahead (launch
		 * start, after a bypassed block or a new coefficient set). */
		const int  ap    = sm.ap;
		const bool aNext = sb + 1 < TBF_BLK / TBF_SUB || hasNext;
#ifndef WH_ABL_HORN
		if (WH_RARE (!sm.aReady))
			sm.ab[ap ^ 1][n] = xin;
		if (aNext)
			sm.ab[ap][n] = (float)((double)(sb + 1 < TBF_BLK / TBF_SUB ? in1 : nx0) + 1e-14);
		wave_sync ();
		if (WH_RARE (!sm.aReady)) {
			const float z0 = st.fz[0][0], z1 = st.fz[0][1];
#ifndef WH_NO_SERIAL
			if (lane == 0)
				wh_serial_v (sm.ab[ap ^ 1], st.fz[0], ha[0], ha[1], false);
#endif
			wave_sync ();
			sm.ab[ap ^ 1][n] = wh_output (sm.ab[ap ^ 1][n], z0, z1, ha);
			wave_sync ();
		}
#endif
		/* the states the pass starts from (horn A's scrubbed when it crosses into the next block) */
		const bool scrubA = sb + 1 == TBF_BLK / TBF_SUB;
		float      zs[4][2];
#pragma unroll
		for (int f = 0; f < 4; f++) {
			zs[f][0] = st.fz[f][0];
			zs[f][1] = st.fz[f][1];
		}
		if (scrubA) {
			zs[0][0] = isnan (zs[0][0]) ? 0.f : zs[0][0];
			zs[0][1] = isnan (zs[0][1]) ? 0.f : zs[0][1];
		}
		const uint32_t wb   = st.outpos & WM; /* the drum rings' window: wave-uniform */
		const bool     wrap = wb + TBF_SUB > (uint32_t)W;
#ifdef WH_NO_SERIAL /* timing experiment only (wrong output): k_whirl without its serial filter passes */
		if (false) {
#elif defined(WH_ABL_HORN) /* timing experiment only (wrong output): horn filters A, B not run in k_whirl */
		if (lane >= 2 && lane < 4) {
#else
		if (lane < 4 && (lane > 0 || aNext)) {
#endif
			float* row = lane == 0 ? sm.ab[ap] : (lane == 1 ? sm.ab[ap ^ 1] : sm.wring[lane]);
			if (WH_RARE (wrap))
				wh_serial<true> (row, lane < 2 ? 0u : wb, lane < 2 ? ~0u : WM, st.fz[lane], fa0, fa1, lane == 0 && scrubA);
			else
				wh_serial_v (row + (lane < 2 ? 0u : wb), st.fz[lane], fa0, fa1, lane == 0 && scrubA);
		}
		wave_sync ();
		/* the filter outputs: horn B -> xf, horn A of the next sub-block in place, the drum
		 * shelves' (then the ring slots are cleared) */
#ifdef WH_ABL_HORN
		sm.xf[4 + n] = xin;
#else
		sm.xf[4 + n] = wh_output (sm.ab[ap ^ 1][n], zs[1][0], zs[1][1], hb);
		if (aNext)
			sm.ab[ap][n] = wh_output (sm.ab[ap][n], zs[0][0], zs[0][1], ha);
#endif
		const float dL = wh_output (sm.wring[2][o], zs[2][0], zs[2][1], K.drf);
		const float dR = wh_output (sm.wring[3][o], zs[3][0], zs[3][1], K.drf);
		sm.wring[2][o] = 0.f;
		sm.wring[3][o] = 0.f;
		if (lane == 0) {
			sm.aReady = aNext;
			sm.ap     = ap ^ 1;
		}
		/* rotor angles, angle = fmod (angle + incr, 1) per sample (src/whirl.cpp:1428-1429):
		 * inside one binade of the angle every sum lands on the same grid, so the run is
		 * a0 + n D exactly (phase_run); otherwise lanes 1, 2 replay the recurrence into
		 * the (consumed) filter scratch */
		double ha, da;
		{
			double       Dh, Dd;
			const double h0 = st.hornAngle, d0 = st.drumAngle;
			const bool   frc = (P.dbg & TBF_DEBUG_FORCE_SERIAL) != 0;
			const bool   okh = phase_run (h0, hornIncr, TBF_SUB, Dh) && !frc;
			const bool   okd = phase_run (d0, drumIncr, TBF_SUB, Dd) && !frc;
			ha = h0 + (double)n * Dh;
			da = d0 + (double)n * Dd;
			double he = h0 + (double)TBF_SUB * Dh, de = d0 + (double)TBF_SUB * Dd;
			if (WH_RARE (!(okh && okd))) { /* wave-uniform: every lane replays the recurrence, lane n keeps step n */
				if (lane == 0)
					atomicOr (P.errFlags, (uint32_t)TBF_PATH_WH_ANGLE);
				double a = h0, b = d0;
				for (int i = 0; i < TBF_SUB; i++) {
					if (!okh && n == i)
						ha = a;
					if (!okd && n == i)
						da = b;
					a = wrap1 (a + hornIncr);
					b = wrap1 (b + drumIncr);
				}
				he = okh ? he : a;
				de = okd ? de : b;
			}
			wave_sync (); /* every lane has read the start angles */
			if (lane == 0) {
				st.hornAngle = he;
				st.drumAngle = de;
			}
		}
		wave_sync ();
		/* reflection filters FILTER_C (src/whirl.cpp:1472-1477), lane-parallel */
		const float xf   = sm.xf[n + 4];
		const float xfp  = n == 0 ? st.z[0] : sm.xf[n + 3];
		const float x1v  = (float)((0.4 * xf) + (0.4 * xfp));
		sm.x1[n + 4]     = x1v;
		const float xdp  = lane_shr1_or (xin, st.z[2]); /* the previous sample's input */
		const float xd1v = (float)((0.4 * xin) + (0.4 * xdp));
		wave_sync ();
		const float x1p  = n == 0 ? st.z[1] : sm.x1[n + 3];
		const float x2v  = (float)((0.4 * x1v) + (0.4 * x1p));
		sm.x2[n + 4]     = x2v;
		const float xd1p = lane_shr1_or (xd1v, st.z[3]);
		const float xd2v = (float)((0.4 * xd1v) + (0.4 * xd1p));
		wave_sync ();

		/* ---- rings (HL, HR, DL, DR) in groups of WH_RG: the group's motions first (their
		 * table loads in flight together), then each ring's ordered adds ---- */
#pragma unroll
		for (int r0 = 0; r0 < 4; r0 += WH_RG) {
			int   mu[WH_RG][3];
			float ma[WH_RG][3], mb[WH_RG][3];
			/* the table positions of all 12 motions, then every table load (18) in flight
			 * together, then the arithmetic: issued motion by motion, each motion's loads
			 * were waited for before the next motion's were issued */
			float h1v[WH_RG][3];
#pragma unroll
			for (int gi = 0; gi < WH_RG; gi++)
#pragma unroll
				for (int q = 0; q < 3; q++) {
					const int p = ((r0 + gi) & 1) + 2 * q;
					/* x 16384 is exact (a power of two), so one fma rounds once where the
					 * reference's multiply-then-add rounds once: the same double */
					if (r0 + gi < 2) /* HN_MOTION, src/whirl.cpp:1434 */
						h1v[gi][q] = (float)__builtin_fma (ha + ((p & 1) ? K.bwAng : K.fwAng), 16384.0, (double)K.hornPhase[p]);
					else /* DR_MOTION, src/whirl.cpp:1457 */
						h1v[gi][q] = (float)__builtin_fma (da, 16384.0, (double)K.hornPhase[p]);
				}
			f2u   dpv[WH_RG][3];
			f4u   b4v[2][3];
			float b5v[2][3];
#pragma unroll
			for (int gi = 0; gi < WH_RG; gi++)
#pragma unroll
				for (int q = 0; q < 3; q++) {
					const int      p   = ((r0 + gi) & 1) + 2 * q;
					const bool     fwd = (p == 0 || p == 3 || p == 4);
					const float*   dsp = r0 + gi < 2 ? (fwd ? hnFwd : hnBwd) : (fwd ? drFwd : drBwd);
					const unsigned hl  = ((unsigned int)floorf (h1v[gi][q])) & 16383u;
					dpv[gi][q]         = *(const f2u*)(dsp + hl); /* dsp[hl], dsp[(hl + 1) & 16383] */
					if (r0 + gi < 2) {
						const unsigned kk = ((unsigned int)roundf (h1v[gi][q])) & 16383u;
						const float*   b  = (fwd ? bbw : bfw) + 5 * kk;
						b4v[gi][q]        = *(const f4u*)b;
						b5v[gi][q]        = b[4];
					}
				}
			/* behind the table loads: the next block's input (used from the second
			 * sub-block on; the second sub-block loads it again, so that every sub-block
			 * issues the same memory operations in the same order and each wait is
			 * counted exactly) and the previous sub-block's output stores */
			if (r0 == 0) {
				nx0 = inNext[lane];
				nx1 = inNext[lane + NL];
				wh_flush (pend);
			}
#pragma unroll
			for (int gi = 0; gi < WH_RG; gi++) {
				const int r = r0 + gi;
#pragma unroll
				for (int q = 0; q < 3; q++) {
					const int   p  = (r & 1) + 2 * q;
					const float h1 = h1v[gi][q], hd = frac1 (h1);
					const f2u   dp = dpv[gi][q];
					const float intp = dp.x * (1.f - hd) + hd * dp.y;
					float       xa, t;
					if (r < 2) {
						/* HN_MOTION, src/whirl.cpp:1432-1453 */
						const float* hist = p < 2 ? sm.xf : (p < 4 ? sm.x1 : sm.x2);
						const f4u    b4   = b4v[gi][q];
						t                 = K.hornSpacing[p] + intp + (float)outpos;
						xa                = b4.x * hist[n + 4];
						xa += b4.y * hist[n + 3];
						xa += b4.z * hist[n + 2];
						xa += b4.w * hist[n + 1];
						xa += b5v[gi][q] * hist[n + 0];
					} else {
						/* DR_MOTION, src/whirl.cpp:1455-1469 */
						xa = p < 2 ? xin : (p < 4 ? xd1v : xd2v);
						t  = K.drumSpacing[p] + intp + (float)outpos;
					}
					const float rr = floorf (t);
					const float qq = xa * (t - rr);
					mu[gi][q]      = (int32_t)((unsigned int)rr) + unwrap;
					ma[gi][q]      = xa - qq;
					mb[gi][q]      = qq;
				}
			}
			/* fast path preconditions (wave votes), per ring: each motion's slot
			 * non-decreasing in n with groups of <= 2 equal slots, and the ring's motions
			 * >= 2 slots apart in source order at every sample (so passes farthest-first
			 * keep the per-slot order: a farther motion reaches a slot only at earlier
			 * samples) */
			bool okr[WH_RG];
			bool allOk = !(P.dbg & TBF_DEBUG_FORCE_SERIAL);
			/* as wave ballots, whose masks the passes reuse: eq (slot == previous lane's),
			 * s1 (slot == previous lane's + 1); monotone = no lane below its predecessor,
			 * groups <= 2 = no two consecutive eq bits */
			uint64_t eqm[WH_RG][3], s1m[WH_RG][3];
#pragma unroll
			for (int gi = 0; gi < WH_RG; gi++) {
				const bool ok = (mu[gi][1] >= mu[gi][0] + 2) && (mu[gi][2] >= mu[gi][1] + 2);
				uint64_t   bad = ~__ballot (ok);
#pragma unroll
				for (int q = 0; q < 3; q++) {
					const int      U  = mu[gi][q];
					const int      Up = lane_shr1 (U);
					const uint64_t e  = __ballot (U == Up) & ~1ull; /* lane 0 has no previous sample */
					bad |= (__ballot (U < Up) & ~1ull) | (e & (e >> 1));
					eqm[gi][q] = e;
					s1m[gi][q] = __ballot (U == Up + 1) & ~1ull;
				}
				okr[gi] = bad == 0 && !(P.dbg & TBF_DEBUG_FORCE_SERIAL);
				allOk   = allOk && okr[gi];
			}
			if (!WH_RARE (!allOk)) {
				/* every ring on its fast path: the rings are independent, so each pass
				 * (farthest motion first) updates all of them in one LDS round trip */
#pragma unroll
				for (int q = 2; q >= 0; q--) {
					motion_pass<W, WH_RG> (sm.wring + r0, mu, ma, mb, eqm, s1m, q);
					wave_sync ();
				}
			} else {
#pragma unroll
				for (int gi = 0; gi < WH_RG; gi++) {
					float* ring = sm.wring[r0 + gi];
					if (okr[gi]) {
						motion_add<W> (ring, mu[gi][2], ma[gi][2], mb[gi][2], lane);
						wave_sync ();
						motion_add<W> (ring, mu[gi][1], ma[gi][1], mb[gi][1], lane);
						wave_sync ();
						motion_add<W> (ring, mu[gi][0], ma[gi][0], mb[gi][0], lane);
						wave_sync ();
					} else {
						/* serial replay in the reference order: sample-major, motions in source order */
						if (lane == 0)
							atomicOr (P.errFlags, (uint32_t)TBF_PATH_WH_MOTION);
						for (int i = 0; i < TBF_SUB; i++) {
		#pragma unroll
							for (int q = 0; q < 3; q++) {
								const uint32_t sl = (uint32_t)__shfl (mu[gi][q], i) & WM;
								const float    aa = __shfl (ma[gi][q], i);
								const float    bb = __shfl (mb[gi][q], i);
								if (lane == 0) {
									ring[sl] += aa;
									ring[(sl + 1) & WM] += bb;
								}
							}
						}
						wave_sync ();
					}
				}
			}
		}
		/* ---- outputs (whirlProc2 outHL/outHR/outDL/outDR + whirlProc3 mix) ---- */
		{
			const float leak = xf * K.leakage;
			const float hL   = K.hornLevel * hlv + leak;
			const float hR   = K.hornLevel * hrv + leak;
			pend.l           = oL + sb * TBF_SUB + n;
			pend.r           = oR + sb * TBF_SUB + n;
			pend.vl          = hL * K.mic[0] + hR * K.mic[1] + dL * K.mic[2] + dR * K.mic[3];
			pend.vr          = hL * K.mic[4] + hR * K.mic[5] + dL * K.mic[6] + dR * K.mic[7];
		}
		/* ---- carry filter taps and histories ---- */
		if (lane == NL - 1) {
			st.z[0] = xf;
			st.z[1] = x1v;
			st.z[2] = xin;
			st.z[3] = xd1v;
		}
		wave_sync ();
		if (lane < 24) { /* history k = lane / 8, entry j = lane % 8, one lane each */
			const int    k = lane >> 3, j = lane & 7;
			const float* h = k == 0 ? sm.xf : (k == 1 ? sm.x1 : sm.x2);
			st.adx[k][(st.adi[k] + j) & 7] = h[4 + TBF_SUB - 1 - j];
		}
		if (lane == 0)
			st.outpos = (st.outpos + TBF_SUB) & 2047u;
		wave_sync ();
	}
	/* NaN scrub (src/whirl.cpp:1622-1630), a lane per value: lanes 0..7 the filter states
	 * fz (horn A's only when it did not run ahead: then it got its scrub when it crossed
	 * into the next block), lanes 8..11 z */
	if (lane < 8) {
		const int f = lane >> 1, j = lane & 1;
		if ((f > 0 || !sm.aReady) && isnan (st.fz[f][j]))
			st.fz[f][j] = 0.f;
	} else if (lane < 12) {
		if (isnan (st.z[lane - 8]))
			st.z[lane - 8] = 0.f;
	}
	if (lane == 0) {
		if (sm.brake & 1) st.hornIncr = 0;
		if (sm.brake & 2) st.drumIncr = 0;
	}
	wave_sync ();
}

static_assert (sizeof (tbf_wh_params) % 4 == 0 && sizeof (tbf_wh_params) <= 4 * NL, "one dword per lane");

template <int W>
__global__ void __attribute__ ((amdgpu_flat_work_group_size (NL, NL), amdgpu_waves_per_eu (W <= 512 ? WH_WAVES : (W <= 1024 ? 2 : 1))))
k_whirl (const tbf_launch P, const tbf_inst_const* __restrict__ cst, const tbf_seg_ctl* __restrict__ ctl)
{
	__shared__ WhLds<W> sm;
	const uint32_t inst = blockIdx.x + P.instBase;
	if (inst >= P.nInst)
		return;
	const tbf_inst_const& K  = cst[inst];
	tbf_wh_state*         S  = &P.st[inst].wh;
	float*                wr = P.wring + (size_t)inst * 4 * W;
	copy_words (&sm.st, S);
	if (threadIdx.x == 0) {
		sm.aReady = 0;
		sm.ap     = 0;
	}
	for (uint32_t i = threadIdx.x; i < 4u * W; i += NL)
		sm.wring[i / W][i % W] = wr[i];
	wave_sync ();
	/* the input (lane n: samples n and n + 64 of a block) is loaded one block ahead, in
	 * the block's first sub-block behind its table loads (stage_whirl), so its latency
	 * overlaps a whole sub-block and no wait for it waits for output stores */
	const float* inBase = P.mid2 + (size_t)inst * P.midStride;
	/* the launch's per-block control (bypass, rotary selection), lane b = block b (<= 64
	 * blocks): read once, so no block waits on the two dependent control loads */
	int byv = 0, rvv = -1, wsv = 0;
	if (threadIdx.x < P.nBlocks) {
		const tbf_seg_ctl& Gb = ctl_of (P, ctl, threadIdx.x, inst);
		byv                   = Gb.whBypass != 0;
		rvv                   = Gb.whRevOption;
		wsv                   = (int)Gb.whSet;
	}
	float c0 = 0.f, c1 = 0.f;
	if (P.nBlocks > 0) {
		c0 = inBase[threadIdx.x];
		c1 = inBase[threadIdx.x + NL];
	}
	/* before the first sub-block's outputs exist, the held store writes 0 to the first
	 * output sample of the lane, which the real output overwrites later (same lane, same
	 * address: in order) */
	WhOut pend;
	pend.l  = P.outL + (size_t)inst * P.outStride + P.outOffset + threadIdx.x;
	pend.r  = P.outR + (size_t)inst * P.outStride + P.outOffset + threadIdx.x;
	pend.vl = pend.vr = 0.f;
	for (uint32_t blk = 0; blk < P.nBlocks; blk++) {
		float*     oL = P.outL + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		float*     oR = P.outR + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		float      n0, n1;
		const bool more = blk + 1 < P.nBlocks;
		/* a new parameter set (MIDI control functions) from this block on */
		const int ws = rl (wsv, blk_lane ((int)blk));
		if (WH_RARE (ws)) {
			const uint32_t* src = (const uint32_t*)(P.whSets + (ws - 1));
			if (threadIdx.x < sizeof (tbf_wh_params) / 4)
				((uint32_t*)&sm.st.prm)[threadIdx.x] = src[threadIdx.x];
			wave_sync ();
		}
		/* horn filter A may run ahead into the next block unless that one is bypassed or
		 * changes its coefficients */
		const int  nx      = blk_lane ((int)blk + 1);
		const bool hasNext = more && !rl (byv, nx) && !rl (wsv, nx);
		stage_whirl<W> (P, sm, rl (byv, blk_lane ((int)blk)) != 0, rl (rvv, blk_lane ((int)blk)), K, c0, c1,
		                inBase + (size_t)(more ? blk + 1 : blk) * TBF_BLK, n0, n1, hasNext, oL, oR, pend);
		c0 = n0;
		c1 = n1;
	}
	if (P.nBlocks > 0)
		wh_flush (pend);
	wave_sync ();
	copy_words (S, &sm.st);
	for (uint32_t i = threadIdx.x; i < 4u * W; i += NL)
		wr[i] = sm.wring[i / W][i % W];
}

/* ------------------------------------------------------------------ k_whirl_split
 * k_whirl with two waves per instance: the horn wave (rings HL, HR: horn filters A / B,
 * FILTER_C on the horn signal, the six HN_MOTIONs, the outputs and mic mix) and the drum
 * wave (rings DL, DR: the drum shelves, FILTER_C on the input, the six DR_MOTIONs).  The
 * two halves of whirlProc2 share nothing within a block but the drum outputs dL / dR,
 * which the drum wave leaves in its ring slots at outpos (just consumed by the shelves)
 * and the horn wave reads after one workgroup barrier per sub-block; the drum wave clears
 * those slots after the next barrier, before its own adds of that sub-block (the adds land
 * >= 79 slots ahead and the ring holds write-ahead + 68 slots, so an add of sub-block k + 1
 * may wrap into window k only after it is cleared).  Each rotor's speed update is its own
 * half of whirl_speed.  So every instance is two waves of about half the instructions
 * (a latency-bound kernel: one wave alone per SIMD ran 7.1 ms per 512 blocks against 9.4
 * at 4 per SIMD, profiles/r05/s26), and the same operations in the same order as k_whirl.
 * The engine launches it where it wins as rendered: rings of 1024 or 2048 samples (k_whirl's
 * LDS leaves it 2 / 1 waves per SIMD; the 96 kHz bench 156.4 -> 151.5 ms per step) and at
 * most one instance per CU (real-time periods: 128 frames p50 0.213 -> 0.208 ms).  Alone it
 * is faster up to 8 instances per CU too (6.34 vs 7.20 ms per 512 blocks at 2048 instances),
 * but rendered beside the other stages the 2048-instance step went 77.6 -> 91.3 ms; at 4096
 * k_whirl's 4 waves per SIMD win outright (9.4 against 14.5 ms in two rounds).
 * profiles/r05/s29, s30. */

#ifndef WHS_WAVES
#define WHS_WAVES 4 /* k_whirl_split waves per SIMD at the 512-sample ring: 128 VGPRs, 8 instances per CU (at 8
                      * per SIMD, 64 VGPRs, all 4096 at once but with spills in the sub-block loop: slower) */
#endif
/* a wave-uniform value moved to scalar registers */
__device__ __forceinline__ float sgpr_f (float v) { return __int_as_float (__builtin_amdgcn_readfirstlane (__float_as_int (v))); }
__device__ __forceinline__ double sgpr_d (double v)
{
	const unsigned long long u = __double_as_longlong (v);
	const unsigned long long lo = (unsigned)__builtin_amdgcn_readfirstlane ((int)(unsigned)u);
	const unsigned long long hi = (unsigned)__builtin_amdgcn_readfirstlane ((int)(unsigned)(u >> 32));
	return __longlong_as_double ((long long)(lo | (hi << 32)));
}

/* one rotor's half of whirl_speed (src/whirl.cpp:174-235, 1219-1374): the horn's or the
 * drum's fields only; brake = 1 when its brake engaged */
template <bool HORN>
__device__ void whirl_speed_rotor (tbf_wh_state& st, const tbf_inst_const& K, int revOpt, int& brake)
{
	double       angle = HORN ? st.hornAngle : st.drumAngle, incr = HORN ? st.hornIncr : st.drumIncr;
	double       target = HORN ? st.hornTarget : st.drumTarget;
	int          acdc   = HORN ? st.hornAcDc : st.drumAcDc;
	const double brakePos = HORN ? st.prm.hnBrakePos : st.prm.drBrakePos;
	if (revOpt >= 0) {
		const int i = revOpt % 9;
		target      = HORN ? K.revHorn[i] : K.revDrum[i];
		if (incr < target)
			acdc = 1;
		else if (target < incr)
			acdc = -1;
	}
	if (acdc) {
		int flywheel = 0;
		if (brakePos > 0 && target == 0 && incr > 0 && incr < (HORN ? K.hnHardstop : K.drHardstop)) {
			const double targetPos = HORN ? fmod (1.25 - brakePos, 1.0) : fmod (brakePos + .75, 1.0);
			if (fabs (angle - targetPos) < (2.0 / 16384)) {
				angle = targetPos;
				incr  = 0;
			} else {
				const float diffinc = (float)(fmod (1. + targetPos - angle, 1.0) / (float)TBF_BLK);
				if (incr > diffinc)
					incr = diffinc;
				else if (incr < K.minspeed)
					incr = K.minspeed;
				flywheel = 1;
			}
		}
		if (!flywheel) {
			const double l = acdc > 0 ? st.prm.lAcc[HORN ? 0 : 2] : st.prm.lAcc[HORN ? 1 : 3];
			incr += (1 - l) * (target - incr);
		}
		if (fabs (target - incr) < K.deadzone) {
			acdc = 0;
			incr = target;
		}
	}
	brake = 0;
	if (brakePos > 0) {
		const double targetPos = HORN ? fmod (1.25 - brakePos, 1.0) : fmod (brakePos + .75, 1.0);
		if (!acdc && incr == 0 && angle != targetPos) {
			brake = 1;
			if (fabs (angle - targetPos) < (2.0 / 16384)) {
				angle = targetPos;
			} else {
				incr = fmod (1. + targetPos - angle, 1.0) / (float)TBF_BLK;
				if (incr > (HORN ? K.hnLimit : K.drLimit))
					incr = HORN ? K.hnLimit : K.drLimit;
			}
		}
	}
	if (HORN) {
		st.hornAngle  = angle;
		st.hornIncr   = incr;
		st.hornTarget = target;
		st.hornAcDc   = acdc;
	} else {
		st.drumAngle  = angle;
		st.drumIncr   = incr;
		st.drumTarget = target;
		st.drumAcDc   = acdc;
	}
}

/* a rotor's angles over a sub-block: lane n gets the angle of sample n (phase_run's closed
 * form, or the literal fmod recurrence replayed); the angle after the sub-block is stored */
__device__ __forceinline__ double wh_angles (const tbf_launch& P, double& stAngle, const double incr, const int n)
{
	double       D;
	const double a0 = stAngle;
	const bool   ok = phase_run (a0, incr, TBF_SUB, D) && !(P.dbg & TBF_DEBUG_FORCE_SERIAL);
	double       an = a0 + (double)n * D, ae = a0 + (double)TBF_SUB * D;
	if (!ok) { /* wave-uniform: every lane replays the recurrence, lane n keeps step n */
		if (n == 0)
			atomicOr (P.errFlags, (uint32_t)TBF_PATH_WH_ANGLE);
		double a = a0;
		for (int i = 0; i < TBF_SUB; i++) {
			if (n == i)
				an = a;
			a = wrap1 (a + incr);
		}
		ae = a;
	}
	wave_sync (); /* every lane has read the start angle */
	if (n == 0)
		stAngle = ae;
	wave_sync ();
	return an;
}

/* the three motions of one ring (HORN: HL or HR, else DL or DR; gi = the ring's channel)
 * and their ordered adds: k_whirl's ring group for one ring, so that a wave holds one
 * ring's motions at a time (the split kernel's waves have 64 VGPRs) */
template <int W, bool HORN>
__device__ __forceinline__ void wh_ring (const tbf_launch& P, WhLds<W>& sm, const tbf_inst_const& K, const double hb,
                                         const int gi, const uint32_t outpos, const int32_t unwrap, const float xin,
                                         const float xd1v, const float xd2v)
{
	const int      n  = threadIdx.x & (NL - 1), lane = n;
	const uint32_t WM = (uint32_t)W - 1u;
	const float*   tF = P.whTab + (HORN ? 0 : 2) * TBF_WH_TSTRIDE;
	const float*   tB = tF + TBF_WH_TSTRIDE;
	float*         ring = sm.wring[(HORN ? 0 : 2) + gi];
	int            mu[1][3];
	float          ma[1][3], mb[1][3], h1v[3];
#pragma unroll
	for (int q = 0; q < 3; q++) { /* HN_MOTION src/whirl.cpp:1434 / DR_MOTION 1457, the fma exact (see k_whirl) */
		/* the phase converted here: hoisted out of the sub-block loop, the six converted
		 * doubles held 12 VGPRs across it and spilled */
		int ph = K.hornPhase[gi + 2 * q];
		asm volatile ("" : "+s"(ph));
		h1v[q] = (float)__builtin_fma (hb, 16384.0, (double)ph);
	}
	f2u   dpv[3];
	f4u   b4v[3];
	float b5v[3];
#pragma unroll
	for (int q = 0; q < 3; q++) {
		const int      p   = gi + 2 * q;
		const bool     fwd = (p == 0 || p == 3 || p == 4);
		const unsigned hl  = ((unsigned int)floorf (h1v[q])) & 16383u;
		dpv[q]             = *(const f2u*)((fwd ? tF : tB) + hl); /* tab[hl], tab[(hl + 1) & 16383] */
		if (HORN) {
			const unsigned kk = ((unsigned int)roundf (h1v[q])) & 16383u;
			const float*   b  = (fwd ? P.whBw + 16384 * 5 : P.whBw) + 5 * kk;
			b4v[q]            = *(const f4u*)b;
			b5v[q]            = b[4];
		}
	}
#pragma unroll
	for (int q = 0; q < 3; q++) {
		const int   p    = gi + 2 * q;
		const float hd   = frac1 (h1v[q]);
		const float intp = dpv[q].x * (1.f - hd) + hd * dpv[q].y;
		float       xa, t;
		if (HORN) { /* HN_MOTION, src/whirl.cpp:1432-1453 */
			const float* hist = p < 2 ? sm.xf : (p < 4 ? sm.x1 : sm.x2);
			t                 = K.hornSpacing[p] + intp + (float)outpos;
			xa                = b4v[q].x * hist[n + 4];
			xa += b4v[q].y * hist[n + 3];
			xa += b4v[q].z * hist[n + 2];
			xa += b4v[q].w * hist[n + 1];
			xa += b5v[q] * hist[n + 0];
		} else { /* DR_MOTION, src/whirl.cpp:1455-1469 */
			xa = p < 2 ? xin : (p < 4 ? xd1v : xd2v);
			t  = K.drumSpacing[p] + intp + (float)outpos;
		}
		const float rr = floorf (t);
		const float qq = xa * (t - rr);
		mu[0][q]       = (int32_t)((unsigned int)rr) + unwrap;
		ma[0][q]       = xa - qq;
		mb[0][q]       = qq;
	}
	/* the fast path's preconditions as wave ballots whose masks the passes reuse (k_whirl) */
	const bool ok  = (mu[0][1] >= mu[0][0] + 2) && (mu[0][2] >= mu[0][1] + 2);
	uint64_t   bad = ~__ballot (ok);
	uint64_t   eqm[1][3], s1m[1][3];
#pragma unroll
	for (int q = 0; q < 3; q++) {
		const int      U  = mu[0][q];
		const int      Up = lane_shr1 (U);
		const uint64_t e  = __ballot (U == Up) & ~1ull;
		bad |= (__ballot (U < Up) & ~1ull) | (e & (e >> 1));
		eqm[0][q] = e;
		s1m[0][q] = __ballot (U == Up + 1) & ~1ull;
	}
	if (bad == 0 && !(P.dbg & TBF_DEBUG_FORCE_SERIAL)) {
#pragma unroll
		for (int q = 2; q >= 0; q--) {
			motion_pass<W, 1> (reinterpret_cast<float (*)[W + WH_PAD]> (ring), mu, ma, mb, eqm, s1m, q);
			wave_sync ();
		}
		return;
	}
	/* the serial replay in the reference order: sample-major, motions in source order */
	{
		if (lane == 0)
			atomicOr (P.errFlags, (uint32_t)TBF_PATH_WH_MOTION);
		for (int i = 0; i < TBF_SUB; i++) {
#pragma unroll
			for (int q = 0; q < 3; q++) {
				const uint32_t sl = (uint32_t)__shfl (mu[0][q], i) & WM;
				const float    aa = __shfl (ma[0][q], i);
				const float    bb = __shfl (mb[0][q], i);
				if (lane == 0) {
					ring[sl] += aa;
					ring[(sl + 1) & WM] += bb;
				}
			}
		}
		wave_sync ();
	}
}

/* the horn wave's block (whirlProc2's horn half + whirlProc3 mix): outputs via the held stores */
template <int W>
__device__ void whirl_horn (const tbf_launch& P, WhLds<W>& sm, const bool bypass, const int revOpt, const tbf_inst_const& K,
                            const float in0, const float in1, const float* __restrict__ inNext, float& nx0, float& nx1,
                            const bool hasNext, float* __restrict__ oL, float* __restrict__ oR, WhOut& pend, uint32_t& opos)
{
	const int     lane = threadIdx.x & (NL - 1), n = lane;
	tbf_wh_state& st   = sm.st;
	if (WH_RARE (bypass)) {
		/* whirlProc2 bypass (src/whirl.cpp:1197-1215) + whirlProc3 mix (see stage_whirl) */
		nx0 = inNext[lane];
		nx1 = inNext[lane + NL];
		wh_flush (pend);
		oL[lane] = in0 * K.mic[0] + in0 * K.mic[1] + 0.f * K.mic[2] + 0.f * K.mic[3];
		oR[lane] = in0 * K.mic[4] + in0 * K.mic[5] + 0.f * K.mic[6] + 0.f * K.mic[7];
		pend.l   = oL + NL + lane;
		pend.r   = oR + NL + lane;
		pend.vl  = in1 * K.mic[0] + in1 * K.mic[1] + 0.f * K.mic[2] + 0.f * K.mic[3];
		pend.vr  = in1 * K.mic[4] + in1 * K.mic[5] + 0.f * K.mic[6] + 0.f * K.mic[7];
		return;
	}
	int brake = 0;
	if (lane == 0) /* a control entry carrying a rotary selection is used for exactly one block */
		whirl_speed_rotor<true> (st, K, revOpt, brake);
	brake = __builtin_amdgcn_readfirstlane (brake);
	wave_sync ();
	/* wave-uniform values in scalar registers (the split kernel's waves have 64 VGPRs) */
	const double   hornIncr = sgpr_d (st.hornIncr);
	const uint32_t WM       = (uint32_t)W - 1u;
	float          ha[5], hb[5];
#pragma unroll
	for (int j = 0; j < 5; j++) {
		ha[j] = sgpr_f (st.prm.hafw[j]);
		hb[j] = sgpr_f (st.prm.hbfw[j]);
	}
	/* serial lanes: 0 horn A (over the next sub-block), 1 horn B (over this one) */
	const float fa0 = lane == 0 ? ha[0] : hb[0];
	const float fa1 = lane == 0 ? ha[1] : hb[1];
	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const uint32_t outpos = (opos + (uint32_t)n) & 2047u;
		const int32_t  unwrap = (int32_t)(opos + (uint32_t)n - outpos); /* 0 or 2048 */
		const float    xin    = (float)((double)(sb == 0 ? in0 : in1) + 1e-14);
		const uint32_t o      = outpos & WM;
		const float    hlv = sm.wring[0][o], hrv = sm.wring[1][o];
		sm.wring[0][o]     = 0.f;
		sm.wring[1][o]     = 0.f;
		if (lane < 4) {
			const int i = lane;
			sm.xf[i]    = st.adx[0][(st.adi[0] + 3 - i) & 7];
			sm.x1[i]    = st.adx[1][(st.adi[1] + 3 - i) & 7];
			sm.x2[i]    = st.adx[2][(st.adi[2] + 3 - i) & 7];
		}
		/* horn A runs one sub-block ahead (see stage_whirl) */
		const int  ap    = sm.ap;
		const bool aNext = sb + 1 < TBF_BLK / TBF_SUB || hasNext;
		if (WH_RARE (!sm.aReady))
			sm.ab[ap ^ 1][n] = xin;
		if (aNext)
			sm.ab[ap][n] = (float)((double)(sb + 1 < TBF_BLK / TBF_SUB ? in1 : nx0) + 1e-14);
		wave_sync ();
		if (WH_RARE (!sm.aReady)) {
			const float z0 = st.fz[0][0], z1 = st.fz[0][1];
			if (lane == 0)
				wh_serial_v (sm.ab[ap ^ 1], st.fz[0], ha[0], ha[1], false);
			wave_sync ();
			sm.ab[ap ^ 1][n] = wh_output (sm.ab[ap ^ 1][n], z0, z1, ha);
			wave_sync ();
		}
		const bool scrubA = sb + 1 == TBF_BLK / TBF_SUB;
		float      zs[2][2];
#pragma unroll
		for (int f = 0; f < 2; f++) {
			zs[f][0] = st.fz[f][0];
			zs[f][1] = st.fz[f][1];
		}
		if (scrubA) {
			zs[0][0] = isnan (zs[0][0]) ? 0.f : zs[0][0];
			zs[0][1] = isnan (zs[0][1]) ? 0.f : zs[0][1];
		}
		if (lane < 2 && (lane > 0 || aNext))
			wh_serial_v (lane == 0 ? sm.ab[ap] : sm.ab[ap ^ 1], st.fz[lane], fa0, fa1, lane == 0 && scrubA);
		wave_sync ();
		sm.xf[4 + n] = wh_output (sm.ab[ap ^ 1][n], zs[1][0], zs[1][1], hb);
		if (aNext)
			sm.ab[ap][n] = wh_output (sm.ab[ap][n], zs[0][0], zs[0][1], ha);
		if (lane == 0) {
			sm.aReady = aNext;
			sm.ap     = ap ^ 1;
		}
		const double ang = wh_angles (P, st.hornAngle, hornIncr, n);
		/* FILTER_C on the horn signal (src/whirl.cpp:1472-1477) */
		const float xf  = sm.xf[n + 4];
		const float xfp = n == 0 ? st.z[0] : sm.xf[n + 3];
		const float x1v = (float)((0.4 * xf) + (0.4 * xfp));
		sm.x1[n + 4]    = x1v;
		wave_sync ();
		const float x1p = n == 0 ? st.z[1] : sm.x1[n + 3];
		const float x2v = (float)((0.4 * x1v) + (0.4 * x1p));
		sm.x2[n + 4]    = x2v;
		wave_sync ();
		/* behind this sub-block's loads: the next block's input and the held output stores */
		nx0 = inNext[lane];
		nx1 = inNext[lane + NL];
		wh_flush (pend);
		wh_ring<W, true> (P, sm, K, ang + K.fwAng, 0, outpos, unwrap, xin, 0.f, 0.f);
		wh_ring<W, true> (P, sm, K, ang + K.bwAng, 1, outpos, unwrap, xin, 0.f, 0.f);
		/* the drum wave's dL / dR of this sub-block, left in its ring slots at outpos */
		__syncthreads ();
		const float dL = sm.wring[2][o], dR = sm.wring[3][o];
		{
			const float leak = xf * K.leakage;
			const float hL   = K.hornLevel * hlv + leak;
			const float hR   = K.hornLevel * hrv + leak;
			pend.l           = oL + sb * TBF_SUB + n;
			pend.r           = oR + sb * TBF_SUB + n;
			pend.vl          = hL * K.mic[0] + hR * K.mic[1] + dL * K.mic[2] + dR * K.mic[3];
			pend.vr          = hL * K.mic[4] + hR * K.mic[5] + dL * K.mic[6] + dR * K.mic[7];
		}
		if (lane == NL - 1) {
			st.z[0] = xf;
			st.z[1] = x1v;
		}
		wave_sync ();
		if (lane < 24) { /* history k = lane / 8, entry j = lane % 8, one lane each */
			const int    k = lane >> 3, j = lane & 7;
			const float* h = k == 0 ? sm.xf : (k == 1 ? sm.x1 : sm.x2);
			st.adx[k][(st.adi[k] + j) & 7] = h[4 + TBF_SUB - 1 - j];
		}
		opos = (opos + TBF_SUB) & 2047u;
		wave_sync ();
	}
	/* NaN scrub (src/whirl.cpp:1622-1630): the horn filters' states (horn A's only when it did
	 * not run ahead) and z[0..1]; the brake */
	if (lane < 4) {
		const int f = lane >> 1, j = lane & 1;
		if ((f > 0 || !sm.aReady) && isnan (st.fz[f][j]))
			st.fz[f][j] = 0.f;
	} else if (lane < 6) {
		if (isnan (st.z[lane - 4]))
			st.z[lane - 4] = 0.f;
	}
	if (lane == 0 && brake)
		st.hornIncr = 0;
	wave_sync ();
}

/* the drum wave's block (whirlProc2's drum half): dL / dR into the ring slots at outpos */
template <int W>
__device__ void whirl_drum (const tbf_launch& P, WhLds<W>& sm, const bool bypass, const int revOpt, const tbf_inst_const& K,
                            const float in0, const float in1, const float* __restrict__ inNext, float& nx0, float& nx1,
                            uint32_t& opos, int& clr)
{
	const int     lane = threadIdx.x & (NL - 1), n = lane;
	tbf_wh_state& st   = sm.st;
	if (WH_RARE (bypass)) {
		nx0 = inNext[lane];
		nx1 = inNext[lane + NL];
		return;
	}
	int brake = 0;
	if (lane == 0)
		whirl_speed_rotor<false> (st, K, revOpt, brake);
	brake = __builtin_amdgcn_readfirstlane (brake);
	wave_sync ();
	const double   drumIncr = sgpr_d (st.drumIncr);
	const uint32_t WM       = (uint32_t)W - 1u;
	for (int sb = 0; sb < TBF_BLK / TBF_SUB; sb++) {
		const uint32_t outpos = (opos + (uint32_t)n) & 2047u;
		const int32_t  unwrap = (int32_t)(opos + (uint32_t)n - outpos);
		const float    xin    = (float)((double)(sb == 0 ? in0 : in1) + 1e-14);
		const uint32_t o      = outpos & WM;
		/* the shelves over this sub-block's ring outputs, in place (lanes 0, 1: DL, DR) */
		const float z20 = st.fz[2][0], z21 = st.fz[2][1], z30 = st.fz[3][0], z31 = st.fz[3][1];
		const uint32_t wb   = opos & WM; /* wave-uniform */
		const bool     wrap = wb + TBF_SUB > (uint32_t)W;
		if (lane < 2) {
			float* row = sm.wring[2 + lane];
			if (WH_RARE (wrap))
				wh_serial<true> (row, wb, WM, st.fz[2 + lane], K.drf[0], K.drf[1], false);
			else
				wh_serial_v (row + wb, st.fz[2 + lane], K.drf[0], K.drf[1], false);
		}
		wave_sync ();
		const float dL = wh_output (sm.wring[2][o], z20, z21, K.drf);
		const float dR = wh_output (sm.wring[3][o], z30, z31, K.drf);
		sm.wring[2][o] = dL; /* handed to the horn wave */
		sm.wring[3][o] = dR;
		__syncthreads ();
		/* the previous window: the horn wave has read it (it reached this barrier after) */
		if (clr >= 0) {
			sm.wring[2][((uint32_t)clr + (uint32_t)n) & WM] = 0.f;
			sm.wring[3][((uint32_t)clr + (uint32_t)n) & WM] = 0.f;
		}
		clr = (int)wb;
		const double ang = wh_angles (P, st.drumAngle, drumIncr, n);
		/* FILTER_C on the input (src/whirl.cpp:1472-1477), by lane shifts */
		const float xdp  = lane_shr1_or (xin, st.z[2]);
		const float xd1v = (float)((0.4 * xin) + (0.4 * xdp));
		const float xd1p = lane_shr1_or (xd1v, st.z[3]);
		const float xd2v = (float)((0.4 * xd1v) + (0.4 * xd1p));
		nx0 = inNext[lane];
		nx1 = inNext[lane + NL];
		wh_ring<W, false> (P, sm, K, ang, 0, outpos, unwrap, xin, xd1v, xd2v);
		wh_ring<W, false> (P, sm, K, ang, 1, outpos, unwrap, xin, xd1v, xd2v);
		if (lane == NL - 1) {
			st.z[2] = xin;
			st.z[3] = xd1v;
		}
		opos = (opos + TBF_SUB) & 2047u;
		wave_sync ();
	}
	if (lane < 4) {
		const int f = 2 + (lane >> 1), j = lane & 1;
		if (isnan (st.fz[f][j]))
			st.fz[f][j] = 0.f;
	} else if (lane < 6) {
		if (isnan (st.z[lane - 2]))
			st.z[lane - 2] = 0.f;
	}
	if (lane == 0 && brake)
		st.drumIncr = 0;
	wave_sync ();
}

template <int W>
__global__ void __attribute__ ((amdgpu_flat_work_group_size (2 * NL, 2 * NL),
                                amdgpu_waves_per_eu (W <= 512 ? WHS_WAVES : (W <= 1024 ? 4 : 2))))
k_whirl_split (const tbf_launch P, const tbf_inst_const* __restrict__ cst, const tbf_seg_ctl* __restrict__ ctl)
{
	__shared__ WhLds<W> sm;
	const uint32_t inst = blockIdx.x + P.instBase;
	if (inst >= P.nInst)
		return;
	const int             tid  = threadIdx.x, lane = tid & (NL - 1);
	const bool            horn = __builtin_amdgcn_readfirstlane (tid >> 6) == 0;
	const tbf_inst_const& K    = cst[inst];
	tbf_wh_state*         S    = &P.st[inst].wh;
	float*                wr   = P.wring + (size_t)inst * 4 * W;
	for (uint32_t i = (uint32_t)tid; i < sizeof (tbf_wh_state) / 4; i += 2 * NL)
		((uint32_t*)&sm.st)[i] = ((const uint32_t*)S)[i];
	if (tid == 0) {
		sm.aReady = 0;
		sm.ap     = 0;
	}
	for (uint32_t i = (uint32_t)tid; i < 4u * W; i += 2 * NL)
		sm.wring[i / W][i % W] = wr[i];
	__syncthreads ();
	uint32_t     opos   = sm.st.outpos;
	const float* inBase = P.mid2 + (size_t)inst * P.midStride;
	int          byv = 0, rvv = -1, wsv = 0;
	if (lane < (int)P.nBlocks) {
		const tbf_seg_ctl& Gb = ctl_of (P, ctl, (uint32_t)lane, inst);
		byv                   = Gb.whBypass != 0;
		rvv                   = Gb.whRevOption;
		wsv                   = (int)Gb.whSet;
	}
	float c0 = 0.f, c1 = 0.f;
	if (P.nBlocks > 0) {
		c0 = inBase[lane];
		c1 = inBase[lane + NL];
	}
	WhOut pend;
	pend.l  = P.outL + (size_t)inst * P.outStride + P.outOffset + lane;
	pend.r  = P.outR + (size_t)inst * P.outStride + P.outOffset + lane;
	pend.vl = pend.vr = 0.f;
	int clr = -1; /* drum wave: the window whose dL / dR slots await clearing */
	for (uint32_t blk = 0; blk < P.nBlocks; blk++) {
		float*     oL = P.outL + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		float*     oR = P.outR + (size_t)inst * P.outStride + P.outOffset + (size_t)blk * TBF_BLK;
		float      n0, n1;
		const bool more = blk + 1 < P.nBlocks;
		/* a new parameter set from this block on: both waves copy it (the same words; the
		 * other wave is past its last read of the old set, k_whirl_split's barriers) */
		const int ws = rl (wsv, blk_lane ((int)blk));
		if (WH_RARE (ws)) {
			const uint32_t* src = (const uint32_t*)(P.whSets + (ws - 1));
			if (lane < (int)(sizeof (tbf_wh_params) / 4))
				((uint32_t*)&sm.st.prm)[lane] = src[lane];
			wave_sync ();
		}
		const int   nx      = blk_lane ((int)blk + 1);
		const bool  hasNext = more && !rl (byv, nx) && !rl (wsv, nx);
		const bool  byp     = rl (byv, blk_lane ((int)blk)) != 0;
		const int   rev     = rl (rvv, blk_lane ((int)blk));
		const float* inNext = inBase + (size_t)(more ? blk + 1 : blk) * TBF_BLK;
#ifndef WHS_ONLY
		if (horn)
			whirl_horn<W> (P, sm, byp, rev, K, c0, c1, inNext, n0, n1, hasNext, oL, oR, pend, opos);
		else
			whirl_drum<W> (P, sm, byp, rev, K, c0, c1, inNext, n0, n1, opos, clr);
#elif WHS_ONLY == 1
		whirl_horn<W> (P, sm, byp, rev, K, c0, c1, inNext, n0, n1, hasNext, oL, oR, pend, opos);
#else
		whirl_drum<W> (P, sm, byp, rev, K, c0, c1, inNext, n0, n1, opos, clr);
#endif
		c0 = n0;
		c1 = n1;
	}
	if (horn && P.nBlocks > 0)
		wh_flush (pend);
	__syncthreads (); /* the horn wave has read the last window's dL / dR */
	if (!horn && clr >= 0) {
		sm.wring[2][((uint32_t)clr + (uint32_t)lane) & (uint32_t)(W - 1)] = 0.f;
		sm.wring[3][((uint32_t)clr + (uint32_t)lane) & (uint32_t)(W - 1)] = 0.f;
	}
	if (horn && lane == 0)
		sm.st.outpos = opos;
	__syncthreads ();
	for (uint32_t i = (uint32_t)tid; i < sizeof (tbf_wh_state) / 4; i += 2 * NL)
		((uint32_t*)S)[i] = ((const uint32_t*)&sm.st)[i];
	for (uint32_t i = (uint32_t)tid; i < 4u * W; i += 2 * NL)
		wr[i] = sm.wring[i / W][i % W];
}

/* ------------------------------------------------------------------ launch */
/* stage k (0 k_tonegen, 1 k_mixpre, 2 k_rv_pre, 3 k_rv_core, 4 k_rv_post, 5 k_whirl) of one
 * launch chunk; the chain mode decides which stages run (tbf_chain_stages) */
extern "C" int tbf_launch_stage (const tbf_launch* P, int k, hipStream_t stream)
{
	if (P->nInst == 0 || P->nBlocks == 0)
		return 0;
	if ((uint64_t)P->nBlocks * TBF_BLK > P->midStride)
		return -22;
	if ((k == 2 || k == 4 || k == 5) && P->nBlocks > NL && P->ctlIdx) /* per-block controls one per lane (blk_lane) */
		return -22;
	const dim3 grid (P->nInst), block (NL);
	const dim3 cgrid ((P->nInst + RVC_CB - 1) / RVC_CB), cblock (RVC_THREADS);
	if (k == 0)
	{
		const uint32_t ns = P->tgSplit > 1 && !P->ctlIdx ? std::min (P->tgSplit, (uint32_t)TG_SPLIT_MAX) : 1u;
		if (ns > P->nBlocks)
			return -22;
		hipLaunchKernelGGL (k_tonegen, grid, dim3 (NL * ns), ns * sizeof (TgLds), stream, *P, P->ctl, P->tpls, P->cst);
	}
	else if (k == 1)
		hipLaunchKernelGGL (k_mixpre, dim3 ((P->nInst + MP_CB - 1) / MP_CB), dim3 (MP_THREADS), 0, stream, *P, P->ctl);
	else if (k == 2)
		hipLaunchKernelGGL (k_rv_pre, cgrid, cblock, 0, stream, *P, P->cst, P->ctl);
	else if (k == 3)
		/* the LDS kernel loads and stores a channel's 129.7 KB of rings per launch; the
		 * streaming kernel moves 24.6 KB per block: below 8 blocks the streaming one
		 * moves fewer bytes (real-time periods of one or two blocks) */
		if (P->rvLds && P->nBlocks >= RVL_MIN_BLOCKS) {
			if (hipMemsetAsync (P->rvWork, 0, sizeof (uint32_t), stream) != hipSuccess)
				return -5;
			const uint32_t pairs = 2 * (P->nInst - P->instBase);
			hipLaunchKernelGGL (k_rv_core_lds, dim3 (P->rvGrid && P->rvGrid < pairs ? P->rvGrid : pairs), dim3 (RVL_THREADS),
			                    0, stream, *P, P->cst);
		} else
			hipLaunchKernelGGL (k_rv_core, dim3 (2 * P->nInst), block, 0, stream, *P, P->cst);
	else if (k == 4)
		hipLaunchKernelGGL (k_rv_post, dim3 ((P->nInst + RVP_CB - 1) / RVP_CB), dim3 (RVP_THREADS), 0, stream, *P, P->cst, P->ctl);
	else if (k == 5) {
		if (P->whSplit) {
			const dim3 sblock (2 * NL);
			switch (P->wringLen) {
				case 512: hipLaunchKernelGGL (k_whirl_split<512>, grid, sblock, 0, stream, *P, P->cst, P->ctl); break;
				case 1024: hipLaunchKernelGGL (k_whirl_split<1024>, grid, sblock, 0, stream, *P, P->cst, P->ctl); break;
				case 2048: hipLaunchKernelGGL (k_whirl_split<2048>, grid, sblock, 0, stream, *P, P->cst, P->ctl); break;
				default: return -22;
			}
		} else
		switch (P->wringLen) {
			case 512: hipLaunchKernelGGL (k_whirl<512>, grid, block, 0, stream, *P, P->cst, P->ctl); break;
			case 1024: hipLaunchKernelGGL (k_whirl<1024>, grid, block, 0, stream, *P, P->cst, P->ctl); break;
			case 2048: hipLaunchKernelGGL (k_whirl<2048>, grid, block, 0, stream, *P, P->cst, P->ctl); break;
			default: return -22;
		}
	} else
		return -22;
	return hipGetLastError () == hipSuccess ? 0 : -5;
}

/* whether k_rv_core_lds can run an instance with these reverb constants: a channel's 12
 * rings fit its LDS ring and every delay leaves a group's reads clear of its writes */
extern "C" int tbf_rv_lds_fits (const tbf_inst_const* k)
{
	/* tap offsets (sin + 1) * vibDepth < 7: the taps stay inside the staged window (72
	 * slots past count, for the group argument below) and the LDS mirror */
	if (!(k->vibDepth >= 0.0 && 2.0 * k->vibDepth < 7.0))
		return 0;
	for (int l = 0; l < 12; l++) {
		/* a group's reads must find only data written before the group: tap lines read up
		 * to 71 slots past count+1, the allpasses read count+1 */
		if (k->delay[l] < RVL_G * TBF_SUB + (l < 8 ? 72 : 0) || k->delay[l] != RVL_DLY[l])
			return 0;
		for (int c = 0; c < 2; c++)
			if ((int)(k->ringOff[c * 13 + l] - k->ringOff[c * 13]) != RVL_OFS[l])
				return 0;
	}
	return 1;
}

/* number of stages the chain mode runs */
extern "C" int tbf_chain_stages (uint32_t chain)
{
	return chain == TBF_CHAIN_TONEGEN || chain == TBF_CHAIN_TAP_PREAMP ? 2 : (chain == TBF_CHAIN_TAP_REVERB ? 5 : 6);
}
