/* tbf_tpl.h -- device template builder interface (tbf_tpl.hip) */
#ifndef TBF_TPL_H
#define TBF_TPL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tbf_types.h"

/* one wheel's writeSamples spectrum (wheels 1..256 -> index 0..255) */
typedef struct tbf_tpl_wheel {
	uint32_t off, len; /* bank offset (= first rand() draw) and length */
	int32_t  np;       /* nonzero partials */
	uint32_t pad;
	double   U;        /* attenuation / sum |amplitude| */
	double   amp[12], hz[12];
} tbf_tpl_wheel;

/* the play matrix's template-independent inputs on the device (tbf::MatrixInputs) */
typedef struct tbf_tpl_mx {
	const tbf_le*   tm;    /* terminal mix, terminal i's list at tm[tmOff[i] .. tmOff[i + 1]) */
	const uint32_t* tmOff; /* TBF_NW + 2 */
	const tbf_le*   tp;    /* the cfg's taper list of key k at tp[tpOff[k] .. tpOff[k + 1]) */
	const uint32_t* tpOff; /* 385 */
	const tbf_le*   xt;    /* the cfg's crosstalk lists, the same way */
	const uint32_t* xtOff; /* 385 */
	const float*    taper; /* [128][9] manual default levels */
	double          wiringXT, floor, minLevel;
	uint32_t        cap;   /* staging entries per key */
} tbf_tpl_mx;

/* k_tpl_matrix + k_tpl_offsets + k_tpl_gather over ntpl templates: freq [ntpl][TBF_NW]
 * and ratio [ntpl][9] (each template's frequency table and bus ratios); the key lists in
 * stage [ntpl * 384][cap] with their lengths in cnt, then packed: key q = t * 384 + k at
 * out[off[q] .. off[q + 1]) (cnt[q] > cap: the list did not fit, the caller fails) */
extern "C" int tbf_tpl_matrix_launch (uint32_t ntpl, const tbf_tpl_mx* mx, const double* freq, const double* ratio,
                                      tbf_contrib* stage, uint32_t* cnt, uint32_t* off, tbf_contrib* out,
                                      hipStream_t s);

/* k_tpl_rand + k_tpl_wave over ntpl templates; lsb/bank indexed by base[t] + draw */
extern "C" int tbf_tpl_launch (uint32_t ntpl, uint32_t maxChunks, uint32_t maxLen, const uint32_t* E61,
                               const uint64_t* total, const uint64_t* base, const tbf_tpl_wheel* wh, uint8_t* lsb,
                               float* bank, double sr, hipStream_t s);

#endif
