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

/* k_tpl_rand + k_tpl_wave over ntpl templates; lsb/bank indexed by base[t] + draw */
extern "C" int tbf_tpl_launch (uint32_t ntpl, uint32_t maxChunks, uint32_t maxLen, const uint32_t* E61,
                               const uint64_t* total, const uint64_t* base, const tbf_tpl_wheel* wh, uint8_t* lsb,
                               float* bank, double sr, hipStream_t s);

#endif
