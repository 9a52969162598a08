/*
 * tbf_calib.hip -- PMC calibration kernels (test hook tbf_debug_calibrate).
 *
 * MI355X_MICROARCH.md: FETCH_SIZE/WRITE_SIZE are calibrated only for 16-B/lane
 * streaming; the reverb ring traffic of tbf_render_kernel is 8-B/lane (64 consecutive
 * doubles per wave instruction).  These kernels stream a known byte count with exactly
 * that pattern so the counters can be converted to bytes for roofline.traffic.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tbf_sin.h"

__global__ void __launch_bounds__ (256) tbf_calib_read_f64 (const double* __restrict__ p, uint64_t n,
                                                          double* __restrict__ sink)
{
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	double         acc    = 0.0;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
		acc += p[i];
	if (acc == 1.2345e300) /* never true for the zero-filled buffer; keeps the loads */
		sink[blockIdx.x] = acc;
}

__global__ void __launch_bounds__ (256) tbf_calib_write_f64 (double* __restrict__ p, uint64_t n)
{
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
		p[i] = (double)i;
}

/* test hook for tbf_sin.h (op 4): buf = n inputs x, then tbf_sin (x), sin (x), tbf_sin2 (x, x'),
 * asin fast path, asin (7 n doubles; x' = the input n / 2 further on) */
__global__ void __launch_bounds__ (256) tbf_check_sin (double* __restrict__ p, uint64_t n)
{
	const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n)
		return;
	const double x = p[i];
	p[n + i]       = tbf_sin (x);
	p[2 * n + i]   = sin (x);
	/* tbf_sin2 on (x, the input n / 2 further on): its results must be the same bits */
	const double x2 = p[(i + n / 2) % n];
	double       r0, r1;
	tbf_sin2 (x, x2, r0, r1);
	p[3 * n + i] = r0;
	p[4 * n + i] = r1;
	/* asin: the polynomial branch where every lane is inside it, else the library */
	const double y = fmin (fmax (x, -1.0), 1.0);
	p[5 * n + i]   = __all (fabs (y) < 0.5) ? tbf_asin_poly (y) : asin (y);
	p[6 * n + i]   = asin (y);
}

/* VALU issue-cost probes (ops 5..12, bench.py VALU_CYC): every wave runs `iters` rounds of 8
 * independent chains of one instruction (inline asm, so the instruction is exactly the
 * one named), enough waves resident for the SIMDs to be issue-bound, not latency-bound.
 * The caller times the launch (HIP events on the stream); wave 0 writes the shader clock
 * it saw (s_memtime cycles over s_memrealtime's 100 MHz ticks) to buf[0..1], so
 * cycles per wave64 instruction per SIMD = time x clock / (waves per SIMD x 32 iters). */
#define CALIB_CHAINS 8
template <int OP>
__global__ void __launch_bounds__ (256) tbf_calib_valu (double* __restrict__ out, uint32_t iters)
{
	const uint64_t t0 = __builtin_amdgcn_s_memtime (), r0 = __builtin_amdgcn_s_memrealtime ();
	double         d[CALIB_CHAINS];
	float          f[CALIB_CHAINS];
	const double   dc = 1.0000001 + 1e-9 * threadIdx.x;
	const float    fc = 1.0001f + 1e-6f * threadIdx.x;
#pragma unroll
	for (int k = 0; k < CALIB_CHAINS; k++) {
		d[k] = 0.5 + 0.01 * k + 1e-7 * threadIdx.x;
		f[k] = 0.5f + 0.01f * k + 1e-5f * threadIdx.x;
	}
	for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
		for (int kr = 0; kr < 4 * CALIB_CHAINS; kr++) { /* 4 rounds of the chains per loop trip */
			const int k = kr % CALIB_CHAINS;
			if (OP == 0) __asm__ __volatile__ ("v_add_f32 %0, %0, %1" : "+v"(f[k]) : "v"(fc));
			if (OP == 1) __asm__ __volatile__ ("v_fma_f32 %0, %0, %1, %1" : "+v"(f[k]) : "v"(fc));
			if (OP == 2) __asm__ __volatile__ ("v_add_f64 %0, %0, %1" : "+v"(d[k]) : "v"(dc));
			if (OP == 3) __asm__ __volatile__ ("v_mul_f64 %0, %0, %1" : "+v"(d[k]) : "v"(dc));
			if (OP == 4) __asm__ __volatile__ ("v_fma_f64 %0, %0, %1, %1" : "+v"(d[k]) : "v"(dc));
			if (OP == 5) __asm__ __volatile__ ("v_sin_f32 %0, %0" : "+v"(f[k]));
			if (OP == 6) __asm__ __volatile__ ("v_rcp_f64 %0, %0" : "+v"(d[k]));
			if (OP == 7) __asm__ __volatile__ ("v_add_u32 %0, %0, %1" : "+v"(f[k]) : "v"(fc));
		}
	}
	double acc = 0.0;
#pragma unroll
	for (int k = 0; k < CALIB_CHAINS; k++)
		acc += d[k] + (double)f[k];
	if (acc == 1.2345e300) /* never: keeps the chains live */
		out[2 + blockIdx.x] = acc;
	if (blockIdx.x == 0 && threadIdx.x == 0) {
		out[0] = (double)(__builtin_amdgcn_s_memtime () - t0);
		out[1] = (double)(__builtin_amdgcn_s_memrealtime () - r0);
	}
}

extern "C" int tbf_launch_calibrate (int op, void* buf, uint64_t n, hipStream_t s)
{
	dim3 grid (4096), block (256);
	if (op == 0)
		hipLaunchKernelGGL (tbf_calib_read_f64, grid, block, 0, s, (const double*)buf, n, (double*)buf);
	else if (op == 1)
		hipLaunchKernelGGL (tbf_calib_write_f64, grid, block, 0, s, (double*)buf, n);
	else if (op == 2) /* the read with every wave's 512 B starting 64 B into a cache line */
		hipLaunchKernelGGL (tbf_calib_read_f64, grid, block, 0, s, (const double*)buf + 8, n - 8, (double*)buf);
	else if (op == 3) /* the write, likewise misaligned */
		hipLaunchKernelGGL (tbf_calib_write_f64, grid, block, 0, s, (double*)buf + 8, n - 8);
	else if (op == 4) /* tbf_sin.h against the library: n inputs, buffer of 7 n doubles */
		hipLaunchKernelGGL (tbf_check_sin, dim3 ((unsigned)((n + 255) / 256)), block, 0, s, (double*)buf, n);
	else if (op >= 5 && op <= 12) {
		/* VALU issue probes: n = iterations; 2048 workgroups of 4 waves = 8 waves per SIMD on
		 * 256 CUs; buf holds >= 2 + 2048 doubles */
		const dim3     g (2048);
		const uint32_t it = (uint32_t)n;
		switch (op - 5) {
			case 0: hipLaunchKernelGGL (tbf_calib_valu<0>, g, block, 0, s, (double*)buf, it); break;
			case 1: hipLaunchKernelGGL (tbf_calib_valu<1>, g, block, 0, s, (double*)buf, it); break;
			case 2: hipLaunchKernelGGL (tbf_calib_valu<2>, g, block, 0, s, (double*)buf, it); break;
			case 3: hipLaunchKernelGGL (tbf_calib_valu<3>, g, block, 0, s, (double*)buf, it); break;
			case 4: hipLaunchKernelGGL (tbf_calib_valu<4>, g, block, 0, s, (double*)buf, it); break;
			case 5: hipLaunchKernelGGL (tbf_calib_valu<5>, g, block, 0, s, (double*)buf, it); break;
			case 6: hipLaunchKernelGGL (tbf_calib_valu<6>, g, block, 0, s, (double*)buf, it); break;
			default: hipLaunchKernelGGL (tbf_calib_valu<7>, g, block, 0, s, (double*)buf, it); break;
		}
	}
	else
		return -22;
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
