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
	else
		return -22;
	return hipGetLastError () == hipSuccess ? 0 : -5;
}
