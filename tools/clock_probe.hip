// SPDX-License-Identifier: GPL-2.0
/*
 * clock_probe.hip - diagnostic, never the product: the shader clock of one
 * CU over time, while other kernels run.  One wave samples s_memtime (the
 * shader clock counter, clock64()) and s_memrealtime (the 100 MHz counter,
 * wall_clock64()) every `period` realtime ticks into out[2 k], out[2 k + 1],
 * until `max` samples or `ticks` realtime ticks have passed: every path
 * ends, so the grid drains.  Runs beside back-to-back RX launches
 * (tools/clock_trace.py) to tell a clock drop from a memory-side slowdown.
 *
 *   hipcc -O2 --offload-arch=gfx950 -fPIC -shared tools/clock_probe.hip \
 *         -o tools/libclock_probe.so
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void __launch_bounds__(64) clock_probe_kernel(unsigned long long *out, int max,
							  unsigned long long period,
							  unsigned long long ticks)
{
	if (threadIdx.x != 0)
		return;
	const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
	unsigned long long next = r0;
	for (int k = 0; k < max; k++) {
		unsigned long long r = __builtin_amdgcn_s_memrealtime();
		while (r < next)
			r = __builtin_amdgcn_s_memrealtime();
		const unsigned long long c = __builtin_readcyclecounter();
		out[2 * k] = r;
		out[2 * k + 1] = c;
		if (r - r0 >= ticks) {
			out[2 * max] = (unsigned long long)(k + 1);
			return;
		}
		next = r + period;
	}
	out[2 * max] = (unsigned long long)max;
}

extern "C" int clock_probe_launch(unsigned long long *d_out, int max, unsigned long long period,
				  unsigned long long ticks, void *stream)
{
	if (!d_out || max <= 0)
		return -1;
	hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d_out,
			   max, period, ticks);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}
