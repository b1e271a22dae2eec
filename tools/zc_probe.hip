// SPDX-License-Identifier: GPL-2.0
// Zero-copy gather probe for the chunked host path: a
// kernel reads each frame's bytes straight out of the page-locked host
// UMEM (mapped into the GPU's address space, as xdpgpu_register_umem
// registers it) and writes them into an HBM mirror at the same offset,
// against the copy engine's pitched copy of the same rows.  One JSON line
// per case: rows, pitch, width, lanes a row, GB/s of row bytes, Mrows/s.
//   hipcc --offload-arch=gfx950 -O2 tools/zc_probe.hip -o tools/zc_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CK(x)                                                                   \
	do {                                                                    \
		hipError_t e_ = (x);                                            \
		if (e_ != hipSuccess) {                                         \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,      \
				hipGetErrorString(e_));                         \
			exit(1);                                                \
		}                                                               \
	} while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

/* rows of (1 << wsh) 16-byte pieces at the offsets addrs[] names */
template <bool NT>
__global__ __launch_bounds__(256) void k_gather(const uint8_t *__restrict__ src,
						uint8_t *__restrict__ dst,
						const uint64_t *__restrict__ addrs, uint32_t n,
						uint32_t wsh)
{
	const size_t total = (size_t)n << wsh;
	for (size_t t = blockIdx.x * 256ull + threadIdx.x; t < total;
	     t += (size_t)gridDim.x * 256) {
		const size_t a = addrs[t >> wsh] + ((t & ((1u << wsh) - 1)) << 4);
		const v4u *s = reinterpret_cast<const v4u *>(src + a);
		v4u v = NT ? __builtin_nontemporal_load(s) : *s;
		*reinterpret_cast<v4u *>(dst + a) = v;
	}
}

int main(int argc, char **argv)
{
	const size_t rows = argc > 1 ? strtoull(argv[1], 0, 0) : (512u << 10);
	/* argv[2]: "r" registered (default, as a caller's UMEM) or "m"
	 * hipHostMalloc'd (xdpgpu_host_alloc); argv[3]: the chunk (pitch) */
	const bool hm = argc > 2 && argv[2][0] == 'm';
	const size_t pitch = argc > 3 ? strtoull(argv[3], 0, 0) : 4096, head = 256;
	const int reps = 5;
	uint8_t *h;
	if (hm) {
		CK(hipHostMalloc((void **)&h, rows * pitch, hipHostMallocMapped));
	} else {
		h = (uint8_t *)aligned_alloc(4096, rows * pitch);
		CK(hipHostRegister(h, rows * pitch, hipHostRegisterMapped));
	}
	memset(h, 1, rows * pitch);
	uint8_t *hd = nullptr;
	CK(hipHostGetDevicePointer((void **)&hd, h, 0));
	uint8_t *d;
	CK(hipMalloc((void **)&d, rows * pitch));
	std::vector<uint64_t> ad(rows), ap(rows);
	for (size_t r = 0; r < rows; r++) {
		ad[r] = r * pitch + head;
		ap[r] = r * 64;          /* packed 64 B frames, for the sequential rate */
	}
	uint64_t *dad, *dap;
	CK(hipMalloc((void **)&dad, rows * 8));
	CK(hipMalloc((void **)&dap, rows * 8));
	CK(hipMemcpy(dad, ad.data(), rows * 8, hipMemcpyHostToDevice));
	CK(hipMemcpy(dap, ap.data(), rows * 8, hipMemcpyHostToDevice));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	printf("{\"mapped_same_va\": %s, \"alloc\": \"%s\", \"pitch\": %zu}\n",
	       hd == h ? "true" : "false", hm ? "hipHostMalloc" : "hipHostRegister", pitch);
	auto timeit = [&](auto fn) {
		double best = 1e30;
		for (int r = 0; r < reps + 1; r++) {
			CK(hipDeviceSynchronize());
			CK(hipEventRecord(e0, 0));
			fn();
			CK(hipEventRecord(e1, 0));
			CK(hipEventSynchronize(e1));
			float ms;
			CK(hipEventElapsedTime(&ms, e0, e1));
			if (r && ms < best)
				best = ms;
		}
		return best;
	};
	for (uint32_t wsh : {2u, 3u, 4u}) {
		const size_t w = 16u << wsh;
		for (int grid : {1024, 4096}) {
			for (int nt = 0; nt < 1; nt++) {
				const double ms = timeit([&] {
					if (nt)
						hipLaunchKernelGGL(k_gather<true>, dim3(grid), dim3(256), 0, 0,
								   hd, d, dad, (uint32_t)rows, wsh);
					else
						hipLaunchKernelGGL(k_gather<false>, dim3(grid), dim3(256), 0, 0,
								   hd, d, dad, (uint32_t)rows, wsh);
				});
				printf("{\"form\": \"gather\", \"nt\": %d, \"rows\": %zu, \"pitch\": %zu, "
				       "\"width\": %zu, \"grid\": %d, \"ms\": %.4f, \"gbps\": %.2f, "
				       "\"mrows\": %.1f}\n", nt, rows, pitch, w, grid, ms,
				       rows * w / ms / 1e6, rows / ms / 1e3);
			}
		}
		const double ms = timeit([&] {
			CK(hipMemcpy2DAsync(d + head, pitch, h + head, pitch, w, rows,
					    hipMemcpyHostToDevice, 0));
		});
		printf("{\"form\": \"copy2d\", \"rows\": %zu, \"pitch\": %zu, \"width\": %zu, "
		       "\"ms\": %.4f, \"gbps\": %.2f, \"mrows\": %.1f}\n", rows, pitch, w, ms,
		       rows * w / ms / 1e6, rows / ms / 1e3);
	}
	/* both at once: the copy engine takes the first k rows (64 B wide) on
	 * one stream while the gather kernel reads the rest on another */
	{
		hipStream_t s1;
		CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
		hipEvent_t f1;
		CK(hipEventCreate(&f1));
		for (double frac : {0.0, 0.25, 0.33, 0.4, 0.5}) {
			const size_t k = (size_t)(rows * frac);
			const double ms = timeit([&] {
				CK(hipStreamWaitEvent(s1, e0, 0));
				if (k)
					CK(hipMemcpy2DAsync(d + head, pitch, h + head, pitch, 64, k,
							    hipMemcpyHostToDevice, s1));
				hipLaunchKernelGGL(k_gather<false>, dim3(4096), dim3(256), 0, 0, hd, d,
						   dad + k, (uint32_t)(rows - k), 2u);
				CK(hipEventRecord(f1, s1));
				CK(hipStreamWaitEvent(0, f1, 0));
			});
			printf("{\"form\": \"copy2d+gather\", \"copy_frac\": %.2f, \"rows\": %zu, "
			       "\"pitch\": %zu, \"width\": 64, \"ms\": %.4f, \"mrows\": %.1f}\n", frac,
			       rows, pitch, ms, rows / ms / 1e3);
		}
	}
	/* packed frames: the whole span, gathered and copied */
	const size_t span = rows * 64;
	for (int grid : {1024, 4096}) {
		const double ms = timeit([&] {
			hipLaunchKernelGGL(k_gather<false>, dim3(grid), dim3(256), 0, 0, hd, d, dap,
					   (uint32_t)rows, 2u);
		});
		printf("{\"form\": \"gather_packed\", \"rows\": %zu, \"grid\": %d, \"ms\": %.4f, "
		       "\"gbps\": %.2f}\n", rows, grid, ms, span / ms / 1e6);
	}
	const double ms = timeit([&] {
		CK(hipMemcpyAsync(d, h, span, hipMemcpyHostToDevice, 0));
	});
	printf("{\"form\": \"copy_packed\", \"bytes\": %zu, \"ms\": %.4f, \"gbps\": %.2f}\n", span,
	       ms, span / ms / 1e6);
	if (hm) {
		CK(hipHostFree(h));
	} else {
		CK(hipHostUnregister(h));
		free(h);
	}
	return 0;
}
