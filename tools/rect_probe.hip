// SPDX-License-Identifier: GPL-2.0
// Host-to-device pitched-copy probe for the chunked host path (DESIGN.md
// §5, "chunked UMEM"): rows of `width` bytes at a 4 KiB pitch from a
// page-locked host buffer into HBM, as xdpgpu_submit copies a batch's
// frames out of the reference's 4 KiB chunks.  Prints one JSON line per
// case: rows, width, streams, copy form, GB/s of row bytes and Mrows/s.
//   hipcc --offload-arch=gfx950 -O2 tools/rect_probe.hip -o tools/rect_probe
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

int main(int argc, char **argv)
{
	const size_t pitch = 4096;
	const size_t rows = argc > 1 ? strtoull(argv[1], 0, 0) : (512u << 10);
	const int reps = 5;
	uint8_t *h, *d;
	/* registered like the caller's UMEM in xdpgpu_register_umem
	 * (hipHostRegisterDefault), or hipHostMalloc'd with argv[2] == "m" */
	const bool hm = argc > 2 && argv[2][0] == 'm';
	if (hm) {
		CK(hipHostMalloc((void **)&h, rows * pitch, 0));
	} else {
		h = (uint8_t *)aligned_alloc(4096, rows * pitch);
		memset(h, 1, rows * pitch);
		CK(hipHostRegister(h, rows * pitch, hipHostRegisterDefault));
	}
	CK(hipMalloc((void **)&d, rows * pitch));
	memset(h, 1, rows * pitch);
	hipStream_t st[8];
	for (int i = 0; i < 8; i++)
		CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	const size_t widths[] = {65, 128, 256, 4096};
	const int nstreams[] = {1, 2, 4, 8};
	for (size_t w : widths) {
		for (int ns : nstreams) {
			double best = 1e30;
			for (int r = 0; r < reps + 1; r++) {
				CK(hipDeviceSynchronize());
				CK(hipEventRecord(e0, st[0]));
				for (int s = 1; s < ns; s++)
					CK(hipStreamWaitEvent(st[s], e0, 0));
				for (int s = 0; s < ns; s++) {
					const size_t r0 = rows * s / ns, r1 = rows * (s + 1) / ns;
					const size_t off = r0 * pitch + 256;
					if (w == pitch)
						CK(hipMemcpyAsync(d + r0 * pitch, h + r0 * pitch,
								  (r1 - r0) * pitch,
								  hipMemcpyHostToDevice, st[s]));
					else
						CK(hipMemcpy2DAsync(d + off, pitch, h + off, pitch, w,
								    r1 - r0, hipMemcpyHostToDevice,
								    st[s]));
				}
				for (int s = 1; s < ns; s++) {
					hipEvent_t ev;
					CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
					CK(hipEventRecord(ev, st[s]));
					CK(hipStreamWaitEvent(st[0], ev, 0));
					CK(hipEventDestroy(ev));
				}
				CK(hipEventRecord(e1, st[0]));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				if (r && ms < best)
					best = ms;
			}
			printf("{\"host\": \"%s\", \"rows\": %zu, \"width\": %zu, \"streams\": %d, \"form\": \"%s\", "
			       "\"ms\": %.4f, \"row_gbps\": %.2f, \"mrows_per_s\": %.1f}\n",
			       hm ? "hipHostMalloc" : "hipHostRegister", rows, w, ns,
			       w == pitch ? "linear" : "2d", best,
			       rows * (double)(w == pitch ? pitch : w) / best / 1e6,
			       rows / best / 1e3);
			fflush(stdout);
		}
	}
	// the copy as many small linear copies (one per 64-row group of
	// consecutive chunks is not possible: rows are not contiguous), for
	// reference: 1-row copies, 4096 of them
	{
		const size_t n = 4096, w = 128;
		CK(hipDeviceSynchronize());
		CK(hipEventRecord(e0, st[0]));
		for (size_t i = 0; i < n; i++)
			CK(hipMemcpyAsync(d + i * pitch + 256, h + i * pitch + 256, w,
					  hipMemcpyHostToDevice, st[0]));
		CK(hipEventRecord(e1, st[0]));
		CK(hipEventSynchronize(e1));
		float ms;
		CK(hipEventElapsedTime(&ms, e0, e1));
		printf("{\"rows\": %zu, \"width\": %zu, \"streams\": 1, \"form\": \"1-row copies\", "
		       "\"ms\": %.4f, \"mrows_per_s\": %.2f}\n", n, w, ms, n / ms / 1e3);
	}
	return 0;
}
