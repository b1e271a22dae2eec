// SPDX-License-Identifier: GPL-2.0
/*
 * hostreg_probe.c - diagnostic, never the product: what the ROCm runtime
 * holds registered (locked / mapped for the GPU) over a host address range.
 * hsa_amd_pointer_info() only looks the address up in the runtime's tables;
 * it touches no page and starts no GPU work, so the probe cannot itself
 * fault.  Loaded by tests/hostreg.py when XDPGPU_HOSTREG_PROBE=1.
 *
 *   gcc -O2 -shared -fPIC -I/opt/rocm/include tools/hostreg_probe.c \
 *       -L/opt/rocm/lib -lhsa-runtime64 -o tools/libhostreg_probe.so
 */
#include <stdint.h>
#include <string.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

static int inited;

int hrp_init(void)
{
	if (inited)
		return 0;
	if (hsa_init() != HSA_STATUS_SUCCESS)
		return -1;
	inited = 1;
	return 0;
}

/* out: type, host base, agent base, size in bytes */
int hrp_info(const void *p, uint64_t *out)
{
	hsa_amd_pointer_info_t in;
	memset(&in, 0, sizeof(in));
	in.size = sizeof(in);
	if (hsa_amd_pointer_info(p, &in, NULL, NULL, NULL) != HSA_STATUS_SUCCESS)
		return -1;
	out[0] = (uint64_t)in.type;
	out[1] = (uint64_t)(uintptr_t)in.hostBaseAddress;
	out[2] = (uint64_t)(uintptr_t)in.agentBaseAddress;
	out[3] = (uint64_t)in.sizeInBytes;
	return 0;
}

/*
 * Every runtime allocation that covers a byte of [p, p + size): the range is
 * walked page by page (and from a found allocation's end on), up to max
 * records of (type, host base, agent base, size).  Returns the count, or -1.
 */
int hrp_scan(const void *p, uint64_t size, uint64_t *out, int max)
{
	const uint64_t pg = 4096;
	uint64_t a = (uint64_t)(uintptr_t)p, end = a + size;
	int n = 0;
	while (a < end && n < max) {
		uint64_t r[4];
		if (hrp_info((const void *)(uintptr_t)a, r))
			return -1;
		if (r[0] != HSA_EXT_POINTER_TYPE_UNKNOWN) {
			memcpy(out + 4 * n, r, sizeof(r));
			n++;
			const uint64_t e = r[1] + r[3];
			a = e > a ? e : a + pg;
			continue;
		}
		a = (a & ~(pg - 1)) + pg;
	}
	return n;
}
