// SPDX-License-Identifier: GPL-2.0
/*
 * hints.hip - XDP hints in front of each frame (xdpgpu_hints_dev).
 *
 * The XDP program of AF_XDP-interaction (af_xdp_kern.c:42-105) writes a
 * metadata struct in front of the frame with bpf_xdp_adjust_meta, its BTF id
 * last; the user program reads the id from the 4 bytes before the frame
 * (xsk_umem__btf_id, lib_xsk_extend.c:16-27) and the struct's members at
 * negative offsets (print_meta_info_via_btf, af_xdp_user.c:813-829).  One
 * lane per frame: the 16 bytes before it as dwords when the frame is 4-byte
 * aligned, as bytes otherwise, and one 16-byte record out.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

namespace {

constexpr int kHintsBlock = 256;

/* the little-endian u32 at umem[at] */
__device__ __forceinline__ uint32_t ld32(const uint8_t *umem, uint64_t at)
{
	if (!(at & 3))
		return *reinterpret_cast<const uint32_t *>(umem + at);
	return (uint32_t)umem[at] | ((uint32_t)umem[at + 1] << 8) |
	       ((uint32_t)umem[at + 2] << 16) | ((uint32_t)umem[at + 3] << 24);
}

__global__ __launch_bounds__(kHintsBlock) void hints_kernel(
	const uint8_t *umem, uint64_t usize, const xdpgpu_desc *desc, uint32_t n,
	uint32_t rx_time_id, uint32_t mark_id, xdpgpu_hints *out)
{
	const uint64_t step = (uint64_t)gridDim.x * kHintsBlock;
	for (uint64_t i = (uint64_t)blockIdx.x * kHintsBlock + threadIdx.x; i < n;
	     i += step) {
		const uint64_t addr = desc[i].addr;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		uint4 r = make_uint4(0, 0, 0, 0);
		if (eff >= 4 && eff <= usize) {
			r.w = ld32(umem, eff - 4);
			if (r.w && r.w == rx_time_id && eff >= 16) {
				/* struct xdp_hints_rx_time, af_xdp_kern.c:47-51 */
				r.x = ld32(umem, eff - 16);
				r.y = ld32(umem, eff - 12);
				r.z = ld32(umem, eff - 8);
			} else if (r.w && r.w == mark_id && eff >= 8) {
				/* struct xdp_hints_mark, af_xdp_kern.c:42-45 */
				r.z = ld32(umem, eff - 8);
			}
		}
		*reinterpret_cast<uint4 *>(out + i) = r;
	}
}

} // namespace

hipError_t launch_hints(const uint8_t *umem, uint64_t usize, const xdpgpu_desc *desc,
			uint32_t n, uint32_t rx_time_id, uint32_t mark_id,
			xdpgpu_hints *out, hipStream_t stream)
{
	uint64_t blocks = ((uint64_t)n + kHintsBlock - 1) / kHintsBlock;
	if (blocks > 8192)
		blocks = 8192;
	hipLaunchKernelGGL(hints_kernel, dim3((uint32_t)blocks), dim3(kHintsBlock), 0,
			   stream, umem, usize, desc, n, rx_time_id, mark_id, out);
	return hipGetLastError();
}

} // namespace xdpgpu
