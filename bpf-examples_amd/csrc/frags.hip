// SPDX-License-Identifier: GPL-2.0
/*
 * frags.hip - multi-buffer packets (XDPGPU_CFG_FRAGS, include/xdpgpu.h).
 *
 * A packet of several descriptors (XDP_PKT_CONTD on all but the last,
 * headers/linux/if_xdp.h:122; IS_EOP_DESC, xdpsock.c:67) has its bytes
 * spread over UMEM chunks.  The RX fast kernel skips its descriptors;
 * frag_count finishes the broken packets (the batch ends inside them, or a
 * fragment lies outside the UMEM) as ABORTED; xdp_rx_packet_kernel
 * (xdp_rx.hip) then reads every complete packet in place: its window from
 * the first fragment, headers and payload sums across the fragments.
 * (Round 2 gathered each packet into a bounce UMEM first and scattered the
 * outputs back: 262 144 x 9000-byte packets in 4096-byte fragments took
 * 1.66 ms that way against 0.61 ms in place; removed.)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

namespace {

constexpr int kFragBlock = 256;
constexpr uint64_t kFragMaxBlocks = 4096;

__device__ __forceinline__ uint64_t frag_eff(const xdpgpu_desc &d)
{
	return (d.addr & ((1ull << 48) - 1)) + (d.addr >> 48);
}

/* the first descriptor of a packet of several */
__device__ __forceinline__ bool packet_head(const FragArgs &a, uint32_t i)
{
	return (a.desc[i].options & XDPGPU_PKT_CONTD) &&
	       !(i && (a.desc[i - 1].options & XDPGPU_PKT_CONTD));
}

/* The packet whose first descriptor is i: its last descriptor and bytes.
 * False when the batch ends inside it, a fragment lies outside the UMEM or
 * the packet does not fit a descriptor's length field. */
__device__ bool packet_walk(const FragArgs &a, uint32_t i, uint32_t &last,
			    uint64_t &total)
{
	bool ok = true;
	total = 0;
	for (uint32_t j = i;; j++) {
		const xdpgpu_desc d = a.desc[j];
		const uint64_t eff = frag_eff(d);
		ok = ok && (uint64_t)d.len <= a.usize && eff <= a.usize - d.len;
		total += d.len;
		last = j;
		if (!(d.options & XDPGPU_PKT_CONTD))
			return ok && total <= 0xffffffffull;
		if (j + 1 == a.n)
			return false;
	}
}

/* the all-zero record and tuple of descriptor k */
__device__ void zero_outputs(const FragArgs &a, uint32_t k)
{
	if (a.res)
		*reinterpret_cast<uint4 *>(a.res + k) = make_uint4(0, 0, 0, 0);
	for (uint32_t b = 0; b < a.tb; b++)
		a.tup[(uint64_t)k * a.tb + b] = 0;
}

/* The packets' first descriptors (a lane per descriptor, grid-strided)
 * walk their fragments; a broken packet is finished here as ABORTED, one
 * frame in the counters (block 0's slot). */
__global__ __launch_bounds__(kFragBlock) void frag_count_kernel(FragArgs a)
{
	const uint64_t step = (uint64_t)gridDim.x * kFragBlock;
	for (uint64_t b = (uint64_t)blockIdx.x * kFragBlock; b < a.n; b += step) {
		const uint64_t i = b + threadIdx.x;
		uint32_t last = 0;
		uint64_t total = 0;
		const bool head = i < a.n && packet_head(a, (uint32_t)i);
		if (!head || packet_walk(a, (uint32_t)i, last, total))
			continue;
		for (uint32_t k = (uint32_t)i; k <= last; k++) {
			a.verdict[k] = XDPGPU_ABORTED;
			zero_outputs(a, k);
		}
		if (a.stats) {
			atomicAdd(&a.stats[CNT_FRAMES], 1ull);
			atomicAdd(&a.stats[CNT_BYTES], (unsigned long long)total);
			atomicAdd(&a.stats[CNT_VERDICT0 + XDPGPU_ABORTED], 1ull);
		}
	}
}

uint32_t frag_blocks(uint64_t items, uint64_t cap)
{
	uint64_t b = (items + kFragBlock - 1) / kFragBlock;
	if (b > cap)
		b = cap;
	return b ? (uint32_t)b : 1u;
}

} // namespace

hipError_t launch_frag_count(const FragArgs &a, hipStream_t stream)
{
	hipLaunchKernelGGL(frag_count_kernel, dim3(frag_blocks(a.n, kFragMaxBlocks)),
			   dim3(kFragBlock), 0, stream, a);
	return hipGetLastError();
}

} // namespace xdpgpu
