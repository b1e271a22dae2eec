// SPDX-License-Identifier: GPL-2.0
/*
 * hostpath.hip - the host path's write-back of ICMPv6 echo replies, and
 * its opt-in gather of a chunked UMEM's frames (umem_gather_kernel below).
 *
 * xdpgpu_submit runs the RX kernels on the slot's device mirror of the
 * host UMEM.  The echo responder (process_packet, af_xdp_user.c:968-1040)
 * rewrites a TX frame in place: MACs, IPv6 addresses, type and checksum,
 * all in its bytes 0-57.  Only those frames may be written back: the rest
 * of the UMEM belongs to the application and the kernel (fill ring frames
 * the NIC may be filling), SURVEY §8b.  So for every descriptor of the
 * batch whose verdict is TX this kernel copies bytes [0, min(len, 64)) of
 * its frame, and nothing else, as compact 80-byte records (EchoRec) that
 * xdpgpu_wait scatters on the host.  (Until round 4 the kernel could also
 * write them straight into the mapped pinned UMEM; no kernel writes host
 * memory any more, and only the opt-in gather reads it)
 * Multi-buffer packets: each fragment of a TX packet has verdict TX, and
 * packet byte p < 64 lies at offset <= p of its fragment, so the fragments'
 * first 64 bytes cover the rewrite.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

namespace {

constexpr int kEchoWave = 64;
constexpr int kEchoBlock = 256;

__device__ __forceinline__ uint32_t rl32(uint32_t v, int l)
{
	return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

/* One lane per descriptor; the wave copies its TX frames one after the
 * other, lane j byte j. */
__global__ __launch_bounds__(kEchoBlock) void echo_writeback_kernel(EchoArgs a)
{
	const int lane = threadIdx.x & (kEchoWave - 1);
	const uint64_t i = (uint64_t)blockIdx.x * kEchoBlock + threadIdx.x;
	bool tx = false;
	uint64_t eff = 0;
	uint32_t w = 0;
	if (i < a.n && a.verdict[i] == XDPGPU_TX) {
		const xdpgpu_desc d = a.desc[i];
		eff = (d.addr & ((1ull << 48) - 1)) + (d.addr >> 48);
		/* a TX verdict implies a frame inside the UMEM; checked anyway */
		tx = (uint64_t)d.len <= a.usize && eff <= a.usize - d.len;
		w = d.len < kEchoBytes ? d.len : kEchoBytes;
	}
	const uint64_t m = __ballot(tx);
	if (!m)
		return;
	uint32_t base = 0;
	if (lane == 0)
		base = atomicAdd(a.nrec, (uint32_t)__popcll(m));
	base = __builtin_amdgcn_readfirstlane(base);
	uint32_t r = 0;
	for (uint64_t k = m; k; k &= k - 1, r++) {
		const int src = __builtin_ctzll(k);
		const uint64_t se = ((uint64_t)rl32((uint32_t)(eff >> 32), src) << 32) |
				    rl32((uint32_t)eff, src);
		const uint32_t sw = rl32(w, src);
		const uint8_t b = (uint32_t)lane < sw ? a.mirror[se + lane] : 0;
		EchoRec *rec = a.rec + base + r;
		rec->b[lane] = b;
		if (lane == 0) {
			rec->eff = se;
			rec->len = sw;
			rec->rsvd = 0;
		}
	}
}

/*
 * UMEM gather (XDPGPU_CFG_UMEM_GATHER): the bytes each
 * descriptor names, [eff, eff + len), and udp_csum's over-read byte
 * eff + len (lib_checksum.h:175-176) where it can lie past the frame,
 * copied from the host UMEM's GPU mapping into the mirror, in the 16-byte
 * pieces that cover them (clamped to the UMEM; the pieces' other bytes are
 * the UMEM's own, copied to the same offsets of this slot's mirror, which
 * no other batch reads).  The over-read byte: a checksum range starts at
 * an even offset (14 + 4 * tags, + the IPv4 header's 4 * ihl or IPv6's 40
 * + 8k) and the parse bounds its end by len, so it ends at len only with
 * len odd; a multi-buffer packet's byte follows its last fragment, whose
 * own length says nothing, so there every fragment takes it (over_all).
 * Offsets decode as the RX kernel's (addr & (2^48 - 1)) + (addr >> 48).
 * Plain loads, nothing written to host memory; a piece the UMEM's end cuts
 * goes byte by byte.  8 lanes a frame, 8 frames a wave, each lane one
 * piece in flight.  With hdesc the descriptors come from the caller's
 * page-locked array (read here, through its GPU mapping) and lane 0 of
 * each frame's group writes the device copy the RX kernel reads.  The
 * bytes read are summed per wave into *nbytes (xdpgpu_host_stats).
 * With poff (XDPGPU_CFG_HOST_COMPACT) the same pieces come from the
 * device copy of the host-packed buffer instead: the host threads copied
 * each frame's pieces, the same 16-byte-aligned bytes clamped the same
 * way, into one page-locked buffer, one transfer brought it over, and this
 * kernel puts them at their UMEM offsets of the mirror.
 */
constexpr int kGatherLanes = 8;
__global__ __launch_bounds__(256) void umem_gather_kernel(GatherArgs a)
{
	const uint32_t sub = threadIdx.x & (kGatherLanes - 1);
	const uint64_t step = (uint64_t)gridDim.x * (256 / kGatherLanes);
	uint64_t mine = 0;
	for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / kGatherLanes; i < a.n;
	     i += step) {
		xdpgpu_desc d;
		if (a.hdesc) {
			d = a.hdesc[i];
			if (sub == 0)
				a.desc[i] = d;
		} else {
			d = a.desc[i];
		}
		const uint64_t eff = (d.addr & ((1ull << 48) - 1)) + (d.addr >> 48);
		/* descriptors outside the UMEM name no bytes */
		if (eff >= a.usize || (uint64_t)d.len > a.usize - eff)
			continue;
		uint64_t hi = eff + d.len + ((a.over_all | d.len) & 1);
		if (hi > a.usize)
			hi = a.usize;
		const uint64_t lo = eff & ~15ull;
		if (sub == 0) {
			const uint64_t r = (hi + 15) & ~15ull;
			mine += (r < a.usize ? r : a.usize) - lo;
		}
		/* the piece's bytes: at their own offsets of the UMEM's view, or
		 * packed (host compaction: the piece at 16 * poff[i]) */
		const uint8_t *src = a.poff ? a.src + 16 * (uint64_t)a.poff[i] - lo : a.src;
		for (uint64_t p = lo + 16 * sub; p < hi; p += 16 * kGatherLanes) {
			if (p + 16 <= a.usize) {
				const uint4 v = *reinterpret_cast<const uint4 *>(src + p);
				*reinterpret_cast<uint4 *>(a.mirror + p) = v;
			} else {
				for (uint64_t b = p; b < a.usize; b++)
					a.mirror[b] = src[b];
			}
		}
	}
	for (int o = 32; o; o >>= 1)
		mine += __shfl_down(mine, o, 64);
	if ((threadIdx.x & 63) == 0 && mine && a.nbytes)
		atomicAdd(a.nbytes, (unsigned long long)mine);
}

} // namespace

hipError_t launch_umem_gather(const GatherArgs &a, hipStream_t stream)
{
	if (!a.n)
		return hipSuccess;
	const uint64_t want = ((uint64_t)a.n * kGatherLanes + 255) / 256;
	const uint32_t blocks = (uint32_t)(want < 4096 ? want : 4096);
	hipLaunchKernelGGL(umem_gather_kernel, dim3(blocks), dim3(256), 0, stream, a);
	return hipGetLastError();
}

hipError_t launch_echo_writeback(const EchoArgs &a, hipStream_t stream)
{
	if (!a.n)
		return hipSuccess;
	const uint32_t blocks = (uint32_t)(((uint64_t)a.n + kEchoBlock - 1) / kEchoBlock);
	hipLaunchKernelGGL(echo_writeback_kernel, dim3(blocks), dim3(kEchoBlock), 0,
			   stream, a);
	return hipGetLastError();
}

} // namespace xdpgpu
