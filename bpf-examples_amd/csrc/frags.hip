// SPDX-License-Identifier: GPL-2.0
/*
 * frags.hip - multi-buffer packets (XDPGPU_CFG_FRAGS, include/xdpgpu.h).
 *
 * A packet of several descriptors (XDP_PKT_CONTD on all but the last,
 * headers/linux/if_xdp.h:122; IS_EOP_DESC, xdpsock.c:67) has its bytes
 * spread over UMEM chunks.  The RX fast kernel skips its descriptors;
 * frag_count finishes the broken packets; by default xdp_rx_packet_kernel
 * (xdp_rx.hip) then reads every complete packet in place (its window from
 * the first fragment, headers and payload sums across the fragments:
 * 262 144 x 9000-byte packets in 4096-byte fragments, 0.61 vs 1.66 ms
 * through the bounce copy).  cfg.tune bit 24 selects the bounce path:
 *  - frag_count: the packets' first descriptors (lane per descriptor) walk
 *    their fragments; complete packets are counted per block with the
 *    bounce bytes they need (frag_scan turns the block totals into
 *    prefixes), the others (the batch ends inside them, or a fragment lies
 *    outside the UMEM) are finished as ABORTED;
 *  - frag_gather: each complete packet, and the byte after its last
 *    fragment (udp_csum's over-read byte), is copied to a bounce UMEM at a
 *    16-byte aligned offset (its block's prefix on, in descriptor order),
 *    one wave per packet with coalesced 16-byte copies where the fragments
 *    allow them, and gets a bounce descriptor; the RX kernels then run over
 *    the bounce batch, one frame per packet;
 *  - frag_scatter: the packet's verdict goes to each of its descriptors,
 *    its record and tuple to the first (all-zero ones to the others), and
 *    an ICMPv6 echo reply's first 64 bytes back into the fragments (the
 *    rewrite of process_packet, af_xdp_user.c:968-1040, touches bytes
 *    0-61).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

namespace {

constexpr int kFragWave = 64;
constexpr int kFragBlock = 256;
constexpr uint64_t kFragMaxBlocks = 4096;
constexpr int kFragScan = 1024;          /* count / gather grid at most */

__device__ __forceinline__ uint64_t frag_eff(const xdpgpu_desc &d)
{
	return (d.addr & ((1ull << 48) - 1)) + (d.addr >> 48);
}

__device__ __forceinline__ uint32_t rl32(uint32_t v, int l)
{
	return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l)
{
	return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
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

/* bounce bytes of a packet: its bytes and the over-read byte, rounded up
 * to 16 */
__device__ __forceinline__ uint64_t bounce_size(uint64_t total)
{
	return (total + 16) & ~15ull;
}

/* the all-zero record and tuple of descriptor k */
__device__ void zero_outputs(const FragArgs &a, uint32_t k)
{
	if (a.res)
		*reinterpret_cast<uint4 *>(a.res + k) = make_uint4(0, 0, 0, 0);
	for (uint32_t b = 0; b < a.tb; b++)
		a.tup[(uint64_t)k * a.tb + b] = 0;
}

/* Wave-cooperative copy of n bytes: 16-byte vectors, four per lane and
 * step (4 KiB per wave-step), when source and destination share their
 * alignment mod 16 (chunk-aligned fragments); dwords when they share it mod
 * 4; bytes otherwise. */
__device__ void wave_copy(uint8_t *dst, const uint8_t *src, uint64_t n, int lane)
{
	uint64_t o = 0;
	const uintptr_t mis = (uintptr_t)dst ^ (uintptr_t)src;
	if (!(mis & 15)) {
		const uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
		o = head < n ? head : n;
		if ((uint64_t)lane < o)
			dst[lane] = src[lane];
		const uint64_t vecs = (n - o) / 16;
		uint4 *dv = reinterpret_cast<uint4 *>(dst + o);
		const uint4 *sv = reinterpret_cast<const uint4 *>(src + o);
		uint64_t w = lane;
		for (; w + 3 * kFragWave < vecs; w += 4 * kFragWave) {
			uint4 t[4];
#pragma unroll
			for (int u = 0; u < 4; u++)
				t[u] = sv[w + u * kFragWave];
#pragma unroll
			for (int u = 0; u < 4; u++)
				dv[w + u * kFragWave] = t[u];
		}
		for (; w < vecs; w += kFragWave)
			dv[w] = sv[w];
		o += 16 * vecs;
	} else if (!(mis & 3)) {
		const uint64_t head = (4 - ((uintptr_t)dst & 3)) & 3;
		o = head < n ? head : n;
		if ((uint64_t)lane < o)
			dst[lane] = src[lane];
		const uint64_t words = (n - o) / 4;
		uint32_t *dw = reinterpret_cast<uint32_t *>(dst + o);
		const uint32_t *sw = reinterpret_cast<const uint32_t *>(src + o);
		for (uint64_t w = lane; w < words; w += kFragWave)
			dw[w] = sw[w];
		o += 4 * words;
	}
	for (uint64_t b = o + lane; b < n; b += kFragWave)
		dst[b] = src[b];
}

/* wave sum and exclusive wave prefix sum of a u64 */
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
	for (int m = kFragWave / 2; m >= 1; m >>= 1) {
		const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kFragWave);
		const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kFragWave);
		v += ((uint64_t)hi << 32) | lo;
	}
	return v;
}

__device__ __forceinline__ uint64_t wave_excl_u64(uint64_t v, int lane)
{
	uint64_t x = v;
#pragma unroll
	for (int d = 1; d < kFragWave; d <<= 1) {
		const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d, kFragWave);
		const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d, kFragWave);
		if (lane >= d)
			x += ((uint64_t)hi << 32) | lo;
	}
	return x - v;
}

/* Count and gather walk the descriptors in the same order: frag_grid(n)
 * blocks, block-strided 256 descriptors at a time.  Count leaves each
 * block's packets and bounce bytes in blk[]; one block turns them into
 * exclusive prefixes; gather places a block's packets from its prefix on,
 * in descriptor order.  No atomics on shared words (a returning device
 * atomic on one word serialises at ~80 per microsecond), and the bounce
 * layout is deterministic. */
__global__ __launch_bounds__(kFragBlock) void frag_count_kernel(FragArgs a)
{
	__shared__ unsigned long long part[2][kFragBlock / kFragWave];
	const int lane = threadIdx.x & (kFragWave - 1), wid = threadIdx.x / kFragWave;
	const uint64_t step = (uint64_t)gridDim.x * kFragBlock;
	uint64_t cnt = 0, bytes = 0;    /* this lane's complete packets */
	for (uint64_t b = (uint64_t)blockIdx.x * kFragBlock; b < a.n; b += step) {
		const uint64_t i = b + threadIdx.x;
		uint32_t last = 0;
		uint64_t total = 0;
		const bool head = i < a.n && packet_head(a, (uint32_t)i);
		const bool ok = head && packet_walk(a, (uint32_t)i, last, total);
		if (ok) {
			cnt++;
			bytes += bounce_size(total);
		}
		if (!head || ok)
			continue;
		/* broken packet: ABORTED here, one frame in the counters */
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
	cnt = wave_sum_u64(cnt);
	bytes = wave_sum_u64(bytes);
	if (lane == 0) {
		part[0][wid] = cnt;
		part[1][wid] = bytes;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		unsigned long long c = 0, y = 0;
		for (int w = 0; w < kFragBlock / kFragWave; w++) {
			c += part[0][w];
			y += part[1][w];
		}
		a.blk[2 * blockIdx.x] = c;
		a.blk[2 * blockIdx.x + 1] = y;
	}
}

/* one block: exclusive prefixes of the g block totals; the grand totals
 * to fc[0] (packets) and fc[1] (bounce bytes) */
__global__ __launch_bounds__(kFragScan) void frag_scan_kernel(FragArgs a, uint32_t g)
{
	__shared__ unsigned long long sc[2][kFragScan];
	const uint32_t t = threadIdx.x;
	const unsigned long long c = t < g ? a.blk[2 * t] : 0, y = t < g ? a.blk[2 * t + 1] : 0;
	sc[0][t] = c;
	sc[1][t] = y;
	__syncthreads();
	for (uint32_t d = 1; d < kFragScan; d <<= 1) {
		const unsigned long long c2 = t >= d ? sc[0][t - d] : 0;
		const unsigned long long y2 = t >= d ? sc[1][t - d] : 0;
		__syncthreads();
		sc[0][t] += c2;
		sc[1][t] += y2;
		__syncthreads();
	}
	if (t < g) {
		a.blk[2 * t] = sc[0][t] - c;
		a.blk[2 * t + 1] = sc[1][t] - y;
	}
	if (t == kFragScan - 1) {
		a.fc[0] = sc[0][t];
		a.fc[1] = sc[1][t];
	}
}

__global__ __launch_bounds__(kFragBlock) void frag_gather_kernel(FragArgs a)
{
	__shared__ unsigned long long wpart[2][kFragBlock / kFragWave];
	const int lane = threadIdx.x & (kFragWave - 1), wid = threadIdx.x / kFragWave;
	const uint64_t step = (uint64_t)gridDim.x * kFragBlock;
	/* where this block's next packet goes */
	uint64_t kbase = a.blk[2 * blockIdx.x], obase = a.blk[2 * blockIdx.x + 1];
	for (uint64_t b = (uint64_t)blockIdx.x * kFragBlock; b < a.n; b += step) {
		const uint64_t i = b + threadIdx.x;
		uint32_t last = 0;
		uint64_t total = 0;
		const bool mine = i < a.n && packet_head(a, (uint32_t)i) &&
				  packet_walk(a, (uint32_t)i, last, total);
		const uint64_t mm = __ballot(mine);
		const uint64_t sz = mine ? bounce_size(total) : 0;
		const uint64_t pre = wave_excl_u64(sz, lane);
		if (lane == kFragWave - 1) {
			wpart[0][wid] = (unsigned long long)__popcll(mm);
			wpart[1][wid] = pre + sz;
		}
		__syncthreads();
		uint64_t kw = kbase, ow = obase, kt = 0, ot = 0;
		for (int w = 0; w < kFragBlock / kFragWave; w++) {
			if (w < wid) {
				kw += wpart[0][w];
				ow += wpart[1][w];
			}
			kt += wpart[0][w];
			ot += wpart[1][w];
		}
		__syncthreads();
		kbase += kt;
		obase += ot;
		const uint64_t off = ow + pre;
		/* a packet past the bounce capacity (only descriptors that
		 * repeat UMEM bytes can get there: the capacity is the UMEM
		 * size plus the per-packet padding) gets an empty bounce
		 * descriptor, which the RX kernels finish as ABORTED */
		const bool fits = off + sz <= a.bounce_cap;
		if (mine) {
			const uint32_t k = (uint32_t)kw + __builtin_amdgcn_mbcnt_hi(
				(uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0));
			*reinterpret_cast<uint4 *>(a.bdesc + k) =
				fits ? make_uint4((uint32_t)off, (uint32_t)(off >> 32),
						  (uint32_t)total, 0u)
				     : make_uint4(0u, 0u, 0u, 0u);
			a.bmap[k] = make_uint2((uint32_t)i, last - (uint32_t)i + 1);
		}
		/* the wave copies its packets one after the other */
		for (uint64_t m = __ballot(mine && fits); m; m &= m - 1) {
			const int src = __builtin_ctzll(m);
			const uint32_t first = rl32((uint32_t)i, src), lst = rl32(last, src);
			uint8_t *dst = a.bounce + rl64(off, src);
			uint64_t at = 0, end = 0;
			for (uint32_t j = first; j <= lst; j++) {
				const xdpgpu_desc d = a.desc[j];
				const uint64_t eff = frag_eff(d);
				wave_copy(dst + at, a.umem + eff, d.len, lane);
				at += d.len;
				end = eff + d.len;
			}
			/* udp_csum's over-read byte, then zeros to the 16-byte end */
			for (uint64_t o = at + lane; o < bounce_size(at); o += kFragWave)
				dst[o] = (o == at && end < a.usize) ? a.umem[end] : 0;
		}
	}
}

__global__ __launch_bounds__(kFragBlock) void frag_scatter_kernel(FragArgs a)
{
	const uint64_t step = (uint64_t)gridDim.x * kFragBlock;
	const uint64_t m = a.fc[0];        /* packets gathered (device count) */
	for (uint64_t k = (uint64_t)blockIdx.x * kFragBlock + threadIdx.x; k < m;
	     k += step) {
		const uint2 mp = a.bmap[k];
		const uint8_t v = a.bverdict[k];
		for (uint32_t f = 0; f < mp.y; f++) {
			a.verdict[mp.x + f] = v;
			if (f)
				zero_outputs(a, mp.x + f);
		}
		if (a.res)
			*reinterpret_cast<uint4 *>(a.res + mp.x) =
				*reinterpret_cast<const uint4 *>(a.bres + k);
		for (uint32_t b = 0; b < a.tb; b++)
			a.tup[(uint64_t)mp.x * a.tb + b] = a.btup[k * a.tb + b];
		if (v != XDPGPU_TX)
			continue;
		/* the echo reply's bytes back into the fragments */
		const uint4 bd = *reinterpret_cast<const uint4 *>(a.bdesc + k);
		const uint8_t *src = a.bounce + (((uint64_t)bd.y << 32) | bd.x);
		const uint64_t want = bd.z < 64u ? bd.z : 64u;
		uint64_t at = 0;
		for (uint32_t f = 0; f < mp.y && at < want; f++) {
			const xdpgpu_desc d = a.desc[mp.x + f];
			const uint64_t eff = frag_eff(d);
			for (uint32_t o = 0; o < d.len && at < want; o++, at++)
				a.umem[eff + o] = src[at];
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
	const uint32_t g = frag_blocks(a.n, kFragScan);
	hipLaunchKernelGGL(frag_count_kernel, dim3(g), dim3(kFragBlock), 0, stream, a);
	hipLaunchKernelGGL(frag_scan_kernel, dim3(1), dim3(kFragScan), 0, stream, a, g);
	return hipGetLastError();
}

hipError_t launch_frag_gather(const FragArgs &a, hipStream_t stream)
{
	hipLaunchKernelGGL(frag_gather_kernel, dim3(frag_blocks(a.n, kFragScan)),
			   dim3(kFragBlock), 0, stream, a);
	return hipGetLastError();
}

hipError_t launch_frag_scatter(const FragArgs &a, hipStream_t stream)
{
	hipLaunchKernelGGL(frag_scatter_kernel, dim3(frag_blocks(a.m, kFragMaxBlocks)),
			   dim3(kFragBlock), 0, stream, a);
	return hipGetLastError();
}

} // namespace xdpgpu
