// SPDX-License-Identifier: GPL-2.0
/*
 * stream_probe.hip - diagnostic (not a test, not the product): the data
 * movement of a single address-order pass over a packed pool, with
 * producer and consumer waves (VERDICT r05 "next" #2 for config 3, IMIX).
 *
 * One block per CU, 16 waves: waves 0-3 produce, 4-15 consume.  A block
 * takes segments of kSeg consecutive descriptors (a global counter); the
 * segment's bytes [A0, A1) stream into an LDS ring of 4 windows of 32 KiB
 * by global_load_lds_dwordx4 (1 KiB an instruction).  In phase k the
 * consumers take the frames that start in window k (their bytes reach
 * into window k + 1 at most, 1.5 KiB), the producers issue window k + 3
 * into the slot window k - 1 left and wait only for window k + 2 (issued
 * a phase earlier), then the block synchronises.  A consumer group of 8
 * lanes takes one frame: its descriptor from HBM, its bytes from the ring
 * (16-byte chunks strided over the 8 lanes), the one's-complement sum of
 * the whole frame reduced over the group, and the frame's outputs as the
 * RX kernel writes them for config 3: a verdict byte, a 16-byte record
 * (the sum, the first words) and a 44-byte tuple (header words).  That is
 * the whole pool read once in address order plus 61 bytes written and 16
 * read a frame; the parse is stood in for by reading the first 64 bytes.
 *
 * Requires descriptors sorted by address with frames inside the pool
 * (the IMIX pool is); outputs are checked by tools/stream_probe.py
 * against a host recompute of the same sums.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

#ifndef SP_PROD
#define SP_PROD 4
#endif
#ifndef SP_WIN_KB
#define SP_WIN_KB 32
#endif
#ifndef SP_GROUP
#define SP_GROUP 8
#endif
constexpr int kWaves = 16, kProd = SP_PROD, kCons = kWaves - kProd;
constexpr int kWin = SP_WIN_KB * 1024, kSlots = 4, kRing = kWin * kSlots;
constexpr int kGroup = SP_GROUP;                /* lanes a frame */
static_assert(kWin % (1024 * kProd) == 0, "whole 1 KiB loads per producer");
/* s_waitcnt vmcnt(one window's loads of a producer wave), nothing else */
constexpr int kLoadsPerWin = kWin / 1024 / kProd;
static_assert(kLoadsPerWin < 64, "vmcnt is 6 bits");
constexpr int kVmcntNew = 0x0f70 | (kLoadsPerWin & 15) | ((kLoadsPerWin >> 4) << 14);
constexpr int kFramesPerRound = kCons * 64 / kGroup;
constexpr uint32_t kSeg = 2048;
constexpr uint32_t kMaxWin = 512;             /* windows a segment       */

struct Args {
	const uint8_t *pool;
	uint64_t usize;
	const uint4 *desc;      /* xdp_desc: addr lo, addr hi, len, options */
	uint32_t n;
	uint8_t *verdict;
	uint4 *rec;
	uint8_t *tup;
	uint32_t *seg_ctr;
};

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ uint32_t add_halves(uint32_t acc, uint32_t x)
{
	return acc + (x & 0xffff) + (x >> 16);
}

__device__ __forceinline__ uint32_t fold16(uint64_t x)
{
	x = (x & 0xffffffffull) + (x >> 32);
	x = (x & 0xffff) + (x >> 16);
	x = (x & 0xffff) + (x >> 16);
	return (uint32_t)((x & 0xffff) + (x >> 16));
}

__global__ __launch_bounds__(1024, 1) void stream_probe_kernel(Args a)
{
	__shared__ __attribute__((aligned(16))) uint8_t ring[kRing];
	/* the segment, and the first frame of each window of it */
	__shared__ uint32_t ctl[2];
	__shared__ uint32_t wstart[kMaxWin + 1];
	/* the segment's descriptors as (offset from A0, length) */
	__shared__ uint2 dl[kSeg];
	const int lane = threadIdx.x & 63;
	const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint32_t nseg = (a.n + kSeg - 1) / kSeg;
	for (;;) {
		if (threadIdx.x == 0)
			ctl[0] = atomicAdd(a.seg_ctr, 1u);
		__syncthreads();
		const uint32_t seg = ctl[0];
		__syncthreads();
		if (seg >= nseg)
			break;
		const uint32_t f0 = seg * kSeg;
		const uint32_t f1 = min(f0 + kSeg, a.n);
		const uint4 dfirst = a.desc[f0], dlast = a.desc[f1 - 1];
		const uint64_t A0 = ((((uint64_t)dfirst.y << 32) | dfirst.x)) & ~15ull;
		uint64_t A1 = ((((uint64_t)dlast.y << 32) | dlast.x) + dlast.z + 1 + 15) & ~15ull;
		if (A1 > ((a.usize + 15) & ~15ull))
			A1 = (a.usize + 15) & ~15ull;
		uint32_t nwin = (uint32_t)((A1 - A0 + kWin - 1) / kWin);
		if (nwin > kMaxWin)
			nwin = kMaxWin;   /* (the probe's pools stay far below) */
		/* windows no frame starts in after the last start: empty */
		for (uint32_t k = threadIdx.x; k <= nwin; k += blockDim.x)
			wstart[k] = f1;
		__syncthreads();
		/* producer: window w's 32 loads of 1 KiB, wave p the p-th of each
		 * four */
		auto produce = [&](uint32_t w) {
			const uint64_t wb = A0 + (uint64_t)w * kWin;
			uint8_t *slot = ring + (w % kSlots) * kWin;
#pragma unroll
			for (int j = 0; j < kWin / 1024 / kProd; j++) {
				const uint32_t off = (uint32_t)(j * kProd + wid) * 1024u;
				uint64_t src = wb + off + 16 * lane;
				/* past the segment: the pool's first bytes (never read) */
				if (src + 16 > A1)
					src = 0;
				__builtin_amdgcn_global_load_lds((const void *)(a.pool + src),
								 (lds_void_t *)(slot + off), 16, 0, 0);
			}
		};
		if (wid < kProd) {
			produce(0);
			if (nwin > 1)
				produce(1);
			if (nwin > 2)
				produce(2);
			__builtin_amdgcn_s_waitcnt(0x0f70);   /* vmcnt(0): windows 0-2 */
		} else {
			/* the window each frame starts in; a frame starting a new
			 * window is that window's first (frames lie in address order,
			 * less than a window apart) */
			for (uint32_t f = f0 + (uint32_t)(threadIdx.x - 64 * kProd); f < f1;
			     f += 64 * kCons) {
				const uint4 dv = a.desc[f];
				const uint64_t eff = ((uint64_t)dv.y << 32) | dv.x;
				const uint32_t w = (uint32_t)((eff - A0) / kWin);
				dl[f - f0] = make_uint2((uint32_t)(eff - A0), dv.z);
				uint32_t wp = 0xffffffffu;
				if (f > f0) {
					const uint4 dp = a.desc[f - 1];
					wp = (uint32_t)(((((uint64_t)dp.y << 32) | dp.x) - A0) / kWin);
				}
				for (uint32_t k = wp + 1; k <= w && k < kMaxWin; k++)
					wstart[k] = f;
			}
		}
		__syncthreads();
		for (uint32_t k = 0; k < nwin; k++) {
			if (wid < kProd) {
				if (k + 3 < nwin) {
					produce(k + 3);
					/* window k + 3's 8 loads may stay in flight */
					__builtin_amdgcn_s_waitcnt(kVmcntNew);
				} else {
					__builtin_amdgcn_s_waitcnt(0x0f70);
				}
			} else {
				/* the frames starting in window k, 96 at a time */
				const uint32_t g = (uint32_t)((wid - kProd) * (64 / kGroup) + lane / kGroup);
				const int sub = lane & (kGroup - 1);
				/* (clamped to the segment: the probe never trusts LDS
				 * for a global address) */
				const uint32_t fb = min(max(wstart[k], f0), f1);
				const uint32_t fe = min(max(wstart[k + 1], fb), f1);
				for (uint32_t f = fb + g; __ballot(f < fe);
				     f += kFramesPerRound) {
					if (f >= fe)
						continue;
					const uint2 dv = dl[f - f0];
					const uint64_t eff = A0 + dv.x;
					const uint32_t len = dv.y;
					/* the frame's bytes from the ring, 16-byte chunks */
					const uint64_t lo = eff & ~15ull;
					const uint64_t hi = (eff + len + 15) & ~15ull;
					uint32_t s = 0;
					for (uint64_t p = lo + 16 * sub; p < hi; p += 16 * kGroup) {
						const uint32_t o = (uint32_t)((p - A0) % kRing);
						const uint4 v = *reinterpret_cast<const uint4 *>(ring + o);
						s = add_halves(add_halves(add_halves(add_halves(s, v.x), v.y), v.z),
							       v.w);
					}
					for (int m = 1; m < kGroup; m <<= 1)
						s += __shfl_xor(s, m, kGroup);
					/* the header words: the frame's first 64 bytes */
					const uint32_t o0 = (uint32_t)((lo - A0) % kRing);
					const uint4 h = *reinterpret_cast<const uint4 *>(
						ring + ((o0 + 16 * (sub & 3)) % kRing));
					const uint32_t hx = __shfl(h.x, (lane & ~(kGroup - 1)) + 1, 64);
					const uint32_t hy = __shfl(h.y, (lane & ~(kGroup - 1)) + 2, 64);
					if (sub == 0) {
						a.verdict[f] = (uint8_t)(4 ^ (fold16(s) & 1));
						a.rec[f] = make_uint4(fold16(s), h.x, hx, len);
					}
					if (sub < 3) {
						uint8_t *t = a.tup + 44ull * f;
						if (sub < 2)
							*reinterpret_cast<uint4 *>(t + 16 * sub) =
								make_uint4(h.x, h.y, hx, hy);
						else
							*reinterpret_cast<uint3 *>(t + 32) = make_uint3(h.z, h.w, s);
					}
				}
			}
			/* no fence: the producers waited for window k + 2 themselves,
			 * the consumers' ring reads are consumed, and their output
			 * stores need not be complete (a __syncthreads would wait for
			 * window k + 3's loads too) */
			__builtin_amdgcn_s_barrier();
		}
		__syncthreads();
	}
}

} // namespace

extern "C" int stream_probe(const void *pool, uint64_t usize, const void *desc, uint32_t n,
			    void *verdict, void *rec, void *tup, uint32_t *d_ctr, int blocks,
			    void *stream)
{
	Args a;
	a.pool = (const uint8_t *)pool;
	a.usize = usize;
	a.desc = (const uint4 *)desc;
	a.n = n;
	a.verdict = (uint8_t *)verdict;
	a.rec = (uint4 *)rec;
	a.tup = (uint8_t *)tup;
	a.seg_ctr = d_ctr;
	if (hipMemsetAsync(d_ctr, 0, 4, (hipStream_t)stream) != hipSuccess)
		return -1;
	hipLaunchKernelGGL(stream_probe_kernel, dim3(blocks), dim3(1024), 0, (hipStream_t)stream,
			   a);
	return hipGetLastError() == hipSuccess ? 0 : -1;
}
