// SPDX-License-Identifier: GPL-2.0
/* Internal interface between the host C-ABI (xdpgpu.cpp) and the kernels
 * (xdp_rx.hip).  Not installed; include/xdpgpu.h is the public boundary. */
#ifndef XDPGPU_INTERNAL_H
#define XDPGPU_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

#include "xdpgpu.h"

namespace xdpgpu {

/* Blocks of THREADS threads of a kernel resident at once on the current
 * device (occupancy x CUs, at most cap), cached per device ordinal.
 * Contexts on different devices, or threads racing on the first call, each
 * compute the same value; the relaxed atomic makes the race benign. */
template <auto KERN, int THREADS>
static uint32_t resident_blocks_dev(uint32_t cap)
{
	constexpr int kMaxDev = 64;
	static std::atomic<uint32_t> cached[kMaxDev];
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess || dev < 0)
		return cap;
	if (dev < kMaxDev) {
		const uint32_t c = cached[dev].load(std::memory_order_relaxed);
		if (c)
			return c;
	}
	int per_cu = 0;
	hipDeviceProp_t prop;
	if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
	    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, KERN, THREADS, 0) !=
		    hipSuccess ||
	    per_cu <= 0)
		return cap;
	uint32_t c = (uint32_t)per_cu * (uint32_t)prop.multiProcessorCount;
	if (c > cap)
		c = cap;
	if (dev < kMaxDev)
		cached[dev].store(c, std::memory_order_relaxed);
	return c;
}

/* Ordering of a wave's LDS-DMA (global_load_lds) tile staging, made
 * explicit.  The builtins __builtin_amdgcn_s_waitcnt and wave_barrier are
 * IntrNoMem intrinsics: they do not keep LDS loads from moving across them,
 * so the order of "read tile t's windows from LDS" and "DMA tile t+1 into
 * the same LDS" would rest on the compiler's alias analysis of the DMA
 * destination (and its vmcnt insertion on the same analysis).  Inline asm
 * with a memory clobber is a barrier for both the IR and the machine
 * scheduler, and the wait instruction itself is emitted as written.
 *  - lds_dma_landed(): before reading LDS a DMA wrote (read after write):
 *    every vector memory op of this wave, the DMA included, has completed.
 *  - lds_reads_done(): before issuing a DMA into LDS this wave has just
 *    read (write after read): the reads have returned their data. */
__device__ __forceinline__ void lds_dma_landed()
{
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void lds_reads_done()
{
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

/* Lane 0's fetch-and-add of v on an LDS counter, returned to every lane.
 * In asm, waiting for its own result: a compiler-visible LDS atomic gets a
 * vmcnt(0) in front of it while LDS-DMA is pending (the compiler cannot
 * tell the counter from the DMA's destination). */
__device__ __forceinline__ uint32_t lds_fetch_add(uint32_t *ctr, uint32_t v, int lane)
{
	uint32_t r = 0;
	if (lane == 0) {
		const uint32_t addr =
			(uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)ctr;
		asm volatile("ds_add_rtn_u32 %0, %1, %2\n\t"
			     "s_waitcnt lgkmcnt(0)"
			     : "=v"(r)
			     : "v"(addr), "v"(v)
			     : "memory");
	}
	return (uint32_t)__builtin_amdgcn_readfirstlane(r);
}


/* Per-block counter slot layout (u64 each); slots summed by xdpgpu_stats. */
enum {
	CNT_FRAMES = 0,
	CNT_BYTES = 1,
	CNT_VERDICT0 = 2, /* .. +4 */
	CNT_L3_BAD = 7,
	CNT_L4_BAD = 8,
	CNT_L4_ABSENT = 9,
	CNT_FRAG = 10,
	CNT_SLOT = 16,
};

/* Upper bound on the RX kernel grid (blocks of 256 threads): 8 per CU on a
 * 256-CU MI355X.  Sizes the per-block counter area. */
constexpr uint32_t kMaxRxBlocks = 2048;
/* Counter slots of a context slot: one per block of the per-block kernels,
 * then one per wave of the double-buffered RX kernel (xdp_rx_db_kernel). */
constexpr uint32_t kStatSlots = kMaxRxBlocks * 5;
/* Global claim counters of xdp_rx_db_kernel's shared tiles (RxArgs.steal):
 * heads per set, u32 words per head (one 128-byte line each). */
constexpr uint32_t kStealHeads = 16, kStealStride = 32;
/* Shared tiles one block may take: twice its share and 32 more, so that the
 * blocks of every head can drain it (each keeps claiming until its head is
 * empty or it reaches the cap; a head has at least floor(nb / heads) >=
 * nb / (2 heads) blocks). */
__host__ __device__ inline uint64_t steal_cap(uint64_t sh, uint64_t nb)
{
	return 2 * ((sh + nb - 1) / nb) + 32;
}

struct RxArgs {
	uint8_t *umem;
	uint64_t usize;
	const xdpgpu_desc *desc;
	uint32_t n;
	uint32_t tuple_fmt;
	uint8_t *verdict;
	xdpgpu_result *res;
	uint8_t *tup;
	uint32_t flags;
	uint32_t initval;
	unsigned long long *stats; /* [kMaxRxBlocks][CNT_SLOT] or null */
	uint32_t *xlist;           /* exception list, xregion per wave      */
	uint32_t *xcount;          /* exception frames per wave             */
	uint32_t *blist;           /* bulk list (payload beyond the header
				    * window), xregion per wave            */
	uint32_t *bcount;          /* bulk frames per wave                  */
	uint4 *ylist;              /* exception frames whose payload sum the
				    * bulk kernel adds: 16 B entries,
				    * xregion per fast-kernel wave region   */
	uint32_t *ycount;          /* entries per region (atomic)           */
	uint32_t ydefer;           /* exception kernel may defer payload sums */
	uint32_t xregion;          /* set by the launcher: entries per wave
				    * region of both lists                  */
	uint32_t nregions;         /* set by the launcher: fast-kernel waves */
	uint32_t force_generic;    /* 1: defer every frame (diagnostic)     */
	uint32_t frags;            /* XDPGPU_CFG_FRAGS: skip the descriptors
				    * of packets of several (frags.hip)     */
	uint32_t diag;             /* set by the launcher: cfg.tune bits 16-17
				    * (diagnostic kernel variants)          */
	uint32_t v6;               /* set by the launcher: the fast shape
				    * includes untagged IPv6/UDP           */
	uint32_t partner;          /* set by the launcher: 2 a wave claims
				    * shared tiles of its own head, then of
				    * the partner head h ^ 4 (default); 1
				    * its own head only (cfg.tune bit 28)  */
	/* xdp_rx_db_kernel's shared tiles: the last steal_tiles tiles of the
	 * batch are claimed at run time from kStealHeads global counters by
	 * any block done with its own (set by the launcher; 0: none) */
	uint32_t *steal;           /* 2 sets x kStealHeads counters, 128 B
				    * apart: a launch uses set steal_set
				    * and zeroes the other for the next    */
	uint32_t steal_set;
	uint32_t steal_16ths;      /* shared tiles = tiles x steal_16ths / 16
				    * (0: none)                            */
	uint32_t steal_tiles;      /* set by the launcher                  */
	uint32_t win;              /* header window: 64, or 128 (a second
				    * half for long frames starting a line) */
	uint64_t xcap;             /* entries of each deferral list        */
};

/* The RX launch (xdp_rx_db_kernel).  ev (nullable): four event slots, the
 * first recorded before the kernel and the second after it (the other two
 * are the round-1 form's, never recorded). */
hipError_t launch_rx(const RxArgs &a, uint32_t max_blocks, hipStream_t stream, uint32_t tune,
		     hipEvent_t *ev);
/* multi-buffer packets read in place (after launch_frag_count): every
 * complete packet of the batch as one frame, outputs to all its
 * descriptors */
hipError_t launch_rx_packets(const RxArgs &a, uint32_t max_blocks, hipStream_t stream);
hipError_t launch_jhash_words(const uint32_t *words, uint32_t nwords, uint32_t stride,
			      uint32_t n, uint32_t initval, uint32_t variant,
			      uint32_t *out, hipStream_t stream);
uint32_t rx_grid_blocks(uint32_t n, uint32_t max_blocks);
uint32_t rx_xregion(uint32_t n, uint32_t blocks);
hipError_t launch_ceiling(const RxArgs &a, uint32_t blocks, hipStream_t stream);

/* Multi-buffer packets (XDPGPU_CFG_FRAGS, frags.hip): finish the packets
 * the batch cannot complete as ABORTED (before launch_rx_packets). */
struct FragArgs {
	uint8_t *umem;
	uint64_t usize;
	const xdpgpu_desc *desc;
	uint32_t n;
	uint8_t *verdict;
	xdpgpu_result *res;        /* nullable */
	uint8_t *tup;              /* nullable */
	uint32_t tb;               /* tuple bytes, 0 without tuples         */
	unsigned long long *stats; /* block 0's counter slot, or null       */
};
hipError_t launch_frag_count(const FragArgs &a, hipStream_t stream);

/* Host path write-back of ICMPv6 echo replies (xdpgpu_submit): for every
 * descriptor of the batch with verdict TX, bytes [0, min(len, 64)) of its
 * frame (the rewrite of process_packet, af_xdp_user.c:990-1037, touches
 * bytes 0-57) go from the slot's device mirror to the host UMEM as compact
 * records the host scatters after xdpgpu_wait (no kernel writes host
 * memory).  Nothing else of the UMEM is written. */
constexpr uint32_t kEchoBytes = 64;
struct EchoRec {
	uint64_t eff;              /* frame's UMEM offset                   */
	uint32_t len;              /* bytes of b[] that are the frame's     */
	uint32_t rsvd;
	uint8_t b[kEchoBytes];
};
static_assert(sizeof(EchoRec) == 80, "echo record layout");
struct EchoArgs {
	const uint8_t *mirror;
	uint64_t usize;
	const xdpgpu_desc *desc;
	const uint8_t *verdict;
	uint32_t n;
	EchoRec *rec;              /* one record per TX frame               */
	uint32_t *nrec;
};
hipError_t launch_echo_writeback(const EchoArgs &a, hipStream_t stream);

/* XDPGPU_CFG_UMEM_GATHER: a batch's frame bytes from the registered host
 * UMEM (its GPU mapping, read only) into the slot's mirror at the same
 * offsets, 16-byte pieces (hostpath.hip) */
struct GatherArgs {
	const uint8_t *src;        /* the host UMEM's device view            */
	uint8_t *mirror;
	uint64_t usize;
	xdpgpu_desc *desc;         /* device copy of the batch's descriptors */
	const xdpgpu_desc *hdesc;  /* non-null: the caller's page-locked array
				    * (device view), read here and copied into
				    * desc for the kernels after */
	uint32_t n;
	uint32_t over_all;         /* 1: every frame's byte len (multi-buffer
				    * packets); 0: odd lengths only          */
	unsigned long long *nbytes;   /* += the bytes read (host stats), or
				       * null                                 */
	/* XDPGPU_CFG_HOST_COMPACT: non-null, src is the batch's pieces packed
	 * on the host (copied to the device in one transfer) and frame i's
	 * piece starts at src + 16 * poff[i] instead of src + (eff & ~15) */
	const uint32_t *poff;
};
hipError_t launch_umem_gather(const GatherArgs &a, hipStream_t stream);

/* jhash (include/jhash.h:25-52) mixing steps, for the device kernels */
__device__ __forceinline__ uint32_t rol32(uint32_t w, uint32_t s)
{
	return (w << s) | (w >> ((32 - s) & 31));
}

#define JH_MIX(a, b, c)                                   \
	do {                                              \
		a -= c; a ^= rol32(c, 4);  c += b;        \
		b -= a; b ^= rol32(a, 6);  a += c;        \
		c -= b; c ^= rol32(b, 8);  b += a;        \
		a -= c; a ^= rol32(c, 16); c += b;        \
		b -= a; b ^= rol32(a, 19); a += c;        \
		c -= b; c ^= rol32(b, 4);  b += a;        \
	} while (0)

#define JH_FINAL(a, b, c)                                 \
	do {                                              \
		c ^= b; c -= rol32(b, 14);                \
		a ^= c; a -= rol32(c, 11);                \
		b ^= a; b -= rol32(a, 25);                \
		c ^= b; c -= rol32(b, 16);                \
		a ^= c; a -= rol32(c, 4);                 \
		b ^= a; b -= rol32(a, 14);                \
		c ^= b; c -= rol32(b, 24);                \
	} while (0)

/* jhash2 (include/jhash.h:114-142) of len words */
__device__ __forceinline__ uint32_t jhash2_dev(const uint32_t *k, uint32_t len, uint32_t initval)
{
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + (len << 2) + initval;
	while (len > 3) {
		a += k[0];
		b += k[1];
		c += k[2];
		JH_MIX(a, b, c);
		len -= 3;
		k += 3;
	}
	switch (len) {
	case 3:
		c += k[2];
		[[fallthrough]];
	case 2:
		b += k[1];
		[[fallthrough]];
	case 1:
		a += k[0];
		JH_FINAL(a, b, c);
		break;
	default:
		break;
	}
	return c;
}

/* nat64 state tables (v6_state_map and v4_reversemap, nat64_kern.c:17-46):
 * 4-way buckets of one 128-byte line, so a lookup touches one line; the
 * home bucket is fastrange(nat64_slot_hash(key), nbuckets), a full bucket
 * overflows into the next (linear probing over buckets).  `meta`: bits 0-3
 * the slots in use, bit 4 an entry of an earlier home bucket lies further
 * on (probing continues past this bucket), bits 8-11 static_conf of the
 * slots (v6 table).  Deleting an entry clears its use bit only. */
constexpr uint32_t kNat64Ovf = 0x10;
struct Nat64V6Bucket {
	uint4 key[4];              /* IPv6 address words as stored          */
	uint32_t val[4];           /* IPv4 address, host order              */
	uint32_t meta;
	uint32_t pad[3];
	unsigned long long last_seen[4];  /* v6_addr_state.last_seen (ns)   */
};
struct Nat64V4Bucket {
	uint32_t key[4];           /* IPv4 address, host order              */
	uint32_t meta;
	uint32_t pad[3];
	uint4 val[4];              /* IPv6 address words                    */
	uint4 pad2[2];
};
static_assert(sizeof(Nat64V6Bucket) == 128 && sizeof(Nat64V4Bucket) == 128,
	      "one cache line per bucket");

__host__ __device__ inline uint32_t nat64_home(uint32_t h, uint32_t nbuckets)
{
	return (uint32_t)(((uint64_t)h * nbuckets) >> 32);
}

/* One slot of a table written by the host after a dynamic-state commit
 * (nat64_patch_kernel): table 0 v6 (key k6, value v4, last_seen), 1 v4
 * (key v4, value k6); the bucket's meta word in both. */
struct Nat64Patch {
	uint32_t table, bucket, slot, meta;
	uint4 k6;
	uint32_t v4, pad;
	unsigned long long last_seen;
	uint4 pad2;
};
static_assert(sizeof(Nat64Patch) == 64, "patch record");

struct Nat64Args {
	uint8_t *umem;
	uint64_t usize;
	const xdpgpu_desc *desc;
	uint32_t n;
	uint8_t *action;
	xdpgpu_desc *out;
	xdpgpu_nat64_cfg cfg;
	Nat64V6Bucket *v6map;
	uint32_t v6nb;             /* buckets */
	const Nat64V4Bucket *v4map;
	uint32_t v4nb;
	/* fast path (ingress, /96 prefix): allowed-source words and masks,
	 * the prefix's first 12 bytes, as LE u32 of the wire bytes */
	uint32_t allow_w[4], allow_m[4], pref_w[3];
	uint32_t fast;             /* 1: fast kernel + list of slow frames */
	uint32_t diag;             /* cfg.tune bits 12-13 (diagnostic A/B):
				    * 1 no map probe, 2 no frame stores */
	uint32_t *xlist;           /* slow frames, xregion per fast wave    */
	uint32_t *xcount;
	uint32_t xregion, nregions;
	uint64_t xcap;             /* entries of the slow list              */
	/* the fast kernel's shared tiles, as RxArgs.steal (xdp_rx_db_kernel):
	 * counters (nullable), their set, and the tiles (set by the
	 * launcher) */
	uint32_t *steal;
	uint32_t steal_set, steal_16ths, steal_tiles;
	/* dynamic state (xdpgpu_nat64_dynamic): a hit stamps last_seen with
	 * the batch clock `now`; a miss, or a hit on an entry that timed out
	 * (last_seen < thr, not static), is left untouched and listed for the
	 * host's in-order commit (miss_idx / miss_src, count in miss_cnt) */
	uint32_t dyn;
	unsigned long long now, thr;
	uint32_t *miss_idx;
	uint4 *miss_src;
	uint32_t *miss_cnt;
	/* the commit's second pass: xlist is the listed frames in order, ov
	 * the IPv4 address each was given (0: SHOT), no table lookup */
	const uint32_t *ov;
};

hipError_t launch_nat64(const Nat64Args &a, uint32_t max_blocks,
			hipStream_t stream);
hipError_t launch_nat64_patch(Nat64V6Bucket *v6map, Nat64V4Bucket *v4map,
			      const Nat64Patch *p, uint32_t np, hipStream_t stream);
uint32_t nat64_slot_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d);

hipError_t launch_hints(const uint8_t *umem, uint64_t usize,
			const xdpgpu_desc *desc, uint32_t n, uint32_t rx_time_id,
			uint32_t mark_id, xdpgpu_hints *out, hipStream_t stream);
hipError_t launch_jhash(const uint8_t *keys, uint32_t key_len,
			uint32_t stride, uint32_t n, uint32_t initval,
			uint32_t *out, hipStream_t stream);
hipError_t launch_ip_fast_csum(const uint8_t *hdrs, uint32_t stride,
			       uint32_t n, uint16_t *out, hipStream_t stream);
hipError_t launch_synproxy(uint8_t *umem, uint64_t usize, const xdpgpu_desc *desc,
			   uint32_t n, const xdpgpu_synproxy_cfg &cfg, uint8_t *verdict,
			   xdpgpu_desc *out, unsigned long long *synacks,
			   unsigned long long *spread, hipStream_t stream);
/* u64 words of the zeroed counter area launch_synproxy needs */
uint32_t synproxy_spread_words();

} // namespace xdpgpu

#endif
