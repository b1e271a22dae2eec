// SPDX-License-Identifier: GPL-2.0
/*
 * xdp_rx.hip - gfx950 kernels for the AF_XDP receive-path transform.
 *
 * One lane per frame, 64 frames (one wavefront) per tile:
 *
 *   1. lane i loads descriptor i of the tile (16 B, coalesced dwordx4);
 *   2. the wave stages the first WIN bytes of its 64 frames into LDS with
 *      "transposed" loads: in load k, lane l fetches 16-byte chunk
 *      (64k + l) mod CPF of frame (64k + l) / CPF, so consecutive lanes read
 *      consecutive chunks and a packed pool is read as contiguous 1 KiB
 *      wave-instructions; a wave with any non-16-byte-aligned frame falls
 *      back to per-lane byte staging (unaligned-chunk UMEMs);
 *   3. each lane parses its own frame out of LDS (row stride WIN+4 bytes so
 *      that 64 lanes reading the same field hit distinct banks), computes
 *      the IPv4 header checksum, the L4 checksum and the jhash flow key;
 *   4. L4 bytes past the window (large frames) are summed cooperatively:
 *      for each such frame the whole wave streams its payload in 1 KiB
 *      coalesced steps and reduces the 64 partial sums across lanes;
 *   5. verdict, 16-byte result and tuple are written coalesced; per-verdict
 *      counters are kept in scalar registers (ballot + popcount) and reduced
 *      once per block at kernel end.
 *
 * Integer work only (no MFMA); the bound is HBM bandwidth.  Every rule
 * below restates the reference (file:line in comments) or the build-defined
 * verdict surface of SURVEY.md §8a; oracle/xdp_oracle.c is the CPU
 * statement of exactly the same pipeline and is what the tests compare to.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

/* Diagnostic builds (-DXDPGPU_DBG, tools/dbg_build.sh): the accesses of the
 * double-buffered kernel and its tail are bounds-checked (codes 1-9; 10:
 * the echo responder's 64-byte reply store); a violation is
 * counted (g_dbg[2 code]) with its value (g_dbg[2 code + 1]) and the access
 * is skipped.  Read by xdpgpu_debug_read. */
#ifdef XDPGPU_DBG
__device__ unsigned long long g_dbg[64];
__device__ __forceinline__ bool dbg_bad(bool bad, uint32_t code, uint64_t val)
{
	if (bad) {
		atomicAdd(&g_dbg[2 * code], 1ull);
		atomicExch(&g_dbg[2 * code + 1], (unsigned long long)val);
	}
	return bad;
}
#define DBG_BAD(c, code, v) dbg_bad((c), (code), (uint64_t)(v))
#else
#define DBG_BAD(c, code, v) false
#endif

/* Timing builds (-DXDPGPU_STAMPS, tools/dbg_build.sh stamps): each wave of
 * the double-buffered kernel records s_memrealtime (100 MHz) at its start
 * (0), the end of its tile loop (1), its end (2), and the time its tail
 * spends in each kind of batch (4-7, STAMP_ADD); read by
 * xdpgpu_stamps_read. */
#ifdef XDPGPU_STAMPS
constexpr int kStampWaves = 8192;
__device__ unsigned long long g_stamp[8 * kStampWaves];
/* k == 0 also records where the wave runs: HW_ID | XCC_ID << 32 */
#define STAMP(wgid, lane, k)                                                   \
	do {                                                                   \
		if ((lane) == 0 && (wgid) < (uint64_t)kStampWaves) {           \
			g_stamp[8 * (wgid) + (k)] = __builtin_amdgcn_s_memrealtime(); \
			if ((k) == 0)                                          \
				g_stamp[8 * (wgid) + 4] = g_stamp[8 * (wgid) + 5] = \
				g_stamp[8 * (wgid) + 6] = g_stamp[8 * (wgid) + 7] = 0; \
			if ((k) == 0)                                          \
				g_stamp[8 * (wgid) + 3] =                      \
					(unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | \
					((unsigned long long)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32); \
		}                                                              \
	} while (0)
/* time (ticks) a wave spends in its tail's exception (4), bulk (5) and
 * payload (6) batches and waiting for the exception batches (7) */
#define STAMP_T0() unsigned long long st_t0_ = __builtin_amdgcn_s_memrealtime()
#define STAMP_ADD(wgid, lane, k)                                               \
	do {                                                                   \
		const unsigned long long st_t1_ = __builtin_amdgcn_s_memrealtime(); \
		if ((lane) == 0 && (wgid) < (uint64_t)kStampWaves)             \
			g_stamp[8 * (wgid) + (k)] += st_t1_ - st_t0_;          \
		st_t0_ = st_t1_;                                               \
	} while (0)
#else
#define STAMP(wgid, lane, k) do { } while (0)
#define STAMP_T0() do { } while (0)
#define STAMP_ADD(wgid, lane, k) do { } while (0)
#endif

/* ------------------------------------------------------------------ */
/* one's-complement helpers                                            */

/* Fold to 16 bits with end-around carry: 0 -> 0, else 1..0xffff, equal to
 * the value mod 0xffff (0xffff standing for 0).  Because every sum on the
 * path is of non-negative terms and, where it matters, provably non-zero
 * (the pseudo header, a version nibble), this makes any summation order
 * bit-exact with lib_checksum.h's sequential loops (SURVEY.md §8a a-C1). */
__device__ __forceinline__ uint32_t fold16(uint64_t x)
{
	x = (x & 0xffffffffull) + (x >> 32);
	x = (x & 0xffffffffull) + (x >> 32);
	uint32_t y = (uint32_t)x;
	y = (y & 0xffff) + (y >> 16);
	y = (y & 0xffff) + (y >> 16);
	return y;
}

/* the sum of a dword's two 16-bit halves (v_sad_u16 against zero) */
__device__ __forceinline__ uint32_t halves(uint32_t d)
{
	return __builtin_amdgcn_sad_u16(d, 0u, 0u);
}

/* acc + the halves of a 16-byte chunk's four dwords, one v_sad_u16 each */
__device__ __forceinline__ uint32_t add_chunk(uint32_t acc, uint4 v)
{
	acc = __builtin_amdgcn_sad_u16(v.x, 0u, acc);
	acc = __builtin_amdgcn_sad_u16(v.y, 0u, acc);
	acc = __builtin_amdgcn_sad_u16(v.z, 0u, acc);
	return __builtin_amdgcn_sad_u16(v.w, 0u, acc);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v)
{
	return ((v & 0xff) << 8) | ((v >> 8) & 0xff);
}

/* Byte mask of the dword at byte position o keeping bytes in [lo, hi). */
__device__ __forceinline__ uint32_t keep_mask(uint64_t o, uint64_t lo,
					      uint64_t hi)
{
	uint64_t st = lo > o ? lo - o : 0;
	uint64_t en = hi > o ? hi - o : 0;
	if (st > 4)
		st = 4;
	if (en > 4)
		en = 4;
	if (en <= st)
		return 0;
	uint32_t nb = (uint32_t)(en - st);
	return (0xffffffffu >> (32 - 8 * nb)) << (8 * (uint32_t)st);
}

/* Byte masks of the four dwords of the 16-byte chunk at p keeping the bytes
 * in [lo, hi): 32-bit arithmetic on the chunk-relative bounds. */
__device__ __forceinline__ uint4 chunk_keep(uint64_t p, uint64_t lo, uint64_t hi)
{
	const int32_t a0 = lo > p ? (int32_t)(lo - p < 16 ? lo - p : 16) : 0;
	const int32_t b0 = hi > p ? (int32_t)(hi - p < 16 ? hi - p : 16) : 0;
	uint32_t m[4];
#pragma unroll
	for (int j = 0; j < 4; j++) {
		int32_t st = a0 - 4 * j, en = b0 - 4 * j;
		st = st < 0 ? 0 : st > 4 ? 4 : st;
		en = en < 0 ? 0 : en > 4 ? 4 : en;
		const uint32_t fe = en ? (0xffffffffu >> ((32 - 8 * en) & 31)) : 0u;
		const uint32_t fs = st ? (0xffffffffu >> ((32 - 8 * st) & 31)) : 0u;
		m[j] = fe & ~fs;
	}
	return make_uint4(m[0], m[1], m[2], m[3]);
}

/* A 128-byte window's second half (RxArgs.win 128): staged for a frame
 * longer than 64 bytes whose first byte starts a 128-byte line (its bytes
 * [64, 128) are then the rest of that line, which the bulk pass would
 * otherwise fetch again) and which the UMEM's 16-byte rounded size holds.
 * The tile loop's DMA (issue_win) and the bulk pass (bulk_batch) decide it
 * the same way. */
__device__ __forceinline__ bool win_hi(const RxArgs &a, uint64_t eff, uint32_t len)
{
	return a.win == 128 && len > 64 && !(eff & 127) &&
	       eff + 128 <= ((a.usize + 15) & ~15ull);
}

/* af_xdp_user.c:590-606 csum16_add / csum16_sub / csum_replace2 */
__device__ __forceinline__ uint32_t c16_add(uint32_t csum, uint32_t addend)
{
	uint32_t r = (csum + addend) & 0xffff;
	return (r + (r < addend ? 1u : 0u)) & 0xffff;
}

__device__ __forceinline__ uint32_t csum_replace2(uint32_t sum, uint32_t old,
						  uint32_t nw)
{
	uint32_t t = c16_add(~sum & 0xffff, ~old & 0xffff);
	return ~c16_add(t, nw) & 0xffff;
}

/* process_packet's echo reply (af_xdp_user.c:968-1040) of an untagged
 * ICMPv6 echo request whose first 64 bytes are d: MACs and addresses
 * swapped, type 129, csum_replace2 of the type word, written over the
 * frame's first 64 bytes at fp as whole 16-byte chunks */
__device__ __forceinline__ void echo_reply_store(uint8_t *fp, const uint32_t (&d)[16])
{
	uint32_t o[16];
	auto byte = [&](int b) -> uint32_t { return (d[b >> 2] >> (8 * (b & 3))) & 0xff; };
	auto src = [&](int b) -> int {
		return b < 6 ? b + 6 : b < 12 ? b - 6 : (b >= 22 && b < 38) ? b + 16
		       : (b >= 38 && b < 54) ? b - 16 : b;
	};
#pragma unroll
	for (int w = 0; w < 16; w++)
		o[w] = byte(src(4 * w)) | (byte(src(4 * w + 1)) << 8) |
		       (byte(src(4 * w + 2)) << 16) | (byte(src(4 * w + 3)) << 24);
	/* byte 54: type 129; bytes 56-57: the check word */
	const uint32_t ck = csum_replace2(d[14] & 0xffff, 0x0080, 0x0081);
	o[13] = (o[13] & 0xff00ffffu) | (129u << 16);
	o[14] = (o[14] & 0xffff0000u) | ck;
	uint4 *fw = reinterpret_cast<uint4 *>(fp);
	fw[0] = make_uint4(o[0], o[1], o[2], o[3]);
	fw[1] = make_uint4(o[4], o[5], o[6], o[7]);
	fw[2] = make_uint4(o[8], o[9], o[10], o[11]);
	fw[3] = make_uint4(o[12], o[13], o[14], o[15]);
}

/* ------------------------------------------------------------------ */
/* jhash (include/jhash.h:25-52), word form; jhash(key, 44) equals
 * jhash2(words, 11) on little-endian (jhash.h:68-142).                 */

/* rol32, JH_MIX, JH_FINAL: xdpgpu_internal.h */

__device__ __forceinline__ uint32_t jhash_key44(const uint32_t k[11],
						uint32_t initval)
{
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + 44u + initval;
	a += k[0]; b += k[1]; c += k[2];
	JH_MIX(a, b, c);
	a += k[3]; b += k[4]; c += k[5];
	JH_MIX(a, b, c);
	a += k[6]; b += k[7]; c += k[8];
	JH_MIX(a, b, c);
	a += k[9]; b += k[10];
	JH_FINAL(a, b, c);
	return c;
}

/* ------------------------------------------------------------------ */
/* frame byte access: LDS window first, global beyond it                */

/* Byte off of the multi-buffer packet whose descriptors are d[head..last]
 * (the concatenation of its fragments, as frags.hip's oracle sees it; the
 * byte one past its end is the one after its last fragment in the UMEM,
 * udp_csum's over-read byte, then zeros).  A walk over the descriptors:
 * only headers past the first fragment, and short first fragments, come
 * here. */
__device__ uint32_t pkt_byte(const uint8_t *umem, uint64_t usize, const xdpgpu_desc *d,
			     uint64_t head, uint32_t last, uint32_t off)
{
	uint64_t end = 0;
	for (uint64_t j = head; j <= last; j++) {
		const xdpgpu_desc x = d[j];
		const uint64_t e = (x.addr & ((1ull << 48) - 1)) + (x.addr >> 48);
		if (off < x.len)
			return umem[e + off];
		off -= x.len;
		end = e + x.len;
	}
	return (off == 0 && end < usize) ? umem[end] : 0u;
}

template <int WIN, bool DEEP>
struct FrameView {
	const uint32_t *w;    /* this lane's LDS row (dword aligned) */
	const uint8_t *umem;  /* UMEM base (wave uniform)            */
	uint64_t eff;         /* this frame's UMEM offset             */
	uint64_t usize;
	/* common path (DEEP false): set when a byte past the window was
	 * wanted; the lane is then parsed again with DEEP true, which reads
	 * such bytes from global memory */
	uint32_t deep;
	/* a multi-buffer packet read in place: bytes from flen on are the
	 * later fragments' (pkt_byte); flen ~0 for a frame */
	uint32_t flen;
	uint32_t plast;
	uint64_t phead;
	const xdpgpu_desc *pdesc;

	__device__ __forceinline__ uint32_t gbyte(uint32_t off) const
	{
		if (off >= flen)
			return pkt_byte(umem, usize, pdesc, phead, plast, off);
		const uint64_t at = eff + off;
		return at < usize ? umem[at] : 0;
	}
	__device__ __forceinline__ uint32_t wd(uint32_t off)
	{
		if constexpr (!DEEP)
			deep |= off >= (uint32_t)WIN;
		return w[(off >> 2) & (WIN / 4 - 1)];
	}
	__device__ __forceinline__ uint32_t b8(uint32_t off)
	{
		if constexpr (DEEP) {
			if (off >= (uint32_t)WIN)
				return gbyte(off);
		}
		return (wd(off) >> ((off & 3) * 8)) & 0xff;
	}
	/* network-order 16-bit field at an even offset (every L2/L3/L4
	 * field position is even: tags are 4 B, header lengths 4 B units) */
	__device__ __forceinline__ uint32_t be16(uint32_t off)
	{
		if constexpr (DEEP) {
			if (off + 1 >= (uint32_t)WIN || (off & 1))
				return (b8(off) << 8) | b8(off + 1);
		}
		const uint32_t d = wd(off);
		return bswap16((off & 2) ? (d >> 16) : (d & 0xffff));
	}
	/* 16 bits as a little-endian load of the wire bytes */
	__device__ __forceinline__ uint32_t le16(uint32_t off)
	{
		return bswap16(be16(off));
	}
	__device__ __forceinline__ uint32_t le32(uint32_t off)
	{
		return le16(off) | (le16(off + 2) << 16);
	}
	/*
	 * Exact integer sum of the bytes in [lo, min(hi, WIN)) weighted as
	 * little-endian dwords at frame-relative positions: byte r counts
	 * 2^(8*(r&3)).  Congruent mod 0xffff to the lib_checksum.h sum of LE
	 * 16-bit words, and 0 only if every byte is 0.  Masks touch only the
	 * first and last dword.
	 */
	__device__ __forceinline__ uint64_t win_sum(uint32_t lo, uint32_t hi) const
	{
		const uint32_t h = hi < (uint32_t)WIN ? hi : (uint32_t)WIN;
		if (lo >= h)
			return 0;
		const uint32_t o0 = lo & ~3u, oL = (h - 1) & ~3u;
		uint64_t s = 0;
		for (uint32_t o = o0; o <= oL; o += 4)
			s += w[o >> 2];
		const uint32_t head = w[o0 >> 2] & ~(0xffffffffu << (8 * (lo & 3)));
		const uint32_t tb = h - oL;          /* 1..4 bytes kept */
		const uint32_t tail = tb >= 4 ? 0u :
				      (w[oL >> 2] & (0xffffffffu << (8 * tb)));
		return s - head - tail;
	}
	/* The same weighting for the bytes of [lo, hi) past the window. */
	__device__ uint64_t glob_sum(uint32_t lo, uint32_t hi)
	{
		if constexpr (!DEEP) {
			deep |= hi > (uint32_t)WIN;
			return 0;
		}
		uint64_t s = 0;
		for (uint32_t o = lo > (uint32_t)WIN ? lo : (uint32_t)WIN; o < hi; o++)
			s += (uint64_t)gbyte(o) << (8 * (o & 3));
		return s;
	}
};

/* weight of the 16-bit word at even frame position x in the sums above */
__device__ __forceinline__ uint64_t word_weight(uint32_t x, uint32_t v)
{
	return (x & 2) ? ((uint64_t)v << 16) : (uint64_t)v;
}

/* ------------------------------------------------------------------ */
/* per-lane parse state, packed: it stays live across the wave's
 * cooperative payload loop, so it is kept to eight registers            */

enum : uint32_t { ST_ABORT = 0, ST_PASS = 2, ST_GO = 0xff };

struct Lane {
	uint32_t m;      /* [7:0] state  [15:8] L4 proto / next header
			  * [23:16] l3 offset  [25:24] VLAN tags  26 ipv4
			  * 27 ipv6  28 frag  29 has_l4  30 has_csum  31 over-read */
	uint32_t l4cl;   /* [15:0] l4 offset  [31:16] L4 checksum length  */
	uint32_t chkvid; /* [15:0] L4 check offset  [27:16] outer VLAN id  */
	uint32_t cks;    /* [15:0] stored IPv4 check  [31:16] stored L4 check */
	uint32_t sums;   /* [15:0] IPv4 header sum  [31:16] L4 window sum;
			  * folded to 16 bits (residue and zero-ness kept),
			  * check words excluded */
	uint32_t sa, da; /* IPv4 addresses: LE loads of the wire bytes */
	uint32_t ports;  /* sport | dport << 16: LE loads of the wire bytes */

	__device__ __forceinline__ uint32_t st() const { return m & 0xff; }
	__device__ __forceinline__ uint32_t nh() const { return (m >> 8) & 0xff; }
	__device__ __forceinline__ uint32_t l3() const { return (m >> 16) & 0xff; }
	__device__ __forceinline__ uint32_t nvlan() const { return (m >> 24) & 3; }
	__device__ __forceinline__ bool ipv4() const { return (m >> 26) & 1; }
	__device__ __forceinline__ bool ipv6() const { return (m >> 27) & 1; }
	__device__ __forceinline__ bool frag() const { return (m >> 28) & 1; }
	__device__ __forceinline__ bool has_l4() const { return (m >> 29) & 1; }
	__device__ __forceinline__ bool has_csum() const { return (m >> 30) & 1; }
	__device__ __forceinline__ uint32_t over() const { return m >> 31; }
	__device__ __forceinline__ uint32_t l4() const { return l4cl & 0xffff; }
	__device__ __forceinline__ uint32_t cl() const { return l4cl >> 16; }
	__device__ __forceinline__ uint32_t rhi() const { return l4() + cl() + over(); }
	__device__ __forceinline__ uint32_t chk() const { return chkvid & 0xffff; }
	__device__ __forceinline__ uint32_t vid() const { return chkvid >> 16; }
	__device__ __forceinline__ uint32_t c3() const { return cks & 0xffff; }
	__device__ __forceinline__ uint32_t c4() const { return cks >> 16; }
	__device__ __forceinline__ uint32_t s3() const { return sums & 0xffff; }
	__device__ __forceinline__ uint32_t s4() const { return sums >> 16; }
};

/* The pipeline of oracle/xdp_oracle.c frame_pipeline(), up to the sums. */
template <int WIN, bool DEEP>
__device__ __forceinline__ Lane parse_lane(FrameView<WIN, DEEP> &F,
					   uint32_t end)
{
	Lane L;
	L.m = ST_ABORT;
	L.l4cl = L.chkvid = L.cks = L.sums = 0;
	L.sa = L.da = L.ports = 0;

	/* parse_ethhdr_vlan, parsing_helpers.h:86-129, VLAN_MAX_DEPTH 2 */
	if (end < 14)
		return L;
	uint32_t proto = F.be16(12);
	uint32_t l3 = 14, nvlan = 0, vid = 0;
#pragma unroll
	for (int i = 0; i < 2; i++) {
		if (proto != 0x8100 && proto != 0x88A8)
			break;
		if (l3 + 4 > end)
			break;
		if (i == 0)
			vid = F.be16(l3) & 0x0fff;
		proto = F.be16(l3 + 2);
		l3 += 4;
		nvlan++;
	}

	/* af_xdp_kern.c:114-148 parse_pkt__is_ARP_or_NDP */
	if (proto == 0x0806) {
		L.m = ST_PASS;
		return L;
	}
	const bool ipv4 = proto == 0x0800;
	const bool ipv6 = proto == 0x86DD;
	uint32_t ip_end = 0, nonfirst = 0, frag = 0, nh = 0, l4 = 0;
	uint32_t s3 = 0, c3 = 0;

	if (ipv6) {
		/* parse_ip6hdr :174-194 + skip_ip6hdrext :139-172 */
		if (l3 + 40 > end)
			return L;
		if ((F.b8(l3) >> 4) != 6)
			return L;
		uint32_t cur = l3 + 40;
		nh = F.b8(l3 + 6);
		int frag_at = -1;
		bool found = false;
		for (int i = 0; i < 6; i++) {
			if (cur + 2 > end)
				return L;
			if (nh == 0 || nh == 60 || nh == 43 || nh == 135) {
				uint32_t hl = F.b8(cur + 1);
				nh = F.b8(cur);
				cur += (hl + 1) * 8;
			} else if (nh == 51) {
				uint32_t hl = F.b8(cur + 1);
				nh = F.b8(cur);
				cur += (hl + 2) * 4;
			} else if (nh == 44) {
				frag_at = (int)cur;
				nh = F.b8(cur);
				cur += 8;
			} else {
				found = true;
				break;
			}
		}
		if (!found)
			return L;
		l4 = cur;
		if (nh == 58) {
			/* parse_icmp6hdr :224-237; NDP 133..137 -> PASS */
			if (cur + 8 > end)
				return L;
			const uint32_t t = F.b8(cur);
			if (t >= 133 && t <= 137) {
				L.m = ST_PASS;
				return L;
			}
		}
		ip_end = l3 + 40 + F.be16(l3 + 4);
		if (ip_end > end || cur > ip_end)
			return L;
		if (frag_at >= 0) {
			frag = 1;
			if (F.be16((uint32_t)frag_at + 2) >> 3)
				nonfirst = 1;
		}
	} else if (ipv4) {
		/* parse_iphdr :196-222 */
		if (l3 + 20 > end)
			return L;
		const uint32_t vihl = F.b8(l3);
		if ((vihl >> 4) != 4)
			return L;
		const uint32_t hl = (vihl & 0xf) * 4;
		if (hl < 20)
			return L;
		if (l3 + hl > end)
			return L;
		nh = F.b8(l3 + 9);
		const uint32_t tot = F.be16(l3 + 2);
		if (tot < hl || l3 + tot > end)
			return L;
		ip_end = l3 + tot;
		l4 = l3 + hl;
		const uint32_t fo = F.be16(l3 + 6) & 0x3fff;
		if (fo) {
			frag = 1;
			if (fo & 0x1fff)
				nonfirst = 1;
		}
		/* header sum with the check word zeroed (af_xdp_user.c:664):
		 * exact integer sum minus the check's own term */
		c3 = F.le16(l3 + 10);
		uint64_t s = F.win_sum(l3, l3 + hl);
		if (l3 + hl > (uint32_t)WIN)
			s += F.glob_sum(l3, l3 + hl);
		s3 = fold16(s - word_weight(l3 + 10, c3));
		L.sa = F.le32(l3 + 12);
		L.da = F.le32(l3 + 16);
	}

	uint32_t has_l4 = 0, has_csum = 0, cl = 0, chk = 0;
	if ((ipv4 || ipv6) && !nonfirst) {
		if (nh == 17) {
			/* parse_udphdr :272-290 */
			if (l4 + 8 > end)
				return L;
			const uint32_t ulen = F.be16(l4 + 4);
			if (ulen < 8)
				return L;
			has_l4 = 1;
			if (!frag) {
				if (l4 + ulen > ip_end)
					return L;
				cl = ulen;
				chk = l4 + 6;
				has_csum = 1;
			}
		} else if (nh == 6) {
			/* parse_tcphdr :295-318 */
			if (l4 + 20 > end)
				return L;
			const uint32_t thl = (F.b8(l4 + 12) >> 4) * 4;
			if (thl < 20 || l4 + thl > end)
				return L;
			has_l4 = 1;
			if (!frag) {
				cl = ip_end - l4;
				if (cl < thl)
					return L;
				chk = l4 + 16;
				has_csum = 1;
			}
		} else if ((nh == 1 && ipv4) || (nh == 58 && ipv6)) {
			/* parse_icmphdr / parse_icmp6hdr :224-252 */
			if (l4 + 8 > end)
				return L;
			has_l4 = 1;
			if (!frag) {
				cl = ip_end - l4;
				if (cl < 8)
					return L;
				chk = l4 + 2;
				has_csum = 1;
			}
		}
		if (has_l4 && (nh == 6 || nh == 17))
			L.ports = F.le16(l4) | (F.le16(l4 + 2) << 16);
	}

	uint32_t over = 0, c4 = 0, s4 = 0;
	if (has_csum) {
		/* udp_csum over-reads one byte for an odd length
		 * (lib_checksum.h:175-176); csum_partial zero-pads (ICMP, v6) */
		over = (ipv4 && nh != 1) ? (cl & 1) : 0;
		c4 = F.le16(chk);
		uint64_t s = F.win_sum(l4, l4 + cl + over);
		if (chk < (uint32_t)WIN)      /* else removed in the wave pass */
			s -= word_weight(chk, c4);
		s4 = fold16(s);
	}
	L.m = ST_GO | (nh << 8) | (l3 << 16) | (nvlan << 24) |
	      ((uint32_t)ipv4 << 26) | ((uint32_t)ipv6 << 27) | (frag << 28) |
	      (has_l4 << 29) | (has_csum << 30) | (over << 31);
	L.l4cl = l4 | (cl << 16);
	L.chkvid = chk | (vid << 16);
	L.cks = c3 | (c4 << 16);
	L.sums = s3 | (s4 << 16);
	return L;
}

/* ------------------------------------------------------------------ */
/* wave helpers                                                         */

__device__ __forceinline__ uint32_t readlane32(uint32_t v, int src)
{
	return (uint32_t)__builtin_amdgcn_readlane((int)v, src);
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v)
{
#pragma unroll
	for (int m = 32; m >= 1; m >>= 1)
		v += (uint32_t)__shfl_xor((int)v, m, kWave);
	return v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v)
{
#pragma unroll
	for (int m = 32; m >= 1; m >>= 1) {
		uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
		uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
		v += ((uint64_t)hi << 32) | lo;
	}
	return v;
}

__device__ __forceinline__ uint4 load_desc(const xdpgpu_desc *d, uint64_t i,
					   uint32_t n)
{
	if (i < n)
		return *reinterpret_cast<const uint4 *>(d + i);
	return make_uint4(0, 0, 0, 0);
}

/* Issue the transposed 16-byte window loads of one tile into registers.
 * In load k, lane l fetches chunk (64k + l) % CPF of frame (64k + l) / CPF,
 * so a packed pool is read as contiguous 1 KiB wave-instructions.  Returns
 * true (and issues nothing) when a frame of the tile is not 16-byte
 * aligned: the caller then stages bytes per lane. */
template <int WIN>
__device__ __forceinline__ bool issue_window(const RxArgs &a, uint4 dv,
					     int lane, uint64_t *dtab,
					     uint4 *fv)
{
	constexpr int CPF = WIN / 16;
	const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
	const uint32_t len = dv.z;
	const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
	const bool valid = (dv.x | dv.y | dv.z) != 0 && (uint64_t)len <= a.usize &&
			   eff <= a.usize - len;
	if (__ballot(valid && (eff & 15)))
		return true;
	/* per-frame staging word: eff << 8 | chunks to load (those starting
	 * at or before len: the udp_csum over-read byte included) */
	uint32_t nch = (len >> 4) + 1;
	if (nch > (uint32_t)CPF)
		nch = CPF;
	dtab[lane] = valid ? ((eff << 8) | nch) : 0ull;
	__builtin_amdgcn_wave_barrier();
#pragma unroll
	for (int k = 0; k < CPF; k++) {
		const int q = k * kWave + lane;
		const uint64_t e = dtab[q / CPF];
		const int ch = q % CPF;
		const uint64_t src = (e >> 8) + 16ull * ch;
		uint4 v = make_uint4(0, 0, 0, 0);
		if ((uint32_t)ch < (uint32_t)(e & 0xff) && src < a.usize) {
			v = *reinterpret_cast<const uint4 *>(a.umem + src);
			if (src + 16 > a.usize) {
				const uint4 m = chunk_keep(src, src, a.usize);
				v.x &= m.x;
				v.y &= m.y;
				v.z &= m.z;
				v.w &= m.w;
			}
		}
		fv[k] = v;
	}
	return false;
}

/* Write the chunks loaded by issue_window into the per-frame LDS rows. */
template <int WIN>
__device__ __forceinline__ void commit_window(uint32_t *win, const uint4 *fv,
					      int lane)
{
	constexpr int CPF = WIN / 16;
	constexpr int SDW = WIN / 4 + 1;
#pragma unroll
	for (int k = 0; k < CPF; k++) {
		const int q = k * kWave + lane;
		uint32_t *dst = win + (q / CPF) * SDW + (q % CPF) * 4;
		dst[0] = fv[k].x;
		dst[1] = fv[k].y;
		dst[2] = fv[k].z;
		dst[3] = fv[k].w;
	}
}

/* ------------------------------------------------------------------ */
/* the RX kernel                                                        */

/* Wave counters (wave-uniform, scalar registers) */
struct Counters {
	uint32_t c[CNT_FRAG + 1];
	uint64_t bytes; /* per lane */
};

/*
 * L4 bytes past the header window, summed by the whole wave: for every lane
 * in `need` the wave streams that frame's range in 1 KiB coalesced steps and
 * reduces the 64 partial sums.  Returns, in the owning lane, the folded sum
 * (frame-relative parity; check word removed if it lies in the range).
 */
template <int WIN>
__device__ __forceinline__ uint32_t ext_sums(const RxArgs &a, bool need,
					     uint64_t eff, uint32_t l4,
					     uint32_t rhi, uint32_t chk,
					     uint32_t c4, int lane)
{
	constexpr int G = 4;   /* frames whose 1 KiB steps are in flight together */
	uint64_t mask = __ballot(need);
	uint32_t out = 0;
	while (mask) {
		int src[G];
		uint64_t lo[G], lim[G], seff[G];
		uint32_t acc[G];
		int nf = 0;
		uint64_t steps = 0;   /* 1 KiB steps of the longest frame */
#pragma unroll
		for (int k = 0; k < G; k++) {
			src[k] = 0;
			lo[k] = lim[k] = seff[k] = 0;
			acc[k] = 0;
			if (mask) {
				const int sl = __builtin_ctzll(mask);
				mask &= mask - 1;
				src[k] = sl;
				seff[k] = ((uint64_t)readlane32((uint32_t)(eff >> 32), sl) << 32) |
					  readlane32((uint32_t)eff, sl);
				const uint32_t sl4 = readlane32(l4, sl);
				const uint64_t hi = seff[k] + readlane32(rhi, sl);
				lo[k] = seff[k] + (sl4 > (uint32_t)WIN ? sl4 : (uint32_t)WIN);
				lim[k] = hi < a.usize ? hi : a.usize;
				const uint64_t st = (lim[k] - (lo[k] & ~15ull) + 1023) / 1024;
				steps = st > steps ? st : steps;
				nf = k + 1;
			}
		}
		for (uint64_t s = 0; s < steps; s++) {
			uint4 v[G];
			uint64_t p[G];
#pragma unroll
			for (int k = 0; k < G; k++) {
				p[k] = (lo[k] & ~15ull) + 1024 * s + 16ull * lane;
				v[k] = make_uint4(0, 0, 0, 0);
				if (k < nf && p[k] < lim[k])
					v[k] = *reinterpret_cast<const uint4 *>(a.umem + p[k]);
			}
#pragma unroll
			for (int k = 0; k < G; k++) {
				if (p[k] < lo[k] || p[k] + 16 > lim[k]) {
					const uint4 m = chunk_keep(p[k], lo[k], lim[k]);
					v[k].x &= m.x;
					v[k].y &= m.y;
					v[k].z &= m.z;
					v[k].w &= m.w;
				}
				acc[k] = add_chunk(acc[k], v[k]);
			}
		}
#pragma unroll
		for (int k = 0; k < G; k++) {
			if (k >= nf)
				break;
			/* exact: a range is at most 64 KiB, so the raw sum of
			 * 16-bit halves fits 32 bits */
			uint32_t t = wave_sum32(acc[k]);
			if (readlane32(chk, src[k]) >= (uint32_t)WIN) {
				const uint32_t c = readlane32(c4, src[k]);
				t -= (seff[k] & 1) ? bswap16(c) : c;
			}
			uint32_t f = fold16(t);
			if (seff[k] & 1)     /* absolute vs frame-relative parity */
				f = bswap16(f);
			if (lane == src[k])
				out = f;
		}
	}
	return out;
}

/*
 * ext_sums for multi-buffer packets read in place: the range [max(l4, WIN),
 * rhi) of each lane in `need` (packet head head..last, logical offsets)
 * streamed by the whole wave fragment by fragment, 4 KiB per wave-step;
 * a fragment whose UMEM offset and packet offset differ in parity is summed
 * with its bytes swapped within each 16-bit half, so that every fragment
 * adds in the packet's own word pairing (exact, the check word removed
 * there).  The byte past the packet is the one after its last fragment.
 */
__device__ __forceinline__ uint32_t swap_in_halves(uint32_t x)
{
	return ((x & 0x00ff00ffu) << 8) | ((x >> 8) & 0x00ff00ffu);
}

/* The payload sums of the multi-buffer packets of a batch (the lanes with
 * need): packet bytes [max(l4, WIN), rhi) summed fragment by fragment, each
 * fragment's part with the parity of its offset in the packet, the check
 * word taken out where it lies past the window.  Four packets at a time,
 * 16 lanes each, 1 KiB of a packet a step (kPktU 16-byte loads a lane):
 * four chains of dependent loads run at once where round 5's form (the
 * whole wave on one packet at a time, 4 KiB a step) ran one.  262 144 x
 * 9000 B packets in 4 KiB fragments: 0.490 vs 0.587-0.602 ms, alternating
 * processes on one box (tools/r06_pk_session.sh); the next fragment's
 * descriptor loaded under the current one's steps was slower (0.505-0.515).
 * The packet kernel runs at two blocks a CU for it (166 VGPRs, no spill;
 * 128 spilled). */
constexpr int kPktG = 4, kPktL = kWave / kPktG, kPktU = 4;
template <int WIN>
__device__ uint32_t pkt_ext_sums(const RxArgs &a, bool need, uint64_t head, uint32_t last,
				 uint32_t l4, uint32_t rhi, uint32_t chk, uint32_t c4,
				 int lane)
{
	const int grp = lane / kPktL, gl = lane % kPktL;
	uint64_t mask = __ballot(need);
	uint32_t out = 0;
	while (mask) {
		/* group g takes the g-th lowest packet left (none: -1) */
		int sl = -1;
		uint64_t m = mask;
#pragma unroll
		for (int g = 0; g < kPktG; g++) {
			const int b = m ? __builtin_ctzll(m) : -1;
			if (g == grp)
				sl = b;
			m &= m - 1;
		}
		mask = m;
		const int src = sl >= 0 ? sl : 0;
		/* (descriptor indices are below a.n, a u32) */
		const uint32_t first = (uint32_t)__shfl((int)(uint32_t)head, src, kWave);
		const uint32_t lst = (uint32_t)__shfl((int)last, src, kWave);
		const uint32_t sl4 = (uint32_t)__shfl((int)l4, src, kWave);
		const uint32_t hi = (uint32_t)__shfl((int)rhi, src, kWave);
		const uint32_t lo = sl4 > (uint32_t)WIN ? sl4 : (uint32_t)WIN;
		uint32_t acc = 0;
		if (sl >= 0) {
			uint32_t o = 0;       /* the fragment's packet offset */
			for (uint32_t j = first; j <= lst && o < hi; j++) {
				const uint4 d = *reinterpret_cast<const uint4 *>(a.desc + j);
				const uint64_t addr = ((uint64_t)d.y << 32) | d.x;
				const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
				const uint32_t dlen = d.z;
				const uint32_t fend = o + dlen + (j == lst ? 1u : 0u);
				const uint32_t x0 = lo > o ? lo : o, x1 = hi < fend ? hi : fend;
				if (x0 < x1) {
					const uint64_t p0 = eff + (x0 - o);
					uint64_t p1 = eff + (x1 - o);
					p1 = p1 < a.usize ? p1 : a.usize;
					const bool sw = ((eff - o) & 1) != 0;
					for (uint64_t b = p0 & ~15ull; b < p1; b += kPktU * 16 * kPktL) {
						uint4 v[kPktU];
						uint64_t q[kPktU];
#pragma unroll
						for (int k = 0; k < kPktU; k++) {
							q[k] = b + 16ull * (gl + kPktL * k);
							v[k] = make_uint4(0, 0, 0, 0);
							if (q[k] < p1)
								v[k] = *reinterpret_cast<const uint4 *>(a.umem + q[k]);
						}
#pragma unroll
						for (int k = 0; k < kPktU; k++) {
							if (q[k] < p0 || q[k] + 16 > p1) {
								const uint4 mk = chunk_keep(q[k], p0, p1);
								v[k].x &= mk.x;
								v[k].y &= mk.y;
								v[k].z &= mk.z;
								v[k].w &= mk.w;
							}
							if (sw) {
								v[k].x = swap_in_halves(v[k].x);
								v[k].y = swap_in_halves(v[k].y);
								v[k].z = swap_in_halves(v[k].z);
								v[k].w = swap_in_halves(v[k].w);
							}
							acc += halves(v[k].x) + halves(v[k].y) + halves(v[k].z) +
							       halves(v[k].w);
						}
					}
				}
				o += dlen;
			}
		}
		/* the group's sum (16 lanes), the check word out, folded */
#pragma unroll
		for (int off = 1; off < kPktL; off <<= 1)
			acc += (uint32_t)__shfl_xor((int)acc, off, kPktL);
		const uint32_t schk = (uint32_t)__shfl((int)chk, src, kWave);
		const uint32_t sc4 = (uint32_t)__shfl((int)c4, src, kWave);
		uint32_t t = acc;
		if (schk >= (uint32_t)WIN)
			t -= sc4;
		const uint32_t f = fold16(t);
		/* to the packet's own lane */
#pragma unroll
		for (int g = 0; g < kPktG; g++) {
			const int sg = __builtin_amdgcn_readlane(sl, g * kPktL);
			const uint32_t fg = (uint32_t)__builtin_amdgcn_readlane((int)f, g * kPktL);
			if (lane == sg)
				out = fg;
		}
	}
	return out;
}

/*
 * The generic pipeline on up to 64 frames (one per lane): any descriptor,
 * any alignment, any header stack the oracle knows.  Used for the frames
 * the fast path defers.  Writes verdict, result and tuple of each frame.
 */
template <int WIN, bool PKT = false>
__device__ __forceinline__ void generic_batch(const RxArgs &a, uint32_t *win,
					      uint64_t *dtab, int lane,
					      uint64_t i, bool active,
					      uint4 *yl, uint32_t *yc,
					      uint32_t (&cnt)[CNT_FRAG + 1],
					      uint64_t &my_bytes)
{
	constexpr int SDW = WIN / 4 + 1;
	/* PKT: lane i is a multi-buffer packet's first descriptor (frags.hip
	 * finished the broken ones), read in place: len is the packet's,
	 * flen its first fragment's */
	uint32_t plast = 0;
	uint64_t ptotal = 0;
	if constexpr (PKT) {
		active = active && (a.desc[i].options & XDPGPU_PKT_CONTD) &&
			 !(i && (a.desc[i - 1].options & XDPGPU_PKT_CONTD));
		if (active) {
			for (uint64_t j = i;; j++) {
				const uint32_t o = a.desc[j].options;
				ptotal += a.desc[j].len;
				if (!(o & XDPGPU_PKT_CONTD) || j + 1 == a.n) {
					plast = (uint32_t)j;
					active = !(o & XDPGPU_PKT_CONTD);
					break;
				}
			}
			for (uint64_t j = i; active && j <= plast; j++) {
				const xdpgpu_desc x = a.desc[j];
				const uint64_t e = (x.addr & ((1ull << 48) - 1)) + (x.addr >> 48);
				active = (uint64_t)x.len <= a.usize && e <= a.usize - x.len;
			}
			active = active && ptotal <= 0xffffffffull;
		}
	}
	const uint4 dv = active ? *reinterpret_cast<const uint4 *>(a.desc + i)
				: make_uint4(0, 0, 0, 0);
	const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
	const uint32_t flen = dv.z;
	const uint32_t len = PKT ? (uint32_t)ptotal : flen;
	const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
	const bool valid = active && (uint64_t)flen <= a.usize &&
			   eff <= a.usize - flen;

	/* stage the header windows */
	uint4 cv[WIN / 16];
	const bool misaligned = issue_window<WIN>(a, dv, lane, dtab, cv);
	if (!misaligned) {
		commit_window<WIN>(win, cv, lane);
	} else {
		/* unaligned-chunk UMEM: per-lane byte staging */
		for (int d = 0; d < WIN / 4; d++) {
			uint32_t wv = 0;
#pragma unroll
			for (int b = 0; b < 4; b++) {
				const uint32_t off = 4 * d + b;
				if (valid && off <= flen && eff + off < a.usize)
					wv |= (uint32_t)a.umem[eff + off] << (8 * b);
			}
			win[lane * SDW + d] = wv;
		}
	}
	if constexpr (PKT) {
		/* a first fragment shorter than the window: the rest of the
		 * window from the later fragments */
		if (valid && flen < (uint32_t)WIN) {
			uint8_t *row = reinterpret_cast<uint8_t *>(win + lane * SDW);
			for (uint32_t off = flen; off < (uint32_t)WIN; off++)
				row[off] = off <= len ? (uint8_t)pkt_byte(a.umem, a.usize, a.desc, i,
									  plast, off)
						      : 0;
		}
	}
	__builtin_amdgcn_wave_barrier();

	/* parse: branch-free window reads; frames whose headers reach past
	 * the window are parsed again with global-memory reads */
	FrameView<WIN, false> F;
	F.w = win + lane * SDW;
	F.umem = a.umem;
	F.eff = eff;
	F.usize = a.usize;
	F.deep = 0;
	F.flen = PKT ? flen : ~0u;
	F.plast = plast;
	F.phead = i;
	F.pdesc = a.desc;
	Lane L = parse_lane<WIN, false>(F, valid ? len : 0u); /* 0: ABORTED */
	if (__ballot(F.deep)) {
		if (F.deep) {
			FrameView<WIN, true> G;
			G.w = F.w;
			G.umem = a.umem;
			G.eff = eff;
			G.usize = a.usize;
			G.deep = 0;
			G.flen = F.flen;
			G.plast = plast;
			G.phead = i;
			G.pdesc = a.desc;
			L = parse_lane<WIN, true>(G, valid ? len : 0u);
		}
	}

	/* a checksum range past the window: the payload sum is deferred to
	 * the bulk kernel (yl entry), except for echo candidates, whose TX
	 * verdict needs it here (and for packets read in place, summed here) */
	const bool echo_cand = (a.flags & XDPGPU_CFG_ICMP6_ECHO) &&
			       L.nvlan() == 0 && L.ipv6() && len >= 62 &&
			       F.b8(20) == 58 && F.b8(54) == 128;
	const bool need_ext = L.st() == ST_GO && L.has_csum() &&
			      L.rhi() > (uint32_t)WIN;
	const bool ydef = !PKT && need_ext && a.ydefer && a.res && !echo_cand &&
			  L.rhi() < 65536u;
	uint32_t ext_sum;
	if constexpr (PKT)
		ext_sum = pkt_ext_sums<WIN>(a, need_ext, i, plast, L.l4(), L.rhi(), L.chk(),
					    L.c4(), lane);
	else
		ext_sum = ext_sums<WIN>(a, need_ext && !ydef, eff, L.l4(), L.rhi(), L.chk(),
					L.c4(), lane);
	uint32_t partial = 0;   /* ydef: the L4 sum without the payload part */

	/* checksums, flow key, verdict */
	uint32_t verdict = L.st() == ST_PASS ? XDPGPU_PASS : XDPGPU_ABORTED;
	uint4 rec = make_uint4(0, 0, 0, 0);
	uint32_t key[11];
#pragma unroll
	for (int j = 0; j < 11; j++)
		key[j] = 0;
	uint32_t l3_bad = 0, l4_bad = 0, absent = 0;
	if (L.st() == ST_GO) {
		const bool ip = L.ipv4() || L.ipv6();
		const uint32_t nh = L.nh(), cl = L.cl(), c4 = L.c4();
		uint32_t flags = 0, l3c = 0, l4c = 0, l3_ok = 1, l4_ok = 0;
		if (L.ipv4()) {
			/* ip_fast_csum, lib_checksum.h:103-106 */
			l3c = ~L.s3() & 0xffff;
			l3_ok = fold16((uint64_t)L.s3() + L.c3()) == 0xffff;
		}
		if (L.has_csum()) {
			const uint64_t body = (uint64_t)L.s4() + ext_sum;
			uint64_t ph = 0;
			if (L.ipv4() && nh != 1) {
				/* udp_csum -> csum_tcpudp_magic,
				 * lib_checksum.h:142-179 */
				ph = (uint64_t)L.sa + L.da + ((uint64_t)(nh + cl) << 8);
			} else if (L.ipv6()) {
				/* csum_ipv6_magic, xdp_synproxy_kern.c:149-172 */
				ph = (uint64_t)__builtin_bswap32(cl) +
				     __builtin_bswap32(nh) +
				     F.win_sum(L.l3() + 8, L.l3() + 40);
			}
			/* ICMPv4: no pseudo header, ~do_csum(msg) */
			partial = fold16(body + ph);
			l4c = ~fold16(body + ph) & 0xffff;
			l4_ok = (~fold16(body + c4 + ph) & 0xffff) == 0;
			if (L.ipv4() && nh == 17 && c4 == 0) {
				absent = 1;
				l4_ok = 1;
			}
		}
		if (L.nvlan())
			flags |= XDPGPU_F_VLAN;
		if (ip) {
			flags |= XDPGPU_F_IP;
			if (L.ipv6())
				flags |= XDPGPU_F_IPV6;
			if (l3_ok)
				flags |= XDPGPU_F_L3_OK;
			if (L.frag())
				flags |= XDPGPU_F_FRAG;
			if (L.has_l4())
				flags |= XDPGPU_F_L4;
			if (L.has_csum() && l4_ok && !ydef)
				flags |= XDPGPU_F_L4_OK;
			if (absent && !ydef)
				flags |= XDPGPU_F_L4_ABSENT;
			/* flow key: pping.h:120-139, v4 mapped as in
			 * pping_kern.c:212-217 */
			if (L.ipv4()) {
				key[2] = 0xffff0000u;
				key[3] = L.sa;
				key[7] = 0xffff0000u;
				key[8] = L.da;
			} else {
#pragma unroll
				for (int j = 0; j < 4; j++) {
					key[j] = F.le32(L.l3() + 8 + 4 * j);
					key[5 + j] = F.le32(L.l3() + 24 + 4 * j);
				}
			}
			key[4] = L.ports & 0xffff;
			key[9] = L.ports >> 16;
			key[10] = nh | ((L.ipv4() ? 2u : 10u) << 16);
		}
		rec.x = jhash_key44(key, a.initval);
		l3_bad = L.ipv4() && !l3_ok;
		l4_bad = L.has_csum() && !l4_ok;
		rec.y = l3c | ((ydef ? 0u : l4c) << 16);
		rec.z = flags | ((ip ? nh : 0u) << 8) | (L.l3() << 16) |
			(L.nvlan() << 24);
		rec.w = ip ? (L.l4() | ((L.has_csum() ? cl : 0u) << 16)) : 0u;

		verdict = XDPGPU_REDIRECT;
		if ((a.flags & XDPGPU_CFG_VERIFY_CSUM) && (l3_bad || l4_bad)) {
			verdict = XDPGPU_DROP;
		} else if ((a.flags & XDPGPU_CFG_ICMP6_ECHO) &&
			   L.nvlan() == 0 && L.ipv6() && len >= 62 &&
			   F.b8(20) == 58 && F.b8(54) == 128) {
			verdict = XDPGPU_TX;   /* rewritten below */
		}
	}
	/* af_xdp_user.c:968-1040 echo responder: each TX lane rewrites its own
	 * frame from its window row (MACs swapped, IPv6 addresses swapped,
	 * type 129, csum_replace2): bytes 0-11 and 20-59 as dwords (the
	 * unchanged bytes among them rewritten with their own values), bytes
	 * one by one for a frame not 4-byte aligned.  (One frame at a time by
	 * the whole wave, a byte per lane: the echo pool's launch 1.38 vs
	 * 1.26 ms.) */
	if (verdict == XDPGPU_TX) {
		const uint32_t *row = win + lane * SDW;
		auto rb = [&](int j) -> uint32_t { return (row[j >> 2] >> ((j & 3) * 8)) & 0xff; };
		auto nb = [&](int j) -> uint32_t {
			if (j < 6)
				return rb(j + 6);
			if (j < 12)
				return rb(j - 6);
			if (j >= 22 && j < 38)
				return rb(j + 16);
			if (j >= 38 && j < 54)
				return rb(j - 16);
			if (j == 54)
				return 129u;
			if (j == 56 || j == 57) {
				const uint32_t ck = csum_replace2(rb(56) | (rb(57) << 8), 0x0080, 0x0081);
				return j == 56 ? (ck & 0xff) : (ck >> 8);
			}
			return rb(j);
		};
		uint8_t *g = a.umem + eff;
		if (PKT && flen < 60) {
			/* the rewritten bytes spread over the fragments */
			uint64_t j = i;
			uint32_t o = 0;
			for (int b = 0; b < 60; b++) {
				while (b >= (int)(o + a.desc[j].len)) {
					o += a.desc[j].len;
					j++;
				}
				const xdpgpu_desc x = a.desc[j];
				const uint64_t e = (x.addr & ((1ull << 48) - 1)) + (x.addr >> 48);
				if (b < 12 || b >= 22)
					a.umem[e + (b - o)] = (uint8_t)nb(b);
			}
		} else if (!(eff & 3)) {
			uint32_t *gw = reinterpret_cast<uint32_t *>(g);
#pragma unroll
			for (int d = 0; d < 15; d++) {
				if (d >= 3 && d < 5)
					continue;
				gw[d] = nb(4 * d) | nb(4 * d + 1) << 8 | nb(4 * d + 2) << 16 |
					nb(4 * d + 3) << 24;
			}
		} else {
			for (int j = 0; j < 60; j++)
				if (j < 12 || j >= 22)
					g[j] = (uint8_t)nb(j);
		}
	}
	const bool rec_live = verdict != XDPGPU_ABORTED && verdict != XDPGPU_PASS;

	/* deferred payload sums: entries appended to this region's list */
	const uint64_t ym = __ballot(active && ydef);
	if (ym) {
		uint32_t base = 0;
		if (lane == 0)
			base = atomicAdd(yc, (uint32_t)__popcll(ym));
		base = __builtin_amdgcn_readfirstlane(base);
		if (active && ydef) {
			const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
				(uint32_t)(ym >> 32),
				__builtin_amdgcn_mbcnt_lo((uint32_t)ym, 0));
			const uint32_t start = L.l4() > (uint32_t)WIN ? L.l4() : (uint32_t)WIN;
			const bool chk_in = L.chk() >= (uint32_t)WIN;
			const uint32_t fl = ((L.ipv4() && L.nh() == 17) ? 1u : 0u) |
					    (chk_in ? 2u : 0u);
			yl[base + rank] = make_uint4((uint32_t)i, partial | (L.c4() << 16),
						     start | ((chk_in ? L.chk() : 0u) << 16),
						     L.rhi() | (fl << 16));
		}
	}

	/* outputs (a deferred frame's verdict is the bulk kernel's) */
	if (active) {
		if (!ydef)
			a.verdict[i] = (uint8_t)verdict;
		if (a.res)
			*reinterpret_cast<uint4 *>(a.res + i) = rec;
		if (a.tup) {
			if (a.tuple_fmt == XDPGPU_TUPLE_V4) {
				uint4 tv = make_uint4(0, 0, 0, 0);
				if (rec_live) {
					const bool ip = L.ipv4() || L.ipv6();
					tv.x = L.ipv4() ? L.sa : 0u;
					tv.y = L.ipv4() ? L.da : 0u;
					tv.z = L.ports;
					tv.w = (ip ? L.nh() : 0u) |
					       ((ip ? (L.ipv4() ? 2u : 10u) : 0u) << 8) |
					       (L.vid() << 16);
				}
				*reinterpret_cast<uint4 *>(a.tup + 16 * i) = tv;
			} else if (a.tuple_fmt == XDPGPU_TUPLE_NET) {
				uint32_t *tp = reinterpret_cast<uint32_t *>(a.tup + 44 * i);
#pragma unroll
				for (int j = 0; j < 11; j++)
					tp[j] = rec_live ? key[j] : 0u;
			}
		}
	}

	if constexpr (PKT) {
		/* the packet's other descriptors: its verdict, all-zero
		 * records and tuples */
		if (active) {
			const uint32_t tb = a.tup ? (a.tuple_fmt == XDPGPU_TUPLE_NET ? 44u :
						     a.tuple_fmt == XDPGPU_TUPLE_V4 ? 16u : 0u)
						  : 0u;
			for (uint64_t j = i + 1; j <= plast; j++) {
				a.verdict[j] = (uint8_t)verdict;
				if (a.res)
					*reinterpret_cast<uint4 *>(a.res + j) = make_uint4(0, 0, 0, 0);
				for (uint32_t b = 0; b < tb; b++)
					a.tup[j * tb + b] = 0;
			}
		}
	}

	/* counters: ballot + popcount (deferred frames: the bulk kernel) */
	const bool own = active && !ydef;
	const bool live = rec_live && !ydef;
	if (a.stats) {
		cnt[CNT_FRAMES] += __popcll(__ballot(own));
#pragma unroll
		for (int v = 0; v < 5; v++)
			cnt[CNT_VERDICT0 + v] +=
				__popcll(__ballot(own && verdict == (uint32_t)v));
		cnt[CNT_L3_BAD] += __popcll(__ballot(live && l3_bad));
		cnt[CNT_L4_BAD] += __popcll(__ballot(live && l4_bad));
		cnt[CNT_L4_ABSENT] += __popcll(__ballot(live && absent));
		cnt[CNT_FRAG] += __popcll(__ballot(live && L.frag()));
	}
	my_bytes += own ? len : 0;
}

/* Counters: a wave's uniform counts into the block's LDS slot, then the
 * block's slot into its own global slot (one read-modify-write per block;
 * xdpgpu_stats sums the slots).  Every thread of the block calls it. */
__device__ __forceinline__ void block_stats_flush(const RxArgs &a,
						  unsigned long long *blk_cnt,
						  const uint32_t (&cnt)[CNT_FRAG + 1],
						  uint64_t my_bytes, int lane)
{
	if (!a.stats)
		return;
	const uint64_t bytes = wave_sum64(my_bytes);
	if (lane == 0) {
		atomicAdd(&blk_cnt[CNT_BYTES], (unsigned long long)bytes);
#pragma unroll
		for (int k = 0; k <= CNT_FRAG; k++)
			if (k != CNT_BYTES && cnt[k])
				atomicAdd(&blk_cnt[k], (unsigned long long)cnt[k]);
	}
	__syncthreads();
	if (threadIdx.x < CNT_SLOT && blk_cnt[threadIdx.x])
		a.stats[(uint64_t)blockIdx.x * CNT_SLOT + threadIdx.x] +=
			blk_cnt[threadIdx.x];
}

/* LE 16-bit loads of the VLAN TPIDs 0x8100 / 0x88A8 (parsing_helpers.h:75) */
__device__ __forceinline__ bool le_is_vlan(uint32_t v)
{
	return (v == 0x0081u) | (v == 0xa888u);
}

/* mask of the first nb (0..4) bytes of a dword: a clamp, one multiply-add
 * and one 64-bit shift (0xffffffff >> 32 is 0 in 64 bits, where the 32-bit
 * shift's count wraps) */
__device__ __forceinline__ uint32_t first_bytes(int32_t nb)
{
	const int32_t c = nb < 0 ? 0 : nb > 4 ? 4 : nb;
	return (uint32_t)(0xffffffffull >> (32 - 8 * c));
}

/* mask's lane set ? b : a (v_cndmask_b32 on a wave-wide lane mask) */
__device__ __forceinline__ uint32_t lane_sel(uint64_t mask, uint32_t a, uint32_t b)
{
	uint32_t r;
	asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(mask));
	return r;
}

/* acc plus the two 16-bit halves of x (v_sad_u16 against zero): the
 * one's-complement sums accumulate 16-bit halves in 32 bits, congruent mod
 * 0xffff to the 32-bit words' sum and zero exactly when it is, so fold16
 * gives the same result with one instruction a word instead of a 64-bit
 * add.  acc must stay far below 2^32 (2^32 is 1 mod 0xffff: a wrap would
 * change the sum): start chains from 0 or a small raw term. */
__device__ __forceinline__ uint32_t add_halves(uint32_t acc, uint32_t x)
{
	return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

typedef __attribute__((address_space(3))) void lds_void_t;

/* non-temporal 16-byte store (streamed outputs, written once) */
typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
typedef unsigned int v3u_t __attribute__((ext_vector_type(3)));
__device__ __forceinline__ void st_nt16(void *p, uint4 r)
{
	v4u_t v = {r.x, r.y, r.z, r.w};
	__builtin_nontemporal_store(v, reinterpret_cast<v4u_t *>(p));
}

/* non-temporal 16-byte load (payload streamed once) */
__device__ __forceinline__ uint4 ld_nt16(const void *p)
{
	const v4u_t v = __builtin_nontemporal_load(reinterpret_cast<const v4u_t *>(p));
	return make_uint4(v.x, v.y, v.z, v.w);
}

/*
 * Bulk kernel: completes the fast-shape frames whose L4 checksum range runs
 * past the 64-byte window, by summing frame bytes [64, end of range) (with
 * udp_csum's over-read byte; zero past the UMEM) into the window sum the
 * fast kernel left in the result record.
 *
 * Per batch of 64 listed frames the wave works as four quarter-waves
 * (G = 16; a diagnostic G = 8 variant uses eight 8-lane groups): a group
 * streams one frame at a time, G lanes x 16 B x U per step, and on
 * finishing a frame takes the next unassigned one of the batch (dynamic,
 * so long and short frames balance).  Per-lane partial sums go to LDS, 16
 * per frame (G = 8 zero-fills the other 8); lane f then adds frame f's 16
 * partials and completes its record.
 * Frames are 16-byte aligned (a fast-shape condition), so absolute and
 * frame-relative 16-bit words coincide.
 */
/* One batch of up to 64 listed frames, wave-wide: the quarter-wave payload
 * streaming described above, then lane f completes frame f's record,
 * verdict and counters.  GEN false: fast-kernel bulk list (u32 indices,
 * 16-byte aligned frames, range [64, end), window sum and check word in the
 * result record).  GEN true: exception-kernel entries (xdpgpu ylist: index,
 * partial sum | check word, range start | check offset, range end | flags;
 * any alignment).  meta: 64 uint4, part4: 256 uint4 of this wave's LDS. */
/* the little-endian 16-bit word at byte offset o (0..14) of a 16-byte
 * chunk */
__device__ __forceinline__ uint32_t u16_at(uint4 x, uint32_t o)
{
	const uint32_t k = (o >> 2) & 3;
	const uint32_t w = k == 0 ? x.x : k == 1 ? x.y : k == 2 ? x.z : x.w;
	const uint32_t w2 = k == 0 ? x.y : k == 1 ? x.z : k == 2 ? x.w : 0u;
	const uint64_t d = ((uint64_t)w2 << 32) | w;
	return (uint32_t)(d >> (8 * (o & 3))) & 0xffff;
}

/* the completed record of a bulk frame: a scattered 16-byte store */
#ifndef XDP_TAIL_REC_NT
#define XDP_TAIL_REC_NT 1
#endif
constexpr bool kTailRecNt = XDP_TAIL_REC_NT != 0;
/* the bulk pass's verdict bytes non-temporal (build knob): IMIX 2.260 vs
 * 2.252 ms plain, alternating processes (tools/gpu_ab_outnt.sh) */
#ifndef XDP_TAIL_VERDICT_NT
#define XDP_TAIL_VERDICT_NT 0
#endif
constexpr bool kTailVerdictNt = XDP_TAIL_VERDICT_NT != 0;
/* bulk frames' provisional verdicts stored by the tile loop, the bulk pass
 * storing only those that change (fast_tile; build knob) */
#ifndef XDP_BULK_VERDICT_TILE
#define XDP_BULK_VERDICT_TILE 1
#endif
constexpr bool kBulkVerdictTile = XDP_BULK_VERDICT_TILE != 0;
/* ARP and NDP (PASS) and the common parse failures (ABORTED) decided in the
 * tile loop (fast_tile's "quick" frames; build knob), so that a pool of
 * otherwise fast frames leaves the tail no exception batch */
#ifndef XDP_QUICK
#define XDP_QUICK 1
#endif
constexpr bool kQuick = XDP_QUICK != 0;
/* a tile of fast and bulk frames only (two in three of config 2's) skips
 * the quick classification after one ballot (build knob): config 2 0.3086 /
 * 0.3097 vs 0.3191 / 0.3145 ms a step, IMIX, 1500 B and echo unchanged,
 * alternating processes (profiles/r04_ab_quick_skip.txt) */
#ifndef XDP_QUICK_SKIP
#define XDP_QUICK_SKIP 1
#endif
/* tiles with no tagged frame skip the tag shift of the window words
 * (fast_tile; build knob): config 2 0.3185 / 0.3315 vs 0.3344 / 0.3406 ms
 * per step without, alternating processes (profiles/r04_ab_untagged.txt) */
#ifndef XDP_UNTAGGED_TILES
#define XDP_UNTAGGED_TILES 1
#endif
constexpr bool kUntaggedTiles = XDP_UNTAGGED_TILES != 0;
/* A 44-byte network_tuple at a dword-aligned address: two 16-byte stores
 * and a 12-byte one (global stores need only dword alignment) */
__device__ __forceinline__ void store_tuple44(uint8_t *p, const uint32_t (&t)[11])
{
	const v4u_t a0 = {t[0], t[1], t[2], t[3]}, a1 = {t[4], t[5], t[6], t[7]};
	const v3u_t a2 = {t[8], t[9], t[10]};
	asm volatile("global_store_dwordx4 %0, %1, off\n\t"
		     "global_store_dwordx4 %0, %2, off offset:16\n\t"
		     "global_store_dwordx3 %0, %3, off offset:32\n\t"
		     "s_nop 2"
		     :: "v"(p), "v"(a0), "v"(a1), "v"(a2) : "memory");
}

/* Who stores an IPv6 frame's network_tuple (build knob): 1 the tile
 * loop, from the window, when it classifies the frame (every tuple sector
 * written in one pass); 0 the bulk pass, from frame bytes [16, 64) it
 * loads again */
#ifndef XDP_TUP6_TILE
#define XDP_TUP6_TILE 1
#endif
constexpr bool kTup6Tile = XDP_TUP6_TILE != 0;

/* Diagnostic builds of the bulk pass (XDP_TAIL_DIAG, never the product):
 * bit 0: no output stores (record, verdict, tuple); bit 1: no payload
 * loads (the range summed as zeros); bit 2: no record store; bit 3: no
 * verdict store; bit 4: the record stored over the frame's n/2 away;
 * bit 5: a load of the record instead of its store; bit 6: lane 0's record
 * alone; bit 7: one dword of each record */
#ifndef XDP_TAIL_DIAG
#define XDP_TAIL_DIAG 0
#endif
/* The bulk pass's record store as a buffer store with these cache-policy
 * bits (A/B knob; -1: the plain non-temporal global store) */
#ifndef XDP_TAIL_REC_AUX
#define XDP_TAIL_REC_AUX -1
#endif
/* Latency probe of the bulk pass (stamps builds only, XDP_LAT_PROBE): per
 * wave, slot 4 counts bulk batches (x100), slot 6 the ticks from a batch's
 * start to its list entry, descriptor and record in registers (an explicit
 * vmcnt(0): with bit 1 clear it also waits for the previous batch's record
 * store, vmcnt retiring in order), slot 7 (bit 1) the ticks of a vmcnt(0)
 * right after the record store */
#if defined(XDPGPU_STAMPS) && defined(XDP_LAT_PROBE)
#define LAT_NOW(v) \
	asm volatile("" ::: "memory"); \
	const unsigned long long v = __builtin_amdgcn_s_memrealtime(); \
	asm volatile("" ::: "memory")
#define LAT_WAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#define LAT_ACC(sid, lane, k, d) \
	do { \
		if ((lane) == 0 && (sid) < (uint64_t)kStampWaves) \
			g_stamp[8 * (sid) + (k)] += (d); \
	} while (0)
#endif
/* Batch-adaptive group size (build knob): 1 smaller groups for batches
 * of short ranges only; 0 always G */
#ifndef XDP_TAIL_ADAPT
#define XDP_TAIL_ADAPT 1
#endif
constexpr bool kTailAdapt = XDP_TAIL_ADAPT != 0;
/* Batches of ranges within 64 bytes streamed in one step (stream_short;
 * build knob, off: DESIGN.md §5.2) */
#ifndef XDP_TAIL_SHORT
#define XDP_TAIL_SHORT 1
#endif
constexpr bool kTailShort = XDP_TAIL_SHORT != 0;
/* Ranges longer than this many bytes streamed from their 128-byte line
 * (bulk_batch; build knob, 0 off): 2 M x 1500 B 0.632 / 0.634 vs 0.658 /
 * 0.661 ms and 3.69 vs 3.89 GB of HBM traffic a launch (the line a step
 * boundary split was fetched twice); IMIX 1.927 / 1.930 vs 1.937 / 1.934;
 * 256 (IMIX's 570-byte frames too) slowed IMIX to 1.96 ms
 * (profiles/r04_ab_line_align.txt) */
#ifndef XDP_TAIL_LINE_AL
#define XDP_TAIL_LINE_AL 640
#endif
/* The bulk pass's payload streaming, G lanes per frame (dynamic frame
 * assignment): every listed frame's partial sums into part (16 per frame,
 * zero-filled for G < 16).  meta: the batch's ranges. */
template <int G, int U, bool NT>
__device__ __forceinline__ void stream_groups(const RxArgs &a, const uint4 *meta,
					      uint32_t *part, int lane, uint32_t nb)
{
	static_assert(G == 16 || G == 8 || G == 4, "group of 16, 8 or 4 lanes per frame");
	const uint32_t sub = lane & (G - 1);
	/* G-lane group streaming with dynamic frame assignment.  Loads under
	 * their lane's range only: a branch-free form (every lane loading, the
	 * chunks outside masked to zero) lets the compiler count loads in
	 * flight, and two steps in flight per group then fit, but it ran 18 %
	 * slower on 1500 B frames and 4 % on IMIX, with or without the second
	 * step (the dead lanes' loads cost more than the overlap gains) */
	uint32_t k = lane / G;             /* this group's frame */
	uint32_t nxt = kWave / G;          /* next unassigned (uniform) */
	bool live = k < nb;
	uint4 m = meta[live ? k : 0];
	uint64_t flo = ((uint64_t)m.y << 32) | m.x;
	uint32_t fnb = m.z, fsk = m.w, o = 0, acc = 0;
	while (__ballot(live)) {
		uint4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t ou = o + 16 * G * u + 16 * sub;
			v[u] = make_uint4(0, 0, 0, 0);
			if (!(XDP_TAIL_DIAG & 2) && live && ou < fnb)
				v[u] = NT ? ld_nt16(a.umem + flo + ou)
					  : *reinterpret_cast<const uint4 *>(a.umem + flo + ou);
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint32_t ou = o + 16 * G * u + 16 * sub;
			if ((ou + 16 > fnb || ou < fsk) && ou < fnb) {
				const uint4 mk = chunk_keep(ou, fsk, fnb);
				v[u].x &= mk.x;
				v[u].y &= mk.y;
				v[u].z &= mk.z;
				v[u].w &= mk.w;
			}
			acc = add_chunk(acc, v[u]);
		}
		o += 16 * G * U;
		const bool done = live && o >= fnb;
		const uint64_t dq = __ballot(done && sub == 0);
		if (dq) {
			if (done) {
				part[16 * k + sub] = acc;   /* the rest: zeroed */
				acc = 0;
				k = nxt + (uint32_t)__popcll(dq & ((1ull << (lane & ~(G - 1))) - 1));
				live = k < nb;
				m = meta[live ? k : 0];
				flo = ((uint64_t)m.y << 32) | m.x;
				fnb = m.z;
				fsk = m.w;
				o = 0;
			}
			nxt += (uint32_t)__popcll(dq);
		}
	}
}

/* A batch whose ranges are all at most 64 bytes from their aligned start
 * (the 128-byte frames of the echo leg): four lanes per frame, each lane
 * loading its 16-byte chunk of four frames (g, g + 16, g + 32, g + 48) at
 * once, so that the whole batch is one round trip; stream_groups<4> would
 * take four dependent steps of 16 frames.  Same partials as stream_groups
 * (part[16 f + chunk], the rest left zero). */
template <bool NT>
__device__ __forceinline__ void stream_short(const RxArgs &a, const uint4 *meta,
					     uint32_t *part, int lane, uint32_t nb)
{
	const uint32_t sub = lane & 3, g = lane >> 2, ou = 16 * sub;
	uint4 v[4], m[4];
#pragma unroll
	for (int u = 0; u < 4; u++) {
		const uint32_t f = g + 16 * u;
		m[u] = meta[f < nb ? f : 0];
		v[u] = make_uint4(0, 0, 0, 0);
		const uint64_t flo = ((uint64_t)m[u].y << 32) | m[u].x;
		if (!(XDP_TAIL_DIAG & 2) && f < nb && ou < m[u].z)
			v[u] = NT ? ld_nt16(a.umem + flo + ou)
				  : *reinterpret_cast<const uint4 *>(a.umem + flo + ou);
	}
#pragma unroll
	for (int u = 0; u < 4; u++) {
		const uint32_t f = g + 16 * u, fnb = m[u].z, fsk = m[u].w;
		if ((ou + 16 > fnb || ou < fsk) && ou < fnb) {
			const uint4 mk = chunk_keep(ou, fsk, fnb);
			v[u].x &= mk.x;
			v[u].y &= mk.y;
			v[u].z &= mk.z;
			v[u].w &= mk.w;
		}
		if (f < nb)
			part[16 * f + sub] = add_chunk(0u, v[u]);
	}
}

/* The bulk pass's records staged in the wave's free LDS (build knob,
 * XDP_REC_STAGE batches, 0 off) and stored XDP_REC_STAGE batches at a
 * time: a 64-lane record store costs the launch about 0.36 us of its CU's
 * time while payload loads stream (EXPERIMENTS.md §5.2, round 6) */
#ifndef XDP_REC_STAGE
#define XDP_REC_STAGE 4
#endif
/* XDP_REC_RELOAD (build knob): 0 stages whole records (16 bytes and the
 * frame index a frame, four batches in the 5 KiB); 1 stages only what the
 * bulk pass adds (the frame index, ~sum and l4 offset a frame, two flag
 * masks a batch: up to nine batches), merged into the tile's record
 * reloaded at the store (a load of that shape is free, a store is not) */
#ifndef XDP_REC_RELOAD
#define XDP_REC_RELOAD 0
#endif
constexpr uint32_t kRecStage = XDP_REC_STAGE;
constexpr bool kRecReload = XDP_REC_RELOAD != 0;
/* records reloaded at once when a full stage is stored (XDP_REC_GROUP) */
#ifndef XDP_REC_GROUP
#define XDP_REC_GROUP 4
#endif
constexpr uint32_t kRecGroup = XDP_REC_GROUP;
static_assert(kRecStage <= (kRecReload ? 9u : 4u),
	      "the tail's free LDS (wave buffer from uint4 320) holds these batches");
/* the staging area: whole records (kRecReload 0) at meta + 320, then the
 * frame indices (~0: none), then (kRecReload 1) the ~sum | l4 << 16 words
 * and the batches' L4_OK / L4_ABSENT masks */
__device__ __forceinline__ uint32_t *stage_idx(uint4 *meta)
{
	return reinterpret_cast<uint32_t *>(meta + 320 + (kRecReload ? 0u : kRecStage * kWave));
}

/* store staged batch s (lane's frame) */
__device__ __forceinline__ void rec_store_staged(const RxArgs &a, uint4 *meta, uint32_t s, int lane)
{
	const uint32_t *ix = stage_idx(meta);
	const uint32_t j = ix[s * kWave + lane];
	if constexpr (!kRecReload) {
		const uint4 r = meta[320 + s * kWave + lane];
		if (j != ~0u)
			st_nt16(a.res + j, r);
	}
}

/* the reload form for batches [s0, s0 + C): C records loaded, merged and
 * stored */
template <uint32_t C>
__device__ __forceinline__ void rec_flush_reload(const RxArgs &a, uint4 *meta, uint32_t s0,
						 int lane)
{
	const uint32_t *ix = stage_idx(meta);
	const uint32_t *pw = ix + kRecStage * kWave;
	const uint64_t *mk = reinterpret_cast<const uint64_t *>(ix + 2 * kRecStage * kWave);
	uint32_t j[C];
	uint4 r[C];
#pragma unroll
	for (uint32_t u = 0; u < C; u++) {
		j[u] = ix[(s0 + u) * kWave + lane];
		r[u] = make_uint4(0, 0, 0, 0);
		if (j[u] != ~0u)
			r[u] = *reinterpret_cast<const uint4 *>(a.res + j[u]);
	}
#pragma unroll
	for (uint32_t u = 0; u < C; u++) {
		const uint32_t p = pw[(s0 + u) * kWave + lane];
		const uint64_t okm = mk[2 * (s0 + u)], abm = mk[2 * (s0 + u) + 1];
		uint4 x = r[u];
		x.y = (x.y & 0xffff) | (p << 16);
		/* (fast_tile's marks in bits 30-31 cleared; nvlan is 0..2) */
		x.z = (x.z & 0x3fffffffu) | (((okm >> lane) & 1) ? XDPGPU_F_L4_OK : 0u) |
		      (((abm >> lane) & 1) ? XDPGPU_F_L4_ABSENT : 0u);
		x.w = (p >> 16) | (x.w & 0xffff0000u);
		if (j[u] != ~0u)
			st_nt16(a.res + j[u], x);
	}
}

/* every staged batch stored (the end of the tail) */
__device__ __forceinline__ void rec_flush(const RxArgs &a, uint4 *meta, uint32_t &nst, int lane)
{
	for (uint32_t s = 0; s < nst; s++) {
		if constexpr (kRecReload)
			rec_flush_reload<1>(a, meta, s, lane);
		else
			rec_store_staged(a, meta, s, lane);
	}
	nst = 0;
}

template <int U, bool NT, bool GEN, int G, int WIN = 64, bool EC = true>
__device__ __forceinline__ void bulk_batch(const RxArgs &a, uint4 *meta,
					   uint4 *part4, int lane,
					   const void *list, uint32_t nb,
					   uint32_t (&cnt)[CNT_FRAG + 1],
					   uint64_t &my_bytes, uint32_t &nst, uint64_t sid = 0)
{
	(void)sid;
#ifdef LAT_NOW
	LAT_NOW(lat0);
#endif
	uint32_t *part = reinterpret_cast<uint32_t *>(part4);
	const bool act = (uint32_t)lane < nb;
	uint4 ye = make_uint4(0, 0, 0, 0);
	uint64_t i;
	if constexpr (GEN) {
		ye = reinterpret_cast<const uint4 *>(list)[act ? lane : 0];
		i = ye.x;
	} else {
		i = reinterpret_cast<const uint32_t *>(list)[act ? lane : 0];
	}
	if (DBG_BAD(i >= a.n, GEN ? 3 : 2, i))
		i = 0;
	const uint4 dv = *reinterpret_cast<const uint4 *>(a.desc + i);
	uint4 rv = *reinterpret_cast<const uint4 *>(a.res + i);
#ifdef LAT_NOW
	LAT_WAIT();
	LAT_NOW(lat1);
	LAT_ACC(sid, lane, 6, lat1 - lat0);
	LAT_ACC(sid, lane, 4, 100ull);
#endif
	/* an IPv6 frame whose 128-byte window summed to byte 128 (fast_tile's
	 * mark in the nvlan byte, cleared here) */
	bool w6 = false, tsh = false;
	if constexpr (!GEN && WIN == 128) {
		w6 = (rv.z >> 31) != 0;
		/* its last bytes summed by the tile (XDP_TAIL_SHARE) */
		tsh = ((rv.z >> 30) & 1) != 0;
		rv.z &= 0x3fffffffu;
	}
	const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
	const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
	const uint32_t cl = rv.w >> 16;
	/* GEN false: the fast shape's records; IPv6/UDP (V6 builds) has its
	 * L4 header 40 bytes after l3 and no over-read byte */
	const bool r6 = !GEN && (rv.z & XDPGPU_F_IPV6);
	/* IPv4 ICMP (V6 builds): no over-read byte either */
	const bool nov = r6 || ((rv.z >> 8) & 0xff) == 1;
	const uint32_t l4 = GEN ? (rv.w & 0xffff) : ((rv.z >> 16) & 0xff) + (r6 ? 40u : 20u);
	const uint32_t rhi = GEN ? (ye.w & 0xffff) : l4 + cl + (nov ? 0u : (cl & 1));
	uint64_t lim = eff + rhi;
	/* (the tile took [the line start, lim)) */
	lim = tsh ? lim & ~127ull : lim;
	lim = lim < a.usize ? lim : a.usize;
	/* an IPv6/UDP frame's network_tuple words (the tile stored none):
	 * frame bytes [16, 64), loaded here so that the round trip overlaps
	 * the payload streaming */
	const bool net6 = !GEN && act && r6 && a.tup && a.tuple_fmt == XDPGPU_TUPLE_NET;
	/* the tile stored it (XDP_TUP6_TILE) unless this pass builds it */
	const bool tup6 = net6 && !kTup6Tile;
	/* an untagged ICMPv6 frame under the echo responder: its first 64
	 * bytes, for the type and the rewrite */
	/* EC false: an instance the launcher never takes with the responder on */
	const bool echo6 = EC && !GEN && act && r6 && (a.flags & XDPGPU_CFG_ICMP6_ECHO) &&
			   ((rv.z >> 8) & 0xff) == 58 && (rv.z >> 24) == 0;
	/* (an echo request's first 64 bytes are loaded after the streaming,
	 * below: the ECHO instance answers most requests in its tile loop, so
	 * a batch rarely holds one, and 16 registers live across the
	 * streaming spilled) */
	uint4 h0 = make_uint4(0, 0, 0, 0), h1 = h0, h2 = h0, h3 = h0;
	if (tup6) {
		h1 = *reinterpret_cast<const uint4 *>(a.umem + eff + 16);
		h2 = *reinterpret_cast<const uint4 *>(a.umem + eff + 32);
		h3 = *reinterpret_cast<const uint4 *>(a.umem + eff + 48);
	}
	/* a "late" IPv6 frame (fast_tile): its check word (and TCP's data
	 * offset) lie in frame bytes [64, 80), which the UMEM holds (both
	 * before l4 + 20 <= len) */
	const uint32_t p6 = (rv.z >> 8) & 0xff;
	const uint32_t chk6 = p6 == 6 ? 16u : p6 == 17 ? 6u : 2u;
	const bool late = r6 && !w6 && l4 + chk6 >= 64;
	uint4 x64 = make_uint4(0, 0, 0, 0);
	if (act && late)
		x64 = *reinterpret_cast<const uint4 *>(a.umem + eff + 64);
	/* absolute range [lo, lim), streamed from its 16-byte aligned start */
	/* from byte 128 where the tile's 128-byte window summed to there: an
	 * IPv4 frame with a staged second half (win_hi), an IPv6 frame
	 * fast_tile marked */
	const uint64_t lo = eff + (GEN ? (ye.z & 0xffff)
				       : (WIN == 128 && (r6 ? w6 : win_hi(a, eff, dv.z))) ? 128u : 64u);
	/* ranges longer than XDP_TAIL_LINE_AL bytes streamed from their 128-byte
	 * line (the group's chunks then cover whole lines and no line is split
	 * between two steps); shorter ones from their 16-byte chunk (0: always) */
	const uint64_t lo_al = lo & (XDP_TAIL_LINE_AL && lim > lo && lim - lo > XDP_TAIL_LINE_AL
					     ? ~127ull : ~15ull);
	uint32_t t = 0;
	meta[lane] = make_uint4((uint32_t)lo_al, (uint32_t)(lo_al >> 32),
				(uint32_t)(lim > lo ? lim - lo_al : 0),
				(uint32_t)(lo - lo_al));
	__builtin_amdgcn_wave_barrier();

	/* the group size: 16 lanes per frame, fewer when every range of the
	 * batch is short (the echo leg's 128-byte frames: 4 lanes, 16 frames
	 * a step instead of 4: 0.64 vs 0.93 ms; one lane per frame, the batch
	 * in one step, 0.81 ms: each load instruction then touches 64 lines) */
	uint32_t mx = act && lim > lo ? (uint32_t)(lim - lo_al) : 0u;
#pragma unroll
	for (int d = 1; d < kWave; d <<= 1)
		mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, kWave));
	/* frame f's 16 partials, zero but for its group's lanes.  The four
	 * 16-byte slots of a lane rotated by lane / 4: lanes l and l + 4 are
	 * 256 bytes apart, one bank row, so an unrotated slot j would put them
	 * on the same banks */
#pragma unroll
	for (int j = 0; j < 4; j++)
		part4[4 * lane + ((j + (lane >> 2)) & 3)] = make_uint4(0, 0, 0, 0);
	__builtin_amdgcn_wave_barrier();
	if (kTailShort && mx <= 64)
		stream_short<NT>(a, meta, part, lane, nb);
	else if (kTailAdapt && mx <= 64 * U)
		stream_groups<4, U, NT>(a, meta, part, lane, nb);
	else if (kTailAdapt && mx <= 128 * U)
		stream_groups<8, U, NT>(a, meta, part, lane, nb);
	else
		stream_groups<G, U, NT>(a, meta, part, lane, nb);
	__builtin_amdgcn_wave_barrier();

	/* lane f completes frame f: exact, a range is < 64 KiB + 64 B so
	 * the raw sum of 16-bit halves fits 32 bits */
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const uint4 x = part4[4 * lane + ((j + (lane >> 2)) & 3)];
		t += x.x + x.y + x.z + x.w;
	}
	uint32_t c4, sum4;
	bool absent, l3_bad;
	if constexpr (GEN) {
		/* the exception kernel's ext_sums arithmetic: check word in
		 * the range removed exactly, absolute vs frame-relative
		 * parity */
		c4 = ye.y >> 16;
		if (ye.w & (2u << 16))
			t -= (eff & 1) ? bswap16(c4) : c4;
		uint32_t f = fold16(t);
		if (eff & 1)
			f = bswap16(f);
		sum4 = fold16((uint64_t)(ye.y & 0xffff) + f);
		absent = (ye.w & (1u << 16)) && c4 == 0;
		l3_bad = (rv.z & XDPGPU_F_IP) && !(rv.z & XDPGPU_F_IPV6) &&
			 !(rv.z & XDPGPU_F_L3_OK);
	} else {
		c4 = rv.w & 0xffff;
		if (late) {
			/* the check word is among the summed halves (an even
			 * frame offset in a range from byte 64): taken out
			 * exactly */
			c4 = u16_at(x64, l4 + chk6 - 64);
			t -= c4;
		}
		sum4 = fold16((uint64_t)(rv.y >> 16) + t);
		absent = !r6 && ((rv.z >> 8) & 0xff) == 17 && c4 == 0;
		l3_bad = !(rv.z & XDPGPU_F_L3_OK);
	}
	/* IPv6/TCP: parse_tcphdr's data offset checks (parsing_helpers.h:
	 * 295-318, and the range at least the header), ABORTED otherwise */
	bool abort6 = false;
	if constexpr (!GEN) {
		const uint32_t thl = ((u16_at(x64, l4 + 12 - 64) & 0xff) >> 4) * 4;
		abort6 = late && p6 == 6 && ((thl < 20) | (l4 + thl > dv.z) | (cl < thl));
	}
	const bool l4_ok = absent || (~fold16((uint64_t)sum4 + c4) & 0xffff) == 0;
	const bool drop = (a.flags & XDPGPU_CFG_VERIFY_CSUM) && (l3_bad || !l4_ok);
	/* process_packet's echo reply (af_xdp_user.c:968-1040) for an echo
	 * request that was not dropped: MACs and addresses swapped, type 129,
	 * csum_replace2 of the type word, written over the first 64 bytes as
	 * whole 16-byte chunks; the record and tuple are the request's */
	if (__ballot(echo6)) {
		if (echo6) {
			h0 = *reinterpret_cast<const uint4 *>(a.umem + eff);
			h1 = *reinterpret_cast<const uint4 *>(a.umem + eff + 16);
			h2 = *reinterpret_cast<const uint4 *>(a.umem + eff + 32);
			h3 = *reinterpret_cast<const uint4 *>(a.umem + eff + 48);
		}
	}
	const bool echo_tx = echo6 && ((h3.y >> 16) & 0xff) == 128 && !drop;
	if (echo_tx && !(XDP_TAIL_DIAG & 1) &&
	    !DBG_BAD(eff + 64 > ((a.usize + 15) & ~15ull), 10, eff)) {
		const uint32_t d[16] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w,
					h2.x, h2.y, h2.z, h2.w, h3.x, h3.y, h3.z, h3.w};
		echo_reply_store(a.umem + eff, d);
	}
	if (XDP_TAIL_DIAG & 1) {
		/* diagnostic: no output stores */
	} else if (act && abort6) {
		/* ABORTED frames carry all-zero records and tuples */
		const uint4 z = make_uint4(0, 0, 0, 0);
		if constexpr (kTailRecNt)
			st_nt16(a.res + i, z);
		else
			*reinterpret_cast<uint4 *>(a.res + i) = z;
		if (net6) {
			const uint32_t tz[11] = {};
			store_tuple44(a.tup + 44 * i, tz);
		} else if (a.tup && a.tuple_fmt == XDPGPU_TUPLE_V4) {
			/* the tile stored the 16-byte tuple */
			*reinterpret_cast<uint4 *>(a.tup + 16 * i) = z;
		}
		a.verdict[i] = (uint8_t)XDPGPU_ABORTED;
		my_bytes += dv.z;
	} else if (act) {
		rv.y = (rv.y & 0xffff) | ((~sum4 & 0xffff) << 16);
		rv.z |= (l4_ok ? XDPGPU_F_L4_OK : 0u) |
			(absent ? XDPGPU_F_L4_ABSENT : 0u);
		rv.w = l4 | (cl << 16);
		if constexpr (XDP_TAIL_DIAG & 4) {
			/* diagnostic: no record store */
		} else if constexpr (XDP_TAIL_DIAG & 16) {
			/* diagnostic: the record stored over another frame's, half
			 * the batch away (a line this pass has not read) */
			st_nt16(a.res + (i + a.n / 2) % a.n, rv);
		} else if constexpr (XDP_TAIL_DIAG & 256) {
			/* diagnostic (pools without exception frames only): the
			 * record stored into the payload list's scratch, lines no
			 * pass of the launch writes */
			st_nt16(a.ylist ? reinterpret_cast<uint4 *>(a.ylist) + i
					: reinterpret_cast<uint4 *>(a.res + i), rv);
		} else if constexpr (XDP_TAIL_DIAG & 32) {
			/* diagnostic: a load of the record instead of its store */
			const uint4 q = ld_nt16(a.res + i);
			my_bytes += q.x == 0x9e3779b9u;
		} else if constexpr (XDP_TAIL_DIAG & 64) {
			/* diagnostic: lane 0's record alone */
			if (lane == 0)
				st_nt16(a.res + i, rv);
		} else if constexpr (XDP_TAIL_DIAG & 128) {
			/* diagnostic: the record's second dword alone */
			__builtin_nontemporal_store(rv.y, reinterpret_cast<uint32_t *>(a.res + i) + 1);
		} else if constexpr (kRecStage > 0) {
			/* staged (rec_flush; the reload form keeps its own words) */
			if constexpr (!kRecReload)
				meta[320 + nst * kWave + lane] = rv;
		} else if constexpr (XDP_TAIL_REC_AUX >= 0) {
			const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
				a.res, 0, 0x7fffffff, 0x00020000);
			__builtin_amdgcn_raw_buffer_store_b128((v4u_t){rv.x, rv.y, rv.z, rv.w}, rr,
							       (uint32_t)(16 * i), 0, XDP_TAIL_REC_AUX);
		} else if constexpr (kTailRecNt)
			st_nt16(a.res + i, rv);
		else
			*reinterpret_cast<uint4 *>(a.res + i) = rv;
#ifdef LAT_NOW
		if constexpr ((XDP_LAT_PROBE & 2) != 0) {
			LAT_NOW(lat2);
			LAT_WAIT();
			LAT_NOW(lat3);
			LAT_ACC(sid, lane, 7, lat3 - lat2);
		}
#endif
		if (tup6) {
			/* the addresses and ports, from the words loaded with
			 * the batch, shifted by the tags (nv dwords; the fast
			 * shape keeps them inside bytes [16, 64)) */
			const uint32_t w0[12] = {h1.x, h1.y, h1.z, h1.w, h2.x, h2.y,
						 h2.z, h2.w, h3.x, h3.y, h3.z, h3.w};   /* dwords 4..15 */
			const uint32_t nv = rv.z >> 24;
			uint32_t w[12];
#pragma unroll
			for (int k = 0; k < 12; k++)
				w[k] = nv == 0 ? w0[k]
				     : nv == 1 ? (k + 1 < 12 ? w0[k + 1] : 0u)
					       : (k + 2 < 12 ? w0[k + 2] : 0u);
			uint32_t t[11];
#pragma unroll
			for (int k = 0; k < 4; k++) {
				t[k] = (w[1 + k] >> 16) | (w[2 + k] << 16);
				t[5 + k] = (w[5 + k] >> 16) | (w[6 + k] << 16);
			}
			/* ports for UDP and TCP; ICMPv6 has none */
			const bool ports = p6 == 17 || p6 == 6;
			t[4] = ports ? w[9] >> 16 : 0u;
			t[9] = ports ? w[10] & 0xffffu : 0u;
			t[10] = p6 | (10u << 16);
			/* three wide stores (the record is dword aligned): eleven
			 * scattered dword stores cost IMIX 0.5 ms of tail stores */
			store_tuple44(a.tup + 44 * i, t);
		}
		const uint8_t vd = echo_tx ? XDPGPU_TX : drop ? XDPGPU_DROP : XDPGPU_REDIRECT;
		/* the tile stored the provisional verdict (kBulkVerdictTile) */
		const uint8_t vprov = (a.flags & XDPGPU_CFG_VERIFY_CSUM) && l3_bad ? XDPGPU_DROP
										 : XDPGPU_REDIRECT;
		if (!(XDP_TAIL_DIAG & 8) && (GEN || !kBulkVerdictTile || vd != vprov)) {
			if constexpr (kTailVerdictNt)
				__builtin_nontemporal_store(vd, a.verdict + i);
			else
				a.verdict[i] = vd;
		}
		my_bytes += dv.z;
	}
	if (a.stats) {
		const bool fin = act && !abort6;
		cnt[CNT_FRAMES] += __popcll(__ballot(act));
		cnt[CNT_VERDICT0 + XDPGPU_ABORTED] += __popcll(__ballot(act && abort6));
		cnt[CNT_VERDICT0 + XDPGPU_DROP] += __popcll(__ballot(fin && drop));
		cnt[CNT_VERDICT0 + XDPGPU_TX] += __popcll(__ballot(fin && echo_tx));
		cnt[CNT_VERDICT0 + XDPGPU_REDIRECT] += __popcll(__ballot(fin && !drop && !echo_tx));
		cnt[CNT_L3_BAD] += __popcll(__ballot(fin && l3_bad));
		cnt[CNT_L4_BAD] += __popcll(__ballot(fin && !l4_ok));
		cnt[CNT_L4_ABSENT] += __popcll(__ballot(fin && absent));
		if constexpr (GEN)
			cnt[CNT_FRAG] += __popcll(__ballot(act && (rv.z & XDPGPU_F_FRAG)));
	}
	if constexpr (kRecStage > 0) {
		const bool st = act && !abort6 && !(XDP_TAIL_DIAG & 1);
		uint32_t *ix = stage_idx(meta);
		ix[nst * kWave + lane] = st ? (uint32_t)i : ~0u;
		if constexpr (kRecReload) {
			ix[(kRecStage + nst) * kWave + lane] = (~sum4 & 0xffff) | (l4 << 16);
			const uint64_t okm = __ballot(st && l4_ok), abm = __ballot(st && absent);
			uint64_t *mk = reinterpret_cast<uint64_t *>(ix + 2 * kRecStage * kWave);
			if (lane == 0) {
				mk[2 * nst] = okm;
				mk[2 * nst + 1] = abm;
			}
		}
		nst = __builtin_amdgcn_readfirstlane(nst + 1);
		if (nst == kRecStage) {
			__builtin_amdgcn_wave_barrier();
			if constexpr (kRecReload) {
				/* groups of kRecGroup reloads in flight */
#pragma unroll
				for (uint32_t s = 0; s + kRecGroup <= kRecStage; s += kRecGroup)
					rec_flush_reload<kRecGroup>(a, meta, s, lane);
				if constexpr (kRecStage % kRecGroup)
					rec_flush_reload<kRecStage % kRecGroup>(
						a, meta, kRecStage - kRecStage % kRecGroup, lane);
			} else {
#pragma unroll
				for (uint32_t s = 0; s < kRecStage; s++)
					rec_store_staged(a, meta, s, lane);
			}
			nst = 0;
		}
	}
	__builtin_amdgcn_wave_barrier();
}

/*
 * Fast kernel, 64-byte header windows staged by LDS-DMA.
 *
 * Per wave and tile of 64 frames: the 256 16-byte chunks of the windows go
 * straight from HBM into LDS with four global_load_lds_dwordx4 (nt); in
 * load k lane l fetches chunk c of frame f = 16k + l/4, and slot 64k + l of
 * the tile buffer receives it, with c = (l & 3) ^ ((f >> 2) & 3): frame f's
 * chunk c then sits in slot 4f + (c ^ ((f >> 2) & 3)), which makes the four
 * ds_read_b128 each lane issues for its own frame bank-conflict free.  The
 * DMA of tile t+1 is issued as soon as tile t is in registers, so it runs
 * under tile t's parse.  Descriptors are prefetched two tiles ahead.
 *
 * Frames of the fast shape (Ethernet + 0..2 VLAN tags + IPv4 ihl 5, not a
 * fragment, + UDP/TCP) whose checksum range lies in the window are finished
 * here.  Fast-shape frames with a longer range get everything but the
 * payload sum here and go to the bulk list; every other frame is deferred
 * to the exception kernel.
 */
/* Hardware hazards the compiler cannot see in inline asm (its hazard
 * recognizer only knows the memory instructions it emitted itself):
 *  - a VALU write of an SGPR (v_readfirstlane of a base address) followed
 *    by a VMEM instruction reading that SGPR needs 5 wait states: every
 *    scalar-base store below starts with s_nop 6 (7, a margin over 5);
 *  - a VALU write of the data VGPRs of a preceding store of more than 8
 *    bytes: the compiler puts 2 wait states there on gfx950 (one was seen
 *    to corrupt the data of the last lanes of 16-lane groups), the 12- and
 *    16-byte stores end with s_nop 2 (3).
 */

/* Output stores of the fast kernels' tile loop, as inline asm.  The
 * compiler's wait insertion treats vmcnt as out of order once loads and
 * stores are both pending (on gfx9-class targets they share the counter),
 * so every wait it places for a descriptor load behind a store would be a
 * full vmcnt(0); the hardware retires them in issue order
 * (MI355X_MICROARCH.md), and stores need no wait of their own here.
 * Asm stores are invisible to that tracking, and its waits for the loads
 * it sees stay counted.  (A counted wait is then also a wait for older
 * asm stores: it only ever waits more, never less.)  The kernels that read
 * these bytes back (rx_tail) wait with vmcnt(0) first. */
__device__ __forceinline__ void st_asm_b8(void *p, uint32_t v)
{
	asm volatile("global_store_byte %0, %1, off" :: "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void st_asm_b32(void *p, uint32_t v)
{
	asm volatile("global_store_dword %0, %1, off" :: "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void st_asm_b128_nt(void *p, uint4 r)
{
	const v4u_t v = {r.x, r.y, r.z, r.w};
	asm volatile("global_store_dwordx4 %0, %1, off nt\n\ts_nop 2" :: "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void st_asm_b128(void *p, uint4 r)
{
	const v4u_t v = {r.x, r.y, r.z, r.w};
	asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 2" :: "v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ void st_asm_b96(void *p, uint32_t x, uint32_t y, uint32_t z)
{
	const v3u_t v = {x, y, z};
	asm volatile("global_store_dwordx3 %0, %1, off\n\ts_nop 2" :: "v"(p), "v"(v) : "memory");
}

/* Wave-uniform 64-bit value in SGPRs.  __builtin_amdgcn_readfirstlane
 * returns int: each half goes through uint32_t before widening, or the low
 * half would be sign-extended over the high one. */
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v)
{
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
	return ((uint64_t)hi << 32) | lo;
}

/* A wave-uniform pointer in SGPRs (the compiler cannot see that a value
 * derived from the wave index is uniform). */
template <typename T>
__device__ __forceinline__ T *uniform_ptr(T *p)
{
	return (T *)(uintptr_t)uniform_u64((uint64_t)(uintptr_t)p);
}

/* The same in the scalar-base form: a wave-uniform 64-bit base in SGPRs
 * and a 32-bit per-lane byte offset, so no 64-bit address is held in
 * VGPRs across the loop. */
__device__ __forceinline__ void st_asm_sb8(const void *base, uint32_t off, uint32_t v)
{
	asm volatile("s_nop 6\n\tglobal_store_byte %0, %1, %2" :: "v"(off), "v"(v), "s"(base)
		     : "memory");
}

__device__ __forceinline__ void st_asm_sb32(const void *base, uint32_t off, uint32_t v)
{
	asm volatile("s_nop 6\n\tglobal_store_dword %0, %1, %2" :: "v"(off), "v"(v), "s"(base)
		     : "memory");
}

__device__ __forceinline__ void st_asm_sb128(const void *base, uint32_t off, uint4 r, bool nt)
{
	const v4u_t v = {r.x, r.y, r.z, r.w};
	if (nt)
		asm volatile("s_nop 6\n\tglobal_store_dwordx4 %0, %1, %2 nt\n\ts_nop 2"
			     :: "v"(off), "v"(v), "s"(base) : "memory");
	else
		asm volatile("s_nop 6\n\tglobal_store_dwordx4 %0, %1, %2\n\ts_nop 2"
			     :: "v"(off), "v"(v), "s"(base) : "memory");
}

__device__ __forceinline__ void st_asm_sb96(const void *base, uint32_t off, uint32_t x,
					    uint32_t y, uint32_t z)
{
	const v3u_t v = {x, y, z};
	asm volatile("s_nop 6\n\tglobal_store_dwordx3 %0, %1, %2\n\ts_nop 2"
		     :: "v"(off), "v"(v), "s"(base) : "memory");
}

/* Per-wave state of the fast kernels' tile loop. */
struct FastWave {
	uint32_t cnt[CNT_FRAG + 1];       /* wave-uniform counters         */
	uint64_t my_bytes;                /* per lane                      */
	uint32_t xq_n, xout, bq_n, bout;  /* queued / flushed deferrals
					   * (uniform): exception, bulk    */
	uint32_t *xq, *bq;                /* LDS queues, 2 x 64 entries    */
	uint32_t *xl, *bl;                /* this wave's list regions (the
					   * block's: xdp_rx_db_kernel)    */
	uint32_t *lcount;                 /* xdp_rx_db_kernel: the block's
					   * list lengths in LDS (2)       */
};

/* Append the frames of the lanes with want set to a list: LDS queue in
 * lane order, flushed 64 entries at a time to this wave's region. */
__device__ __forceinline__ void defer_append(bool want, uint64_t i, uint32_t *q,
					     uint32_t &qn, uint32_t *gl,
					     uint32_t &gout, int lane)
{
	const uint64_t dm = __ballot(want);
	if (!dm)
		return;
	const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
		(uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0));
	if (want)
		q[qn + rank] = (uint32_t)i;
	qn += (uint32_t)__popcll(dm);
	if (qn >= (uint32_t)kWave) {
		__builtin_amdgcn_wave_barrier();
		st_asm_b32(gl + gout + lane, q[lane]);
		gout += kWave;
		const uint32_t rest = q[kWave + lane];
		__builtin_amdgcn_wave_barrier();
		q[lane] = rest;
		qn -= kWave;
	}
}

/*
 * One tile of the fast kernels, after its 64-byte windows are in F:
 * fast-shape classification, deferral of the other frames, and for fast
 * frames the checksums, flow key, hash, tuple, record, verdict and
 * counters.  Frames of the fast shape (Ethernet + 0..2 VLAN tags + IPv4
 * ihl 5, not a fragment, + UDP/TCP) whose checksum range lies in the window
 * are finished here; fast-shape frames with a longer range get everything
 * but the payload sum and go to the bulk list; every other frame goes to
 * the exception list.
 */
/* A fast tile's outputs, kept in registers from its step to the next one,
 * whose stores they are (xdp_rx_db_kernel).  The flow key of a fast-shape
 * frame varies only in saddr, daddr, ports and protocol (IPv4 mapped into
 * ::ffff:0:0/96), so the record, the verdict and the V4 or network_tuple
 * layouts all rebuild from these words. */
struct TileOut {
	uint64_t t0;       /* first frame of the tile (wave-uniform)        */
	uint32_t li;       /* this lane's frame in the tile                 */
	uint32_t fl;       /* bit 0: verdict store, bit 1: record and tuple,
			    * bit 2: IPv6 (network_tuple: the bulk
			    * pass's; 16-byte tuple: stored here)      */
	uint32_t verdict;
	uint32_t sa, da, ports, proto, vid;
	uint4 rec;
};

/* The stores of a TileOut: exactly kTileStores buffer stores over the
 * tile's records whatever the configuration (the double-buffered kernel's
 * counted wait relies on the number), a lane with nothing to store, and a
 * store the configuration does not need, at an offset past its resource's
 * size (dropped by the hardware); no branches. */
constexpr int kTileStores = 5;
/* cache policy (buffer aux bits) of the tile's verdict, record and 16-byte
 * tuple stores: build knobs for A/B (0 plain, 2 non-temporal).  Config 2,
 * alternating processes (tools/gpu_ab_stores.sh): non-temporal verdicts
 * 0.3292 vs 0.3376 ms plain; plain records and tuples 0.400 ms */
#ifndef XDP_VERDICT_AUX
#define XDP_VERDICT_AUX 2
#endif
#ifndef XDP_REC_AUX
#define XDP_REC_AUX 2
#endif
#ifndef XDP_TUP4_AUX
#define XDP_TUP4_AUX 2
#endif
__device__ __forceinline__ void store_tile(const RxArgs &a, const TileOut &o)
{
	constexpr uint32_t kOff = 0x80000000u;
	constexpr int kFmt = 0x00020000;      /* gfx9 raw buffer dword 3 */
	const bool bad = DBG_BAD(o.t0 >= a.n || (o.t0 & (kWave - 1)), 9, o.t0);
	const uint32_t fl = bad ? 0u : o.fl;
	const __amdgpu_buffer_rsrc_t rv =
		__builtin_amdgcn_make_buffer_rsrc(a.verdict + o.t0, 0, kWave, kFmt);
	__builtin_amdgcn_raw_buffer_store_b8((uint8_t)o.verdict, rv,
					     (fl & (kBulkVerdictTile ? 3 : 1)) ? o.li : kOff, 0,
					     XDP_VERDICT_AUX);
	const bool out = fl & 2;
	/* a missing output: a resource of no records over the verdicts */
	const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
		a.res ? (void *)(a.res + o.t0) : (void *)a.verdict, 0,
		a.res ? 16 * kWave : 0, kFmt);
	__builtin_amdgcn_raw_buffer_store_b128((v4u_t){o.rec.x, o.rec.y, o.rec.z, o.rec.w},
					       rr, out ? 16 * o.li : kOff, 0, XDP_REC_AUX);
	const bool net = a.tuple_fmt == XDPGPU_TUPLE_NET;
	const bool tup = a.tup && (net || a.tuple_fmt == XDPGPU_TUPLE_V4);
	const uint32_t tb = net ? 44u : 16u;
	const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
		tup ? (void *)(a.tup + tb * o.t0) : (void *)a.verdict, 0,
		tup ? (int)(tb * kWave) : 0, kFmt);
	/* an IPv6 frame's network_tuple is the bulk pass's (its addresses
	 * are not among the words kept here); its 16-byte tuple is stored
	 * here */
	const bool tout = out && !((fl & 4) && net);
	const uint32_t b = tout ? tb * o.li : kOff;
	/* a quick frame's tuple (fl bit 3): all zero */
	const uint32_t zq = (fl & 8) ? 0u : ~0u;
	const uint32_t ipv = ((fl & 4) ? 10u : 2u) & zq;
	const v4u_t w0 = net ? (v4u_t){0u, 0u, 0xffff0000u & zq, o.sa}
			     : (v4u_t){o.sa, o.da, o.ports, o.proto | (ipv << 8) | (o.vid << 16)};
	/* 16-byte tuples: whole lines, streamed (nt).  44-byte tuples: the
	 * lanes' 16-byte pieces straddle lines that other stores of the tile
	 * complete, so they stay in L2 to merge there (nt: 2x the loop time on
	 * IMIX) */
	if (net) {
		__builtin_amdgcn_raw_buffer_store_b128(w0, rt, b, 0, 0);
	} else {
		__builtin_amdgcn_raw_buffer_store_b128(w0, rt, b, 0, XDP_TUP4_AUX);
	}
	__builtin_amdgcn_raw_buffer_store_b128((v4u_t){o.ports & 0xffff, 0u, 0u, 0xffff0000u & zq},
					       rt, net && tout ? b + 16 : kOff, 0, 0);
	__builtin_amdgcn_raw_buffer_store_b96((v3u_t){o.da, o.ports >> 16,
						      o.proto | ((2u << 16) & zq)},
					      rt, net && tout ? b + 32 : kOff, 0, 0);
}

/* Append to the block's list without an LDS queue: the wave reserves its
 * entries with one LDS atomic on the list's length, and each deferred lane
 * stores its index at its rank (a partial line per store; deferrals are
 * rare on the fast shapes). */
__device__ __forceinline__ void defer_direct(bool want, uint64_t i, uint32_t *gl,
					     uint32_t *lcount, int lane, uint32_t xcap)
{
	const uint64_t dm = __ballot(want);
	if (!dm)
		return;
	const uint32_t base = lds_fetch_add(lcount, (uint32_t)__popcll(dm), lane);
	const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
		(uint32_t)(dm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0));
	if (want && !DBG_BAD(base + rank >= xcap, 7, base + rank))
		st_asm_sb32(uniform_ptr(gl), (base + rank) * 4u, (uint32_t)i);
}

/* NW: window words a lane holds, 16 (64-byte windows) or 32 (128-byte
 * windows, RxArgs.win: a frame's bytes [64, 128) are staged too when it
 * is longer than 64 bytes and starts a 128-byte line, win_hi below) */
/* A 128-byte window's second half as read_tile_w2 reduces it (so that
 * its 16 words need no registers past the read): the sum of the frame's
 * words 16 + nv .. 31 (nv VLAN tags), and its words 16 + nv and 17 + nv
 * (the tag-shifted words 16 and 17: IPv6/TCP's data offset and check
 * word).  Its words 16 and 17 themselves are F[16], F[17]. */
struct WinHi {
	uint64_t s2;
	uint32_t w16, w17;
	/* XDP_TAIL_SHARE: bit 16 set when the next lane's window held this
	 * frame's last bytes (its range ends in the first half of the line
	 * the next frame starts halfway into), their sum folded in bits 0-15 */
	uint32_t tail;
};
/* The line a 64-byte-offset frame starts in: its first half is the end of
 * the frame before it, which the bulk pass would fetch again.  With
 * XDP_TAIL_SHARE the window DMA stages that first half in the second
 * half's slot (no bytes the line fetch does not bring anyway) and the
 * previous lane's frame, a bulk frame whose range ends there, takes its
 * sum: the bulk pass streams that frame only to the line start. */
#ifndef XDP_TAIL_SHARE
#define XDP_TAIL_SHARE 1
#endif
/* diagnostic builds only (instruction-count and timing probes, wrong
 * outputs): parts of the tile loop's compute left out.  1 the second half's
 * reduction (read_tile_w2), 2 the jhash, 4 the IPv6 shape, 8 the quick
 * classification, 16 the counters, 32 the deferrals (no tail work), 64 the
 * 128-byte tile loop's output stores */
#ifndef XDP_TILE_DIAG
#define XDP_TILE_DIAG 0
#endif
constexpr bool kTailShare = XDP_TAIL_SHARE != 0;

/* ECHO (128-byte windows with the echo responder on): an untagged ICMPv6
 * echo request whose range ends inside the window is answered here too */
template <bool LQ, bool ST = true, bool V6 = false, int NW = 16, bool ECHO = false>
__device__ __forceinline__ void fast_tile(const RxArgs &a, const uint32_t (&F)[18],
					  uint4 dv, uint64_t i, bool active,
					  bool dma, int lane, FastWave &w,
					  TileOut *to = nullptr, const WinHi *wh = nullptr)
{
	static_assert(NW == 16 || NW == 32, "64- or 128-byte windows");
	const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
	const uint32_t len = dv.z;
	const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
	const bool staged = dma & active & (len >= 14) & ((uint64_t)len <= a.usize) &
			    (eff <= a.usize - len) & !(eff & 15) &
			    (eff + 64 <= ((a.usize + 15) & ~15ull));
	/* the second half was staged (128-byte windows) */
	const bool hi = NW == 32 && win_hi(a, eff, len);

	/* 2. fast-shape classification, branch free (bitwise &/| on
	 * flags, selects).  r[j] = frame dword j + nv */
	const bool v1 = le_is_vlan(F[3] & 0xffff);
	const bool v2 = v1 & le_is_vlan(F[4] & 0xffff);
	const uint32_t nv = (uint32_t)v1 + (uint32_t)v2;
	/* masks, not selects: a select chain over F is turned into a
	 * dynamically indexed private array (scratch) by the compiler */
	uint32_t r[16];
	if (kUntaggedTiles && !__ballot(v1)) {
		/* a tile with no tagged frame (config 2's every tile): the
		 * words as they are, 65 VALU instructions of 500 fewer */
#pragma unroll
		for (int j = 3; j < 16; j++)
			r[j] = F[j];
	} else {
		/* two selects a word on the lanes' tag masks, as asm: written
		 * as C selects the compiler turns the words into a dynamically
		 * indexed private array (scratch) */
		const uint64_t k1 = __ballot(v1), k2 = __ballot(v2);
#pragma unroll
		for (int j = 3; j < 16; j++)
			r[j] = lane_sel(k2, lane_sel(k1, F[j], F[j + 1]), F[j + 2]);
	}
	const uint32_t l3 = 14 + 4 * nv, l4 = l3 + 20;
	const uint32_t tot = bswap16(r[4] & 0xffff);
	const uint32_t proto = r[5] >> 24;
	const bool udp = proto == 17;
	/* V6 builds (the 44-byte network_tuple and no tuple: IMIX) also take
	 * IPv4 ICMP: the message sum with no pseudo header and no over-read
	 * byte (an odd length zero padded, do_csum), no ports in the key */
	const bool icmp = V6 && proto == 1;
	const uint32_t thl = ((r[11] >> 20) & 0xf) * 4;
	const uint32_t cl = udp ? bswap16(r[9] >> 16) : tot - 20;
	const bool ok_udp = (len >= l4 + 8) & (cl >= 8) & (l4 + cl <= l3 + tot);
	const bool ok_tcp = (len >= l4 + 20) & (thl >= 20) & (l4 + thl <= len) &
			    (cl >= thl);
	const bool ok_icmp = (len >= l4 + 8) & (cl >= 8);
	bool fast = (!a.force_generic) & staged &
		    ((r[3] & 0x00ffffffu) == 0x00450008u) &
		    ((r[5] & 0xff3fu) == 0) & (udp | (proto == 6) | icmp) &
		    (tot >= 20) & (l3 + tot <= len) &
		    (udp ? ok_udp : icmp ? ok_icmp : ok_tcp);
	/* a checksum range (with udp_csum's odd over-read byte) that ends
	 * past the window: the bulk kernel adds the payload sum */
	const bool shape = fast;
	const uint32_t over = icmp ? 0u : (cl & 1);
	/* the window ends at 64, or at 128 where the second half was staged
	 * (its words, masked by the range, come summed in wh) */
	fast = shape & (l4 + cl + over <= (hi ? 128u : 64u));
	bool bulk = shape & !fast & (a.res != nullptr);

	/* V6: IPv6 with no extension header behind 0..2 VLAN tags, in the
	 * shifted words r (r[j] = frame dword j + nv, zero past the window),
	 * with the generic parse's conditions (parse_ip6hdr, parse_udphdr,
	 * parse_tcphdr, parse_icmp6hdr):
	 *  - UDP behind at most one tag (its length at l4 + 4 in the window),
	 *    the range its length;
	 *  - TCP behind at most one tag (both ports in the window), the range
	 *    the payload length; its data offset lies past the window, so the
	 *    bulk pass checks it (ABORTED when parse_tcphdr would fail);
	 *  - ICMPv6 (its type in the window) other than NDP (PASS,
	 *    af_xdp_kern.c:114-148), the range the payload length; with the
	 *    echo responder, an untagged echo request is answered by the bulk
	 *    pass once its checksum verifies (process_packet,
	 *    af_xdp_user.c:968-1040).
	 * csum_ipv6_magic, an odd length zero padded, a stored 0 not absent.
	 * A check word at or past byte 64 (TCP; UDP behind a tag; ICMPv6
	 * behind two) is "late": the bulk pass reads it, and the data offset,
	 * from frame bytes [64, 80). */
	bool v6 = false, i6 = false, t6 = false, full6 = false, fast6 = false, echo_el = false;
	uint32_t ulen6 = 0, nh6 = 0;
	if constexpr (V6 && !(XDP_TILE_DIAG & 4)) {
		const uint32_t plen = bswap16(r[4] >> 16);
		nh6 = r[5] & 0xff;
		const uint32_t ity = (r[13] >> 16) & 0xff;
		const bool u6 = nh6 == 17;
		t6 = nh6 == 6;
		i6 = (nh6 == 58) & (plen >= 8) & !((ity >= 133) & (ity <= 137));
		ulen6 = u6 ? bswap16(r[14] >> 16) : plen;
		v6 = (!a.force_generic) & staged & ((r[3] & 0xffffu) == 0xdd86u) &
		     (((r[3] >> 20) & 0xf) == 6) & (l3 + 40 + plen <= len) &
		     ((u6 & (nv <= 1) & (ulen6 >= 8) & (ulen6 <= plen)) | i6 |
		      (t6 & (nv <= 1) & (plen >= 20))) &
		     (a.res != nullptr);
		i6 = i6 & v6;
		t6 = t6 & v6;
		if constexpr (NW == 32) {
			/* 128-byte windows: a staged IPv6 frame (full6) is
			 * summed to its range end or byte 128 here, its check
			 * word and TCP's data offset taken from the window (a
			 * data offset that fails parse_tcphdr is left to the bulk
			 * pass's late path, which ABORTs it); a range that ends
			 * inside the window is finished here (an untagged echo
			 * request under the responder too: the ECHO instance
			 * answers it below) */
			const uint32_t thl6 = ((wh->w16 >> 20) & 0xf) * 4;
			const uint32_t re6 = 54 + 4 * nv + ulen6;
			full6 = hi & v6 &
				(!t6 | ((thl6 >= 20) & (54 + 4 * nv + thl6 <= len) & (thl6 <= ulen6)));
			/* (the launcher takes the ECHO instance whenever the responder is on) */
			echo_el = ECHO & i6 & (nv == 0);
			fast6 = full6 & (re6 <= 128u);
		}
		/* through the bulk pass (which also reads a late check word)
		 * unless finished in a 128-byte window; a payload inside the
		 * window is an empty range there */
		bulk = bulk | (v6 & !fast6);
		fast = fast | fast6;
	}

	/* Quick frames (kQuick, the per-CU kernel): verdicts parse_lane
	 * decides from bytes the window holds, with all-zero records and
	 * tuples (generic_batch's outputs for ABORTED and PASS):
	 *  - a runt (len < 14: parse_ethhdr_vlan fails, in bounds or not);
	 *  - for a staged frame of at least 64 bytes (its tags all consumed,
	 *    every byte read below lies in the frame and the window):
	 *    ARP behind 0..2 tags (PASS); untagged-or-tagged IPv6 with no
	 *    extension header and an ICMPv6 type 133..137 (NDP: PASS); IPv6
	 *    with a version other than 6 (ABORTED); IPv4 whose header
	 *    fails parse_iphdr (version, ihl, header or tot_len past the
	 *    frame, tot_len below the header: ABORTED), and with a 20-byte
	 *    header, not a later fragment, whose UDP length, TCP data offset
	 *    or ICMP length fails parse_udphdr / parse_tcphdr /
	 *    parse_icmphdr or runs past tot_len (ABORTED).
	 * Every other frame the fast shape does not take stays an exception. */
	bool quick = false;
	uint32_t qv = XDPGPU_ABORTED;
	if (!LQ && kQuick && !(XDP_TILE_DIAG & 8) && (!XDP_QUICK_SKIP || __ballot(active & !fast & !bulk))) {
		const uint32_t et = r[3] & 0xffff;
		const bool big = (!a.force_generic) & staged & (len >= 64);
		const bool arp = big & (et == 0x0608u);
		const uint32_t vihl = (r[3] >> 16) & 0xff, hl = (vihl & 15) * 4;
		const bool hdr_bad = ((vihl >> 4) != 4) | (hl < 20) | (l3 + hl > len) |
				     (tot < hl) | (l3 + tot > len);
		const uint32_t fo = bswap16(r[5] & 0xffff) & 0x3fff;
		const bool fragb = fo != 0, nonfirst = (fo & 0x1fff) != 0;
		const uint32_t ulen = bswap16(r[9] >> 16);
		const bool udp_bad = (proto == 17) & ((ulen < 8) | (!fragb & (l4 + ulen > l3 + tot)));
		const bool tcp_bad = (proto == 6) &
				     ((thl < 20) | (l4 + thl > len) | (!fragb & (tot - 20 < thl)));
		const bool icmp_bad = (proto == 1) & !fragb & (tot - 20 < 8);
		const bool abort4 = big & (et == 0x0008u) &
				    (hdr_bad | ((hl == 20) & !nonfirst & (udp_bad | tcp_bad | icmp_bad)));
		const bool ip6 = big & (et == 0xdd86u);
		const bool ver6 = ((r[3] >> 20) & 0xf) == 6;
		const uint32_t ty6 = (r[13] >> 16) & 0xff;
		const bool ndp = ip6 & ver6 & ((r[5] & 0xff) == 58) & (ty6 >= 133) & (ty6 <= 137) &
				 (len >= l3 + 48);
		const bool abort6 = ip6 & !ver6;
		const bool runt = (!a.force_generic) & (len < 14);
		quick = active & !fast & !bulk & (runt | arp | ndp | abort4 | abort6);
		qv = (arp | ndp) ? XDPGPU_PASS : XDPGPU_ABORTED;
	}

	/* 3. defer the frames of other shapes to the exception list and
	 * the long ones to the bulk list of this wave */
	if constexpr (LQ) {
		defer_append(active && !fast && !bulk, i, w.xq, w.xq_n, w.xl, w.xout, lane);
		defer_append(bulk, i, w.bq, w.bq_n, w.bl, w.bout, lane);
	} else {
		if constexpr (!(XDP_TILE_DIAG & 32)) {
			defer_direct(active && !fast && !bulk && !quick, i, w.xl, w.lcount, lane,
				     a.xregion);
			defer_direct(bulk, i, w.bl, w.lcount + 1, lane, a.xregion);
		}
	}

	/* 4. fast frames: flow key, hash, tuple, checksums, verdict */
	const uint32_t sa = (r[6] >> 16) | (r[7] << 16);
	const uint32_t da = (r[7] >> 16) | (r[8] << 16);
	const uint32_t ports = icmp ? 0u : (r[8] >> 16) | (r[9] << 16);
	/* IPv4 header sum, check word (r6 low half) excluded */
	/* (the sums are of 16-bit halves in 32 bits, add_halves: congruent
	 * mod 0xffff to the words' sums, so every fold16 below is unchanged) */
	const uint32_t s3 = add_halves(add_halves(add_halves(add_halves(add_halves(
		r[3] >> 16, r[4]), r[5]), r[6] >> 16), r[7]), r[8] & 0xffffu);
	const uint32_t c3 = r[6] & 0xffff;
	const uint32_t c4 = udp ? (r[10] & 0xffff) : icmp ? (r[9] & 0xffff) : (r[12] >> 16);
	/* L4 sum over [34, end) of the shifted frame with the pseudo
	 * header, check word excluded; udp_csum's odd-length over-read
	 * byte included (lib_checksum.h:142-179).  For a bulk frame the
	 * window part: frame bytes [l4, 64), or [l4, 128) with a staged
	 * second half (hi: its words past r's come summed in wh->s2).  r holds
	 * frame words up to 15 + nv; those past 15 count only for hi. */
	const int32_t e0 = (int32_t)(34 + cl + over);
	const int32_t e = (NW == 16 || hi) ? e0 : min(e0, (int32_t)(64 - 4 * nv));
	uint32_t s4 = add_halves(icmp ? 0u : add_halves(add_halves((proto + cl) << 8, sa), da),
				 r[8] >> 16);
	if constexpr (NW == 32)
		s4 += hi ? (uint32_t)wh->s2 : 0u;
	/* first_bytes(e - 4 j) as one clamp and one 64-bit shift */
	const int32_t sb = 32 - 8 * e;
#pragma unroll
	for (int j = 9; j < 16; j++) {
		uint32_t m = (uint32_t)(0xffffffffull >> min(max(sb + 32 * j, 0), 32));
		if (j == 9)
			m &= icmp ? 0xffff0000u : 0xffffffffu;
		if (j == 10)
			m &= udp ? 0xffff0000u : 0xffffffffu;
		if (j == 12)
			m &= udp || icmp ? 0xffffffffu : 0x0000ffffu;
		s4 = add_halves(s4, r[j] & m);
	}
	uint32_t key[11] = {0, 0, 0xffff0000u, sa, ports & 0xffff,
			    0, 0, 0xffff0000u, da, ports >> 16,
			    proto | (2u << 16)};
	uint32_t s3v = s3, s4v = s4;
	uint32_t c3v = c3, c4v = c4, clv = cl, l4v = l4, protov = proto;
	bool udpv = udp;
	if constexpr (V6 && !(XDP_TILE_DIAG & 4)) {
		/* the v6 frame's terms (selected per lane: branch free), in the
		 * shifted words: L4 at 54, addresses at 22-53 */
		/* (from 0: a raw first term near 2^32 would wrap the 32-bit sum) */
		uint32_t p6 = add_halves(add_halves(0u, __builtin_bswap32(ulen6)),
					 __builtin_bswap32(nh6));
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const uint32_t sk = (r[5 + k] >> 16) | (r[6 + k] << 16);
			const uint32_t dk = (r[9 + k] >> 16) | (r[10 + k] << 16);
			p6 = add_halves(add_halves(p6, sk), dk);
			key[k] = v6 ? sk : key[k];
			key[5 + k] = v6 ? dk : key[5 + k];
		}
		const int32_t e6 = (int32_t)(54 + ulen6);
		/* L4 bytes [54, 64 - 4 nv) of the window (r is zero past it);
		 * the check word left out where it lies inside: ICMPv6 at
		 * 56-57, UDP at 60-61 (TCP's, at 70-71, never does) */
		const bool u6 = v6 & !i6 & !t6;
		/* r's words past frame byte 64 count only for full6 (with
		 * 64-byte windows they are zero) */
		const uint32_t r14 = (NW == 16 || nv < 2 || full6) ? r[14] : 0u;
		const uint32_t r15 = (NW == 16 || nv < 1 || full6) ? r[15] : 0u;
		uint32_t s46 = add_halves(add_halves(add_halves(p6, r[13] >> 16),
					   r14 & first_bytes(e6 - 56) & (i6 ? 0xffff0000u : ~0u)),
					   r15 & first_bytes(e6 - 60) & (u6 ? 0xffff0000u : ~0u));
		if constexpr (NW == 32)
			/* the second half (TCP's check word left out by the
			 * read) */
			s46 += full6 ? (uint32_t)wh->s2 : 0u;
		key[4] = v6 ? (i6 ? 0u : r[13] >> 16) : key[4];
		key[9] = v6 ? (i6 ? 0u : r[14] & 0xffffu) : key[9];
		key[10] = v6 ? (nh6 | (10u << 16)) : key[10];
		s4v = v6 ? s46 : s4v;
		s3v = v6 ? 0xffffu : s3v;        /* no IPv6 header checksum: l3 ok */
		c3v = v6 ? 0u : c3v;
		/* the check word where the window holds it (0: late, the bulk
		 * pass loads it) */
		uint32_t c6 = 0;
		if constexpr (NW == 32)
			c6 = full6 ? (i6 ? r[14] & 0xffffu : u6 ? r[15] & 0xffffu : wh->w17 >> 16) : 0u;
		c4v = v6 ? (full6 ? c6
			    : i6 ? (nv <= 1 ? r[14] & 0xffffu : 0u)
			    : u6 && nv == 0 ? r[15] & 0xffffu : 0u)
			 : c4v;
		clv = v6 ? ulen6 : clv;
		l4v = v6 ? 54u + 4 * nv : l4v;
		protov = v6 ? nh6 : protov;
		udpv = udpv & !v6;               /* a stored 0 is not absent */
	}
	/* a bulk frame whose last bytes the next lane summed (XDP_TAIL_SHARE;
	 * not an IPv6 frame the bulk pass streams from byte 64, whose check
	 * word it takes out of its own sum) */
	bool tshare = false;
	if constexpr (NW == 32 && kTailShare) {
		tshare = bulk & ((wh->tail >> 16) & 1) & (!v6 | full6);
		s4v += tshare ? (wh->tail & 0xffffu) : 0u;
	}
	const uint32_t l3c = v6 ? 0u : ~fold16(s3v) & 0xffff;
	const bool l3_ok = fold16((uint64_t)s3v + c3v) == 0xffff;
	const uint32_t sum4 = fold16(s4v);
	const uint32_t l4c = ~sum4 & 0xffff;
	const bool absent = udpv && c4v == 0;
	const bool l4_ok = absent || (~fold16((uint64_t)sum4 + c4v) & 0xffff) == 0;
	const bool drop = (a.flags & XDPGPU_CFG_VERIFY_CSUM) && (!l3_ok || !l4_ok);
	/* the echo responder (ECHO): a finished untagged echo request that
	 * was not dropped is answered in place (the bulk pass's reply) */
	bool echo_tx = false;
	if constexpr (V6 && NW == 32 && ECHO) {
		echo_tx = fast6 & echo_el & (((r[13] >> 16) & 0xff) == 128) & !drop;
		if (echo_tx && !DBG_BAD(eff + 64 > ((a.usize + 15) & ~15ull), 10, eff)) {
			const uint32_t d[16] = {F[0], F[1], F[2], F[3], F[4], F[5], F[6], F[7],
						F[8], F[9], F[10], F[11], F[12], F[13], F[14], F[15]};
			echo_reply_store(a.umem + eff, d);
		}
	}
	/* a bulk frame's record carries its window sum in the l4_csum field
	 * and its check word in l4_off until the bulk pass completes it */
	uint4 rec;
	rec.x = (XDP_TILE_DIAG & 2) ? key[0] ^ key[8] : jhash_key44(key, a.initval);
	rec.y = l3c | ((fast ? l4c : sum4) << 16);
	rec.z = XDPGPU_F_IP | XDPGPU_F_L4 | (nv ? XDPGPU_F_VLAN : 0u) |
		(v6 ? XDPGPU_F_IPV6 : 0u) |
		(l3_ok ? XDPGPU_F_L3_OK : 0u) |
		(fast && l4_ok ? XDPGPU_F_L4_OK : 0u) |
		(fast && absent ? XDPGPU_F_L4_ABSENT : 0u) |
		(protov << 8) | (l3 << 16) | (nv << 24);
	rec.w = (fast ? l4v : c4v) | (clv << 16);
	/* an IPv6 bulk frame summed to byte 128 in its window (full6): the
	 * nvlan byte's top bit tells the bulk pass, which clears it */
	if constexpr (NW == 32)
		rec.z |= ((full6 & !fast6) ? 0x80000000u : 0u) | (tshare ? 0x40000000u : 0u);
	/* the verdict stored with the tile: a fast frame's, and a bulk frame's
	 * provisional one (DROP for a bad IPv4 header under verification,
	 * else REDIRECT), which the bulk pass overwrites only when the frame's
	 * final verdict differs (a bad L4 checksum, an echo reply, ABORTED):
	 * the tile's verdict bytes are one coalesced store, the bulk pass's
	 * scattered single bytes partial-line writes (kBulkVerdictTile) */
	const bool vdrop = fast ? drop : ((a.flags & XDPGPU_CFG_VERIFY_CSUM) && !l3_ok);
	const uint32_t vid = nv ? (bswap16(F[3] >> 16) & 0x0fff) : 0u;
	const uint4 tv4 = make_uint4(sa, da, ports, proto | (2u << 8) | (vid << 16));
	const bool out = fast || bulk;
	if constexpr (LQ) {
		if (out) {
			/* the tile's first frame index (wave-uniform): scalar
			 * bases, per-lane offsets of at most 64 records */
			const uint64_t t0 = uniform_u64(i);
			uint32_t li = (uint32_t)(i - t0);
			if (fast || kBulkVerdictTile)
				st_asm_sb8(a.verdict + t0, li,
					   vdrop ? XDPGPU_DROP : XDPGPU_REDIRECT);
			if (a.res)
				st_asm_sb128(a.res + t0, 16 * li, rec, true);
			if (a.tup) {
				if (a.tuple_fmt == XDPGPU_TUPLE_V4) {
					st_asm_sb128(a.tup + 16 * t0, 16 * li, tv4, true);
				} else if (a.tuple_fmt == XDPGPU_TUPLE_NET) {
					/* 44-byte records: dword aligned */
					const uint8_t *tb = a.tup + 44 * t0;
					st_asm_sb128(tb, 44 * li,
						     make_uint4(key[0], key[1], key[2], key[3]),
						     false);
					st_asm_sb128(tb, 44 * li + 16,
						     make_uint4(key[4], key[5], key[6], key[7]),
						     false);
					st_asm_sb96(tb, 44 * li + 32, key[8], key[9], key[10]);
				}
			}
		}
	} else if constexpr (ST) {
		/* the outputs, stored by the next step (store_tile) */
		to->t0 = uniform_u64(i);   /* all lanes active: lane 0 */
		to->li = (uint32_t)(i - to->t0);
		to->fl = (fast || quick ? 1u : 0u) | (out || quick ? 2u : 0u) | (v6 ? 4u : 0u) |
			 (quick ? 8u : 0u);
		to->verdict = quick ? qv : echo_tx ? XDPGPU_TX : vdrop ? XDPGPU_DROP : XDPGPU_REDIRECT;
		/* an IPv6 frame's 16-byte tuple: no addresses, its ports (none
		 * for ICMPv6), ipv 10 (emit_tuple's layout); a quick frame's:
		 * zero */
		to->sa = v6 || quick ? 0u : sa;
		to->da = v6 || quick ? 0u : da;
		to->ports = quick ? 0u : v6 ? (i6 ? 0u : (r[13] >> 16) | (r[14] << 16)) : ports;
		to->proto = quick ? 0u : v6 ? nh6 : proto;
		to->vid = quick ? 0u : vid;
		to->rec = quick ? make_uint4(0, 0, 0, 0) : rec;
		if constexpr (V6 && kTup6Tile) {
			/* an IPv6 frame's network_tuple now, from the window
			 * (the deferred stores keep four words of a tuple) */
			if (v6 && active && a.tup && a.tuple_fmt == XDPGPU_TUPLE_NET)
				store_tuple44(a.tup + 44 * i, key);
		}
	}
	w.my_bytes += fast || quick ? len : 0;
	/* counters (wave-uniform: ballots outside divergent code) */
	if (!(XDP_TILE_DIAG & 16) && a.stats) {
		w.cnt[CNT_FRAMES] += __popcll(__ballot(fast || quick));
		if constexpr (!LQ && kQuick) {
			w.cnt[CNT_VERDICT0 + XDPGPU_PASS] += __popcll(__ballot(quick && qv == XDPGPU_PASS));
			w.cnt[CNT_VERDICT0 + XDPGPU_ABORTED] +=
				__popcll(__ballot(quick && qv == XDPGPU_ABORTED));
		}
		w.cnt[CNT_VERDICT0 + XDPGPU_DROP] += __popcll(__ballot(fast && drop));
		w.cnt[CNT_VERDICT0 + XDPGPU_REDIRECT] += __popcll(__ballot(fast && !drop && !echo_tx));
		if constexpr (ECHO)
			w.cnt[CNT_VERDICT0 + XDPGPU_TX] += __popcll(__ballot(echo_tx));
		w.cnt[CNT_L3_BAD] += __popcll(__ballot(fast && !l3_ok));
		w.cnt[CNT_L4_BAD] += __popcll(__ballot(fast && !l4_ok));
		w.cnt[CNT_L4_ABSENT] += __popcll(__ballot(fast && absent));
	}
}

/* End of a fast kernel's tile loop: the queued deferrals to the wave's
 * list regions and the list lengths to global memory. */
__device__ __forceinline__ void rx_flush_lists(const RxArgs &a, const FastWave &w,
					       uint64_t wgid, int lane)
{
	__builtin_amdgcn_wave_barrier();
	if ((uint32_t)lane < w.xq_n)
		w.xl[w.xout + lane] = w.xq[lane];
	if ((uint32_t)lane < w.bq_n)
		w.bl[w.bout + lane] = w.bq[lane];
	if (lane == 0) {
		a.xcount[wgid] = w.xout + w.xq_n;
		a.bcount[wgid] = w.bout + w.bq_n;
		a.ycount[wgid] = 0;   /* filled by the exception pass */
	}
}

/* Counters of a wave into its block's LDS slot (lane 0; the block's
 * slot goes to global memory in block_stats_flush). */
__device__ __forceinline__ void wave_stats_to_lds(const RxArgs &a,
						  unsigned long long *blk_cnt,
						  const uint32_t (&cnt)[CNT_FRAG + 1],
						  uint64_t my_bytes, int lane)
{
	if (!a.stats)
		return;
	const uint64_t bytes = wave_sum64(my_bytes);
	if (lane == 0) {
		atomicAdd(&blk_cnt[CNT_BYTES], (unsigned long long)bytes);
#pragma unroll
		for (int k = 0; k <= CNT_FRAG; k++)
			if (k != CNT_BYTES && cnt[k])
				atomicAdd(&blk_cnt[k], (unsigned long long)cnt[k]);
	}
}

/*
 * Tail phase of the double-buffered fast kernel: the block finishes its
 * deferred frames, the exception batches, the bulk batches and the
 * exception frames' deferred payload sums, from one queue of batches (an
 * LDS counter, ctl[3]); each wave reuses its own
 * LDS: win (64 rows of 17 dwords) and gtab (64 u64) for the exception
 * batches, meta (64 uint4) and part (256 uint4) for the bulk batches.
 * Called by every wave of the block (barriers) after a vmcnt(0) and a
 * barrier that end the tile loop.  A wave's vmcnt(0) before each barrier
 * makes its list entries, outputs and payload-list entries visible to the
 * block's other waves, whose L1 lines for them are never loaded before
 * (read-once lists).
 */
/* the tail's payload streaming: groups of kTailG lanes per frame, kTailU
 * 16-byte loads per lane and step (1 KiB per frame and step; 4-lane
 * groups of 8 loads, every load of a 570-byte IMIX payload useful, ran
 * 8 % slower on IMIX and 13 % on 1500 B: the loads of an instruction
 * then touch 16 frames) */
/* (8-lane groups since round 4's 128-byte windows, with the bulk ranges
 * starting at byte 128: IMIX 1.864 / 1.859 vs 1.884 / 1.885 ms, 2 M x
 * 1500 B 0.589 / 0.590 vs 0.604 / 0.602, the echo leg and config 2
 * unchanged, alternating processes, profiles/r04_ab_tail_g8.txt; six
 * loads a lane spilled: IMIX 2.10 ms) */
#ifndef XDP_TAIL_G
#define XDP_TAIL_G 8
#endif
#ifndef XDP_TAIL_U
#define XDP_TAIL_U 4
#endif
constexpr int kTailG = XDP_TAIL_G, kTailU = XDP_TAIL_U;
template <int WIN, bool EC>
__device__ __forceinline__ void rx_tail(const RxArgs &a, const FastWave &w,
					uint64_t rb, uint32_t xc, uint32_t bc,
					int wid, int nw, uint32_t *ctl, int lane,
					uint32_t *win,
					uint64_t *gtab, uint4 *meta, uint4 *part4,
					uint32_t (&cnt)[CNT_FRAG + 1], uint64_t &my_bytes)
{
	uint4 *yl = a.ylist + rb * a.xregion;
	uint32_t *yc = a.ycount + rb;
	/* One queue of batches, each wave claiming the next: the exception
	 * batches (which list the exception frames' long payloads), the bulk
	 * batches, then those payload batches.  A wave that reaches the
	 * payload batches first waits until every exception batch is done
	 * (ctl[5] counts them, each after a vmcnt(0) that makes its list
	 * entries visible): by then only batches already claimed remain. */
	const uint32_t nbb = (bc + kWave - 1) / kWave, nxb = (xc + kWave - 1) / kWave;
	uint32_t ycn = 0, nyb = 0;
	/* staged batches of records (kRecStage) */
	uint32_t nst = 0;
	bool ready = nxb == 0;
	STAMP_T0();
	for (;;) {
		const uint32_t q = lds_fetch_add(ctl + 3, 1, lane);
		if (q < nxb) {
			const uint32_t b = q * kWave;
			const bool act = b + lane < xc;
			uint64_t i = act ? w.xl[b + lane] : 0;
			const bool bad = act && DBG_BAD(i >= a.n, 1, i);
			i = bad ? 0 : i;
			generic_batch<64>(a, win, gtab, lane, i, act && !bad, yl, yc, cnt,
					  my_bytes);
			lds_dma_landed();
			(void)lds_fetch_add(ctl + 5, 1, lane);
			STAMP_ADD(rb * nw + wid, lane, 4);
			continue;
		}
		if (q < nxb + nbb) {
			const uint32_t b = (q - nxb) * kWave;
			bulk_batch<kTailU, true, false, kTailG, WIN, EC>(
				a, meta, part4, lane, w.bl + b,
				bc - b < (uint32_t)kWave ? bc - b : kWave, cnt, my_bytes, nst,
				rb * nw + wid);
			STAMP_ADD(rb * nw + wid, lane, 5);
			continue;
		}
		if (!ready) {
			while (lds_fetch_add(ctl + 5, 0, lane) < nxb)
				__builtin_amdgcn_s_sleep(2);
			ready = true;
			STAMP_ADD(rb * nw + wid, lane, 7);
		}
		if (!nyb && !ycn) {
			/* the count the exception batches' atomics left (read at
			 * the L2, where they were made) */
			if (lane == 0)
				ycn = atomicAdd(yc, 0u);
			ycn = __builtin_amdgcn_readfirstlane(ycn);
			nyb = (ycn + kWave - 1) / kWave;
		}
		const uint32_t yq = q - nxb - nbb;
		if (yq >= nyb)
			break;
		const uint32_t b = yq * kWave;
		bulk_batch<kTailU, true, true, kTailG>(
			a, meta, part4, lane, yl + b, ycn - b < (uint32_t)kWave ? ycn - b : kWave,
			cnt, my_bytes, nst);
		STAMP_ADD(rb * nw + wid, lane, 6);
	}
	if constexpr (kRecStage > 0)
		rec_flush(a, meta, nst, lane);
}

/*
 * Fast kernel, double-buffered (the default RX launch).
 *
 * Each wave keeps two tiles' window DMAs in flight: tile k is read from
 * its LDS buffer while tile k+1's DMA is landing in the other one, and
 * tile k+2's DMA goes into tile k's buffer once tile k is done.  The two
 * buffers are distinct __shared__ variables, so the compiler's LDS-DMA
 * tracking tells them apart; the explicit wait is a counted vmcnt:
 *
 *   per iteration, in order: [wait] [read buffer k] [tile k: compute,
 *   deferrals, stores] [DMA tile k+2 -> buffer k (4 ops)] [descriptor
 *   load, tile k+3 (1 op)]
 *
 * so at the start of iteration k at least 6 vector-memory ops (the
 * descriptor load of iteration k-2, the 4 DMA ops and the descriptor load
 * of iteration k-1) were issued after tile k's DMA; vmcnt counts loads,
 * stores and LDS-DMA together in issue order (MI355X_MICROARCH.md), so
 * vmcnt(6) means tile k's windows have landed, while tile k+1's DMA may
 * still be in flight.  Every DMA and descriptor load is issued
 * unconditionally (past the end they read the UMEM's first 64 bytes and
 * the last descriptor), which keeps the count a lower bound.
 *
 * 4 waves per SIMD (the two buffers need 160 KB of LDS per CU at that
 * occupancy), 128 VGPRs: room for the tail phase (rx_tail) inline, so
 * one launch does the whole batch.
 */
/* One tile's inputs out of the double-buffered LDS, in one asm block:
 * the counted wait vmcnt(5) (see xdp_rx_db_kernel), this lane's 64-byte
 * window
 * (four conflict-free ds_read_b128) and the descriptor of the tile two
 * steps ahead (one ds_read_b128), then the wait for the reads.  In asm
 * because no compiler-visible access may touch LDS the DMA writes: its
 * wait insertion would add vmcnt(0) (it treats LDS-DMA and other vector
 * memory ops as completing out of order), and in one block so that no
 * use of the results is scheduled before their lgkmcnt wait. */
typedef __attribute__((address_space(3))) uint4 lds_uint4_t;
template <int N>
__device__ __forceinline__ void read_tile_db(const uint4 *win, const uint4 *dslot,
					     int lane, uint32_t (&F)[18], uint4 &dn)
{
	/* one address VGPR per buffer: the lane's slot 4 lane + (c ^ sw) is
	 * p ^ 16 c for p = its slot sw (the per-wave buffers are 64-byte
	 * aligned, so the XOR touches only bits 4-5); the chunk addresses are
	 * made in the asm, so that the compiler keeps no four-register set of
	 * loop-invariant LDS addresses live over the tile loop (they were what
	 * the 128-VGPR budget spilled) */
	const int sw = (lane >> 2) & 3;
	const lds_uint4_t *lw = (const lds_uint4_t *)win;
	const lds_uint4_t *ld = (const lds_uint4_t *)dslot;
	const uint32_t p = (uint32_t)(uintptr_t)(lw + 4 * lane + sw);
	const uint32_t ad = (uint32_t)(uintptr_t)(ld + lane);
	v4u_t v0, v1, v2, v3, vd;
	uint32_t t1, t2, t3;
#define XDP_READ_TILE(N)                                                        \
	asm volatile("s_waitcnt vmcnt(" #N ")\n\t"                              \
		     "v_xor_b32 %5, 16, %8\n\t"                                \
		     "v_xor_b32 %6, 32, %8\n\t"                                \
		     "v_xor_b32 %7, 48, %8\n\t"                                \
		     "ds_read_b128 %0, %8\n\t"                                  \
		     "ds_read_b128 %1, %5\n\t"                                  \
		     "ds_read_b128 %2, %6\n\t"                                  \
		     "ds_read_b128 %3, %7\n\t"                                  \
		     "ds_read_b128 %4, %9\n\t"                                  \
		     "s_waitcnt lgkmcnt(0)"                                     \
		     : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(vd),   \
		       "=&v"(t1), "=&v"(t2), "=&v"(t3)                          \
		     : "v"(p), "v"(ad)                                          \
		     : "memory")
	if constexpr (N == 10)
		XDP_READ_TILE(10);
	else
		XDP_READ_TILE(5);
#undef XDP_READ_TILE
	F[0] = v0.x; F[1] = v0.y; F[2] = v0.z; F[3] = v0.w;
	F[4] = v1.x; F[5] = v1.y; F[6] = v1.z; F[7] = v1.w;
	F[8] = v2.x; F[9] = v2.y; F[10] = v2.z; F[11] = v2.w;
	F[12] = v3.x; F[13] = v3.y; F[14] = v3.z; F[15] = v3.w;
	F[16] = F[17] = 0;
	dn = make_uint4(vd.x, vd.y, vd.z, vd.w);
}

/* The 128-byte window form (xdp_rx_db_kernel WIN 128): a lane's two
 * halves out of the two buffers (the first 64 bytes in win0, bytes
 * [64, 128) in win1, each in the tile layout above) and the descriptor of
 * the tile two steps ahead, after the counted wait vmcnt(N). */
template <int N, bool V6>
__device__ __forceinline__ void read_tile_w2(const RxArgs &a, const uint4 *win0,
					     const uint4 *win1, const uint4 *dslot, int lane,
					     uint32_t (&F)[18], WinHi &wh, uint4 &dn, uint4 dv,
					     bool st_ok)
{
	/* the addresses as in read_tile_db: one VGPR for the lane's window
	 * slots (win1 is win0 + 4 KiB: the instructions' offset field) */
	const int sw = (lane >> 2) & 3;
	const lds_uint4_t *l0 = (const lds_uint4_t *)win0;
	const lds_uint4_t *ld = (const lds_uint4_t *)dslot;
	(void)win1;
	const uint32_t p = (uint32_t)(uintptr_t)(l0 + 4 * lane + sw);
	const uint32_t ad = (uint32_t)(uintptr_t)(ld + lane);
	v4u_t v0, v1, v2, v3, v4, v5, v6, v7, vd;
	uint32_t x1, x2, x3;
#define XDP_READ_W2(N)                                                          \
	asm volatile("s_waitcnt vmcnt(" #N ")\n\t"                             \
		     "v_xor_b32 %9, 16, %12\n\t"                               \
		     "v_xor_b32 %10, 32, %12\n\t"                              \
		     "v_xor_b32 %11, 48, %12\n\t"                              \
		     "ds_read_b128 %0, %12\n\t"                                \
		     "ds_read_b128 %1, %9\n\t"                                 \
		     "ds_read_b128 %2, %10\n\t"                                \
		     "ds_read_b128 %3, %11\n\t"                                \
		     "ds_read_b128 %4, %12 offset:4096\n\t"                    \
		     "ds_read_b128 %5, %9 offset:4096\n\t"                     \
		     "ds_read_b128 %6, %10 offset:4096\n\t"                    \
		     "ds_read_b128 %7, %11 offset:4096\n\t"                    \
		     "ds_read_b128 %8, %13\n\t"                                \
		     "s_waitcnt lgkmcnt(0)"                                     \
		     : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3), "=&v"(v4),   \
		       "=&v"(v5), "=&v"(v6), "=&v"(v7), "=&v"(vd),              \
		       "=&v"(x1), "=&v"(x2), "=&v"(x3)                          \
		     : "v"(p), "v"(ad)                                          \
		     : "memory")
	if constexpr (N == 1)
		XDP_READ_W2(1);
	else
		XDP_READ_W2(0);
#undef XDP_READ_W2
	const v4u_t vv[4] = {v0, v1, v2, v3};
#pragma unroll
	for (int k = 0; k < 4; k++) {
		F[4 * k] = vv[k].x;
		F[4 * k + 1] = vv[k].y;
		F[4 * k + 2] = vv[k].z;
		F[4 * k + 3] = vv[k].w;
	}
	/* the second half, reduced now (WinHi): the words past the frame's
	 * tags, each masked by the range end fast_tile derives (the same
	 * fields: an IPv4 frame's L4 range, with udp_csum's over-read byte
	 * and, in V6 builds, ICMP's none; an IPv6 frame's UDP length or
	 * payload length), an IPv6/TCP check word (bytes 70-71 shifted) out;
	 * fast_tile uses the sum only for the shapes it takes */
	const uint32_t A[34] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
				v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w,
				v4.x, v4.y, v4.z, v4.w, v5.x, v5.y, v5.z, v5.w,
				v6.x, v6.y, v6.z, v6.w, v7.x, v7.y, v7.z, v7.w, 0u, 0u};
#pragma unroll
	for (int k = 0; k < 18; k++)
		F[k] = A[k];
	const bool t1 = le_is_vlan(A[3] & 0xffff);
	const bool t2 = t1 & le_is_vlan(A[4] & 0xffff);
	const uint32_t nvt = (uint32_t)t1 + (uint32_t)t2;
	/* a header word past the tags: two selects (the frame's words are not
	 * shifted: the sums below move the range end by the tags instead) */
	const uint64_t k1 = __ballot(t1), k2 = __ballot(t2);
	auto shw = [&](int j) -> uint32_t {
		return lane_sel(k2, lane_sel(k1, A[j], A[j + 1]), A[j + 2]);
	};
	if constexpr ((XDP_TILE_DIAG & 1) != 0) {
		wh.s2 = 0;
		wh.w16 = wh.w17 = 0;
		wh.tail = 0;
		dn = make_uint4(vd.x, vd.y, vd.z, vd.w);
		return;
	}
	const uint32_t w3 = shw(3), w4 = shw(4), w5 = shw(5);
	const bool is6 = (w3 & 0xffff) == 0xdd86u;
	const uint32_t proto = w5 >> 24, nh6 = w5 & 0xff;
	const uint32_t tot = bswap16(w4 & 0xffff), plen = bswap16(w4 >> 16);
	const uint32_t cl = proto == 17 ? bswap16(shw(9) >> 16) : tot - 20;
	const uint32_t e4 = 34 + cl + ((V6 && proto == 1) ? 0u : (cl & 1));
	const uint32_t e6 = 54 + (nh6 == 17 ? bswap16(shw(14) >> 16) : plen);
	const int32_t e = (int32_t)(is6 ? e6 : e4);
	const uint32_t w16 = shw(16), w17 = shw(17);
	/* the tag-shifted words 16..31 masked by the range end e are the
	 * frame's words 16 + nv..31 masked by the frame-relative end E; the
	 * shifted word 17 of an IPv6/TCP frame keeps only its low half (the
	 * check word at shifted bytes 70-71 is left out) */
	const int32_t E = (e > 0 ? e : 0) + 4 * (int32_t)nvt;
	const bool tcp6 = is6 && nh6 == 6;
	/* words 16 and 17 count only past the tags; an IPv6/TCP frame's
	 * shifted word 17 keeps its low half */
	auto wmask = [&](int k) -> uint32_t {
		uint32_t m = ~0u;
		if (k == 16)
			m = t1 ? 0u : m;
		if (k == 17)
			m = t2 ? 0u : m;
		if (k >= 17 && k <= 19)
			m &= (tcp6 && (uint32_t)k == 17 + nvt) ? 0x0000ffffu : ~0u;
		return m;
	};
	uint32_t s2 = 0;
	if (!__ballot((E > 64) & (E < 128))) {
		/* no range ends inside the second half (IMIX, 1500 B: 64-byte
		 * frames end before it, the long ones after): each lane's words
		 * count whole or not at all */
#pragma unroll
		for (int k = 16; k < 32; k++)
			s2 = add_halves(s2, A[k] & wmask(k));
		s2 = E >= 128 ? s2 : 0u;
	} else {
		/* byte masks first_bytes(E - 4 k) as one clamp and one 64-bit
		 * shift each: the shift 32 - 8 (E - 4 k) clamped to [0, 32] */
		const int32_t sb = 32 - 8 * E;
#pragma unroll
		for (int k = 16; k < 32; k++) {
			const int32_t sh = min(max(sb + 32 * k, 0), 32);
			const uint32_t m = (uint32_t)(0xffffffffull >> sh) & wmask(k);
			s2 = add_halves(s2, A[k] & m);
		}
	}
	wh.s2 = s2;
	wh.w16 = w16;
	wh.w17 = w17;
	wh.tail = 0;
	if constexpr (kTailShare) {
		/* this lane's range end, absolute, to the next lane; the end of
		 * the previous lane's, back */
		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool staged = st_ok & (len >= 14) & ((uint64_t)len <= a.usize) &
				    (eff <= a.usize - len) & !(eff & 15) &
				    (eff + 64 <= ((a.usize + 15) & ~15ull));
		/* (a frame starting 64-byte aligned only: its bulk range then
		 * starts 64-byte aligned too, so it starts at or before the line
		 * start wherever it ends inside that line's first half; a frame
		 * starting 16 bytes before the line would have its window and the
		 * next lane's half-line overlap) */
		const uint64_t Eabs = (eff & 63) ? 0ull : eff + (uint32_t)E;
		const uint64_t Ep =
			((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(Eabs >> 32), 1, kWave) << 32) |
			(uint32_t)__shfl_up((int)(uint32_t)Eabs, 1, kWave);
		/* win1 holds [eff - 64, eff) for a staged frame 64 bytes into its
		 * line (issue_win2) */
		const bool lo = staged & ((eff & 127) == 64) & (lane > 0) & (Ep > eff - 64) &
				(Ep <= eff);
		uint32_t snd = 0;
		/* (a tile with no such frame skips the sum) */
		if (__ballot(lo)) {
			const int32_t m = lo ? (int32_t)(Ep - (eff - 64)) : 0;
			const int32_t sb = 32 - 8 * m;
			uint32_t ts = 0;
#pragma unroll
			for (int j = 0; j < 16; j++) {
				const int32_t sh = min(max(sb + 32 * j, 0), 32);
				ts = add_halves(ts, A[16 + j] & (uint32_t)(0xffffffffull >> sh));
			}
			snd = lo ? 0x10000u | fold16(ts) : 0u;
		}
		const uint32_t rcv = (uint32_t)__shfl_down((int)snd, 1, kWave);
		wh.tail = lane < kWave - 1 ? rcv : 0u;
	}
	dn = make_uint4(vd.x, vd.y, vd.z, vd.w);
}

/* Per-wave LDS of the double-buffered kernel, in uint4: two window buffers
 * (256 each) and two descriptor slots (64 each), 10 KiB; kCuWaves waves per
 * block, one block per CU. */
constexpr int kDbWave = 2 * 256 + 2 * 64;
#ifndef XDP_CU_WAVES
#define XDP_CU_WAVES 15
#endif
constexpr int kCuWaves = XDP_CU_WAVES;
constexpr int kCuBlock = kCuWaves * kWave;

/*
 * Fast kernel, double-buffered: the default RX launch.
 *
 * Each wave keeps two tiles in flight: the window DMA of tile k+1 (and the
 * descriptor DMA of tiles k+2, k+3) land while tile k is processed.  Step k
 * on tile t_k, buffer and slot b = k & 1, in issue order:
 *
 *   [wait vmcnt(10); read window t_k from W[b], descriptor t_{k+2} from
 *   D[b]] [output stores of t_{k-1}: kTileStores = 5 ops] [DMA windows of
 *   t_{k+2} -> W[b]: 4 ops] [DMA descriptors t_{k+4} -> D[b]: 1 op]
 *   [tile t_k: compute, deferral stores; outputs kept for step k+1]
 *
 * Descriptor t_{k+2} was DMA'd at step k-2, after the window DMA of t_k,
 * and step k-1 issued 10 ops (5 stores, 5 DMAs) after both; vmcnt counts
 * loads, stores and LDS-DMA together in issue order, so vmcnt(10) means
 * both of step k's inputs have landed while the previous step's stores
 * may still be in flight (a wait that also covered them, vmcnt(5), cost
 * 11 % on config 2).  The count is exact only because every step issues
 * the same ops: store_tile always issues its 5 stores (those a
 * configuration does not need go out of range and are dropped), every DMA
 * is issued unconditionally (past the batch end a window DMA reads the
 * UMEM's first 64 bytes and a descriptor DMA the last descriptor), and the
 * deferral stores only add younger ops.  The prologue issues its DMAs and
 * one empty store_tile in an order that meets the count for steps 0 and 1.
 * (An earlier vmcnt(10) that assumed 5 stores where a configuration
 * issued 3 read stale windows: the count must not depend on the
 * configuration.)  The descriptor of t_k itself (for the compute) was read
 * at step k-2 and travels in registers.
 *
 * Nothing the loop consumes from memory is a compiler-visible load
 * (read_tile_db), so the compiler's wait insertion, which treats vmcnt as
 * out of order once LDS-DMA is pending, never adds a vmcnt(0) to the loop.
 * The output stores are buffer stores issued unconditionally (a lane with
 * nothing to store is out of the resource's range), so the loop has no
 * store branches.
 *
 * One block per CU, kCuWaves waves, tiles claimed at run time.  With a
 * static share per wave (64 tiles each on config 2) the waves of a CU
 * finished 140-170 us apart in a 370 us launch, in the order they were
 * dispatched (rank correlation 0.94, tools/stamps.py): the SIMD's issue
 * arbitration favours its oldest wave, which ran its share twice as fast
 * as the youngest.  So the block's tiles (b, b + nb, b + 2 nb, ... for
 * block b of nb) are handed out by an LDS counter, one claim per step,
 * made 5 steps ahead of the tile's compute (the pipeline needs the tile
 * for its descriptor DMA 4 steps ahead): an LDS atomic, waited on by
 * lgkmcnt, never by vmcnt.  Deferred frames go to the block's lists (an
 * LDS atomic reserves each wave's entries), counters to a per-wave slot,
 * and the tail phase (rx_tail) splits the block's lists over its waves in
 * the same launch, on the same LDS, once the last DMA has landed.
 *
 * 15 waves per CU (4, 4, 4, 3 per SIMD: 15 x 10 KiB of buffers and the
 * block's counters in the CU's 160 KiB), 128 VGPRs.
 *
 * Shared tiles: the block's own tiles (above) are the first part of the
 * batch; the rest (12/16 by default, RxArgs.steal_tiles) is claimed at run
 * time, two tiles per claim, from 16 global counters (block b: counter b
 * mod 16), so the CUs that run faster take more: with static shares the
 * CUs' loop ends spread over 30 us of a 330 us launch.  Config 2: 0.3226
 * vs 0.3435 ms without, in one process (tools/gpu_ab_steal.sh).
 */
/* DIAG (diagnostic A/B, cfg.tune bits 16-17): 1 = no compute (the
 * window's XOR stored as verdict, record and tuple: the same memory
 * traffic), 2 = the full compute with no output stores. */
/* cache policy of the tile loop's descriptor DMA (build knob for A/B):
 * plain.  Non-temporal ran config 2 at 0.3249 vs 0.3298 ms
 * (tools/gpu_ab_desc.sh) but the maximum-size frames test then raised an
 * illegal memory access (tests/test_max_frames.py, round-2 evidence run);
 * not understood, not used */
#ifndef XDP_DESC_AUX
#define XDP_DESC_AUX 0
#endif
/* cache policy of the tile loop's window DMA (build knob for A/B): nt */
#ifndef XDP_WIN_AUX
#define XDP_WIN_AUX 2
#endif
/* WIN 128 (RxArgs.win): 128-byte windows, the two buffers holding one
 * tile's two halves (single-buffered: tile k+1's DMA is issued as tile k
 * is read), so the LDS and the waves per CU stay as they are; not with
 * FRAGS or DIAG. */
template <bool FRAGS, int DIAG = 0, bool V6 = false, int WIN = 64, bool ECHO = false>
__global__ __launch_bounds__(kCuBlock, 1) void xdp_rx_db_kernel(RxArgs a)
{
	static_assert(WIN == 64 || (WIN == 128 && !FRAGS && !DIAG), "128-byte windows: the RX default only");
	static_assert(!ECHO || (V6 && WIN == 128), "the tile loop's echo responder: V6, 128-byte windows");
	/* 64-byte aligned: read_tile_db and read_tile_w2 address a lane's window
	 * slots by XOR inside each wave's 64-byte aligned buffers */
	__shared__ __attribute__((aligned(64))) uint4 lds_all[kCuWaves * kDbWave];
	/* the block's tile claims, list lengths (exception, bulk) and the
	 * tail's batch claims (its two passes) */
	__shared__ uint32_t ctl[8];
	/* the counted wait: the 5 DMAs of the step before and, but for the
	 * no-store variant, the kTileStores output stores issued after them
	 * (kept in the count, so that no step waits for stores) */
	constexpr int kWaitN = DIAG == 2 ? 5 : 5 + kTileStores;
	static_assert(kWaitN == 5 || kWaitN == 10, "read_tile_db's waits");

	const int lane = threadIdx.x & (kWave - 1);
	/* the wave index in an SGPR: every per-wave base (LDS buffers) is
	 * then scalar, and no such pointer occupies VGPRs (where the
	 * allocator spilled one to scratch, and each reload waited
	 * vmcnt(0)).  The LDS-DMA ordering does not rest on the compiler's
	 * view of these pointers (read_tile_db). */
	const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
	uint4 *wl = lds_all + wid * kDbWave;
	uint4 *win0 = wl, *win1 = wl + 256, *dsl0 = wl + 512, *dsl1 = wl + 576;
	const uint64_t rb = blockIdx.x, nb = gridDim.x;
	const uint64_t wgid = rb * kCuWaves + wid;

	if (threadIdx.x == 0) {
		ctl[0] = ctl[1] = ctl[2] = ctl[3] = ctl[4] = ctl[5] = ctl[6] = ctl[7] = 0;
		a.ycount[rb] = 0;      /* filled by the exception pass */
	}
	/* the next launch's shared-tile counters (this launch's set was
	 * zeroed by the one before) */
	if (rb == 0 && threadIdx.x < kStealHeads && a.steal)
		a.steal[((a.steal_set ^ 1) * kStealHeads + threadIdx.x) * kStealStride] = 0;
	lds_dma_landed();
	__syncthreads();

	const uint32_t nfr = a.n;
	const uint64_t ntiles = ((uint64_t)nfr + kWave - 1) / kWave;
	FastWave w = {};
	w.xl = a.xlist + rb * a.xregion;
	w.bl = a.blist + rb * a.xregion;
	w.lcount = ctl + 1;
	STAMP(wgid, lane, 0);

	const bool dma = !a.force_generic && a.usize >= 64;
	/* the block's own tiles are those below own, its k-th b + k nb; the
	 * shared ones above are claimed after them (a.steal_tiles).  (Other
	 * orders, measured and rejected: a contiguous range per block, 0.3504
	 * vs 0.3448 ms; each round of nb tiles rotated over the blocks, 11 %
	 * slower; adjacent pairs per block, 0.3222 vs 0.3179 ms; the order
	 * shifted by s XCDs, no s ahead: DESIGN.md §5.2) */
	const uint64_t shared = FRAGS || DIAG ? 0 : a.steal_tiles;
	const uint64_t own = ntiles - shared;
	auto tile_of = [&](uint64_t k) -> uint64_t {
		const uint64_t t = rb + k * nb;
		return t < own ? t : ntiles;
	};
	/* the block's next cnt tiles: claim indices k .. k + cnt-1 */
	auto claim = [&](uint32_t cnt) -> uint64_t {
		return (uint64_t)lds_fetch_add(&ctl[0], cnt, lane);
	};
	/* descriptor index of lane's frame in tile tt, clamped to the batch */
	auto desc_at = [&](uint64_t tt) -> uint64_t {
		const uint64_t i = tt * kWave + lane;
		return i < nfr ? i : nfr - 1;
	};
	/* DMA of a tile's 64-byte windows into buf; the
	 * frame offsets reach the loading lanes by lane shuffles */
	auto issue_win = [&](uint4 dv, bool live, uint4 *buf) {
		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool ok = live & dma & (len >= 14) & ((uint64_t)len <= a.usize) &
				(eff <= a.usize - len) & !(eff & 15) &
				(eff + 64 <= ((a.usize + 15) & ~15ull));
		const uint64_t e = ok ? eff : 0ull;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int f = 16 * k + (lane >> 2);
			const int c = (lane & 3) ^ ((f >> 2) & 3);
			uint64_t ef =
				((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e >> 32), f, kWave) << 32) |
				(uint32_t)__shfl((int)(uint32_t)e, f, kWave);
			if (DBG_BAD(ef + 16 * c + 16 > ((a.usize + 15) & ~15ull), 4, ef))
				ef = 0;
			__builtin_amdgcn_global_load_lds(
				(const void *)(a.umem + ef + 16 * c),
				(lds_void_t *)(buf + kWave * k), 16, 0, XDP_WIN_AUX);
		}
	};
	/* WIN 128: a tile's first halves into win0 and, for the frames
	 * win_hi takes, bytes [64, 128) into win1 (others: the UMEM's first
	 * 64 bytes, unused) */
	auto issue_win2 = [&](uint4 dv, bool live) {
		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool ok = live & dma & (len >= 14) & ((uint64_t)len <= a.usize) &
				(eff <= a.usize - len) & !(eff & 15) &
				(eff + 64 <= ((a.usize + 15) & ~15ull));
		const uint64_t e = ok ? eff : 0ull;
		const uint64_t e2 = ok && win_hi(a, eff, len) ? eff + 64
				  : kTailShare && ok && (eff & 127) == 64 ? eff - 64 : 0ull;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int f = 16 * k + (lane >> 2);
			const int c = (lane & 3) ^ ((f >> 2) & 3);
			uint64_t ef =
				((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e >> 32), f, kWave) << 32) |
				(uint32_t)__shfl((int)(uint32_t)e, f, kWave);
			uint64_t eg =
				((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e2 >> 32), f, kWave) << 32) |
				(uint32_t)__shfl((int)(uint32_t)e2, f, kWave);
			if (DBG_BAD(ef + 16 * c + 16 > ((a.usize + 15) & ~15ull), 4, ef))
				ef = 0;
			if (DBG_BAD(eg + 16 * c + 16 > ((a.usize + 15) & ~15ull), 4, eg))
				eg = 0;
			__builtin_amdgcn_global_load_lds(
				(const void *)(a.umem + ef + 16 * c),
				(lds_void_t *)(win0 + kWave * k), 16, 0, XDP_WIN_AUX);
			__builtin_amdgcn_global_load_lds(
				(const void *)(a.umem + eg + 16 * c),
				(lds_void_t *)(win1 + kWave * k), 16, 0, XDP_WIN_AUX);
		}
	};
	/* DMA of a tile's 64 descriptors into a slot (lane l: descriptor l) */
	auto issue_desc = [&](uint64_t tt, uint4 *slot) {
		uint64_t di = desc_at(tt);
		if (DBG_BAD(di >= nfr, 5, di))
			di = 0;
		__builtin_amdgcn_global_load_lds((const void *)(a.desc + di),
						 (lds_void_t *)slot, 16, 0, XDP_DESC_AUX);
	};
	/* the previous step's outputs, stored after this step's wait (the
	 * first step stores an empty TileOut: every lane out of range) */
	TileOut pend = {};
	/* step on tile t, whose descriptor dv travels in registers: the
	 * window DMA of tile tw (2 steps ahead, its descriptor from the slot:
	 * returned), the descriptor DMA of tile td (4 ahead), the claim of
	 * the tile 5 ahead (into tn) */
	auto step = [&](uint64_t t, uint4 *win, uint4 *dsl, uint4 dv, uint64_t tw,
			uint64_t td, uint64_t &tn) -> uint4 {
		const uint64_t i = t * kWave + lane;
		bool skip = false;
		if constexpr (FRAGS) {
			const uint32_t contd = dv.w & XDPGPU_PKT_CONTD;
			uint32_t prev = (uint32_t)__shfl_up((int)contd, 1, kWave);
			if (lane == 0)
				prev = t ? a.desc[t * kWave - 1].options & XDPGPU_PKT_CONTD : 0u;
			skip = (contd | prev) != 0;
		}
		const bool active = (i < nfr) & !skip;
		uint32_t F[18];
		uint4 dn;
		read_tile_db<kWaitN>(win, dsl, lane, F, dn);
		if constexpr (DIAG != 1 && DIAG != 2)
			store_tile(a, pend);
		issue_win(dn, tw < ntiles, win);
		issue_desc(td, dsl);
		tn = tile_of(claim(1));
		if constexpr (DIAG == 1) {
			uint32_t x = dv.x ^ dv.z;
#pragma unroll
			for (int k = 0; k < 16; k++)
				x ^= F[k];
			const uint64_t t0 = t * kWave;
			const uint32_t li = (uint32_t)lane;
			const __amdgpu_buffer_rsrc_t rv =
				__builtin_amdgcn_make_buffer_rsrc(a.verdict + t0, 0, kWave, 0x00020000);
			const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
				a.res + t0, 0, 16 * kWave, 0x00020000);
			const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
				a.tup + 16 * t0, 0, 16 * kWave, 0x00020000);
			const uint32_t off = active ? li : 0x80000000u;
			__builtin_amdgcn_raw_buffer_store_b8((uint8_t)x, rv, off, 0, 0);
			__builtin_amdgcn_raw_buffer_store_b128((v4u_t){x, x, x, x}, rr,
							       active ? 16 * li : off, 0, 2);
			__builtin_amdgcn_raw_buffer_store_b128((v4u_t){x, 0, x, 0}, rt,
							       active ? 16 * li : off, 0, 2);
		} else {
			fast_tile<false, DIAG != 2, V6>(a, F, dv, i, active, dma, lane, w, &pend);
		}
		return dn;
	};

	/* WIN 128: step on tile t (descriptor dv), single-buffered: the
	 * counted wait is for the windows the previous step issued (only its
	 * descriptor DMA, and any deferral stores, are younger), then the
	 * previous tile's stores, tile tw's windows (its descriptor dnext,
	 * read a step earlier), the descriptor DMA of tile td (4 ahead into
	 * this step's slot, read 2 steps ahead as now) and the claim */
	auto step2 = [&](uint64_t t, uint4 *dsl, uint4 dv, uint4 dnext, uint64_t tw,
			 uint64_t td, uint64_t &tn) -> uint4 {
		const uint64_t i = t * kWave + lane;
		const bool active = i < nfr;
		uint32_t F[18];
		WinHi wh;
		uint4 dn;
		read_tile_w2<1, V6>(a, win0, win1, dsl, lane, F, wh, dn, dv, active && dma);
		if constexpr (!(XDP_TILE_DIAG & 64))
			store_tile(a, pend);
		issue_win2(dnext, tw < ntiles);
		issue_desc(td, dsl);
		tn = tile_of(claim(1));
		fast_tile<false, true, V6, 32, ECHO>(a, F, dv, i, active, dma, lane, w, &pend, &wh);
		return dn;
	};

	/* the wave's tiles T0 < T1 < ...: the first five claimed at once */
	const uint64_t first = claim(5);
	uint64_t q0 = tile_of(first), q1 = tile_of(first + 1), q2 = tile_of(first + 2),
		 q3 = tile_of(first + 3), q4 = tile_of(first + 4), q5;
	if (WIN == 128 && q0 < ntiles) {
		/* prologue: descriptors of T0 and T1 in registers; descriptor
		 * DMA T2, windows T0, descriptor DMA T3 (one op younger than
		 * T0's windows, as every later step has) */
		const uint4 d0 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(q0));
		const uint4 d1 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(q1));
		issue_desc(q2, dsl0);
		issue_win2(d0, true);
		issue_desc(q3, dsl1);
		uint4 c0 = d0, c1 = d1;
		for (;;) {
			const uint4 n0 = step2(q0, dsl0, c0, c1, q1, q4, q5);
			q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5;
			if (q0 >= ntiles)
				break;
			const uint4 n1 = step2(q0, dsl1, c1, n0, q1, q4, q5);
			q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5;
			if (q0 >= ntiles)
				break;
			c0 = n0;
			c1 = n1;
		}
		store_tile(a, pend);   /* the last tile's outputs */
	} else if (WIN == 64 && q0 < ntiles) {
		/* prologue: descriptors of the first two tiles in registers;
		 * then, in this order, descriptor DMA T2, window DMA T0,
		 * descriptor DMA T3, window DMA T1: at least 5 ops younger than
		 * both of step 0's and of step 1's inputs */
		const uint4 d0 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(q0));
		const uint4 d1 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(q1));
		issue_desc(q2, dsl0);
		issue_win(d0, true, win0);
		issue_desc(q3, dsl1);
		issue_win(d1, q1 < ntiles, win1);
		/* kTileStores ops younger than step 0's and step 1's windows
		 * (dropped: every lane out of range), as every later step has
		 * the previous step's stores */
		if constexpr (DIAG != 2)
			store_tile(a, pend);
		uint4 dc0 = d0, dc1 = d1;
		for (;;) {
			const uint4 n0 = step(q0, win0, dsl0, dc0, q2, q4, q5);
			q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5;
			if (q0 >= ntiles)
				break;
			const uint4 n1 = step(q0, win1, dsl1, dc1, q2, q4, q5);
			q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5;
			if (q0 >= ntiles)
				break;
			dc0 = n0;
			dc1 = n1;
		}
		if constexpr (DIAG != 1 && DIAG != 2)
			store_tile(a, pend);   /* the last tile's outputs */
	}
	/* Shared tiles: with its own tiles done, the wave claims the tiles of
	 * its block's head (block b: head b mod heads) two at a time from the
	 * head's global counter, each claim first reserving two of the
	 * block's steal_cap() slots (its list regions hold that many more
	 * tiles), until the head is empty.  CUs run their own tiles at
	 * rates up to 10 % apart (tools/stamps.py); the shared tiles go to
	 * whichever are done first. */
	if (shared) {
		const uint64_t heads = min((uint64_t)kStealHeads, nb);
		const uint32_t cap = (uint32_t)steal_cap(shared, nb);
		lds_dma_landed();   /* the loop's last DMAs into win0/dsl0 */
		/* a.partner heads in turn: with its own head empty, the wave goes
		 * on with head h ^ 4, whose blocks run on the XCD 4 away (the
		 * other half of the chip), until that is empty too (the default,
		 * 2); with 8, then h ^ 2, h ^ 6, h ^ 1, ... (every XCD's head of
		 * its set).  The first wave of the block to find a head empty
		 * tells the others (bit r of ctl[7]).  Within one process the
		 * two halves of the chip drain their heads 12 us apart, the
		 * same half last in every launch (which half changes with the
		 * buffers' placement; tools/stamps.py per_launch); the partner
		 * head evens them: config 2 0.2969 / 0.2989 vs 0.3007 / 0.3032
		 * ms without, in one process; every XCD's heads 0.3058 / 0.3079
		 * (the XCDs of one half drain together, and a move there only
		 * adds a late pair; not kept). */
		const int rounds = heads % 8 == 0 && a.partner > 1 ? 2 : 1;
		for (int round = 0; round < rounds; ++round) {
			if (round && (__builtin_amdgcn_readfirstlane(ctl[7]) >> round) & 1)
				continue;
			const uint64_t h = (rb % heads) ^ ((0x73516240u >> (4 * round)) & 7);
			uint32_t *ctr = a.steal + (a.steal_set * kStealHeads + h) * kStealStride;
			/* A claim v is head h's tiles 2v and 2v + 1, the j-th being
			 * own + j heads + h, so that a tile goes to the XCD (b mod 8)
			 * the own-tile order gives it; the launcher makes own a
			 * multiple of the heads.  (A tile's XCD matters: an order that
			 * moved the blocks through all positions of each round ran 11 %
			 * slower.)  claim() reserves two of the block's slots first and
			 * returns lane 0's claim (no claim over the cap). */
			auto claim2 = [&]() -> uint32_t {
				uint32_t v = 0x7fffffffu;
				if (lds_fetch_add(&ctl[6], 2, lane) + 2 <= cap && lane == 0)
					v = atomicAdd(ctr, 1u);
				return v;
			};
			auto first_of = [&](uint32_t v) -> uint64_t {
				const uint64_t t = own + (uint64_t)__builtin_amdgcn_readfirstlane(v) * 2 * heads + h;
				return t < ntiles ? t : ntiles;
			};
			auto second_of = [&](uint64_t t) -> uint64_t {
				const uint64_t u = t + heads;
				return u < ntiles ? u : ntiles;
			};
			uint64_t c0 = own + h < ntiles ? first_of(claim2()) : ntiles;
			if (round && c0 >= ntiles && lane == 0)
				atomicOr(&ctl[7], 1u << round);
			if (c0 < ntiles) {
				/* per pair: descriptors, windows and the next claim in
				 * flight, one wait, then the two tiles.  (Pipelined over
				 * pairs, each buffer refilled as soon as read: 0.3361 vs
				 * 0.3250 ms on config 2, one process.) */
				for (; WIN == 128;) {
					/* one tile's two halves at a time: the second
					 * tile's DMA issued as the first is read */
					const uint64_t c1 = second_of(c0);
					const uint4 d0 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(c0));
					const uint4 d1 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(c1));
					issue_win2(d0, true);
					const uint32_t vn = claim2();
					uint32_t F[18];
					WinHi wh;
					uint4 dn;
					lds_dma_landed();
					const uint64_t i0 = c0 * kWave + lane;
					read_tile_w2<0, V6>(a, win0, win1, dsl0, lane, F, wh, dn, d0,
							    i0 < nfr && dma);
					issue_win2(d1, c1 < ntiles);
					fast_tile<false, true, V6, 32, ECHO>(a, F, d0, i0, i0 < nfr, dma, lane, w,
								       &pend, &wh);
					store_tile(a, pend);
					if (c1 >= ntiles)
						break;
					lds_dma_landed();
					const uint64_t i1 = c1 * kWave + lane;
					read_tile_w2<0, V6>(a, win0, win1, dsl0, lane, F, wh, dn, d1,
							    i1 < nfr && dma);
					fast_tile<false, true, V6, 32, ECHO>(a, F, d1, i1, i1 < nfr, dma, lane, w,
								       &pend, &wh);
					store_tile(a, pend);
					c0 = first_of(vn);
					if (c0 >= ntiles)
						break;
				}
				for (; WIN == 64;) {
					const uint64_t c1 = second_of(c0);
					const uint4 d0 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(c0));
					const uint4 d1 = *reinterpret_cast<const uint4 *>(a.desc + desc_at(c1));
					issue_win(d0, true, win0);
					issue_win(d1, c1 < ntiles, win1);
					const uint32_t vn = claim2();
					uint32_t F[18];
					uint4 dn;
					lds_dma_landed();
					read_tile_db<10>(win0, dsl0, lane, F, dn);
					const uint64_t i0 = c0 * kWave + lane;
					fast_tile<false, true, V6>(a, F, d0, i0, i0 < nfr, dma, lane, w, &pend);
					store_tile(a, pend);
					if (c1 >= ntiles)
						break;
					read_tile_db<10>(win1, dsl1, lane, F, dn);
					const uint64_t i1 = c1 * kWave + lane;
					fast_tile<false, true, V6>(a, F, d1, i1, i1 < nfr, dma, lane, w, &pend);
					store_tile(a, pend);
					c0 = first_of(vn);
					if (c0 >= ntiles)
						break;
				}
			}
			lds_dma_landed();   /* a claim left outstanding at a break */
		}
	}
	STAMP(wgid, lane, 1);

	/* tail phase: the block's deferred frames, split over its waves, on
	 * the same LDS once every DMA has landed (rx_tail waits) */
	lds_dma_landed();
	__syncthreads();
	const uint32_t xc = ctl[1], bc = ctl[2];
	/* the bulk pass answers echo requests in a 64-byte window build and
	 * those the ECHO instance's tiles left to it */
	rx_tail<WIN, V6 && (WIN == 64 || ECHO)>(a, w, rb, xc, bc, wid, kCuWaves, ctl, lane, reinterpret_cast<uint32_t *>(wl),
		reinterpret_cast<uint64_t *>(wl + 272), wl, wl + kWave, w.cnt, w.my_bytes);

	/* counters: this wave's own slot (kMaxRxBlocks..: per-wave slots) */
	if (a.stats) {
		const uint64_t bytes = wave_sum64(w.my_bytes);
		unsigned long long *slot = a.stats + (kMaxRxBlocks + wgid) * CNT_SLOT;
		if (lane <= CNT_FRAG && !DBG_BAD(kMaxRxBlocks + wgid >= kStatSlots, 8, wgid)) {
			uint64_t v = 0;
#pragma unroll
			for (int k = 0; k <= CNT_FRAG; k++)
				if (lane == k)
					v = k == CNT_BYTES ? bytes : w.cnt[k];
			if (v)
				slot[lane] += v;
		}
	}
	STAMP(wgid, lane, 2);
}

/* Multi-buffer packets read in place (XDPGPU_CFG_FRAGS, after
 * frag_count): a lane per descriptor, the packets' first descriptors
 * through generic_batch<WIN, true>, grid-strided over the batch's tiles. */
template <int WIN>
__global__ __launch_bounds__(kBlock, 2) void xdp_rx_packet_kernel(RxArgs a)
{
	constexpr int SDW = WIN / 4 + 1;
	__shared__ uint32_t lds[kWavesPerBlock * kWave * SDW + 8];
	__shared__ uint64_t dtab_all[kWavesPerBlock * kWave];
	__shared__ unsigned long long blk_cnt[CNT_SLOT];

	const int lane = threadIdx.x & (kWave - 1);
	const int wid = threadIdx.x / kWave;
	uint32_t *win = lds + wid * kWave * SDW;
	uint64_t *dtab = dtab_all + wid * kWave;
	if (threadIdx.x < CNT_SLOT)
		blk_cnt[threadIdx.x] = 0;
	__syncthreads();

	const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
	const uint64_t ntiles = ((uint64_t)a.n + kWave - 1) / kWave;
	uint32_t cnt[CNT_FRAG + 1] = {};
	uint64_t my_bytes = 0;
	for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wid; t < ntiles; t += nwaves) {
		const uint64_t i = t * kWave + lane;
		generic_batch<WIN, true>(a, win, dtab, lane, i < a.n ? i : 0, i < a.n, nullptr,
					 nullptr, cnt, my_bytes);
	}

	block_stats_flush(a, blk_cnt, cnt, my_bytes, lane);
}

/* Memory ceiling for the RX traffic pattern (diagnostic): the same
 * descriptor, transposed 64-byte window loads and 33 bytes of stores per
 * frame, with no parse.  Its bandwidth is what the RX kernel can approach. */
__global__ __launch_bounds__(kBlock) void xdp_ceiling_kernel(RxArgs a)
{
	__shared__ uint64_t dtab_all[kWavesPerBlock * kWave];
	const int lane = threadIdx.x & (kWave - 1);
	const int wid = threadIdx.x / kWave;
	uint64_t *dtab = dtab_all + wid * kWave;
	const uint64_t ntiles = ((uint64_t)a.n + kWave - 1) / kWave;
	const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
	for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wid; t < ntiles;
	     t += nwaves) {
		const uint64_t i = t * kWave + lane;
		const uint4 dv = load_desc(a.desc, i, a.n);
		dtab[lane] = ((uint64_t)dv.y << 32) | dv.x;
		__builtin_amdgcn_wave_barrier();
		uint32_t x = dv.z;
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int q = k * kWave + lane;
			const uint64_t src = dtab[q >> 2] + 16ull * (q & 3);
			if (src + 16 <= a.usize) {
				uint4 v = *reinterpret_cast<const uint4 *>(a.umem + src);
				x ^= v.x ^ v.y ^ v.z ^ v.w;
			}
		}
		if (i < a.n) {
			a.verdict[i] = (uint8_t)x;
			*reinterpret_cast<uint4 *>(a.res + i) = make_uint4(x, x, x, x);
			*reinterpret_cast<uint4 *>(a.tup + 16 * i) = make_uint4(x, 0, x, 0);
		}
	}
}

hipError_t launch_ceiling(const RxArgs &a, uint32_t blocks, hipStream_t stream)
{
	hipLaunchKernelGGL(xdp_ceiling_kernel, dim3(blocks), dim3(kBlock), 0,
			   stream, a);
	return hipGetLastError();
}

uint32_t rx_grid_blocks(uint32_t n, uint32_t max_blocks)
{
	uint64_t tiles = ((uint64_t)n + kWave - 1) / kWave;
	uint64_t blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
	if (blocks > max_blocks)
		blocks = max_blocks;
	if (blocks > kMaxRxBlocks)
		blocks = kMaxRxBlocks;
	if (blocks == 0)
		blocks = 1;
	return (uint32_t)blocks;
}

/* Blocks of a kernel resident at once on the device (occupancy x CUs). */
template <auto KERN>
static uint32_t resident_blocks()
{
	return resident_blocks_dev<KERN, kBlock>(kMaxRxBlocks);
}

/* The default RX launch: one double-buffered fast kernel with its tail
 * phase (xdp_rx_db_kernel). */
static hipError_t launch_db(RxArgs a, uint32_t max_blocks, hipStream_t stream,
			    hipEvent_t *ev)
{
	uint32_t cap = a.frags ? resident_blocks_dev<xdp_rx_db_kernel<true>, kCuBlock>(kMaxRxBlocks)
			       : resident_blocks_dev<xdp_rx_db_kernel<false>, kCuBlock>(kMaxRxBlocks);
	const uint32_t diag = a.diag;
	if (cap < max_blocks)
		max_blocks = cap;
	/* one block per CU, fewer when the batch has fewer tiles than waves */
	const uint64_t ntiles = ((uint64_t)a.n + kWave - 1) / kWave;
	uint64_t blocks = (ntiles + kCuWaves - 1) / kCuWaves;
	if (blocks > max_blocks)
		blocks = max_blocks;
	if (blocks == 0)
		blocks = 1;
	/* list regions per block: its share of the tiles */
	auto share = [&](uint64_t own) -> uint64_t { return (own + blocks - 1) / blocks; };
	a.xregion = (uint32_t)(share(ntiles) * kWave);
	a.nregions = (uint32_t)blocks;
	/* shared tiles (xdp_rx_db_kernel): the last ntiles x steal_16ths / 16,
	 * for batches of at least 64 tiles per block; a block's region then
	 * holds its own tiles and up to steal_cap() shared ones */
	a.steal_tiles = 0;
	if (a.steal && a.steal_16ths && !a.frags && !diag &&
	    ntiles >= 64 * blocks) {
		/* own a multiple of twice the heads (xdp_rx_db_kernel's head
		 * orders) */
		const uint64_t own = (ntiles - ntiles * min(a.steal_16ths, 16u) / 16) &
				     ~(uint64_t)(2 * kStealHeads - 1);
		const uint64_t sh = ntiles - own;
		const uint64_t xr = (share(own) + steal_cap(sh, blocks)) * kWave;
		if (xr * blocks <= a.xcap && xr <= 0xffffffffull) {
			a.steal_tiles = (uint32_t)sh;
			a.xregion = (uint32_t)xr;
		}
	}
	/* 128-byte windows: the default kernel only */
	if (a.win != 128 || a.frags || diag)
		a.win = 64;
	if (ev)
		(void)hipEventRecord(ev[0], stream);
	const dim3 grid((uint32_t)blocks), blk(kCuBlock);
	if (a.frags)
		hipLaunchKernelGGL((xdp_rx_db_kernel<true>), grid, blk, 0, stream, a);
	else if (a.win == 128 && a.v6 && (a.flags & XDPGPU_CFG_ICMP6_ECHO))
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 0, true, 128, true>), grid, blk, 0, stream, a);
	else if (a.win == 128 && a.v6)
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 0, true, 128>), grid, blk, 0, stream, a);
	else if (a.win == 128)
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 0, false, 128>), grid, blk, 0, stream, a);
	else if (diag == 1)
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 1>), grid, blk, 0, stream, a);
	else if (diag == 2)
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 2>), grid, blk, 0, stream, a);
	else if (a.v6)
		hipLaunchKernelGGL((xdp_rx_db_kernel<false, 0, true>), grid, blk, 0, stream, a);
	else
		hipLaunchKernelGGL((xdp_rx_db_kernel<false>), grid, blk, 0, stream, a);
	const hipError_t e = hipGetLastError();
	/* one event after the kernel: every further record on the stream
	 * (round 1's three-kernel pairs) added its own few microseconds to
	 * the measured span */
	if (ev && e == hipSuccess)
		(void)hipEventRecord(ev[1], stream);
	return e;
}

uint32_t rx_xregion(uint32_t n, uint32_t blocks)
{
	const uint64_t ntiles = ((uint64_t)n + kWave - 1) / kWave;
	const uint64_t nwaves = (uint64_t)blocks * kWavesPerBlock;
	return (uint32_t)(((ntiles + nwaves - 1) / nwaves) * kWave);
}

hipError_t launch_rx_packets(const RxArgs &a, uint32_t max_blocks, hipStream_t stream)
{
	const uint64_t tiles = ((uint64_t)a.n + kWave - 1) / kWave;
	uint64_t blocks = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
	uint32_t cap = resident_blocks<xdp_rx_packet_kernel<64>>();
	cap = cap < max_blocks ? cap : max_blocks;
	blocks = blocks < cap ? blocks : cap;
	if (!blocks)
		return hipSuccess;
	hipLaunchKernelGGL(xdp_rx_packet_kernel<64>, dim3((uint32_t)blocks), dim3(kBlock), 0,
			   stream, a);
	return hipGetLastError();
}

hipError_t launch_rx(const RxArgs &a, uint32_t max_blocks, hipStream_t stream, uint32_t tune,
		     hipEvent_t *ev)
{
	RxArgs b = a;
	/* bits 16-17: diagnostic variants (no compute, no stores) */
	b.diag = (tune >> 16) & 3;
	/* IPv6 in the fast shape (IMIX's IPv6 frames) for the 44-byte
	 * network_tuple and no tuple, and with the echo responder (its
	 * requests are IPv6); bit 18 turns it off.  The 16-byte IPv4 tuple
	 * otherwise keeps the IPv4-only kernel (config 2), whose registers it
	 * would cost. */
	b.v6 = (a.tuple_fmt != XDPGPU_TUPLE_V4 || (a.flags & XDPGPU_CFG_ICMP6_ECHO)) &&
	       !((tune >> 18) & 1);
	/* bit 28: after its own head, a wave claims no shared tiles of the
	 * partner head (the default goes on with the head in the other half
	 * of the chip) */
	b.partner = (tune >> 28) & 1 ? 1 : 2;
	return launch_db(b, max_blocks, stream, ev);
}

/* ------------------------------------------------------------------ */
/* primitives                                                           */

/* jhash over arbitrary keys, one lane per key (jhash.h:68-105) */
__global__ __launch_bounds__(kBlock) void jhash_kernel(const uint8_t *keys,
						       uint32_t key_len,
						       uint32_t stride,
						       uint32_t n,
						       uint32_t initval,
						       uint32_t *out)
{
	const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
	if (i >= n)
		return;
	const uint8_t *k = keys + i * stride;
	uint32_t len = key_len;
	uint32_t a, b, c;
	a = b = c = 0xdeadbeefu + len + initval;
	while (len > 12) {
		uint32_t w[3];
		for (int j = 0; j < 3; j++)
			w[j] = (uint32_t)k[4 * j] | ((uint32_t)k[4 * j + 1] << 8) |
			       ((uint32_t)k[4 * j + 2] << 16) |
			       ((uint32_t)k[4 * j + 3] << 24);
		a += w[0];
		b += w[1];
		c += w[2];
		JH_MIX(a, b, c);
		len -= 12;
		k += 12;
	}
	if (len) {
		uint32_t t[3] = {0, 0, 0};
		for (uint32_t j = 0; j < len; j++)
			t[j >> 2] += (uint32_t)k[j] << (8 * (j & 3));
		a += t[0];
		b += t[1];
		c += t[2];
		JH_FINAL(a, b, c);
	}
	out[i] = c;
}

/* ip_fast_csum (lib_checksum.h:103-106) with any summation order */
__global__ __launch_bounds__(kBlock) void ip_fast_csum_kernel(
	const uint8_t *hdrs, uint32_t stride, uint32_t n, uint16_t *out)
{
	const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
	if (i >= n)
		return;
	const uint8_t *h = hdrs + i * stride;
	const uint32_t bytes = (h[0] & 0xf) * 4;
	uint64_t s = 0;
	for (uint32_t o = 0; o + 1 < bytes; o += 2)
		s += (uint32_t)h[o] | ((uint32_t)h[o + 1] << 8);
	out[i] = (uint16_t)(~fold16(s) & 0xffff);
}

#ifdef XDPGPU_STAMPS
} // namespace xdpgpu
extern "C" int xdpgpu_stamps_read(unsigned long long *out)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(xdpgpu::g_stamp), sizeof(xdpgpu::g_stamp)) !=
	    hipSuccess)
		return -5;
	return 0;
}
namespace xdpgpu {
#endif

#ifdef XDPGPU_DBG
} // namespace xdpgpu
extern "C" int xdpgpu_debug_read(unsigned long long *out)
{
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(xdpgpu::g_dbg), sizeof(xdpgpu::g_dbg)) !=
	    hipSuccess)
		return -5;
	static const unsigned long long z[64] = {};
	return hipMemcpyToSymbol(HIP_SYMBOL(xdpgpu::g_dbg), z, sizeof(z)) == hipSuccess ? 0 : -5;
}
namespace xdpgpu {
#endif

hipError_t launch_jhash(const uint8_t *keys, uint32_t key_len,
			uint32_t stride, uint32_t n, uint32_t initval,
			uint32_t *out, hipStream_t stream)
{
	const uint32_t blocks = (n + kBlock - 1) / kBlock;
	if (!blocks)
		return hipSuccess;
	hipLaunchKernelGGL(jhash_kernel, dim3(blocks), dim3(kBlock), 0, stream,
			   keys, key_len, stride, n, initval, out);
	return hipGetLastError();
}

/* jhash2 (include/jhash.h:114-142) over n keys of nwords u32 at stride
 * words (variant 0), or jhash_1word / 2words / 3words (jhash.h:145-170:
 * __jhash_nwords with initval + JHASH_INITVAL + 4 nwords; variant =
 * nwords, words past nwords zero). */
__global__ __launch_bounds__(kBlock) void jhash_words_kernel(const uint32_t *words,
							     uint32_t nwords,
							     uint32_t stride, uint32_t n,
							     uint32_t initval,
							     uint32_t variant,
							     uint32_t *out)
{
	const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
	if (i >= n)
		return;
	const uint32_t *k = words + i * stride;
	uint32_t a, b, c;
	if (variant) {
		const uint32_t iv = initval + 0xdeadbeefu + (variant << 2);
		a = k[0] + iv;
		b = (variant > 1 ? k[1] : 0u) + iv;
		c = (variant > 2 ? k[2] : 0u) + iv;
		JH_FINAL(a, b, c);
		out[i] = c;
		return;
	}
	uint32_t len = nwords;
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
	out[i] = c;
}

hipError_t launch_jhash_words(const uint32_t *words, uint32_t nwords, uint32_t stride,
			      uint32_t n, uint32_t initval, uint32_t variant,
			      uint32_t *out, hipStream_t stream)
{
	const uint32_t blocks = (n + kBlock - 1) / kBlock;
	if (!blocks)
		return hipSuccess;
	hipLaunchKernelGGL(jhash_words_kernel, dim3(blocks), dim3(kBlock), 0, stream,
			   words, nwords, stride, n, initval, variant, out);
	return hipGetLastError();
}

hipError_t launch_ip_fast_csum(const uint8_t *hdrs, uint32_t stride,
			       uint32_t n, uint16_t *out, hipStream_t stream)
{
	const uint32_t blocks = (n + kBlock - 1) / kBlock;
	if (!blocks)
		return hipSuccess;
	hipLaunchKernelGGL(ip_fast_csum_kernel, dim3(blocks), dim3(kBlock), 0,
			   stream, hdrs, stride, n, out);
	return hipGetLastError();
}

} // namespace xdpgpu
