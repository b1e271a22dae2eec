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

__device__ __forceinline__ uint32_t halves(uint32_t d)
{
	return (d & 0xffff) + (d >> 16);
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

/* ------------------------------------------------------------------ */
/* jhash (include/jhash.h:25-52), word form; jhash(key, 44) equals
 * jhash2(words, 11) on little-endian (jhash.h:68-142).                 */

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

template <int WIN>
struct FrameView {
	const uint32_t *w;  /* this lane's LDS row (dword aligned)   */
	const uint8_t *g;   /* umem + eff                             */
	uint64_t gleft;     /* umem bytes from eff to the end         */

	__device__ __forceinline__ uint32_t b8(uint32_t off) const
	{
		if (off < (uint32_t)WIN)
			return (w[off >> 2] >> ((off & 3) * 8)) & 0xff;
		return off < gleft ? g[off] : 0;
	}
	/* network-order 16-bit field */
	__device__ __forceinline__ uint32_t be16(uint32_t off) const
	{
		if (off + 1 < (uint32_t)WIN && !(off & 1)) {
			uint32_t d = w[off >> 2];
			uint32_t h = (off & 2) ? (d >> 16) : (d & 0xffff);
			return bswap16(h);
		}
		return (b8(off) << 8) | b8(off + 1);
	}
	/* 16 bits as a little-endian load of the wire bytes */
	__device__ __forceinline__ uint32_t le16(uint32_t off) const
	{
		return bswap16(be16(off));
	}
	__device__ __forceinline__ uint32_t le32(uint32_t off) const
	{
		return le16(off) | (le16(off + 2) << 16);
	}
	/* Sum of LE u16 words (frame-relative parity) of the bytes in
	 * [lo, hi) with [x, x+2) treated as zero, window part only. */
	__device__ __forceinline__ uint32_t win_sum(uint32_t lo, uint32_t hi,
						    uint32_t x) const
	{
		uint32_t h = hi < (uint32_t)WIN ? hi : (uint32_t)WIN;
		uint32_t s = 0;
		for (uint32_t o = lo & ~3u; o < h; o += 4) {
			uint32_t d = w[o >> 2];
			d &= keep_mask(o, lo, h) & ~keep_mask(o, x, x + 2);
			s += halves(d);
		}
		return s;
	}
	/* Same, bytes past the window, one lane on its own (rare: deep
	 * headers only). */
	__device__ uint32_t glob_sum(uint32_t lo, uint32_t hi, uint32_t x) const
	{
		uint32_t s = 0;
		for (uint32_t o = lo > (uint32_t)WIN ? lo : (uint32_t)WIN; o < hi;
		     o++) {
			uint32_t v = o < gleft ? g[o] : 0;
			if (o - x < 2)
				v = 0;
			s += (o & 1) ? (v << 8) : v;
		}
		return s;
	}
};

/* ------------------------------------------------------------------ */
/* per-lane parse state                                                 */

enum : uint32_t { ST_ABORT = 0, ST_PASS = 2, ST_GO = 0xff };

struct Lane {
	uint32_t st;
	uint32_t l3, l4, nvlan, vid;
	uint32_t ipv4, ipv6, nh;
	uint32_t frag, has_l4, has_csum;
	uint32_t cl, chk;       /* L4 checksum length, check offset      */
	uint32_t rhi;           /* end of the summed L4 range (+over-read) */
	uint32_t s3, c3;        /* IPv4 header sum (check zeroed), stored */
	uint32_t s4, c4;        /* L4 sum window part (check zeroed)      */
	uint32_t sa[4], da[4];
	uint32_t sp, dp;
};

/* The pipeline of oracle/xdp_oracle.c frame_pipeline(), up to the sums. */
template <int WIN>
__device__ __forceinline__ void parse_lane(const FrameView<WIN> &F,
					   uint32_t end, Lane &L)
{
	L.st = ST_ABORT;
	L.l3 = L.l4 = L.nvlan = L.vid = 0;
	L.ipv4 = L.ipv6 = L.nh = 0;
	L.frag = L.has_l4 = L.has_csum = 0;
	L.cl = L.chk = L.rhi = 0;
	L.s3 = L.c3 = L.s4 = L.c4 = 0;
	L.sp = L.dp = 0;
#pragma unroll
	for (int j = 0; j < 4; j++)
		L.sa[j] = L.da[j] = 0;

	/* parse_ethhdr_vlan, parsing_helpers.h:86-129, VLAN_MAX_DEPTH 2 */
	if (end < 14)
		return;
	uint32_t proto = F.be16(12);
	uint32_t c = 14;
#pragma unroll
	for (int i = 0; i < 2; i++) {
		if (proto != 0x8100 && proto != 0x88A8)
			break;
		if (c + 4 > end)
			break;
		if (i == 0)
			L.vid = F.be16(c) & 0x0fff;
		proto = F.be16(c + 2);
		c += 4;
		L.nvlan++;
	}
	L.l3 = c;
	const uint32_t l3 = c;

	/* af_xdp_kern.c:114-148 parse_pkt__is_ARP_or_NDP */
	if (proto == 0x0806) {
		L.st = ST_PASS;
		return;
	}
	L.ipv4 = (proto == 0x0800);
	L.ipv6 = (proto == 0x86DD);
	uint32_t ip_end = 0, nonfirst = 0;
	int frag_at = -1;

	if (L.ipv6) {
		/* parse_ip6hdr :174-194 + skip_ip6hdrext :139-172 */
		if (l3 + 40 > end)
			return;
		if ((F.b8(l3) >> 4) != 6)
			return;
		uint32_t cur = l3 + 40;
		uint32_t nh = F.b8(l3 + 6);
		bool found = false;
		for (int i = 0; i < 6; i++) {
			if (cur + 2 > end)
				return;
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
			return;
		L.nh = nh;
		L.l4 = cur;
		if (nh == 58) {
			/* parse_icmp6hdr :224-237; NDP 133..137 -> PASS */
			if (cur + 8 > end)
				return;
			uint32_t t = F.b8(cur);
			if (t >= 133 && t <= 137) {
				L.st = ST_PASS;
				return;
			}
		}
		ip_end = l3 + 40 + F.be16(l3 + 4);
		if (ip_end > end || cur > ip_end)
			return;
		if (frag_at >= 0) {
			L.frag = 1;
			if (F.be16((uint32_t)frag_at + 2) >> 3)
				nonfirst = 1;
		}
#pragma unroll
		for (int j = 0; j < 4; j++) {
			L.sa[j] = F.le32(l3 + 8 + 4 * j);
			L.da[j] = F.le32(l3 + 24 + 4 * j);
		}
	} else if (L.ipv4) {
		/* parse_iphdr :196-222 */
		if (l3 + 20 > end)
			return;
		uint32_t vihl = F.b8(l3);
		if ((vihl >> 4) != 4)
			return;
		uint32_t hl = (vihl & 0xf) * 4;
		if (hl < 20)
			return;
		if (l3 + hl > end)
			return;
		L.nh = F.b8(l3 + 9);
		uint32_t tot = F.be16(l3 + 2);
		if (tot < hl || l3 + tot > end)
			return;
		ip_end = l3 + tot;
		L.l4 = l3 + hl;
		uint32_t fo = F.be16(l3 + 6) & 0x3fff;
		if (fo) {
			L.frag = 1;
			if (fo & 0x1fff)
				nonfirst = 1;
		}
		/* header sum with the check word zeroed (af_xdp_user.c:664) */
		L.c3 = F.le16(l3 + 10);
		L.s3 = F.win_sum(l3, l3 + hl, l3 + 10);
		if (l3 + hl > (uint32_t)WIN)
			L.s3 += F.glob_sum(l3, l3 + hl, l3 + 10);
		L.sa[0] = F.le32(l3 + 12);
		L.da[0] = F.le32(l3 + 16);
	}

	if ((L.ipv4 || L.ipv6) && !nonfirst) {
		const uint32_t l4 = L.l4;
		const uint32_t nh = L.nh;
		if (nh == 17) {
			/* parse_udphdr :272-290 */
			if (l4 + 8 > end)
				return;
			uint32_t ulen = F.be16(l4 + 4);
			if (ulen < 8)
				return;
			L.has_l4 = 1;
			if (!L.frag) {
				if (l4 + ulen > ip_end)
					return;
				L.cl = ulen;
				L.chk = l4 + 6;
				L.has_csum = 1;
			}
		} else if (nh == 6) {
			/* parse_tcphdr :295-318 */
			if (l4 + 20 > end)
				return;
			uint32_t thl = (F.b8(l4 + 12) >> 4) * 4;
			if (thl < 20 || l4 + thl > end)
				return;
			L.has_l4 = 1;
			if (!L.frag) {
				uint32_t cl = ip_end - l4;
				if (cl < thl)
					return;
				L.cl = cl;
				L.chk = l4 + 16;
				L.has_csum = 1;
			}
		} else if ((nh == 1 && L.ipv4) || (nh == 58 && L.ipv6)) {
			/* parse_icmphdr / parse_icmp6hdr :224-252 */
			if (l4 + 8 > end)
				return;
			L.has_l4 = 1;
			if (!L.frag) {
				uint32_t cl = ip_end - l4;
				if (cl < 8)
					return;
				L.cl = cl;
				L.chk = l4 + 2;
				L.has_csum = 1;
			}
		}
		if (L.has_l4 && (nh == 6 || nh == 17)) {
			L.sp = F.le16(l4);
			L.dp = F.le16(l4 + 2);
		}
	}

	if (L.has_csum) {
		/* udp_csum over-reads one byte for an odd length
		 * (lib_checksum.h:175-176); csum_partial zero-pads (ICMP, v6) */
		uint32_t over = (L.ipv4 && L.nh != 1) ? (L.cl & 1) : 0;
		L.rhi = L.l4 + L.cl + over;
		L.c4 = F.le16(L.chk);
		L.s4 = F.win_sum(L.l4, L.rhi, L.chk);
	}
	L.st = ST_GO;
}

/* ------------------------------------------------------------------ */
/* wave helpers                                                         */

__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src)
{
	return (uint32_t)__shfl((int)v, src, kWave);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src)
{
	uint32_t lo = shfl32((uint32_t)v, src);
	uint32_t hi = shfl32((uint32_t)(v >> 32), src);
	return ((uint64_t)hi << 32) | lo;
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

/* ------------------------------------------------------------------ */
/* the RX kernel                                                        */

template <int WIN>
__global__ __launch_bounds__(kBlock) void xdp_rx_kernel(RxArgs a)
{
	constexpr int CPF = WIN / 16;      /* 16-B chunks per frame window */
	constexpr int SDW = WIN / 4 + 1;   /* LDS row stride in dwords      */
	__shared__ uint32_t lds[kWavesPerBlock * kWave * SDW];
	__shared__ unsigned long long blk_cnt[CNT_SLOT];

	const int lane = threadIdx.x & (kWave - 1);
	const int wid = threadIdx.x / kWave;
	uint32_t *win = lds + wid * kWave * SDW;
	const uint32_t *row = win + lane * SDW;

	if (threadIdx.x < CNT_SLOT)
		blk_cnt[threadIdx.x] = 0;
	__syncthreads();

	const uint64_t ntiles = ((uint64_t)a.n + kWave - 1) / kWave;
	const uint64_t nwaves = (uint64_t)gridDim.x * kWavesPerBlock;
	uint64_t cnt_frames = 0, cnt_v[5] = {0, 0, 0, 0, 0};
	uint64_t cnt_l3 = 0, cnt_l4 = 0, cnt_abs = 0, cnt_frag = 0;
	uint64_t my_bytes = 0;

	for (uint64_t t = (uint64_t)blockIdx.x * kWavesPerBlock + wid;
	     t < ntiles; t += nwaves) {
		const uint64_t i = t * kWave + lane;
		const bool active = i < a.n;

		/* 1. descriptor */
		uint64_t addr = 0;
		uint32_t len = 0;
		if (active) {
			uint4 dv = *reinterpret_cast<const uint4 *>(a.desc + i);
			addr = ((uint64_t)dv.y << 32) | dv.x;
			len = dv.z;
		}
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool valid = active && (uint64_t)len <= a.usize &&
				   eff <= a.usize - len;

		/* 2. stage the header window into LDS */
		const uint64_t misaligned = __ballot(valid && (eff & 15));
		if (misaligned == 0) {
#pragma unroll
			for (int k = 0; k < CPF; k++) {
				const int q = k * kWave + lane;
				const int f = q / CPF;
				const int ch = q % CPF;
				const uint64_t feff = shfl64(eff, f);
				const uint32_t flen = shfl32(len, f);
				const uint32_t fval = shfl32(valid ? 1u : 0u, f);
				const uint64_t src = feff + 16ull * ch;
				uint4 v = make_uint4(0, 0, 0, 0);
				if (fval && 16u * ch <= flen && src < a.usize) {
					v = *reinterpret_cast<const uint4 *>(a.umem + src);
					if (src + 16 > a.usize) {
						v.x &= keep_mask(src, src, a.usize);
						v.y &= keep_mask(src + 4, src, a.usize);
						v.z &= keep_mask(src + 8, src, a.usize);
						v.w &= keep_mask(src + 12, src, a.usize);
					}
				}
				uint32_t *dst = win + f * SDW + ch * 4;
				dst[0] = v.x;
				dst[1] = v.y;
				dst[2] = v.z;
				dst[3] = v.w;
			}
		} else {
			/* unaligned-chunk UMEM: per-lane byte staging */
			for (int d = 0; d < WIN / 4; d++) {
				uint32_t wv = 0;
#pragma unroll
				for (int b = 0; b < 4; b++) {
					const uint32_t off = 4 * d + b;
					if (valid && off <= len && eff + off < a.usize)
						wv |= (uint32_t)a.umem[eff + off] << (8 * b);
				}
				win[lane * SDW + d] = wv;
			}
		}
		__builtin_amdgcn_wave_barrier();

		/* 3. per-lane parse */
		FrameView<WIN> F;
		F.w = row;
		F.g = a.umem + eff;
		F.gleft = a.usize - (valid ? eff : a.usize);
		Lane L;
		parse_lane<WIN>(F, valid ? len : 0u, L);   /* end 0 -> ABORTED */

		/* 4. cooperative sum of L4 bytes past the window */
		const bool need_ext = L.st == ST_GO && L.has_csum &&
				      L.rhi > (uint32_t)WIN;
		uint64_t ext_mask = __ballot(need_ext);
		uint32_t ext_sum = 0;
		while (ext_mask) {
			const int src = __builtin_ctzll(ext_mask);
			ext_mask &= ext_mask - 1;
			const uint64_t seff = shfl64(eff, src);
			const uint32_t sl4 = shfl32(L.l4, src);
			const uint32_t srhi = shfl32(L.rhi, src);
			const uint32_t schk = shfl32(L.chk, src);
			const uint64_t lo = seff + (sl4 > (uint32_t)WIN ? sl4 : (uint32_t)WIN);
			const uint64_t hi = seff + srhi;
			const uint64_t x = seff + schk;
			const uint64_t lim = hi < a.usize ? hi : a.usize;
			uint32_t acc = 0;
			for (uint64_t p = (lo & ~15ull) + 16ull * lane; p < lim;
			     p += 16ull * kWave) {
				uint4 v = *reinterpret_cast<const uint4 *>(a.umem + p);
				v.x &= keep_mask(p, lo, lim) & ~keep_mask(p, x, x + 2);
				v.y &= keep_mask(p + 4, lo, lim) & ~keep_mask(p + 4, x, x + 2);
				v.z &= keep_mask(p + 8, lo, lim) & ~keep_mask(p + 8, x, x + 2);
				v.w &= keep_mask(p + 12, lo, lim) & ~keep_mask(p + 12, x, x + 2);
				acc += halves(v.x) + halves(v.y) + halves(v.z) + halves(v.w);
			}
			acc = wave_sum32(fold16(acc));
			uint32_t s = fold16(acc);
			if (seff & 1)        /* absolute vs frame-relative parity */
				s = bswap16(s);
			if (lane == src)
				ext_sum = s;
		}

		/* 5. checksums, flow key, verdict */
		uint32_t verdict = L.st == ST_PASS ? XDPGPU_PASS : XDPGPU_ABORTED;
		uint4 rec = make_uint4(0, 0, 0, 0);
		uint32_t key[11];
#pragma unroll
		for (int j = 0; j < 11; j++)
			key[j] = 0;
		uint32_t l3_bad = 0, l4_bad = 0, absent = 0;
		if (L.st == ST_GO) {
			const bool ip = L.ipv4 || L.ipv6;
			uint32_t flags = 0, l3c = 0, l4c = 0, l3_ok = 1, l4_ok = 0;
			if (L.ipv4) {
				/* ip_fast_csum, lib_checksum.h:103-106 */
				l3c = ~fold16(L.s3) & 0xffff;
				l3_ok = fold16((uint64_t)L.s3 + L.c3) == 0xffff;
			}
			if (L.has_csum) {
				const uint64_t body = (uint64_t)L.s4 + ext_sum;
				if (L.ipv4 && L.nh != 1) {
					/* udp_csum -> csum_tcpudp_magic,
					 * lib_checksum.h:142-179 */
					const uint64_t ph = (uint64_t)L.sa[0] + L.da[0] +
						((uint64_t)(L.nh + L.cl) << 8);
					l4c = ~fold16(body + ph) & 0xffff;
					l4_ok = (~fold16(body + L.c4 + ph) & 0xffff) == 0;
					if (L.nh == 17 && L.c4 == 0) {
						absent = 1;
						l4_ok = 1;
					}
				} else if (L.ipv4) {
					/* ICMP: ~do_csum(msg) */
					l4c = ~fold16(body) & 0xffff;
					l4_ok = (~fold16(body + L.c4) & 0xffff) == 0;
				} else {
					/* csum_ipv6_magic, xdp_synproxy_kern.c:149-172 */
					uint64_t ph = (uint64_t)__builtin_bswap32(L.cl) +
						      __builtin_bswap32(L.nh);
#pragma unroll
					for (int j = 0; j < 4; j++)
						ph += (uint64_t)L.sa[j] + L.da[j];
					l4c = ~fold16(body + ph) & 0xffff;
					l4_ok = (~fold16(body + L.c4 + ph) & 0xffff) == 0;
				}
			}
			if (L.nvlan)
				flags |= XDPGPU_F_VLAN;
			if (ip) {
				flags |= XDPGPU_F_IP;
				if (L.ipv6)
					flags |= XDPGPU_F_IPV6;
				if (l3_ok)
					flags |= XDPGPU_F_L3_OK;
				if (L.frag)
					flags |= XDPGPU_F_FRAG;
				if (L.has_l4)
					flags |= XDPGPU_F_L4;
				if (L.has_csum && l4_ok)
					flags |= XDPGPU_F_L4_OK;
				if (absent)
					flags |= XDPGPU_F_L4_ABSENT;
				/* flow key: pping.h:120-139, v4 mapped as in
				 * pping_kern.c:212-217 */
				if (L.ipv4) {
					key[2] = 0xffff0000u;
					key[3] = L.sa[0];
					key[7] = 0xffff0000u;
					key[8] = L.da[0];
				} else {
					key[0] = L.sa[0]; key[1] = L.sa[1];
					key[2] = L.sa[2]; key[3] = L.sa[3];
					key[5] = L.da[0]; key[6] = L.da[1];
					key[7] = L.da[2]; key[8] = L.da[3];
				}
				key[4] = L.sp;
				key[9] = L.dp;
				key[10] = L.nh | ((L.ipv4 ? 2u : 10u) << 16);
			}
			const uint32_t hash = jhash_key44(key, a.initval);
			l3_bad = L.ipv4 && !l3_ok;
			l4_bad = L.has_csum && !l4_ok;
			rec.x = hash;
			rec.y = l3c | (l4c << 16);
			rec.z = flags | ((ip ? L.nh : 0u) << 8) | (L.l3 << 16) |
				(L.nvlan << 24);
			rec.w = ip ? (L.l4 | ((L.has_csum ? L.cl : 0u) << 16)) : 0u;

			verdict = XDPGPU_REDIRECT;
			if ((a.flags & XDPGPU_CFG_VERIFY_CSUM) && (l3_bad || l4_bad)) {
				verdict = XDPGPU_DROP;
			} else if ((a.flags & XDPGPU_CFG_ICMP6_ECHO) &&
				   L.nvlan == 0 && L.ipv6 && len >= 62 &&
				   F.b8(20) == 58 && F.b8(54) == 128) {
				/* af_xdp_user.c:968-1040 echo responder */
				uint8_t *g = a.umem + eff;
				for (int j = 0; j < 6; j++) {
					uint8_t t0 = (uint8_t)F.b8(j);
					g[j] = (uint8_t)F.b8(6 + j);
					g[6 + j] = t0;
				}
				for (int j = 0; j < 16; j++) {
					uint8_t t0 = (uint8_t)F.b8(22 + j);
					g[22 + j] = (uint8_t)F.b8(38 + j);
					g[38 + j] = t0;
				}
				g[54] = 129;
				uint32_t ck = csum_replace2(F.le16(56), 0x0080, 0x0081);
				g[56] = (uint8_t)ck;
				g[57] = (uint8_t)(ck >> 8);
				verdict = XDPGPU_TX;
			}
		}
		const bool rec_live = verdict != XDPGPU_ABORTED && verdict != XDPGPU_PASS;

		/* 6. outputs */
		if (active) {
			a.verdict[i] = (uint8_t)verdict;
			if (a.res)
				*reinterpret_cast<uint4 *>(a.res + i) = rec;
			if (a.tup) {
				if (a.tuple_fmt == XDPGPU_TUPLE_V4) {
					uint4 tv = make_uint4(0, 0, 0, 0);
					if (rec_live) {
						tv.x = L.ipv4 ? L.sa[0] : 0u;
						tv.y = L.ipv4 ? L.da[0] : 0u;
						tv.z = L.sp | (L.dp << 16);
						tv.w = ((L.ipv4 || L.ipv6) ? L.nh : 0u) |
						       (((L.ipv4 || L.ipv6) ? (L.ipv4 ? 2u : 10u) : 0u) << 8) |
						       (L.vid << 16);
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

		/* 7. counters (scalar: ballot + popcount) */
		cnt_frames += __popcll(__ballot(active));
#pragma unroll
		for (int v = 0; v < 5; v++)
			cnt_v[v] += __popcll(__ballot(active && verdict == (uint32_t)v));
		cnt_l3 += __popcll(__ballot(rec_live && l3_bad));
		cnt_l4 += __popcll(__ballot(rec_live && l4_bad));
		cnt_abs += __popcll(__ballot(rec_live && absent));
		cnt_frag += __popcll(__ballot(rec_live && L.frag));
		my_bytes += active ? len : 0;
	}

	if (a.stats) {
		const uint64_t bytes = wave_sum64(my_bytes);
		if (lane == 0) {
			atomicAdd(&blk_cnt[CNT_FRAMES], (unsigned long long)cnt_frames);
			atomicAdd(&blk_cnt[CNT_BYTES], (unsigned long long)bytes);
#pragma unroll
			for (int v = 0; v < 5; v++)
				atomicAdd(&blk_cnt[CNT_VERDICT0 + v],
					  (unsigned long long)cnt_v[v]);
			atomicAdd(&blk_cnt[CNT_L3_BAD], (unsigned long long)cnt_l3);
			atomicAdd(&blk_cnt[CNT_L4_BAD], (unsigned long long)cnt_l4);
			atomicAdd(&blk_cnt[CNT_L4_ABSENT], (unsigned long long)cnt_abs);
			atomicAdd(&blk_cnt[CNT_FRAG], (unsigned long long)cnt_frag);
		}
		__syncthreads();
		if (threadIdx.x < CNT_SLOT)
			a.stats[(uint64_t)blockIdx.x * CNT_SLOT + threadIdx.x] +=
				blk_cnt[threadIdx.x];
	}
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

hipError_t launch_rx(const RxArgs &a, uint32_t window, uint32_t blocks,
		     hipStream_t stream)
{
	if (window == 128)
		hipLaunchKernelGGL(xdp_rx_kernel<128>, dim3(blocks), dim3(kBlock),
				   0, stream, a);
	else
		hipLaunchKernelGGL(xdp_rx_kernel<64>, dim3(blocks), dim3(kBlock),
				   0, stream, a);
	return hipGetLastError();
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
