// SPDX-License-Identifier: GPL-2.0
/*
 * nat64.hip - the nat64-bpf translator (nat64-bpf/nat64_kern.c) as a batch
 * transform over UMEM frames on gfx950, BASELINE config 4.
 *
 * One lane per frame, 64 frames per wave-tile.  Frame bytes [-32, 96) (the
 * 32 bytes in front hold an IPv4 -> IPv6 frame's grown header) are staged
 * into a per-lane LDS row with transposed 16-byte loads (consecutive lanes
 * read consecutive chunks of one frame), falling back to byte loads for
 * frames that are not 16-byte aligned or sit at the UMEM edges.  The lane
 * then follows nat64_handler (nat64_kern.c:875-890) on its row: parse,
 * prefix and state checks, the new IP header, the ICMP rewrite and the
 * incremental checksum updates, writing the translated header bytes back
 * into the row.  Finally the rewritten span goes to HBM as dword stores
 * (byte stores only where the frame is not 4-byte aligned or the span's
 * edge is not).  Headers past the staged window (long IPv6 extension
 * chains) are read from HBM.
 *
 * The static v6_state_map / v4_reversemap are hash tables in HBM of
 * 4-way, 128-byte buckets (one line per lookup), built by the host
 * (xdpgpu.cpp, xdpgpu_internal.h).
 *
 * Checksum arithmetic: bpf_csum_diff and bpf_l4_csum_replace restated mod
 * 0xffff (see oracle/nat64_oracle.c for the derivation): each update is
 * c' = ~F((~c + delta) mod 0xffff), F(0) = 0xffff.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xdpgpu_internal.h"

namespace xdpgpu {

namespace {

constexpr int kWaveN = 64;
constexpr int kWavesN = 4;
constexpr int kBlockN = kWaveN * kWavesN;
constexpr int kRowDw = 33;        /* 128 B row + 4 B pad (bank spread) */
constexpr int kFront = 32;        /* row byte 0 = frame byte -32 */
constexpr int kWinEnd = 96;       /* staged frame bytes [-32, 96) */

__device__ __forceinline__ uint32_t slot_hash(uint32_t a, uint32_t b, uint32_t c,
					      uint32_t d)
{
	uint32_t h = a * 0x9E3779B1u ^ b * 0x85EBCA77u ^ c * 0xC2B2AE3Du ^
		     d * 0x27D4EB2Fu;
	h ^= h >> 15;
	h *= 0x2C1B3C6Du;
	h ^= h >> 13;
	return h;
}

/* x mod 0xffff for x < 2^32 */
__device__ __forceinline__ uint32_t mod_ffff(uint32_t x)
{
	x = (x & 0xffff) + (x >> 16);
	x = (x & 0xffff) + (x >> 16);
	return x == 0xffff ? 0 : x;
}

/* one bpf_l4_csum_replace on checksum c (LE u16 as stored) */
__device__ __forceinline__ uint32_t csum_upd(uint32_t c, uint32_t delta)
{
	const uint32_t v = mod_ffff(mod_ffff(~c & 0xffff) + delta);
	const uint32_t f = v ? v : 0xffff;
	return ~f & 0xffff;
}

struct Row {
	uint8_t *rb;          /* LDS row: rb[kFront + o] = frame byte o */
	const uint8_t *g;     /* frame in HBM, for bytes past the window */

	__device__ __forceinline__ uint32_t b(int o) const
	{
		return o < kWinEnd ? rb[kFront + o] : g[o];
	}
	__device__ __forceinline__ uint32_t be16(int o) const
	{
		return (b(o) << 8) | b(o + 1);
	}
	__device__ __forceinline__ uint32_t be32(int o) const
	{
		return (be16(o) << 16) | be16(o + 2);
	}
	__device__ __forceinline__ uint32_t le16(int o) const
	{
		return b(o) | (b(o + 1) << 8);
	}
	__device__ __forceinline__ void put(int o, uint32_t v) const
	{
		rb[kFront + o] = (uint8_t)v;
	}
	/* sum mod 0xffff of the LE 16-bit words of [o, o+n), n even */
	__device__ __forceinline__ uint32_t words(int o, int n) const
	{
		uint32_t s = 0;
		for (int k = 0; k < n; k += 2)
			s += le16(o + k);
		return mod_ffff(s);
	}
};

/* N header bytes built byte by byte, kept as N / 4 words in registers
 * (byte k at bits 8 (k & 3) of word k >> 2): every index is a constant once
 * the loops are unrolled, but for the RFC 6052 positions of the IPv4
 * address, which the prefix length picks at run time (set_dyn: a select
 * per possible position).  A byte array would live in scratch. */
template <int N>
struct Bytes {
	uint32_t w[N / 4];

	__device__ __forceinline__ uint32_t operator[](int k) const
	{
		return (w[k >> 2] >> (8 * (k & 3))) & 0xff;
	}
	__device__ __forceinline__ void set(int k, uint32_t v)
	{
		const int sh = 8 * (k & 3);
		w[k >> 2] = (w[k >> 2] & ~(0xffu << sh)) | ((v & 0xff) << sh);
	}
	__device__ __forceinline__ void zero()
	{
#pragma unroll
		for (int j = 0; j < N / 4; j++)
			w[j] = 0;
	}
	/* byte k, LO <= k < HI, k not known at compile time */
	template <int LO, int HI>
	__device__ __forceinline__ void set_dyn(int k, uint32_t v)
	{
#pragma unroll
		for (int j = LO; j < HI; j++)
			if (k == j)
				set(j, v);
	}
};

/* bpf_csum_diff(from, .., to, ..) mod 0xffff from the two word sums */
__device__ __forceinline__ uint32_t diff_mod(uint32_t from, uint32_t to)
{
	return mod_ffff(to + 0xffff - from);
}

/* bpf_l4_csum_replace at frame offset co of the row */
__device__ __forceinline__ void row_csum(const Row &R, int co, uint32_t delta,
					 bool mangled0)
{
	uint32_t c = R.le16(co);
	if (mangled0 && c == 0)
		return;
	c = csum_upd(c, delta);
	if (mangled0 && c == 0)
		c = 0xffff;
	R.put(co, c & 0xff);
	R.put(co + 1, c >> 8);
}

/* sum of the (LE words of the) pseudo header of update_icmp_checksum
 * (nat64_kern.c:120-158) from an IPv6 header at v6 bytes */
__device__ __forceinline__ uint32_t icmp_ph_sum(const Bytes<40> &v6)
{
	uint32_t s = 0;
	for (int k = 8; k < 40; k += 2)
		s += v6[k] | (v6[k + 1] << 8);
	s += v6[4] | (v6[5] << 8);        /* .len = payload_len (a __be16) */
	s += 58u << 8;                    /* .nh, last byte */
	return mod_ffff(s);
}

/* update_icmp_checksum: icmp header at frame offset h of the row (already
 * rewritten), old[8] the original */
__device__ __forceinline__ void icmp_csum(const Row &R, int h, const uint8_t *old,
					  const Bytes<40> &v6, bool add)
{
	const uint32_t ph = icmp_ph_sum(v6);
	const int co = h + 2;
	row_csum(R, co, add ? ph : diff_mod(ph, 0), false);
	const uint32_t hb = old[0] | (old[1] << 8), ha = R.le16(h);
	row_csum(R, co, diff_mod(hb, ha), false);
	const uint32_t ub = mod_ffff((old[4] | (old[5] << 8)) + (old[6] | (old[7] << 8)));
	const uint32_t ua = mod_ffff(R.le16(h + 4) + R.le16(h + 6));
	bool same = true;
	for (int k = 4; k < 8; k++)
		same = same && old[k] == R.b(h + k);
	if (!same)
		row_csum(R, co, diff_mod(ub, ua), false);
}

__device__ __forceinline__ void put_be32r(const Row &R, int o, uint32_t v)
{
	R.put(o, v >> 24);
	R.put(o + 1, v >> 16);
	R.put(o + 2, v >> 8);
	R.put(o + 3, v);
}

/* rewrite_icmpv6 (nat64_kern.c:644-739) at frame offset h */
__device__ bool rewrite_icmpv6(const Row &R, int h, const Bytes<40> &v6)
{
	uint8_t old[8];
	for (int k = 0; k < 8; k++)
		old[k] = (uint8_t)R.b(h + k);
	uint32_t t = old[0], c = old[1], nt = t, nc = c;
	switch (t) {
	case 128: nt = 8; break;
	case 129: nt = 0; break;
	case 1:
		nt = 3;
		if (c == 0 || c == 2 || c == 3) nc = 1;
		else if (c == 1) nc = 10;
		else if (c == 4) nc = 3;
		else return false;
		break;
	case 2: {
		nt = 3;
		nc = 4;
		const uint32_t mtu = ((uint32_t)old[4] << 24 | (uint32_t)old[5] << 16 |
				      (uint32_t)old[6] << 8 | old[7]) - 20;
		if (mtu > 0xffff)
			return false;
		R.put(h + 6, mtu >> 8);
		R.put(h + 7, mtu);
		break;
	}
	case 3: nt = 11; break;
	case 4:
		if (c == 0) {
			nt = 12;
			nc = 0;
			const uint32_t ptr = (uint32_t)old[4] << 24 | (uint32_t)old[5] << 16 |
					     (uint32_t)old[6] << 8 | old[7];
			uint32_t r;
			if (ptr == 0 || ptr == 1) r = ptr;
			else if (ptr == 4 || ptr == 5) r = 2;
			else if (ptr == 6) r = 9;
			else if (ptr == 7) r = 8;
			else if (ptr >= 8 && ptr <= 23) r = 12;
			else if (ptr >= 24 && ptr <= 39) r = 16;
			else return false;
			R.put(h + 4, r);
		} else if (c == 1) {
			nt = 3;
			nc = 2;
		} else {
			return false;
		}
		break;
	default:
		return false;
	}
	R.put(h, nt);
	R.put(h + 1, nc);
	icmp_csum(R, h, old, v6, false);
	return true;
}

/* rewrite_icmp (nat64_kern.c:325-441) at frame offset h */
__device__ bool rewrite_icmp(const Row &R, int h, const Bytes<40> &v6)
{
	uint8_t old[8];
	for (int k = 0; k < 8; k++)
		old[k] = (uint8_t)R.b(h + k);
	uint32_t t = old[0], c = old[1], nt = t, nc = c;
	switch (t) {
	case 8: nt = 128; break;
	case 0: nt = 129; break;
	case 3:
		nt = 1;
		switch (c) {
		case 0: case 1: case 5: case 6: case 7: case 8: case 11: case 12:
			nc = 0;
			break;
		case 2:
			nt = 4;
			nc = 1;
			put_be32r(R, h + 4, 6);
			break;
		case 3: nc = 4; break;
		case 4: {
			nt = 2;
			nc = 0;
			uint32_t mtu = (((uint32_t)old[6] << 8) | old[7]) + 20;
			if (mtu < 1280)
				mtu = 1280;
			put_be32r(R, h + 4, mtu);
			break;
		}
		case 9: case 10: case 13: case 15: nc = 1; break;
		default: return false;
		}
		break;
	case 12: {
		if (c == 1)
			return false;
		nt = 4;
		nc = 0;
		const uint32_t r = old[4];
		uint32_t p;
		if (r == 0) p = 0;
		else if (r == 1) p = 1;
		else if (r == 2 || r == 3) p = 4;
		else if (r == 8) p = 7;
		else if (r == 9) p = 6;
		else if (r >= 12 && r <= 15) p = 8;
		else if (r >= 16 && r <= 19) p = 24;
		else return false;
		put_be32r(R, h + 4, p);
		break;
	}
	default:
		return false;
	}
	R.put(h, nt);
	R.put(h + 1, nc);
	icmp_csum(R, h, old, v6, true);
	return true;
}

/* RFC 6052 byte positions of the embedded IPv4 address per prefix length
 * (v4addr_to_v6 / v6addr_to_v4, nat64_kern.c:180-323); pref_end is the
 * number of prefix bytes kept (bytes [pref_end, 16) of the prefix are 0,
 * except /64 keeps 8 and the u octet 8 is 0) */
__device__ __forceinline__ bool v4pos(uint32_t plen, int (&pos)[4], int &pref_end)
{
	/* 96: bytes 12-15; 64: 9-12; 56: 7, 9-11; 48: 6, 7, 9, 10; 40: 5-7, 9;
	 * 32: 4-7 -- from byte plen / 8 on, the u octet (byte 8) skipped below
	 * /96.  (Arithmetic rather than a switch: the positions then stay in
	 * registers.) */
	const int base = (int)(plen >> 3);
	for (int k = 0; k < 4; k++)
		pos[k] = base + k + (plen <= 64 && base + k >= 8 ? 1 : 0);
	pref_end = base;
	return plen == 96 || plen == 64 || plen == 56 || plen == 48 || plen == 40 || plen == 32;
}

struct Tables {
	Nat64V6Bucket *v6map;
	uint32_t v6nb;
	const Nat64V4Bucket *v4map;
	uint32_t v4nb;
	uint32_t dyn;              /* Nat64Args.dyn, .now, .thr */
	unsigned long long now, thr;
};

/* v6_state_map lookup (nat64_handle_v6, nat64_kern.c:809-828): the IPv4
 * address (host order) of the source's entry, one 128-byte bucket per
 * probe.  With dynamic state a hit stamps last_seen with the batch clock
 * (nat64_kern.c:821-823), and an entry that has timed out (last_seen <
 * now - timeout_ns, not static: check_item, :543-561) counts as a miss:
 * an earlier frame of the batch may reclaim it, which only the host's
 * in-order commit can tell. */
__device__ uint32_t lookup_v6(const Tables &T, const uint32_t (&w)[4], bool &found)
{
	uint32_t b = nat64_home(slot_hash(w[0], w[1], w[2], w[3]), T.v6nb);
	for (uint32_t probe = 0; probe < T.v6nb; probe++) {
		Nat64V6Bucket *B = T.v6map + b;
		const uint32_t meta = B->meta;
		uint32_t hit = 0;
#pragma unroll
		for (int j = 0; j < 4; j++) {
			const uint4 k = B->key[j];
			hit |= ((k.x == w[0]) & (k.y == w[1]) & (k.z == w[2]) & (k.w == w[3]))
				       ? 1u << j : 0u;
		}
		hit &= meta;
		if (hit) {
			const uint32_t j = (uint32_t)__builtin_ctz(hit);
			if (T.dyn) {
				const unsigned long long ls = B->last_seen[j];
				if (!((meta >> (8 + j)) & 1) && ls < T.thr) {
					found = false;
					return 0;
				}
				if (ls != T.now)
					B->last_seen[j] = T.now;
			}
			found = true;
			return B->val[j];
		}
		if (!(meta & kNat64Ovf))
			break;
		b = b + 1 == T.v6nb ? 0 : b + 1;
	}
	found = false;
	return 0;
}

__device__ bool lookup_v4(const Tables &T, uint32_t v4, uint32_t (&w)[4])
{
	uint32_t b = nat64_home(slot_hash(v4, 0, 0, 0), T.v4nb);
	for (uint32_t probe = 0; probe < T.v4nb; probe++) {
		const Nat64V4Bucket *B = T.v4map + b;
		const uint4 k = *reinterpret_cast<const uint4 *>(B->key);
		const uint32_t hit = B->meta & ((k.x == v4 ? 1u : 0u) | (k.y == v4 ? 2u : 0u) |
						(k.z == v4 ? 4u : 0u) | (k.w == v4 ? 8u : 0u));
		if (hit) {
			const uint4 v = B->val[__builtin_ctz(hit)];
			w[0] = v.x;
			w[1] = v.y;
			w[2] = v.z;
			w[3] = v.w;
			return true;
		}
		if (!(B->meta & kNat64Ovf))
			break;
		b = b + 1 == T.v4nb ? 0 : b + 1;
	}
	return false;
}

/* List the wave's frames that need the host's commit (dynamic state):
 * one atomic per wave on the list length. */
__device__ __forceinline__ void miss_append(const Nat64Args &a, bool miss, uint32_t i,
					    uint4 src, int lane)
{
	const uint64_t m = __ballot(miss);
	if (!m)
		return;
	const int lead = __builtin_ffsll((long long)m) - 1;
	uint32_t base = 0;
	if (lane == lead)
		base = atomicAdd(a.miss_cnt, (uint32_t)__popcll(m));
	base = __shfl(base, lead);
	const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
							__builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
	if (miss) {
		a.miss_idx[base + rank] = i;
		a.miss_src[base + rank] = src;
	}
}

struct Plan {
	int lo, hi;       /* frame-relative span rewritten in the row */
	int co;           /* extra 2-byte store (TCP checksum) or -1 */
};

/* Opt-in XDPGPU_NAT64_F_ICMP_INNER (include/xdpgpu.h; not in the
 * reference: the FIXMEs at nat64_kern.c:438 and :736).  The IPv6 header
 * embedded in an ICMPv6 error at frame offset ii becomes h4i, built by the
 * outer rules of nat64_handle_v6 (:830-850).  v6 is the outer header (its
 * source maps to src4).  False: not translatable (the frame is dropped).
 * Rare frames: byte reads through the row, past it from HBM. */
__device__ bool inner_v6_to_v4(const Row &R, uint32_t len, int ii, uint32_t oplen,
			       const Bytes<40> &v6, uint32_t src4, const Nat64Args &a,
			       const Tables &T, Bytes<20> &h4i)
{
	if ((uint32_t)ii + 40 > len || oplen < 48 || (R.b(ii) >> 4) != 6)
		return false;
	const uint32_t nh = R.b(ii + 6);
	if (nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135)
		return false;
	int p4[4], pend;
	if (!v4pos(a.cfg.v6_plen, p4, pend))
		return false;
	for (int k = 0; k < 16; k++) {
		const uint32_t v = k < pend ? R.b(ii + 8 + k) : 0u;
		if (v != a.cfg.v6_prefix[k])
			return false;
	}
	bool same = true;
	for (int k = 0; k < 16; k++)
		same = same && R.b(ii + 24 + k) == v6[8 + k];
	uint32_t d4 = src4;
	if (!same) {
		/* static state only: a dynamic entry is the error's own source */
		if (T.dyn)
			return false;
		uint32_t w[4];
		for (int k = 0; k < 4; k++)
			w[k] = R.b(ii + 24 + 4 * k) | R.b(ii + 25 + 4 * k) << 8 |
			       R.b(ii + 26 + 4 * k) << 16 | R.b(ii + 27 + 4 * k) << 24;
		bool found;
		d4 = lookup_v6(T, w, found);
		if (!found)
			return false;
	}
	h4i.zero();
	h4i.set(0, 0x45);
	h4i.set(1, ((R.b(ii) & 0x0f) << 4) | (R.b(ii + 1) >> 4));
	const uint32_t tot = R.be16(ii + 4) + 20;
	h4i.set(2, tot >> 8);
	h4i.set(3, tot);
	h4i.set(6, 0x40);
	h4i.set(8, R.b(ii + 7));
	h4i.set(9, nh == 58 ? 1 : nh);
	for (int k = 0; k < 4; k++)
		h4i.set(12 + k, R.b(ii + 8 + p4[k]));
	h4i.set(16, d4 >> 24);
	h4i.set(17, d4 >> 16);
	h4i.set(18, d4 >> 8);
	h4i.set(19, d4);
	uint32_t s = 0;
	for (int k = 0; k < 20; k += 2)
		s += h4i[k] | (h4i[k + 1] << 8);
	s = (s & 0xffff) + (s >> 16);
	s = (s & 0xffff) + (s >> 16);
	s = ~s & 0xffff;
	h4i.set(10, s);
	h4i.set(11, s >> 8);
	return true;
}

/* The IPv4 header (IHL ihl) embedded in an ICMPv4 error at ii becomes h6i,
 * by the outer rules of nat64_handle_v4 (:497-519). */
__device__ bool inner_v4_to_v6(const Row &R, uint32_t len, int ii, uint32_t otot,
			       const Nat64Args &a, const Tables &T, Bytes<40> &h6i,
			       uint32_t &ihl)
{
	if ((uint32_t)ii + 20 > len || (R.b(ii) >> 4) != 4)
		return false;
	ihl = (R.b(ii) & 0xf) * 4;
	if (ihl < 20 || (uint32_t)ii + ihl > len || otot < 28 + ihl)
		return false;
	if (R.be16(ii + 6) & ~0x4000u)
		return false;
	uint32_t w[4];
	if (!lookup_v4(T, R.be32(ii + 12), w))
		return false;
	int p4[4], pend;
	if (!v4pos(a.cfg.v6_plen, p4, pend))
		return false;
	h6i.zero();
	const int keep = a.cfg.v6_plen == 64 ? 8 : pend;
	for (int k = 0; k < 16; k++)
		if (k < keep)
			h6i.set(24 + k, a.cfg.v6_prefix[k]);
	for (int k = 0; k < 4; k++)
		h6i.template set_dyn<24, 40>(24 + p4[k], R.b(ii + 16 + k));
	for (int k = 0; k < 4; k++)
		h6i.w[2 + k] = w[k];
	const uint32_t tos = R.b(ii + 1), proto = R.b(ii + 9);
	h6i.set(0, 6 << 4 | ((tos & 0x70) >> 4));
	h6i.set(1, tos << 4);
	const uint32_t pl = (R.be16(ii + 2) - ihl) & 0xffff;
	h6i.set(4, pl >> 8);
	h6i.set(5, pl);
	h6i.set(6, proto == 1 ? 58 : proto);
	h6i.set(7, R.b(ii + 8));
	return true;
}

/* nat64_handle_v6 (nat64_kern.c:741-873); INNER: the opt-in ICMP-error
 * inner header (its own instantiation, so the reference build keeps its
 * registers) */
template <bool INNER>
__device__ uint32_t handle_v6(const Row &R, uint32_t len, int l3, uint64_t eff,
			      const Nat64Args &a, const Tables &T, Plan &P,
			      int64_t &shift, uint32_t ovv, uint4 &srcw)
{
	if ((uint32_t)l3 + 40 > len || (R.b(l3) >> 4) != 6)
		return XDPGPU_TC_ACT_OK;          /* parse_ip6hdr */
	const uint32_t nexthdr = R.b(l3 + 6);
	/* skip_ip6hdrext (parsing_helpers.h:139-172) */
	int pos = l3 + 40;
	int ip_type = -1;
	uint32_t nh = nexthdr;
	for (int k = 0; k < 6; k++) {
		if ((uint32_t)pos + 2 > len)
			break;
		if (nh == 0 || nh == 60 || nh == 43 || nh == 135) {
			const uint32_t n2 = R.b(pos);
			pos += (R.b(pos + 1) + 1) * 8;
			nh = n2;
		} else if (nh == 51) {
			const uint32_t n2 = R.b(pos);
			pos += (R.b(pos + 1) + 2) * 4;
			nh = n2;
		} else if (nh == 44) {
			nh = R.b(pos);
			pos += 8;
		} else {
			ip_type = (int)nh;
			break;
		}
	}
	if (ip_type < 0)
		return XDPGPU_TC_ACT_OK;
	/* v6addr_to_v4 + prefix compare */
	int p4[4], pend;
	if (!v4pos(a.cfg.v6_plen, p4, pend))
		return XDPGPU_TC_ACT_OK;
	uint8_t d4[4];
	for (int k = 0; k < 4; k++)
		d4[k] = (uint8_t)R.b(l3 + 24 + p4[k]);
	for (int k = 0; k < 16; k++) {
		const uint32_t v = k < pend ? R.b(l3 + 24 + k) : 0u;
		if (v != a.cfg.v6_prefix[k])
			return XDPGPU_TC_ACT_OK;
	}
	if ((uint32_t)ip_type != nexthdr)
		return XDPGPU_TC_ACT_SHOT;
	const uint32_t dst = (uint32_t)d4[0] << 24 | (uint32_t)d4[1] << 16 |
			     (uint32_t)d4[2] << 8 | d4[3];
	if (!dst || (dst & 0xFF000000u) == 0x7F000000u || (dst & 0xF0000000u) == 0xE0000000u)
		return XDPGPU_TC_ACT_SHOT;
	/* allowed_v6_src: the single LPM entry */
	if (!a.cfg.allow_plen)
		return XDPGPU_TC_ACT_SHOT;
	for (uint32_t bit = 0; bit < a.cfg.allow_plen; bit++) {
		const uint32_t sh = 7 - (bit & 7);
		if (((R.b(l3 + 8 + (bit >> 3)) >> sh) & 1) !=
		    ((uint32_t)(a.cfg.allow_prefix[bit >> 3] >> sh) & 1))
			return XDPGPU_TC_ACT_SHOT;
	}
	uint32_t w[4];
	for (int k = 0; k < 4; k++)
		w[k] = R.b(l3 + 8 + 4 * k) | R.b(l3 + 9 + 4 * k) << 8 |
		       R.b(l3 + 10 + 4 * k) << 16 | R.b(l3 + 11 + 4 * k) << 24;
	/* the state: from the table, or (commit pass) the host's decision */
	uint32_t src;
	if (a.ov) {
		if (!ovv)
			return XDPGPU_TC_ACT_SHOT;    /* alloc_new_state failed */
		src = ovv;
	} else {
		bool found;
		src = lookup_v6(T, w, found);
		if (!found) {
			srcw = make_uint4(w[0], w[1], w[2], w[3]);
			return XDPGPU_NAT64_NO_STATE;
		}
	}

	/* the original IPv6 header, kept for the checksum updates */
	Bytes<40> v6;
	for (int k = 0; k < 40; k++)
		v6.set(k, R.b(l3 + k));
	Bytes<20> h4;
	h4.zero();
	h4.set(0, 0x45);
	h4.set(1, ((v6[0] & 0x0f) << 4) | (v6[1] >> 4));
	const uint32_t tot = (v6[4] << 8 | v6[5]) + 20;
	h4.set(2, tot >> 8);
	h4.set(3, tot);
	h4.set(6, 0x40);
	h4.set(8, v6[7]);
	h4.set(9, nexthdr);
	h4.set(12, src >> 24);
	h4.set(13, src >> 16);
	h4.set(14, src >> 8);
	h4.set(15, src);
	for (int k = 0; k < 4; k++)
		h4.set(16 + k, d4[k]);
	const int l4 = l3 + 40;
	P.co = -1;
	int l4_end = l4;            /* rewritten L4 bytes [l4, l4_end) */
	bool inner = false;
	Bytes<20> h4i;
	if (nexthdr == 58) {
		if ((uint32_t)l4 + 8 > len || l4 + 8 > kWinEnd)
			return XDPGPU_TC_ACT_SHOT;
		const uint32_t t0 = R.b(l4);
		inner = INNER && t0 >= 1 && t0 <= 4;
		if (inner && !inner_v6_to_v4(R, len, l4 + 8, v6[4] << 8 | v6[5], v6,
					     src, a, T, h4i))
			return XDPGPU_TC_ACT_SHOT;
		if (!rewrite_icmpv6(R, l4, v6))
			return XDPGPU_TC_ACT_SHOT;
		h4.set(9, 1);
		l4_end = l4 + 8;
		if (inner) {
			/* 40 header bytes out of the ICMP message, 20 in */
			uint32_t to = 0;
			for (int k = 0; k < 20; k += 2)
				to += h4i[k] | (h4i[k + 1] << 8);
			row_csum(R, l4 + 2, diff_mod(R.words(l4 + 8, 40), mod_ffff(to)), false);
			h4.set(2, v6[4]);
			h4.set(3, v6[5]);
		}
	} else if (nexthdr == 6 || nexthdr == 17) {
		const int co = l4 + (nexthdr == 6 ? 16 : 6);
		if ((uint32_t)co + 2 <= len && co + 2 <= kWinEnd) {
			uint32_t from = 0, to = 0;
			for (int k = 8; k < 40; k += 2)
				from += v6[k] | (v6[k + 1] << 8);
			for (int k = 12; k < 20; k += 2)
				to += h4[k] | (h4[k + 1] << 8);
			row_csum(R, co, diff_mod(mod_ffff(from), mod_ffff(to)), nexthdr == 17);
			if (nexthdr == 17)
				l4_end = l4 + 8;
			else
				P.co = co;
		}
	}
	/* csum_fold_helper(bpf_csum_diff(0, 0, hdr, 20, 0)) */
	uint32_t s = 0;
	for (int k = 0; k < 20; k += 2)
		s += h4[k] | (h4[k + 1] << 8);
	s = (s & 0xffff) + (s >> 16);
	s = (s & 0xffff) + (s >> 16);
	s = ~s & 0xffff;
	h4.set(10, s);
	h4.set(11, s >> 8);
	if (inner) {
		/* [L2][IPv4][ICMP][inner IPv4] end where the inner IPv6 header
		 * did: written straight to HBM from the row and registers (the
		 * frame starts 40 bytes later); nothing left for the row's
		 * write-back */
		uint8_t *g = a.umem + eff + 40;
		for (int k = 0; k < 20; k++)
			g[l3 + 28 + k] = h4i[k];
		for (int k = 0; k < 8; k++)
			g[l3 + 20 + k] = (uint8_t)R.b(l4 + k);
		for (int k = 0; k < 20; k++)
			g[l3 + k] = h4[k];
		for (int k = 0; k < l3; k++)
			g[k] = k == 12 ? 0x08 : k == 13 ? 0x00 : (uint8_t)R.b(k);
		P.lo = P.hi = 0;
		shift = 40;
		return XDPGPU_TC_ACT_REDIRECT;
	}
	/* the L2 header moves 20 bytes forward (back to front: l3 may exceed
	 * 20), h_proto = 0x0800, then the IPv4 header */
	for (int k = l3 - 1; k >= 0; k--)
		R.put(20 + k, R.b(k));
	R.put(32, 0x08);
	R.put(33, 0x00);
	for (int k = 0; k < 20; k++)
		R.put(20 + l3 + k, h4[k]);
	P.lo = 20;
	P.hi = l4_end > l3 + 40 ? l4_end : l3 + 40;
	shift = 20;
	return XDPGPU_TC_ACT_REDIRECT;
}

/* nat64_handle_v4 (nat64_kern.c:443-541) */
template <bool INNER>
__device__ uint32_t handle_v4(const Row &R, uint32_t len, int l3, uint64_t eff,
			      const Nat64Args &a, const Tables &T, Plan &P,
			      int64_t &shift)
{
	if ((uint32_t)l3 + 20 > len || (R.b(l3) >> 4) != 4)
		return XDPGPU_TC_ACT_OK;          /* parse_iphdr */
	const uint32_t ihl = (R.b(l3) & 0xf) * 4;
	if (ihl < 20 || (uint32_t)l3 + ihl > len)
		return XDPGPU_TC_ACT_OK;
	const uint32_t dst = R.be32(l3 + 16);
	if ((dst & a.cfg.v4_mask) != a.cfg.v4_prefix)
		return XDPGPU_TC_ACT_OK;
	if (ihl != 20 || (R.be16(l3 + 6) & ~0x4000u))
		return XDPGPU_TC_ACT_SHOT;
	uint32_t w[4];
	if (!lookup_v4(T, dst, w))
		return XDPGPU_TC_ACT_SHOT;
	int p4[4], pend;
	if (!v4pos(a.cfg.v6_plen, p4, pend))
		return XDPGPU_TC_ACT_SHOT;
	Bytes<40> v6;
	v6.zero();
	/* v4addr_to_v6: prefix bytes, then the address bytes */
	const int keep = a.cfg.v6_plen == 64 ? 8 : pend;
	for (int k = 0; k < 16; k++)
		if (k < keep)
			v6.set(8 + k, a.cfg.v6_prefix[k]);
	for (int k = 0; k < 4; k++)
		v6.template set_dyn<8, 24>(8 + p4[k], R.b(l3 + 12 + k));
	for (int k = 0; k < 4; k++)
		v6.w[6 + k] = w[k];
	const uint32_t tos = R.b(l3 + 1), proto = R.b(l3 + 9);
	v6.set(0, 6 << 4 | ((tos & 0x70) >> 4));
	v6.set(1, tos << 4);
	const uint32_t pl = (R.be16(l3 + 2) - 20) & 0xffff;
	v6.set(4, pl >> 8);
	v6.set(5, pl);
	v6.set(6, proto);
	v6.set(7, R.b(l3 + 8));
	/* the bytes in front the frame may grow into (cfg.headroom) */
	const uint64_t room = a.cfg.headroom && a.cfg.headroom < eff ? a.cfg.headroom : eff;
	if (room < 20)
		return XDPGPU_TC_ACT_SHOT;        /* no headroom to grow */
	const int l4 = l3 + 20;
	P.co = -1;
	int l4_end = l4;
	if (proto == 1) {
		if ((uint32_t)l4 + 8 > len || l4 + 8 > kWinEnd)
			return XDPGPU_TC_ACT_SHOT;
		const uint32_t t0 = R.b(l4);
		const bool inner = INNER && (t0 == 3 || t0 == 11 || t0 == 12);
		Bytes<40> h6i;
		uint32_t ihl_i = 0, grow = 0;
		if (inner) {
			if (!inner_v4_to_v6(R, len, l4 + 8, R.be16(l3 + 2), a, T, h6i, ihl_i))
				return XDPGPU_TC_ACT_SHOT;
			grow = 40 - ihl_i;
			if (room < 20 + grow)
				return XDPGPU_TC_ACT_SHOT;
			/* the pseudo header's length is the new payload_len */
			const uint32_t pl2 = (pl + grow) & 0xffff;
			v6.set(4, pl2 >> 8);
			v6.set(5, pl2);
		}
		if (!rewrite_icmp(R, l4, v6))
			return XDPGPU_TC_ACT_SHOT;
		v6.set(6, 58);
		l4_end = l4 + 8;
		if (inner) {
			uint32_t to = 0;
			for (int k = 0; k < 40; k += 2)
				to += h6i[k] | (h6i[k + 1] << 8);
			row_csum(R, l4 + 2, diff_mod(R.words(l4 + 8, (int)ihl_i), mod_ffff(to)),
				 false);
			/* [L2][IPv6][ICMPv6][inner IPv6] end where the inner
			 * IPv4 header did: the frame starts 20 + grow earlier */
			const int sh = 20 + (int)grow;
			uint8_t *g = a.umem + eff - sh;
			for (int k = 0; k < l3; k++)
				g[k] = k == 12 ? 0x86 : k == 13 ? 0xDD : (uint8_t)R.b(k);
			for (int k = 0; k < 40; k++)
				g[l3 + k] = v6[k];
			for (int k = 0; k < 8; k++)
				g[l3 + 40 + k] = (uint8_t)R.b(l4 + k);
			for (int k = 0; k < 40; k++)
				g[l3 + 48 + k] = h6i[k];
			P.lo = P.hi = 0;
			shift = -sh;
			return XDPGPU_TC_ACT_REDIRECT;
		}
	} else if (proto == 6 || proto == 17) {
		const int co = l4 + (proto == 6 ? 16 : 6);
		if ((uint32_t)co + 2 <= len && co + 2 <= kWinEnd) {
			uint32_t from = 0, to = 0;
			for (int k = 12; k < 20; k += 2)
				from += R.b(l3 + k) | (R.b(l3 + k + 1) << 8);
			for (int k = 8; k < 40; k += 2)
				to += v6[k] | (v6[k + 1] << 8);
			row_csum(R, co, diff_mod(mod_ffff(from), mod_ffff(to)), proto == 17);
			if (proto == 17)
				l4_end = l4 + 8;
			else
				P.co = co;
		}
	}
	/* the L2 header moves 20 bytes back, h_proto = 0x86DD, then the
	 * IPv6 header */
	for (int k = 0; k < l3; k++)
		R.put(k - 20, R.b(k));
	R.put(-8, 0x86);
	R.put(-7, 0xDD);
	for (int k = 0; k < 40; k++)
		R.put(l3 - 20 + k, v6[k]);
	P.lo = -20;
	P.hi = l4_end > l4 ? l4_end : l4;
	shift = -20;
	return XDPGPU_TC_ACT_REDIRECT;
}

} // namespace

/* 4 waves a SIMD for the reference's translation (113 VGPRs, nothing in
 * scratch; left to itself the compiler took 150 and 3 waves: ingress 1.021
 * vs 1.010 ms); the ICMP-inner instance keeps its 3 (at 4 it spilled) */
template <bool INNER>
__global__ __launch_bounds__(kBlockN, INNER ? 3 : 4) void xdp_nat64_kernel(Nat64Args a)
{
	__shared__ uint32_t rows_all[kWavesN * kWaveN * kRowDw];
	__shared__ uint64_t dtab_all[kWavesN * kWaveN];
	const int lane = threadIdx.x & (kWaveN - 1);
	const int wid = threadIdx.x / kWaveN;
	uint32_t *rows = rows_all + wid * kWaveN * kRowDw;
	uint64_t *dtab = dtab_all + wid * kWaveN;
	uint8_t *rb = reinterpret_cast<uint8_t *>(rows + lane * kRowDw);
	const Tables T = {a.v6map, a.v6nb, a.v4map, a.v4nb, a.dyn, a.now, a.thr};
	const uint64_t us16 = (a.usize + 15) & ~15ull;

	/* work: every frame (a.xlist null) or the fast kernel's slow-frame
	 * lists, one (region, batch of 64) item at a time */
	const uint64_t nwaves = (uint64_t)gridDim.x * kWavesN;
	const uint64_t nitems = a.xlist ? (uint64_t)a.nregions * (a.xregion / kWaveN)
				       : ((uint64_t)a.n + kWaveN - 1) / kWaveN;
	for (uint64_t t = (uint64_t)blockIdx.x * kWavesN + wid; t < nitems; t += nwaves) {
		uint64_t i;
		bool active;
		uint32_t ovv = 0;
		if (a.xlist) {
			const uint32_t r = (uint32_t)(t % a.nregions);
			const uint32_t b = (uint32_t)(t / a.nregions) * kWaveN;
			const uint32_t cnt = a.xcount[r];
			if (b >= cnt)
				continue;
			active = b + lane < cnt;
			const uint64_t li = (uint64_t)r * a.xregion + b + lane;
			i = active ? a.xlist[li] : 0;
			if (a.ov && active)
				ovv = a.ov[li];
		} else {
			i = t * kWaveN + lane;
			active = i < a.n;
		}
		const uint4 dv = active ? *reinterpret_cast<const uint4 *>(a.desc + i)
					: make_uint4(0, 0, 0, 0);
		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool valid = active && (uint64_t)len <= a.usize && eff <= a.usize - len;

		/* stage frame bytes [-32, 96): transposed 16-byte loads for
		 * aligned frames with the whole span inside the UMEM */
		const bool fastld = valid && !(eff & 15) && eff >= (uint64_t)kFront &&
				    eff - kFront + 128 <= us16;
		dtab[lane] = fastld ? eff - kFront : ~0ull;
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int k = 0; k < 8; k++) {
			const int q = k * kWaveN + lane;
			const int f = q >> 3, c = q & 7;
			const uint64_t base = dtab[f];
			uint4 v = make_uint4(0, 0, 0, 0);
			if (base != ~0ull)
				v = *reinterpret_cast<const uint4 *>(a.umem + base + 16 * c);
			uint32_t *dst = rows + f * kRowDw + 4 * c;
			dst[0] = v.x;
			dst[1] = v.y;
			dst[2] = v.z;
			dst[3] = v.w;
		}
		__builtin_amdgcn_wave_barrier();
		if (valid && !fastld) {
			for (int j = 0; j < 128; j++) {
				const int64_t o = (int64_t)eff - kFront + j;
				rb[j] = (o >= 0 && (uint64_t)o < a.usize) ? a.umem[o] : 0;
			}
		}

		/* nat64_handler (nat64_kern.c:875-890) */
		const Row R = {rb, a.umem + eff};
		uint32_t act = valid ? XDPGPU_TC_ACT_OK : XDPGPU_TC_ACT_SHOT;
		Plan P = {0, 0, -1};
		int64_t shift = 0;
		uint4 srcw = make_uint4(0, 0, 0, 0);
		if (valid && len >= 14) {
			/* parse_ethhdr (parsing_helpers.h:86-137) */
			int l3 = 14;
			uint32_t proto = R.be16(12);
			for (int k = 0; k < 2; k++) {
				if (proto != 0x8100 && proto != 0x88A8)
					break;
				if ((uint32_t)l3 + 4 > len)
					break;
				proto = R.be16(l3 + 2);
				l3 += 4;
			}
			if (a.cfg.direction == XDPGPU_NAT64_EGRESS && proto == 0x0800)
				act = handle_v4<INNER>(R, len, l3, eff, a, T, P, shift);
			else if (a.cfg.direction == XDPGPU_NAT64_INGRESS && proto == 0x86DD)
				act = handle_v6<INNER>(R, len, l3, eff, a, T, P, shift, ovv, srcw);
		}
		if (a.dyn && !a.ov)
			miss_append(a, active && act == XDPGPU_NAT64_NO_STATE, (uint32_t)i, srcw,
				    lane);

		/* write back the rewritten span [P.lo, P.hi) of the row (the
		 * translated frame ends where the original did) and the TCP
		 * checksum */
		if (act == XDPGPU_TC_ACT_REDIRECT) {
			const int hi = P.hi < (int)len ? P.hi : (int)len;
			uint8_t *g = a.umem + eff;
			int o = P.lo;
			if (!(eff & 3)) {
				for (; o + 4 <= hi; o += 4)
					*reinterpret_cast<uint32_t *>(g + o) =
						*reinterpret_cast<const uint32_t *>(rb + kFront + o);
			}
			for (; o < hi; o++)
				g[o] = rb[kFront + o];
			if (P.co >= 0) {
				g[P.co] = rb[kFront + P.co];
				g[P.co + 1] = rb[kFront + P.co + 1];
			}
		}
		if (active) {
			a.action[i] = (uint8_t)act;
			uint4 od = dv;
			if (act == XDPGPU_TC_ACT_REDIRECT) {
				const uint64_t na = eff + shift;
				od.x = (uint32_t)na;
				od.y = (uint32_t)(na >> 32);
				od.z = (uint32_t)((int64_t)len - shift);
			}
			*reinterpret_cast<uint4 *>(a.out + i) = od;
		}
		__builtin_amdgcn_wave_barrier();
	}
}

/* ------------------------------------------------------------------ */
/* Fast kernels (EG false: IPv6 -> IPv4, config 4; EG true: IPv4 -> IPv6)
 * for untagged, 16-byte aligned frames of the common shapes under a /96
 * prefix.  Ingress: no extension header.  The 64-byte window of a
 * tile is staged by LDS-DMA as in the RX fast kernel (conflict-free slot
 * swizzle); everything else happens in registers: field extraction at
 * fixed offsets, the static-map probe, the IPv4 header and its checksum,
 * the incremental L4 update (TCP's check word at 70 is a second, narrow
 * load).  The frame's new first 64 bytes are staged in LDS and written
 * back transposed (four lanes per frame, whole 64-byte sectors).  Frames of other
 * shapes go to the wave's slow list (xdp_nat64_kernel). */

typedef __attribute__((address_space(3))) void lds_void_n;

__device__ __forceinline__ uint32_t halves2(uint32_t x)
{
	return (x & 0xffff) + (x >> 16);
}

__device__ __forceinline__ uint32_t bswap16n(uint32_t x)
{
	return ((x & 0xff) << 8) | ((x >> 8) & 0xff);
}

/* IPv6 -> IPv4 of one lane's frame (nat64_handle_v6 order): decides the
 * action or sends the frame to the slow list; a translated frame's new
 * bytes [0, 64) go to its swizzled LDS slots */
__device__ __forceinline__ void ingress_tile(const Nat64Args &a, const Tables &T,
					     const uint32_t (&F)[16], uint64_t eff,
					     uint32_t len, bool valid, bool staged,
					     uint4 *obuf, uint64_t *otab, int lane,
					     uint32_t &act, bool &slow, bool &xlate, uint4 &srcw)
{
	const int osw = (lane >> 2) & 3;
	/* classification (nat64_handler, nat64_handle_v6 order) */
	const uint32_t et = F[3] & 0xffff;
	const bool vlan = (et == 0x0081u) | (et == 0xa888u);
	const bool is6 = et == 0xdd86u;
	const uint32_t nh = F[5] & 0xff;
	const bool ext = (nh == 0) | (nh == 43) | (nh == 44) | (nh == 51) |
			 (nh == 60) | (nh == 135);
	const bool hdr_ok = (len >= 56) & (((F[3] >> 20) & 0xf) == 6);
	uint32_t s[4], d[4];
#pragma unroll
	for (int k = 0; k < 4; k++) {
		s[k] = (F[5 + k] >> 16) | (F[6 + k] << 16);
		d[k] = (F[9 + k] >> 16) | (F[10 + k] << 16);
	}
	const bool inpref = (d[0] == a.pref_w[0]) & (d[1] == a.pref_w[1]) &
			    (d[2] == a.pref_w[2]);
	const uint32_t dst = __builtin_bswap32(d[3]);
	const bool special = (dst == 0) | ((dst & 0xFF000000u) == 0x7F000000u) |
			     ((dst & 0xF0000000u) == 0xE0000000u);
	const bool allowed = (a.cfg.allow_plen != 0) &
			     ((s[0] & a.allow_m[0]) == a.allow_w[0]) &
			     ((s[1] & a.allow_m[1]) == a.allow_w[1]) &
			     ((s[2] & a.allow_m[2]) == a.allow_w[2]) &
			     ((s[3] & a.allow_m[3]) == a.allow_w[3]);
	const uint32_t itype = (F[13] >> 16) & 0xff;
	const bool icmp_ok = (itype == 128) | (itype == 129);

	/* decided here: invalid (SHOT), len < 14 or not IPv6 (OK),
	 * parse failure (OK), outside the prefix (OK), SHOT cases,
	 * and the translatable shapes; the rest is slow */
	slow = false;
	act = XDPGPU_TC_ACT_OK;
	xlate = false;
	if (!valid) {
		act = XDPGPU_TC_ACT_SHOT;
	} else if (len < 14) {
		act = XDPGPU_TC_ACT_OK;
	} else if (!staged) {
		slow = true;
	} else if (vlan) {
		slow = true;
	} else if (!is6 || !hdr_ok) {
		act = XDPGPU_TC_ACT_OK;           /* also len < 56 */
	} else if (len < 64) {
		slow = true;   /* the 16-byte stores stay inside the frame */
	} else if (ext) {
		slow = true;
	} else if (!inpref) {
		act = XDPGPU_TC_ACT_OK;
	} else if (special || !allowed) {
		act = XDPGPU_TC_ACT_SHOT;
	} else if (nh == 58 && (!icmp_ok || len < 62)) {
		slow = true;
	} else {
		xlate = true;
	}
	uint32_t v4 = 0;
	if (xlate) {
		bool found;
		if (a.diag & 1) {
			found = true;
			v4 = 0x0A630001u;
		} else {
			v4 = lookup_v6(T, s, found);
		}
		if (!found) {
			xlate = false;
			act = XDPGPU_NAT64_NO_STATE;
			srcw = make_uint4(s[0], s[1], s[2], s[3]);
		} else {
			act = XDPGPU_TC_ACT_REDIRECT;
		}
	}
	/* TCP's check word (bytes 70-71) lies past the window */
	uint32_t e68 = 0;
	const bool tcp_upd = xlate && nh == 6 && len >= 72;
	if (tcp_upd)
		e68 = *reinterpret_cast<const uint32_t *>(a.umem + eff + 68);

	const bool put = xlate && !(a.diag & 2);
	otab[lane] = put ? eff : ~0ull;
	if (put) {
		const uint32_t h3 = __builtin_bswap32(v4);        /* src, LE word */
		const uint32_t h4 = d[3];
		const uint32_t tos = (((F[3] >> 16) & 0xf) << 4) | (F[3] >> 28);
		const uint32_t tot = (bswap16n(F[4] >> 16) + 20) & 0xffff;
		const uint32_t ttl = (F[5] >> 8) & 0xff;
		const uint32_t p4 = nh == 58 ? 1u : nh;
		/* IPv4 header checksum (csum_fold_helper of the header):
		 * LE 16-bit words; frag_off is the wire bytes 0x40 0x00
		 * (DF), the LE word 0x0040 */
		uint32_t hs = halves2(0x45u | (tos << 8) | (bswap16n(tot) << 16)) +
			      0x0040u + (ttl | (p4 << 8)) + halves2(h3) + halves2(h4);
		hs = (hs & 0xffff) + (hs >> 16);
		hs = (hs & 0xffff) + (hs >> 16);
		const uint32_t chk4 = ~hs & 0xffff;
		/* the pseudo header's address words, v6 and v4 */
		uint32_t s6 = 0;
#pragma unroll
		for (int k = 0; k < 4; k++)
			s6 += halves2(s[k]) + halves2(d[k]);
		s6 = mod_ffff(s6);
		const uint32_t s4 = mod_ffff(halves2(h3) + halves2(h4));
		uint32_t o13 = (h4 >> 16) | (F[13] & 0xffff0000u);
		uint32_t o14 = F[14], o15 = F[15];
		if (nh == 17) {
			/* update_l4_checksum, BPF_F_MARK_MANGLED_0 */
			uint32_t c = F[15] & 0xffff;
			if (c) {
				c = csum_upd(c, diff_mod(s6, s4));
				if (!c)
					c = 0xffff;
			}
			o15 = (F[15] & 0xffff0000u) | c;
		} else if (nh == 6) {
			if (tcp_upd) {
				const uint32_t c = csum_upd(e68 >> 16, diff_mod(s6, s4));
				e68 = (e68 & 0xffff) | (c << 16);
			}
		} else if (nh == 58) {
			/* rewrite_icmpv6, echo: pseudo header out, type word */
			const uint32_t ph = mod_ffff(s6 + (F[4] >> 16) + (58u << 8));
			const uint32_t code = (F[13] >> 24) & 0xff;
			const uint32_t nt = itype == 128 ? 8u : 0u;
			const uint32_t hb = itype | (code << 8), ha = nt | (code << 8);
			const uint32_t delta = mod_ffff(diff_mod(ph, 0) + diff_mod(hb, ha));
			const uint32_t c = csum_upd(F[14] & 0xffff, delta);
			o13 = (h4 >> 16) | (ha << 16);
			o14 = (F[14] & 0xffff0000u) | c;
		}
		/* frame bytes [0, 64): unchanged [0, 20) (rewritten so
		 * that the stores are whole 64-byte sectors), the L2
		 * header moved to 20 with h_proto 0x0800, the IPv4
		 * header at 34, the L4 bytes at 54; staged in LDS in the
		 * swizzled slots of the header buffer's layout */
		obuf[4 * lane + (0 ^ osw)] = make_uint4(F[0], F[1], F[2], F[3]);
		obuf[4 * lane + (1 ^ osw)] = make_uint4(F[4], F[0], F[1], F[2]);
		obuf[4 * lane + (2 ^ osw)] =
			make_uint4(0x0008u | (0x45u << 16) | (tos << 24),
				   bswap16n(tot), 0x40u | (ttl << 16) | (p4 << 24),
				   chk4 | (h3 << 16));
		obuf[4 * lane + (3 ^ osw)] =
			make_uint4((h3 >> 16) | (h4 << 16), o13, o14, o15);
		if (tcp_upd)
			*reinterpret_cast<uint32_t *>(a.umem + eff + 68) = e68;
	}
}

/* IPv4 -> IPv6 of one lane's frame (nat64_handle_v4, nat64_kern.c:443-541,
 * under a /96 prefix): untagged, ihl 5, at least 64 bytes and 32 bytes of
 * headroom.  ICMP echo request/reply is rewritten here, other ICMP types go
 * to the slow list.  The frame grows 20 bytes to the front: its new bytes
 * [-20, 0) are stored by the lane (a dword and a 16-byte chunk), the new
 * bytes [0, 64) go to its swizzled LDS slots.  Position p of the new frame
 * layout, relative to the old frame start: [-20, -8) the MACs, [-8, -6)
 * h_proto 0x86DD, [-6, 34) the IPv6 header, [34, ...) the L4 bytes in
 * place (the L4 header does not move). */
__device__ __forceinline__ void egress_tile(const Nat64Args &a, const Tables &T,
					    const uint32_t (&F)[16], uint64_t eff,
					    uint32_t len, bool valid, bool staged,
					    uint4 *obuf, uint64_t *otab, int lane,
					    uint32_t &act, bool &slow, bool &xlate)
{
	const int osw = (lane >> 2) & 3;
	const uint32_t et = F[3] & 0xffff;
	const bool vlan = (et == 0x0081u) | (et == 0xa888u);
	const bool is4 = et == 0x0008u;
	const uint32_t vihl = (F[3] >> 16) & 0xff;
	const uint32_t s4 = (F[6] >> 16) | (F[7] << 16);   /* saddr, LE word */
	const uint32_t d4 = (F[7] >> 16) | (F[8] << 16);   /* daddr */
	const uint32_t dst = __builtin_bswap32(d4);
	const bool inpref = (dst & a.cfg.v4_mask) == a.cfg.v4_prefix;
	/* frag_off other than DF: the LE word of wire bytes 20-21 */
	const bool frag = (F[5] & 0xffbfu) != 0;
	const uint32_t proto = F[5] >> 24;
	const uint32_t itype = (F[8] >> 16) & 0xff;
	const bool echo = (itype == 8) | (itype == 0);

	slow = false;
	act = XDPGPU_TC_ACT_OK;
	xlate = false;
	if (!valid) {
		act = XDPGPU_TC_ACT_SHOT;
	} else if (len < 14) {
		act = XDPGPU_TC_ACT_OK;
	} else if (!staged || vlan) {
		slow = true;
	} else if (!is4) {
		act = XDPGPU_TC_ACT_OK;
	} else if (vihl != 0x45 || len < 64 || eff < 32 ||
		   (a.cfg.headroom && a.cfg.headroom < 20)) {
		slow = true;   /* options / other versions; short; no room */
	} else if (!inpref) {
		act = XDPGPU_TC_ACT_OK;
	} else if (frag) {
		act = XDPGPU_TC_ACT_SHOT;
	} else if (proto == 1 && !echo) {
		slow = true;
	} else {
		xlate = true;
	}
	uint32_t w[4] = {0, 0, 0, 0};
	if (xlate) {
		bool found = true;
		if (a.diag & 1) {
			w[0] = 0x20010db8u;
			w[3] = dst;
		} else {
			found = lookup_v4(T, dst, w);
		}
		if (found) {
			act = XDPGPU_TC_ACT_REDIRECT;
		} else {
			xlate = false;
			act = XDPGPU_TC_ACT_SHOT;
		}
	}

	const bool put = xlate && !(a.diag & 2);
	otab[lane] = put ? eff : ~0ull;
	if (!put)
		return;
	const uint32_t tos = F[3] >> 24;
	const uint32_t pl = (bswap16n(F[4] & 0xffff) - 20) & 0xffff;
	const uint32_t ttl = (F[5] >> 16) & 0xff;
	const uint32_t nh = proto == 1 ? 58u : proto;
	/* priority and flow label as v4addr_to_v6's caller writes them */
	const uint32_t b0 = 0x60u | ((tos & 0x70u) >> 4), b1 = (tos << 4) & 0xff;
	/* the pseudo header's address words, v4 and v6 */
	const uint32_t from = mod_ffff(halves2(s4) + halves2(d4));
	uint32_t to = halves2(a.pref_w[0]) + halves2(a.pref_w[1]) +
		      halves2(a.pref_w[2]) + halves2(s4);
#pragma unroll
	for (int k = 0; k < 4; k++)
		to += halves2(w[k]);
	to = mod_ffff(to);
	const uint32_t delta = diff_mod(from, to);
	uint32_t n13 = (w[3] >> 16) | (F[8] & 0xffff0000u);
	uint32_t n14 = F[9], n15 = F[10], n17 = F[12];
	if (proto == 17) {
		/* update_l4_checksum, BPF_F_MARK_MANGLED_0 */
		uint32_t c = F[10] & 0xffff;
		if (c) {
			c = csum_upd(c, delta);
			if (!c)
				c = 0xffff;
		}
		n15 = (F[10] & 0xffff0000u) | c;
	} else if (proto == 6) {
		n17 = (F[12] & 0xffff) | (csum_upd(F[12] >> 16, delta) << 16);
	} else if (proto == 1) {
		/* rewrite_icmp, echo: type word, pseudo header in */
		const uint32_t ph = mod_ffff(to + bswap16n(pl) + (58u << 8));
		const uint32_t code = F[8] >> 24;
		const uint32_t nt = itype == 8 ? 128u : 129u;
		const uint32_t hb = itype | (code << 8), ha = nt | (code << 8);
		const uint32_t c = csum_upd(F[9] & 0xffff, mod_ffff(ph + diff_mod(hb, ha)));
		n13 = (w[3] >> 16) | (ha << 16);
		n14 = (F[9] & 0xffff0000u) | c;
	}
	/* new bytes [-20, 0): MACs, h_proto, version/priority/flow label,
	 * payload_len */
	*reinterpret_cast<uint32_t *>(a.umem + eff - 20) = F[0];
	*reinterpret_cast<uint4 *>(a.umem + eff - 16) =
		make_uint4(F[1], F[2], 0xDD86u | (b0 << 16) | (b1 << 24), bswap16n(pl) << 16);
	/* new bytes [0, 64): nexthdr, hop limit, the addresses, the L4 header */
	obuf[4 * lane + (0 ^ osw)] =
		make_uint4(nh | (ttl << 8) | (a.pref_w[0] << 16),
			   (a.pref_w[0] >> 16) | (a.pref_w[1] << 16),
			   (a.pref_w[1] >> 16) | (a.pref_w[2] << 16),
			   (a.pref_w[2] >> 16) | (s4 << 16));
	obuf[4 * lane + (1 ^ osw)] =
		make_uint4((s4 >> 16) | (w[0] << 16), (w[0] >> 16) | (w[1] << 16),
			   (w[1] >> 16) | (w[2] << 16), (w[2] >> 16) | (w[3] << 16));
	obuf[4 * lane + (2 ^ osw)] = make_uint4(n13, n14, n15, F[11]);
	obuf[4 * lane + (3 ^ osw)] = make_uint4(n17, F[13], F[14], F[15]);
}

/* One block per CU (kCuWavesN waves), tiles claimed at run time from an LDS
 * counter as in the RX kernel (xdp_rx.hip, xdp_rx_db_kernel): with a static
 * share per wave the SIMD's issue arbitration, which favours its oldest
 * wave, lets the waves of a CU finish far apart.  Block b's tiles are b,
 * b + nb, ...; a wave claims the tile two steps ahead of its compute (the
 * descriptor load and the window DMA run one and two steps ahead).  Slow
 * frames go to the block's list (an LDS atomic reserves each wave's 64
 * entries), which xdp_nat64_kernel walks as one region per block. */
constexpr int kCuWavesN = 16;
/* the fast kernel's action and output-descriptor stores non-temporal
 * (build knob for A/B): ingress 1.006 vs 1.048 ms with plain stores,
 * alternating processes (tools/gpu_ab_outnt.sh) */
#ifndef XDP_NAT64_OUT_NT
#define XDP_NAT64_OUT_NT 1
#endif
constexpr bool kOutNt = XDP_NAT64_OUT_NT != 0;
typedef uint32_t v4u_n __attribute__((ext_vector_type(4)));
/* the window DMA's cache policy: plain, not non-temporal — the frame's
 * lines are rewritten in place right after (an in-place rewrite of 64 of
 * each 128 bytes: 0.83 ms per 16 M frames with plain loads, 1.18 ms with
 * non-temporal ones, tools/hbm_probe stride) */
#ifndef XDP_NAT64_WIN_AUX
#define XDP_NAT64_WIN_AUX 0
#endif
constexpr int kWinAux = XDP_NAT64_WIN_AUX;
/* the translated frame sectors' stores (build knob for A/B, bit 0
 * ingress, bit 1 egress): plain or non-temporal.  Egress 1.510 vs 1.617 ms
 * with non-temporal stores; ingress 0.974 vs 0.971 ms (one box) */
#ifndef XDP_NAT64_FRAME_NT
#define XDP_NAT64_FRAME_NT 2
#endif
constexpr int kCuBlockN = kCuWavesN * kWaveN;

template <bool EG>
__global__ __launch_bounds__(kCuBlockN, 1) void xdp_nat64_fast_kernel(Nat64Args a)
{
	__shared__ uint4 buf_all[kCuWavesN * 4 * kWaveN];
	__shared__ uint64_t dtab_all[kCuWavesN * kWaveN];
	__shared__ uint32_t xq_all[kCuWavesN * 2 * kWaveN];
	/* translated first 64 bytes of each frame, stored transposed */
	__shared__ uint4 obuf_all[kCuWavesN * 4 * kWaveN];
	__shared__ uint64_t otab_all[kCuWavesN * kWaveN];
	/* the block's tile claims, slow-list length, shared-tile slots */
	__shared__ uint32_t ctl[3];
	const int lane = threadIdx.x & (kWaveN - 1);
	const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWaveN);
	uint4 *buf = buf_all + wid * 4 * kWaveN;
	uint64_t *dtab = dtab_all + wid * kWaveN;
	uint32_t *xq = xq_all + wid * 2 * kWaveN;
	uint4 *obuf = obuf_all + wid * 4 * kWaveN;
	uint64_t *otab = otab_all + wid * kWaveN;
	const Tables T = {a.v6map, a.v6nb, a.v4map, a.v4nb, a.dyn, a.now, a.thr};

	if (threadIdx.x == 0)
		ctl[0] = ctl[1] = ctl[2] = 0;
	const uint64_t rb = blockIdx.x, nb = gridDim.x;
	/* the next launch's shared-tile counters (this launch's set was
	 * zeroed by the one before) */
	if (rb == 0 && threadIdx.x < kStealHeads && a.steal)
		a.steal[((a.steal_set ^ 1) * kStealHeads + threadIdx.x) * kStealStride] = 0;
	__syncthreads();

	const uint64_t ntiles = ((uint64_t)a.n + kWaveN - 1) / kWaveN;
	/* Shared tiles, as in xdp_rx_db_kernel: the block's own tiles b,
	 * b + nb, ... below own, then those above, one per claim from the
	 * global counter of head b mod heads (tile own + v heads + h), each
	 * claim first reserving one of the block's steal_cap() slots.  A
	 * claim is issued one step before its tile is needed and read after
	 * the next step's full wait, so its round trip is hidden. */
	const uint64_t shared = a.steal ? a.steal_tiles : 0;
	const uint64_t own = ntiles - shared;
	const uint64_t heads = min((uint64_t)kStealHeads, nb), h = rb % heads;
	uint32_t *ctr = a.steal + (a.steal_set * kStealHeads + h) * kStealStride;
	const uint32_t scap = (uint32_t)steal_cap(shared, nb);
	bool stealing = false;
	uint32_t vpend = 0x7fffffffu;
	auto gclaim = [&]() -> uint32_t {
		uint32_t v = 0x7fffffffu;
		if (lds_fetch_add(&ctl[2], 1, lane) < scap && lane == 0)
			v = atomicAdd(ctr, 1u);
		return v;
	};
	uint32_t *xl = a.xlist + rb * a.xregion;
	uint32_t xq_n = 0;
	const uint64_t us16 = (a.usize + 15) & ~15ull;
	const bool dma = a.usize >= 64;
	auto claim = [&](uint32_t cnt) -> uint64_t {
		return rb + (uint64_t)lds_fetch_add(&ctl[0], cnt, lane) * nb;
	};
	/* the next tile: an own tile, else the shared tile of the claim
	 * pending since the last step (the first one claimed now) */
	auto next_tile = [&]() -> uint64_t {
		if (!stealing) {
			const uint64_t t = claim(1);
			if (t < own)
				return t;
			stealing = true;
			if (!shared)
				return ntiles;
			vpend = gclaim();
		}
		const uint32_t v = __builtin_amdgcn_readfirstlane(vpend);
		const uint64_t t = v < 0x7fffffffu ? own + (uint64_t)v * heads + h : ntiles;
		return t < ntiles ? t : ntiles;
	};
	/* 64 queued slow frames to the block's list */
	auto flush = [&](uint32_t cnt) {
		const uint32_t base = lds_fetch_add(&ctl[1], cnt, lane);
		if ((uint32_t)lane < cnt)
			xl[base + lane] = xq[lane];
	};

	auto ld_desc = [&](uint64_t tt) -> uint4 {
		uint64_t i = tt * kWaveN + lane;
		i = i < a.n ? i : a.n - 1;
		return *reinterpret_cast<const uint4 *>(a.desc + i);
	};
	auto issue = [&](uint4 dv, bool live) {
		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool ok = live & dma & ((uint64_t)len <= a.usize) &
				(eff <= a.usize - len) & !(eff & 15) & (eff + 64 <= us16);
		dtab[lane] = ok ? eff : 0ull;
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int f = 16 * k + (lane >> 2);
			const int c = (lane & 3) ^ ((f >> 2) & 3);
			__builtin_amdgcn_global_load_lds(
				(const void *)(a.umem + dtab[f] + 16 * c),
				(lds_void_n *)(buf + kWaveN * k), 16, 0, kWinAux);
		}
	};

	/* the wave's tiles: qa (in the buffer), qb (its descriptor loaded) */
	uint64_t qa = next_tile();
	if (stealing && qa < ntiles)
		vpend = gclaim();
	uint64_t qb = next_tile();
	if (stealing && qb < ntiles)
		vpend = gclaim();
	uint4 dcur = make_uint4(0, 0, 0, 0), dnext = dcur;
	if (qa < ntiles) {
		dcur = ld_desc(qa);
		dnext = ld_desc(qb);
		issue(dcur, true);
	}
	while (qa < ntiles) {
		const uint64_t i = qa * kWaveN + lane;
		const bool active = i < a.n;
		const uint4 dv = dcur;
		uint32_t F[16];
		lds_dma_landed();
		{
			const int sw = (lane >> 2) & 3;
#pragma unroll
			for (int c = 0; c < 4; c++) {
				const uint4 v = buf[4 * lane + (c ^ sw)];
				F[4 * c] = v.x;
				F[4 * c + 1] = v.y;
				F[4 * c + 2] = v.z;
				F[4 * c + 3] = v.w;
			}
		}
		lds_reads_done();
		__builtin_amdgcn_wave_barrier();
		/* resolved before this step's first vector memory op: a pending
		 * claim has landed in the wait above */
		const uint64_t qc = next_tile();
		dcur = dnext;
		issue(dcur, qb < ntiles);
		if (stealing && qc < ntiles)
			vpend = gclaim();
		dnext = ld_desc(qc);

		const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
		const uint32_t len = dv.z;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		const bool valid = active & ((uint64_t)len <= a.usize) & (eff <= a.usize - len);
		const bool staged = valid & dma & !(eff & 15) & (eff + 64 <= us16);

		uint32_t act;
		bool slow, xlate;
		if constexpr (EG) {
			egress_tile(a, T, F, eff, len, valid, staged, obuf, otab, lane, act,
				    slow, xlate);
		} else {
			uint4 srcw = make_uint4(0, 0, 0, 0);
			ingress_tile(a, T, F, eff, len, valid, staged, obuf, otab, lane, act,
				     slow, xlate, srcw);
			if (a.dyn)
				miss_append(a, active && !slow && act == XDPGPU_NAT64_NO_STATE,
					    (uint32_t)i, srcw, lane);
		}

		/* slow frames to the block's list */
		{
			const uint64_t dm = __ballot(active && slow);
			if (dm) {
				const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
					(uint32_t)(dm >> 32),
					__builtin_amdgcn_mbcnt_lo((uint32_t)dm, 0));
				if (active && slow)
					xq[xq_n + rank] = (uint32_t)i;
				xq_n += (uint32_t)__popcll(dm);
				if (xq_n >= (uint32_t)kWaveN) {
					__builtin_amdgcn_wave_barrier();
					flush(kWaveN);
					const uint32_t rest = xq[kWaveN + lane];
					__builtin_amdgcn_wave_barrier();
					xq[lane] = rest;
					xq_n -= kWaveN;
				}
			}
		}

		/* transposed stores: in store k lane l writes chunk l & 3 of
		 * frame 16k + l / 4, so four lanes write one frame's 64 bytes
		 * as a whole sector */
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int f = 16 * k + (lane >> 2);
			const int c = lane & 3;
			const uint64_t e = otab[f];
			if (e != ~0ull) {
				const uint4 v = obuf[4 * f + (c ^ ((f >> 2) & 3))];
				if constexpr (((XDP_NAT64_FRAME_NT >> (EG ? 1 : 0)) & 1) != 0) {
					const v4u_n v4 = {v.x, v.y, v.z, v.w};
					__builtin_nontemporal_store(
						v4, reinterpret_cast<v4u_n *>(a.umem + e + 16 * c));
				} else {
					*reinterpret_cast<uint4 *>(a.umem + e + 16 * c) = v;
				}
			}
		}
		__builtin_amdgcn_wave_barrier();
		if (active && !slow) {
			if constexpr (kOutNt)
				__builtin_nontemporal_store((uint8_t)act, a.action + i);
			else
				a.action[i] = (uint8_t)act;
			uint4 od = dv;
			if (xlate) {
				/* the frame starts 20 bytes later (IPv4) or
				 * earlier (IPv6) */
				const uint64_t na = EG ? eff - 20 : eff + 20;
				od.x = (uint32_t)na;
				od.y = (uint32_t)(na >> 32);
				od.z = EG ? len + 20 : len - 20;
			}
			if constexpr (kOutNt) {
				const v4u_n o4 = {od.x, od.y, od.z, od.w};
				__builtin_nontemporal_store(o4, reinterpret_cast<v4u_n *>(a.out + i));
			} else {
				*reinterpret_cast<uint4 *>(a.out + i) = od;
			}
		}
		qa = qb;
		qb = qc;
	}
	__builtin_amdgcn_wave_barrier();
	if (xq_n)
		flush(xq_n);
	lds_dma_landed();
	__syncthreads();
	if (threadIdx.x == 0)
		a.xcount[rb] = ctl[1];
}

template <auto KERN>
static uint32_t resident_n()
{
	return resident_blocks_dev<KERN, kBlockN>(1024);
}

/* the fast kernel's grid: one block per CU, fewer for short batches */
uint32_t nat64_grid(uint32_t n, uint32_t max_blocks)
{
	uint32_t cap = resident_blocks_dev<xdp_nat64_fast_kernel<false>, kCuBlockN>(1024);
	if (cap > max_blocks)
		cap = max_blocks;
	uint64_t tiles = ((uint64_t)n + kWaveN - 1) / kWaveN;
	uint64_t blocks = (tiles + kCuWavesN - 1) / kCuWavesN;
	if (blocks > cap)
		blocks = cap;
	return blocks ? (uint32_t)blocks : 1u;
}

/* the general kernel: the reference's translation, or with
 * XDPGPU_NAT64_F_ICMP_INNER its own instantiation; blocks 0 = as many as
 * are resident */
static hipError_t launch_slow(const Nat64Args &a, uint32_t blocks, uint32_t max_blocks,
			      uint32_t need, hipStream_t stream)
{
	const bool inner = a.cfg.flags & XDPGPU_NAT64_F_ICMP_INNER;
	if (!blocks) {
		blocks = inner ? resident_n<xdp_nat64_kernel<true>>()
			       : resident_n<xdp_nat64_kernel<false>>();
		if (blocks > max_blocks)
			blocks = max_blocks;
		if (blocks > need)
			blocks = need ? need : 1u;
	}
	if (inner)
		hipLaunchKernelGGL(xdp_nat64_kernel<true>, dim3(blocks), dim3(kBlockN), 0,
				   stream, a);
	else
		hipLaunchKernelGGL(xdp_nat64_kernel<false>, dim3(blocks), dim3(kBlockN), 0,
				   stream, a);
	return hipGetLastError();
}

hipError_t launch_nat64(const Nat64Args &a0, uint32_t max_blocks, hipStream_t stream)
{
	Nat64Args a = a0;
	if (a.ov) {
		/* the commit pass: the general kernel over the listed frames
		 * (xlist, one region of xregion entries, its count in xcount) */
		return launch_slow(a, 0, max_blocks,
				   (a.xregion / kWaveN + kWavesN - 1) / kWavesN, stream);
	}
	if (a.fast) {
		const uint32_t blocks = nat64_grid(a.n, max_blocks);
		/* one slow-list region per block: its share of the tiles, and
		 * with shared tiles (batches of at least 64 tiles per block) up
		 * to steal_cap() more */
		a.nregions = blocks;
		const uint64_t tiles = ((uint64_t)a.n + kWaveN - 1) / kWaveN;
		a.xregion = (uint32_t)(((tiles + a.nregions - 1) / a.nregions) * kWaveN);
		a.steal_tiles = 0;
		if (a.steal && a.steal_16ths && !a.diag && tiles >= 64ull * blocks) {
			const uint64_t own = (tiles - tiles * min(a.steal_16ths, 16u) / 16) &
					     ~(uint64_t)(kStealHeads - 1);
			const uint64_t sh = tiles - own;
			const uint64_t xr =
				((own + blocks - 1) / blocks + steal_cap(sh, blocks)) * kWaveN;
			if (xr * blocks <= a.xcap && xr <= 0xffffffffull) {
				a.steal_tiles = (uint32_t)sh;
				a.xregion = (uint32_t)xr;
			}
		}
		if (a.cfg.direction == XDPGPU_NAT64_EGRESS)
			hipLaunchKernelGGL(xdp_nat64_fast_kernel<true>, dim3(blocks),
					   dim3(kCuBlockN), 0, stream, a);
		else
			hipLaunchKernelGGL(xdp_nat64_fast_kernel<false>, dim3(blocks),
					   dim3(kCuBlockN), 0, stream, a);
		hipError_t e = hipGetLastError();
		if (e != hipSuccess)
			return e;
		return launch_slow(a, 0, max_blocks, ~0u, stream);
	}
	a.xlist = nullptr;
	uint64_t tiles = ((uint64_t)a.n + kWaveN - 1) / kWaveN;
	uint64_t blocks = (tiles + kWavesN - 1) / kWavesN;
	if (blocks > max_blocks)
		blocks = max_blocks;
	if (!blocks)
		return hipSuccess;
	return launch_slow(a, (uint32_t)blocks, max_blocks, ~0u, stream);
}

/* The host's dynamic-state commit: changed slots and their buckets' meta
 * words (all patches of one bucket carry its final meta). */
__global__ void nat64_patch_kernel(Nat64V6Bucket *v6map, Nat64V4Bucket *v4map,
				   const Nat64Patch *p, uint32_t np)
{
	const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
	if (k >= np)
		return;
	const Nat64Patch q = p[k];
	if (q.table == 0) {
		Nat64V6Bucket *B = v6map + q.bucket;
		if (q.slot < 4) {
			B->key[q.slot] = q.k6;
			B->val[q.slot] = q.v4;
			B->last_seen[q.slot] = q.last_seen;
		}
		B->meta = q.meta;
	} else {
		Nat64V4Bucket *B = v4map + q.bucket;
		if (q.slot < 4) {
			B->key[q.slot] = q.v4;
			B->val[q.slot] = q.k6;
		}
		B->meta = q.meta;
	}
}

hipError_t launch_nat64_patch(Nat64V6Bucket *v6map, Nat64V4Bucket *v4map,
			      const Nat64Patch *p, uint32_t np, hipStream_t stream)
{
	if (!np)
		return hipSuccess;
	hipLaunchKernelGGL(nat64_patch_kernel, dim3((np + 255) / 256), dim3(256), 0, stream,
			   v6map, v4map, p, np);
	return hipGetLastError();
}

uint32_t nat64_slot_hash(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
{
	uint32_t h = a * 0x9E3779B1u ^ b * 0x85EBCA77u ^ c * 0xC2B2AE3Du ^
		     d * 0x27D4EB2Fu;
	h ^= h >> 15;
	h *= 0x2C1B3C6Du;
	h ^= h >> 13;
	return h;
}

} // namespace xdpgpu
