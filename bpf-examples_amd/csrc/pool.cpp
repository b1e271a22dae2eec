// SPDX-License-Identifier: GPL-2.0
/*
 * pool.cpp - synthetic UMEM pool generator (host).
 *
 * Stands in for the traffic a NIC would write into an AF_XDP UMEM.  Frame
 * geometry follows xdpsock (xdpsock.c:873-889): a declared size S carries
 * S-4 bytes of L2 data plus a 4-byte FCS slot.  Two replicated-base-frame
 * kinds reproduce the reference generators byte for byte:
 *   XDPGPU_POOL_XDPSOCK     gen_eth_hdr_data (xdpsock.c:893-971),
 *                           desc.len = S-4 (PKT_SIZE, xdpsock.c:1554-1564)
 *   XDPGPU_POOL_AFXDP_USER  gen_base_pkt (af_xdp_user.c:629-700),
 *                           desc.len = S (af_xdp_user.c:886,900)
 * and two randomized kinds implement BASELINE.json configs 2 and 3
 * (SURVEY.md §8d): every frame is a function of (seed, index) only, so the
 * pool is identical for any thread count.
 */
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include <thread>
#include <vector>

#include "xdpgpu.h"

namespace {

/* ---- deterministic randomness (splitmix64) ---- */
struct Rng {
	uint64_t s;
	explicit Rng(uint64_t seed) : s(seed) {}
	uint64_t next()
	{
		uint64_t z = (s += 0x9E3779B97F4A7C15ull);
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		return z ^ (z >> 31);
	}
	uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};

uint64_t mix64(uint64_t x)
{
	Rng r(x);
	return r.next();
}

/* ---- byte helpers ---- */
inline void put_be16(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 8);
	p[1] = (uint8_t)v;
}
inline void put_le16(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)v;
	p[1] = (uint8_t)(v >> 8);
}
inline uint32_t get_le16(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8);
}
inline uint32_t get_le32(const uint8_t *p)
{
	return get_le16(p) | (get_le16(p + 2) << 16);
}

/* ---- generator-side checksum (RFC 1071 sums; the oracle, not this, is
 * what outputs are checked against) ---- */
uint64_t sum16(const uint8_t *p, uint32_t len)
{
	uint64_t s = 0;
	uint32_t i;
	for (i = 0; i + 1 < len; i += 2)
		s += get_le16(p + i);
	if (len & 1)
		s += p[len - 1];
	return s;
}

uint32_t fold(uint64_t s)
{
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	return (uint32_t)s;
}

void ipv4_fix_csum(uint8_t *ip)
{
	uint32_t hl = (ip[0] & 0xf) * 4;
	ip[10] = ip[11] = 0;
	put_le16(ip + 10, ~fold(sum16(ip, hl)) & 0xffff);
}

/* udp_csum() of lib_checksum.h: words over ceil(len/2) (odd: the next byte
 * joins as the high half), pseudo header, no 0 -> 0xffff mapping. */
void l4v4_fix_csum(uint8_t *ip, uint8_t *l4, uint32_t len, uint32_t proto,
		   uint32_t chk_off)
{
	l4[chk_off] = l4[chk_off + 1] = 0;
	uint64_t s = 0;
	for (uint32_t i = 0; i < len; i += 2)
		s += get_le16(l4 + i);
	s += get_le32(ip + 12);
	s += get_le32(ip + 16);
	s += (uint64_t)(proto + len) << 8;
	put_le16(l4 + chk_off, ~fold(s) & 0xffff);
}

void icmp4_fix_csum(uint8_t *l4, uint32_t len)
{
	l4[2] = l4[3] = 0;
	put_le16(l4 + 2, ~fold(sum16(l4, len)) & 0xffff);
}

void l4v6_fix_csum(uint8_t *ip6, uint8_t *l4, uint32_t len, uint32_t proto,
		   uint32_t chk_off)
{
	l4[chk_off] = l4[chk_off + 1] = 0;
	uint64_t s = sum16(l4, len) + sum16(ip6 + 8, 32);
	s += __builtin_bswap32(len) & 0xffff;
	s += __builtin_bswap32(len) >> 16;
	s += __builtin_bswap32(proto) >> 16;
	put_le16(l4 + chk_off, ~fold(s) & 0xffff);
}

/* lib_checksum.h:7-21 semantics (pattern in network order, tail bytes
 * continue the pattern) */
void fill_pattern(uint8_t *dst, uint32_t pattern, uint32_t size)
{
	uint8_t b[4] = { (uint8_t)(pattern >> 24), (uint8_t)(pattern >> 16),
			 (uint8_t)(pattern >> 8), (uint8_t)pattern };
	for (uint32_t i = 0; i < size; i++)
		dst[i] = b[i & 3];
}

/* ---- frame kinds ---- */
enum Expect : uint8_t {
	E_ABORTED = XDPGPU_ABORTED,
	E_DROP = XDPGPU_DROP,
	E_PASS = XDPGPU_PASS,
	E_REDIRECT = XDPGPU_REDIRECT,
};

struct Flow {
	uint32_t saddr, daddr; /* wire-order values as LE u32 of the bytes */
	uint16_t sport, dport;
	uint8_t s6[16], d6[16];
};

Flow flow_of(uint64_t seed, uint32_t f)
{
	Flow fl;
	uint64_t h = mix64(seed * 0x100000001B3ull + f);
	uint64_t h2 = mix64(h);
	uint8_t sa[4] = { 10, (uint8_t)(h >> 8), (uint8_t)(h >> 16), (uint8_t)(h >> 24) };
	uint8_t da[4] = { 172, (uint8_t)(16 + ((h >> 32) & 15)), (uint8_t)(h >> 40),
			  (uint8_t)(h >> 48) };
	memcpy(&fl.saddr, sa, 4);
	memcpy(&fl.daddr, da, 4);
	fl.sport = (uint16_t)(1024 + (h2 % 60000));
	fl.dport = (uint16_t)((h2 >> 20) & 1 ? 53 + ((h2 >> 24) % 8000) : 443);
	/* 2001:db8::/32 sources, 64:ff9b::/96-style destinations */
	static const uint8_t spfx[8] = { 0x20, 0x01, 0x0d, 0xb8, 0, 0, 0, 0 };
	memcpy(fl.s6, spfx, 8);
	for (int i = 0; i < 8; i++)
		fl.s6[8 + i] = (uint8_t)(h2 >> (8 * i));
	memset(fl.d6, 0, 16);
	fl.d6[0] = 0x20;
	fl.d6[1] = 0x01;
	fl.d6[2] = 0x0d;
	fl.d6[3] = 0xb9;
	for (int i = 0; i < 8; i++)
		fl.d6[8 + i] = (uint8_t)(h >> (8 * i));
	return fl;
}

struct Gen {
	const xdpgpu_pool_spec *sp;
	uint32_t stride; /* fixed stride kinds */
};

/* Build an Ethernet header (+ tags) at p; returns the L3 offset. */
uint32_t put_eth(uint8_t *p, const uint8_t *dmac, const uint8_t *smac,
		 uint32_t ethertype, int ntags, uint16_t vid, uint16_t pri)
{
	memcpy(p, dmac, 6);
	memcpy(p + 6, smac, 6);
	uint32_t off = 12;
	for (int t = 0; t < ntags; t++) {
		uint32_t tpid = (ntags == 2 && t == 0) ? 0x88A8 : 0x8100;
		put_be16(p + off, tpid);
		uint32_t tci = (uint32_t)((vid + t) & 0x0fff) | ((uint32_t)(pri & 7) << 13);
		put_be16(p + off + 2, tci);
		off += 4;
	}
	put_be16(p + off, ethertype);
	return off + 2;
}

void put_ipv4(uint8_t *ip, uint32_t tot, uint32_t proto, uint32_t saddr,
	      uint32_t daddr, uint32_t ttl)
{
	ip[0] = 0x45;
	ip[1] = 0;
	put_be16(ip + 2, tot);
	put_be16(ip + 4, 0);
	put_be16(ip + 6, 0);
	ip[8] = (uint8_t)ttl;
	ip[9] = (uint8_t)proto;
	memcpy(ip + 12, &saddr, 4);
	memcpy(ip + 16, &daddr, 4);
	ipv4_fix_csum(ip);
}

void put_ipv6(uint8_t *ip, uint32_t plen, uint32_t nh, const uint8_t *s6,
	      const uint8_t *d6)
{
	ip[0] = 0x60;
	ip[1] = ip[2] = ip[3] = 0;
	put_be16(ip + 4, plen);
	ip[6] = (uint8_t)nh;
	ip[7] = 64;
	memcpy(ip + 8, s6, 16);
	memcpy(ip + 24, d6, 16);
}

const uint8_t kDefDmac[6] = { 0x3c, 0xfd, 0xfe, 0x9e, 0x7f, 0x71 };
const uint8_t kDefSmac[6] = { 0xec, 0xb1, 0xd7, 0x98, 0x3a, 0xc0 };

void rand_bytes(Rng &r, uint8_t *p, uint32_t n)
{
	uint32_t i = 0;
	for (; i + 8 <= n; i += 8) {
		uint64_t v = r.next();
		memcpy(p + i, &v, 8);
	}
	if (i < n) {
		uint64_t v = r.next();
		memcpy(p + i, &v, n - i);
	}
}

/* One randomized frame (kinds UDP4 / IMIX).  Writes at most `cap` bytes at
 * p; returns the descriptor length, sets *expect. */
uint32_t gen_random_frame(const xdpgpu_pool_spec *sp, uint64_t idx, uint8_t *p,
			  uint32_t S, uint8_t *expect)
{
	Rng r(mix64(sp->seed ^ (idx * 0xD1B54A32D192ED03ull)));
	const bool imix = sp->kind == XDPGPU_POOL_IMIX;
	const uint32_t fbits = sp->flow_bits ? sp->flow_bits : 20;
	const uint32_t L2 = S - 4;
	memset(p, 0, S);
	uint32_t u = r.below(1000000);
	Flow fl = flow_of(sp->seed, r.below(1u << fbits));
	*expect = E_REDIRECT;

	/* special traffic first */
	uint32_t acc = sp->ppm_arp;
	if (u < acc) {
		uint32_t o = put_eth(p, kDefDmac, kDefSmac, 0x0806, 0, 0, 0);
		put_be16(p + o, 1);          /* htype ethernet */
		put_be16(p + o + 2, 0x0800); /* ptype IPv4 */
		p[o + 4] = 6;
		p[o + 5] = 4;
		put_be16(p + o + 6, 1);      /* request */
		memcpy(p + o + 8, kDefSmac, 6);
		memcpy(p + o + 14, &fl.saddr, 4);
		memcpy(p + o + 24, &fl.daddr, 4);
		*expect = E_PASS;
		return S;
	}
	acc += sp->ppm_ndp;
	if (u < acc || (u < acc + sp->ppm_echo6)) {
		const bool ndp = u < acc;
		uint32_t o = put_eth(p, kDefDmac, kDefSmac, 0x86DD, 0, 0, 0);
		uint32_t len = L2 - o - 40;
		if (len < 8)
			len = 8; /* 64-byte frames: the ICMPv6 header uses the FCS slot */
		put_ipv6(p + o, len, 58, fl.s6, fl.d6);
		uint8_t *ic = p + o + 40;
		ic[0] = ndp ? (uint8_t)(133 + r.below(5)) : 128;
		ic[1] = 0;
		rand_bytes(r, ic + 4, len - 4);
		l4v6_fix_csum(p + o, ic, len, 58, 2);
		*expect = ndp ? E_PASS : E_REDIRECT;
		return S;
	}
	acc += sp->ppm_echo6;

	/* regular traffic */
	uint32_t size = S;
	int tags = 0;
	bool v6 = false;
	uint32_t l4p = 17;
	int nexts = 0;
	uint32_t doff = 5;
	if (imix) {
		uint32_t c = r.below(12);
		size = c < 7 ? 64 : c < 11 ? 570 : 1500;
		uint32_t tv = r.below(100);
		tags = tv < 20 ? 1 : tv < 22 ? 2 : 0;
		/* 30 % of the pool IPv6, all of it in the
		 * 570/1500 B classes (5/12 of the frames): 72 % of those */
		const uint64_t v6ppm = sp->ppm_v6 ? sp->ppm_v6 : 300000;
		const uint64_t big = v6ppm * 12 / 5;
		v6 = size > 64 && r.below(1000000) < (big < 1000000 ? big : 1000000);
		uint32_t pv = r.below(100);
		l4p = pv < 80 ? 17 : pv < 95 ? 6 : (v6 ? 58 : 1);
		if (v6 && r.below(100) < 5)
			nexts = 1 + (int)r.below(3);
		doff = 5 + r.below(11);
	}
	const uint32_t FL2 = size - 4;
	uint32_t o = put_eth(p, kDefDmac, kDefSmac, v6 ? 0x86DD : 0x0800, tags,
			     (uint16_t)(1 + (fl.sport & 0x7ff)), (uint16_t)(fl.dport & 7));
	uint32_t l3 = o;
	uint32_t iphl = v6 ? 40 + 8 * nexts : 20;
	uint32_t room = FL2 - l3 - iphl; /* L4 bytes */
	if (l4p == 6) {
		if (room < 20)
			l4p = 17;
		else if (doff * 4 > room)
			doff = room / 4;
	}
	uint8_t *l4 = p + l3 + iphl;
	if (l4p == 17) {
		put_be16(l4, fl.sport);
		put_be16(l4 + 2, fl.dport);
		put_be16(l4 + 4, room);
		rand_bytes(r, l4 + 8, room - 8);
	} else if (l4p == 6) {
		put_be16(l4, fl.sport);
		put_be16(l4 + 2, fl.dport);
		uint64_t sq = r.next();
		memcpy(l4 + 4, &sq, 8);
		l4[12] = (uint8_t)(doff << 4);
		l4[13] = 0x18; /* PSH|ACK */
		put_be16(l4 + 14, 501 + (uint32_t)(sq >> 48) % 60000);
		l4[18] = l4[19] = 0;
		for (uint32_t k = 20; k < doff * 4; k++)
			l4[k] = 1; /* NOP options */
		rand_bytes(r, l4 + doff * 4, room - doff * 4);
	} else {
		l4[0] = l4p == 58 ? 128 : 8; /* echo request */
		l4[1] = 0;
		rand_bytes(r, l4 + 4, room - 4);
	}
	if (v6) {
		uint32_t nh = l4p;
		/* extension chain written back to front */
		static const uint8_t ext_types[3] = { 0, 60, 43 }; /* HOP, DST, RT */
		put_ipv6(p + l3, room + 8 * nexts, nexts ? ext_types[0] : l4p, fl.s6,
			 fl.d6);
		for (int e = 0; e < nexts; e++) {
			uint8_t *eh = p + l3 + 40 + 8 * e;
			eh[0] = (uint8_t)(e + 1 < nexts ? ext_types[e + 1] : nh);
			eh[1] = 0;
			if (ext_types[e] == 43) {
				eh[2] = 0; /* routing type 0 */
				eh[3] = 0; /* segments left */
			} else {
				eh[2] = 1; /* PadN, 4 bytes */
				eh[3] = 4;
			}
		}
		l4v6_fix_csum(p + l3, l4, room, l4p, l4p == 6 ? 16 : l4p == 17 ? 6 : 2);
	} else {
		put_ipv4(p + l3, 20 + room, l4p, fl.saddr, fl.daddr, 64);
		if (l4p == 1)
			icmp4_fix_csum(l4, room);
		else
			l4v4_fix_csum(p + l3, l4, room, l4p, l4p == 6 ? 16 : 6);
	}
	uint32_t dlen = size;
	uint32_t chk = l4p == 6 ? 16 : l4p == 17 ? 6 : 2;

	/* corruption classes */
	if (u < acc + sp->ppm_malformed) {
		*expect = E_ABORTED;
		uint32_t m = r.below(5);
		if (m == 0) {
			dlen = r.below(14);                 /* runt */
		} else if (m == 1) {
			p[l3] = v6 ? 0x50 : 0x55;           /* wrong version */
		} else if (m == 2 && !v6) {
			p[l3] = 0x44;                       /* ihl < 5 */
		} else if (l4p == 17) {
			put_be16(l4 + 4, m == 3 ? 5 : room + 512); /* bad UDP len */
		} else {
			dlen = l3 + 10;                     /* truncated IP */
		}
		return dlen;
	}
	acc += sp->ppm_malformed;
	if (u < acc + sp->ppm_bad_l3 && !v6) {
		p[l3 + 10] ^= 0x5a;                     /* bad header checksum */
		*expect = E_DROP;
		return dlen;
	}
	acc += sp->ppm_bad_l3;
	if (u < acc + sp->ppm_bad_l4) {
		uint32_t c = get_le16(l4 + chk);
		uint32_t nc = c ^ 0x0100;
		if (nc == 0 || nc == 0xffff)
			nc = c ^ 0x0300;
		put_le16(l4 + chk, nc);
		*expect = E_DROP;
		return dlen;
	}
	/* a legitimately zero UDP/IPv4 checksum reads as "absent": fine */
	return dlen;
}

/* Base frame of xdpsock gen_eth_hdr_data() / af_xdp_user gen_base_pkt(). */
uint32_t gen_base_frame(const xdpgpu_pool_spec *sp, uint8_t *p)
{
	const bool xs = sp->kind == XDPGPU_POOL_XDPSOCK;
	const uint32_t S = sp->frame_size;
	const uint32_t L2 = S - 4;
	static const uint8_t afx_dmac[6] = { 0xbc, 0xee, 0x7b, 0xda, 0xc2, 0x62 };
	static const uint8_t afx_smac[6] = { 0x24, 0x5e, 0xbe, 0x57, 0xf1, 0x64 };
	const uint8_t zero6[6] = { 0, 0, 0, 0, 0, 0 };
	const uint8_t *dmac = memcmp(sp->dmac, zero6, 6) ? sp->dmac :
			      xs ? kDefDmac : afx_dmac;
	const uint8_t *smac = memcmp(sp->smac, zero6, 6) ? sp->smac :
			      xs ? kDefSmac : afx_smac;
	memset(p, 0, S);
	int tags = (xs && sp->vlan) ? 1 : 0;
	uint32_t l3 = put_eth(p, dmac, smac, 0x0800, tags, sp->vlan_id, sp->vlan_pri);
	uint32_t saddr = sp->saddr, daddr = sp->daddr;
	if (!saddr) {
		uint8_t a[4] = { 10, 10, 10, 16 }, b[4] = { 192, 168, 44, 1 };
		memcpy(&saddr, xs ? a : b, 4);
	}
	if (!daddr) {
		uint8_t a[4] = { 10, 10, 10, 32 }, b[4] = { 192, 168, 44, 3 };
		memcpy(&daddr, xs ? a : b, 4);
	}
	uint32_t ip_len = L2 - l3;
	uint32_t udp_len = ip_len - 20;
	uint8_t *udp = p + l3 + 20;
	put_be16(udp, 0x1000);
	put_be16(udp + 2, 0x1000);
	put_be16(udp + 4, udp_len);
	uint32_t pat = sp->fill_pattern ? sp->fill_pattern :
		       xs ? 0x12345678u : 0x41424344u;
	fill_pattern(udp + 8, pat, udp_len - 8);
	put_ipv4(p + l3, ip_len, 17, saddr, daddr, 64);
	l4v4_fix_csum(p + l3, udp, udp_len, 17, 6);
	return xs ? L2 : S;
}

/* ---- NAT64 pools (BASELINE config 4) ---- */
const uint8_t kPref64[16] = { 0, 0x64, 0xff, 0x9b, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0 };
const uint8_t kAllow[16] = { 0x20, 0x01, 0x0d, 0xb8, 0, 1, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0 };
constexpr uint32_t kV4Pool = 0x0A630000u; /* 10.99.0.0/16 */
constexpr uint32_t kNat64Map = 65533;     /* nat64.c:396 for a /16 */

void nat64_src(uint8_t *a6, uint32_t k)
{
	memcpy(a6, kAllow, 16);
	a6[12] = (uint8_t)(k >> 24);
	a6[13] = (uint8_t)(k >> 16);
	a6[14] = (uint8_t)(k >> 8);
	a6[15] = (uint8_t)k;
}

/* a public IPv4 address (not 0/8, 10/8, 127/8, >= 224/4) */
void public_v4(uint64_t h, uint8_t *a4)
{
	a4[0] = (uint8_t)(11 + (h % 200));
	if (a4[0] == 127)
		a4[0] = 128;
	a4[1] = (uint8_t)(h >> 8);
	a4[2] = (uint8_t)(h >> 16);
	a4[3] = (uint8_t)(1 + ((h >> 24) % 254));
}

enum : uint8_t { A_OK = XDPGPU_TC_ACT_OK, A_SHOT = XDPGPU_TC_ACT_SHOT,
		 A_REDIR = XDPGPU_TC_ACT_REDIRECT, A_NOSTATE = XDPGPU_NAT64_NO_STATE };

/* config 4 (ingress): IPv6/UDP, 10 % TCP, ppm_echo6 ICMPv6 echo, toward
 * 64:ff9b::a.b.c.d from 2001:db8:1:2::k; corruption classes reuse the ppm
 * knobs: bad_l3 = dst outside pref64 (OK), bad_l4 = source not allowed
 * (SHOT), ndp = allowed source without mapping (NO_STATE), arp = ARP (OK),
 * malformed = ext header / reserved v4 dst / truncation / bad version /
 * untranslatable ICMPv6 / UDP checksum 0. */
uint32_t gen_nat64_frame(const xdpgpu_pool_spec *sp, uint64_t idx, uint8_t *p,
			 uint32_t S, uint8_t *expect)
{
	Rng r(mix64(sp->seed ^ (idx * 0xD1B54A32D192ED03ull)));
	const uint32_t L2 = S - 4;
	const uint32_t fbits = sp->flow_bits ? sp->flow_bits : 16;
	memset(p, 0, S);
	uint32_t u = r.below(1000000);
	uint32_t k = 1 + r.below((1u << fbits) < kNat64Map ? (1u << fbits) : kNat64Map);
	uint64_t h = r.next();
	*expect = A_REDIR;

	uint32_t acc = sp->ppm_arp;
	if (u < acc) {
		uint32_t o = put_eth(p, kDefDmac, kDefSmac, 0x0806, 0, 0, 0);
		put_be16(p + o, 1);
		put_be16(p + o + 2, 0x0800);
		p[o + 4] = 6;
		p[o + 5] = 4;
		put_be16(p + o + 6, 1);
		*expect = A_OK;
		return S;
	}
	if (sp->kind == XDPGPU_POOL_NAT64_V4) {
		/* egress: public source toward 10.99.0.0 + k */
		uint8_t sa[4], da[4] = { 10, 99, (uint8_t)(k >> 8), (uint8_t)k };
		public_v4(h, sa);
		uint32_t o = put_eth(p, kDefDmac, kDefSmac, 0x0800, 0, 0, 0);
		uint32_t room = L2 - o - 20;
		uint32_t pv = r.below(100), proto = pv < 80 ? 17 : pv < 90 ? 6 : 1;
		uint8_t *l4 = p + o + 20;
		if (proto == 1) {
			uint32_t t = r.below(8);
			l4[0] = t < 5 ? 8 : t == 5 ? 0 : t == 6 ? 3 : 12;
			l4[1] = l4[0] == 3 ? (uint8_t)r.below(16) : 0;
			rand_bytes(r, l4 + 4, room - 4);
			if (l4[0] == 12)
				l4[4] = (uint8_t)r.below(20);
			icmp4_fix_csum(l4, room);
			if ((l4[0] == 3 && (l4[1] == 14 || l4[1] > 15)) ||
			    (l4[0] == 12 && ((l4[4] > 3 && l4[4] != 8 && l4[4] != 9 && l4[4] < 12) ||
					     l4[4] > 19)))
				*expect = A_SHOT;
		} else {
			put_be16(l4, 1024 + (uint32_t)(h >> 32) % 60000);
			put_be16(l4 + 2, 443);
			if (proto == 17) {
				put_be16(l4 + 4, room);
			} else {
				l4[12] = 5 << 4;
				l4[13] = 0x18;
			}
			rand_bytes(r, l4 + (proto == 17 ? 8 : 20), room - (proto == 17 ? 8 : 20));
		}
		uint32_t saddr, daddr;
		memcpy(&saddr, sa, 4);
		memcpy(&daddr, da, 4);
		put_ipv4(p + o, 20 + room, proto, saddr, daddr, 64);
		if (proto != 1)
			l4v4_fix_csum(p + o, l4, room, proto, proto == 6 ? 16 : 6);
		acc += sp->ppm_bad_l3;
		if (u < acc) {          /* destination outside the v4 pool */
			p[o + 17] = 98;
			ipv4_fix_csum(p + o);
			*expect = A_OK;
		} else if (u < acc + sp->ppm_ndp) { /* no reverse mapping */
			p[o + 18] = 0xff;
			p[o + 19] = 0xfe;
			ipv4_fix_csum(p + o);
			*expect = A_SHOT;
		} else if (u < acc + sp->ppm_ndp + sp->ppm_malformed) {
			put_be16(p + o + 6, 0x2000 | (uint32_t)r.below(8)); /* MF */
			ipv4_fix_csum(p + o);
			*expect = A_SHOT;
		}
		return S;
	}

	/* ingress: IPv6 */
	uint8_t s6[16], d6[16], a4[4];
	nat64_src(s6, k);
	public_v4(h, a4);
	memcpy(d6, kPref64, 12);
	memcpy(d6 + 12, a4, 4);
	uint32_t o = put_eth(p, kDefDmac, kDefSmac, 0x86DD, 0, 0, 0);
	uint32_t room = L2 - o - 40;
	uint32_t pv = r.below(1000000);
	uint32_t proto = pv < sp->ppm_echo6 ? 58 : pv < sp->ppm_echo6 + 100000 ? 6 : 17;
	uint8_t *l4 = p + o + 40;
	if (proto == 58) {
		l4[0] = 128;
		rand_bytes(r, l4 + 4, room - 4);
	} else {
		put_be16(l4, 1024 + (uint32_t)(h >> 32) % 60000);
		put_be16(l4 + 2, 53);
		if (proto == 17) {
			put_be16(l4 + 4, room);
		} else {
			l4[12] = 5 << 4;
			l4[13] = 0x18;
		}
		rand_bytes(r, l4 + (proto == 17 ? 8 : 20), room - (proto == 17 ? 8 : 20));
	}
	const uint32_t chk = proto == 6 ? 16 : proto == 17 ? 6 : 2;
	acc += sp->ppm_bad_l3;
	if (u < acc) {
		d6[1] = 0x65;                           /* outside pref64 */
		*expect = A_OK;
	} else if (u < acc + sp->ppm_bad_l4) {
		s6[6] = 0x99;                           /* source not allowed */
		*expect = A_SHOT;
	} else if (u < acc + sp->ppm_bad_l4 + sp->ppm_ndp) {
		nat64_src(s6, kNat64Map + 1 + r.below(1000)); /* no mapping */
		*expect = A_NOSTATE;
	}
	put_ipv6(p + o, room, proto, s6, d6);
	l4v6_fix_csum(p + o, l4, room, proto, chk);
	acc += sp->ppm_bad_l4 + sp->ppm_ndp;
	if (u >= acc && u < acc + sp->ppm_malformed) {
		uint32_t m = r.below(6);
		if (m == 0) {
			p[o + 6] = 0;                   /* hop-by-hop ext header */
			l4[0] = (uint8_t)proto;
			l4[1] = 0;
			*expect = A_SHOT;
		} else if (m == 1) {
			p[o + 36] = 127;                /* dst 127.x.x.x */
			*expect = A_SHOT;
		} else if (m == 2) {
			*expect = A_OK;                 /* truncated IPv6 header */
			return o + 20 + r.below(20);
		} else if (m == 3) {
			p[o] = 0x50;                    /* version 5 */
			*expect = A_OK;
		} else if (m == 4 && proto == 58) {
			l4[0] = 135;                    /* NDP: not translatable */
			*expect = A_SHOT;
		} else if (proto == 17) {
			l4[6] = l4[7] = 0;              /* UDP checksum 0: kept */
		}
	}
	return S;
}

uint32_t frame_size_of(const xdpgpu_pool_spec *sp, uint64_t idx)
{
	if (sp->kind != XDPGPU_POOL_IMIX)
		return sp->frame_size;
	Rng r(mix64(sp->seed ^ (idx * 0xD1B54A32D192ED03ull)));
	uint32_t u = r.below(1000000);
	(void)r.below(1u << (sp->flow_bits ? sp->flow_bits : 20));
	if (u < sp->ppm_arp + sp->ppm_ndp + sp->ppm_echo6)
		return sp->frame_size ? sp->frame_size : 64;
	uint32_t c = r.below(12);
	return c < 7 ? 64 : c < 11 ? 570 : 1500;
}

uint32_t stride_for(const xdpgpu_pool_spec *sp, uint32_t size)
{
	if (sp->stride)
		return sp->stride;
	return (size + sp->headroom + 63) & ~63u;
}

} // namespace

extern "C" {

void xdpgpu_pool_spec_default(xdpgpu_pool_spec *spec, uint32_t kind,
			      uint32_t frame_size, uint64_t seed)
{
	memset(spec, 0, sizeof(*spec));
	spec->kind = kind;
	spec->frame_size = frame_size ? frame_size : 64;
	spec->seed = seed;
	spec->flow_bits = 20;
	if (kind == XDPGPU_POOL_UDP4 || kind == XDPGPU_POOL_IMIX) {
		/* 1 % bad L3, 1 % bad L4, 0.5 % malformed,
		 * 0.1 % ARP, 0.1 % NDP */
		spec->ppm_bad_l3 = 10000;
		spec->ppm_bad_l4 = 10000;
		spec->ppm_malformed = 5000;
		spec->ppm_arp = 1000;
		spec->ppm_ndp = 1000;
		spec->ppm_echo6 = 0;
	}
	if (kind == XDPGPU_POOL_IMIX) {
		spec->frame_size = 64; /* size of special (ARP/NDP) frames */
		spec->ppm_v6 = 300000; /* 70 % IPv4 / 30 % IPv6 */
	}
	if (kind == XDPGPU_POOL_NAT64 || kind == XDPGPU_POOL_NAT64_V4) {
		/* config 4: 128 B frames, 10 % ICMPv6 echo; 0.5 % of each
		 * corruption class */
		spec->frame_size = frame_size ? frame_size : 128;
		spec->flow_bits = 16;
		spec->ppm_echo6 = 100000;
		spec->ppm_bad_l3 = 5000;
		spec->ppm_bad_l4 = 5000;
		spec->ppm_ndp = 5000;
		spec->ppm_arp = 1000;
		spec->ppm_malformed = 5000;
		/* the IPv6 header grows the frame 20 bytes to the front: 64
		 * bytes of headroom, frames 64-byte aligned as at an AF_XDP
		 * chunk's XDP_PACKET_HEADROOM */
		if (kind == XDPGPU_POOL_NAT64_V4)
			spec->headroom = 64;
	}
	spec->vlan_id = 1;
}

int xdpgpu_nat64_pool_config(uint32_t direction, xdpgpu_nat64_cfg *cfg,
			     xdpgpu_nat64_map *map, uint32_t nmap)
{
	if (!cfg || (nmap && !map) || nmap > kNat64Map)
		return -EINVAL;
	memset(cfg, 0, sizeof(*cfg));
	memcpy(cfg->v6_prefix, kPref64, 16);
	cfg->v6_plen = 96;
	cfg->v4_prefix = kV4Pool;
	cfg->v4_mask = 0xFFFF0000u;
	memcpy(cfg->allow_prefix, kAllow, 16);
	cfg->allow_plen = 64;
	cfg->direction = direction;
	for (uint32_t k = 1; k <= nmap; k++) {
		nat64_src(map[k - 1].v6, k);
		map[k - 1].v4 = kV4Pool + k;
		map[k - 1].rsvd = 0;
	}
	return 0;
}

uint64_t xdpgpu_pool_size(const xdpgpu_pool_spec *spec, uint32_t n)
{
	if (!spec)
		return 0;
	if (spec->kind != XDPGPU_POOL_IMIX || spec->stride)
		return (uint64_t)n * stride_for(spec, spec->frame_size) + 64;
	uint64_t total = 0;
	for (uint32_t i = 0; i < n; i++)
		total += stride_for(spec, frame_size_of(spec, i));
	return total + 64;
}

int xdpgpu_pool_generate(const xdpgpu_pool_spec *spec, uint8_t *umem,
			 uint64_t umem_size, xdpgpu_desc *descs, uint32_t n,
			 uint8_t *expect)
{
	if (!spec || !umem || !descs)
		return -EINVAL;
	const bool nat64 = spec->kind == XDPGPU_POOL_NAT64 ||
			   spec->kind == XDPGPU_POOL_NAT64_V4;
	const bool random = spec->kind == XDPGPU_POOL_UDP4 ||
			    spec->kind == XDPGPU_POOL_IMIX || nat64;
	if (spec->kind > XDPGPU_POOL_NAT64_V4)
		return -EINVAL;
	uint32_t S = spec->frame_size;
	if (spec->kind != XDPGPU_POOL_IMIX && (S < 64 || S > 9728))
		return -EINVAL;

	/* descriptor addresses (prefix sum of strides) */
	uint64_t off = 0;
	for (uint32_t i = 0; i < n; i++) {
		uint32_t sz = frame_size_of(spec, i);
		uint32_t st = stride_for(spec, sz);
		if (st < sz + spec->headroom)
			return -EINVAL;
		descs[i].addr = off + spec->headroom;
		descs[i].len = sz;
		descs[i].options = 0;
		off += st;
	}
	if (off > umem_size)
		return -ENOSPC;

	if (!random) {
		/* replicate one base frame */
		uint8_t base[9728];
		uint32_t len = gen_base_frame(spec, base);
		for (uint32_t i = 0; i < n; i++) {
			memcpy(umem + descs[i].addr, base, S);
			descs[i].len = len;
			if (expect)
				expect[i] = E_REDIRECT;
		}
		return 0;
	}

	uint32_t threads = spec->threads;
	if (!threads)
		threads = std::thread::hardware_concurrency();
	if (threads < 1)
		threads = 1;
	if (threads > 64)
		threads = 64;
	if (n < 65536)
		threads = 1;
	auto work = [&](uint32_t lo, uint32_t hi) {
		for (uint32_t i = lo; i < hi; i++) {
			uint8_t e;
			uint32_t sz = frame_size_of(spec, i);
			descs[i].len = nat64 ?
				gen_nat64_frame(spec, i, umem + descs[i].addr, sz, &e) :
				gen_random_frame(spec, i, umem + descs[i].addr, sz, &e);
			if (expect)
				expect[i] = e;
		}
	};
	if (threads == 1) {
		work(0, n);
	} else {
		std::vector<std::thread> th;
		uint32_t per = (n + threads - 1) / threads;
		for (uint32_t t = 0; t < threads; t++) {
			uint32_t lo = t * per, hi = lo + per;
			if (lo > n)
				lo = n;
			if (hi > n)
				hi = n;
			th.emplace_back(work, lo, hi);
		}
		for (auto &x : th)
			x.join();
	}
	return 0;
}

} // extern "C"
