// SPDX-License-Identifier: GPL-2.0
/*
 * nat64_oracle.c - TEST INFRASTRUCTURE ONLY: the parity oracle of the
 * nat64 transform (xdpgpu_nat64_dev).
 *
 * A plain-C restatement of nat64-bpf/nat64_kern.c, function by function,
 * operating on UMEM frames instead of an sk_buff.  nat64_kern.c is a BPF
 * program (it needs a BPF target, libbpf's bpf_helpers.h and the kernel's
 * helpers), so it cannot be built here; nothing of it is copied.  Two things
 * it calls live outside the reference and are restated from their published
 * semantics:
 *   - bpf_csum_diff(from, n, to, m, seed) (bpf.h:2321-2346): csum_partial
 *     of the 32-bit words ~from[..], to[..] plus seed;
 *   - bpf_l4_csum_replace(skb, off, from, to, flags) (bpf.h:1880-1910):
 *     size 0: *c = csum_fold(csum_add(to, ~csum_unfold(*c)));
 *     size 2/4: *c = csum_fold(csum_partial({~from, to}, 8, ~csum_unfold(*c)));
 *     BPF_F_MARK_MANGLED_0: a stored 0 is left alone, a 0 result becomes
 *     0xffff.
 * Every operand of a csum_fold here is nonzero (~csum_unfold(c) has its
 * high 16 bits set), so each result is fixed by its value mod 0xffff:
 * c' = ~F((~c + delta) mod 0xffff) with F(0) = 0xffff.  That is what
 * nat64_upd() computes.  Parity of this part is pinned by the RFC 6052
 * address vectors and by full checksum recomputation of every translated
 * frame in the tests, not by a reference build ("parity unpinned" at the
 * kernel-helper boundary).
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

static inline uint16_t be16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }
static inline uint32_t be32(const uint8_t *p)
{
	return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
}
static inline void put_be16(uint8_t *p, uint16_t v) { p[0] = v >> 8; p[1] = v & 0xff; }
static inline void put_be32(uint8_t *p, uint32_t v)
{
	p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}
static inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }
static inline void put_le16(uint8_t *p, uint16_t v) { p[0] = v & 0xff; p[1] = v >> 8; }

/* sum of the little-endian 16-bit words of n (even) bytes, mod 0xffff */
static uint32_t words_mod(const uint8_t *p, int n)
{
	uint64_t s = 0;
	for (int i = 0; i < n; i += 2)
		s += le16(p + i);
	return (uint32_t)(s % 0xffff);
}

/* bpf_csum_diff(from, fn, to, tn, 0) mod 0xffff (~w == -w mod 0xffff) */
static uint32_t csum_diff_mod(const uint8_t *from, int fn, const uint8_t *to, int tn)
{
	uint32_t f = fn ? words_mod(from, fn) : 0, t = tn ? words_mod(to, tn) : 0;
	return (t + 0xffff - f) % 0xffff;
}

/* one bpf_l4_csum_replace on the stored checksum c with a diff mod 0xffff */
static uint16_t nat64_upd(uint16_t c, uint32_t delta)
{
	uint32_t v = ((uint32_t)(~c & 0xffff) % 0xffff + delta) % 0xffff;
	uint32_t f = v ? v : 0xffff;
	return (uint16_t)(~f & 0xffff);
}

/* bpf_l4_csum_replace(skb, off, 0, diff, flags) on the checksum at c */
static void l4_csum_replace(uint8_t *c, uint32_t delta, int mangled0)
{
	uint16_t v = le16(c);
	if (mangled0 && v == 0)
		return;
	v = nat64_upd(v, delta);
	if (mangled0 && v == 0)
		v = 0xffff;
	put_le16(c, v);
}

/* v4addr_to_v6 (nat64_kern.c:180-243), addresses as wire bytes */
int oracle_v4addr_to_v6(const uint8_t a4[4], uint8_t a6[16], const uint8_t pref[16],
			int plen)
{
	memset(a6, 0, 16);
	switch (plen) {
	case 96: memcpy(a6, pref, 12); memcpy(a6 + 12, a4, 4); break;
	case 64: memcpy(a6, pref, 8); a6[9] = a4[0]; a6[10] = a4[1]; a6[11] = a4[2]; a6[12] = a4[3]; break;
	case 56: memcpy(a6, pref, 8); a6[7] = a4[0]; a6[9] = a4[1]; a6[10] = a4[2]; a6[11] = a4[3]; break;
	case 48: memcpy(a6, pref, 6); a6[6] = a4[0]; a6[7] = a4[1]; a6[9] = a4[2]; a6[10] = a4[3]; break;
	case 40: memcpy(a6, pref, 5); a6[5] = a4[0]; a6[6] = a4[1]; a6[7] = a4[2]; a6[9] = a4[3]; break;
	case 32: memcpy(a6, pref, 4); memcpy(a6 + 4, a4, 4); break;
	default: return 0;
	}
	return 1;
}

/* v6addr_to_v4 (nat64_kern.c:249-323) */
int oracle_v6addr_to_v4(const uint8_t a6[16], int plen, uint8_t a4[4], uint8_t pref[16])
{
	memset(pref, 0, 16);
	switch (plen) {
	case 96: memcpy(a4, a6 + 12, 4); memcpy(pref, a6, 12); break;
	case 64: a4[0] = a6[9]; a4[1] = a6[10]; a4[2] = a6[11]; a4[3] = a6[12]; memcpy(pref, a6, 8); break;
	case 56: a4[0] = a6[7]; a4[1] = a6[9]; a4[2] = a6[10]; a4[3] = a6[11]; memcpy(pref, a6, 8); pref[7] = 0; break;
	case 48: a4[0] = a6[6]; a4[1] = a6[7]; a4[2] = a6[9]; a4[3] = a6[10]; memcpy(pref, a6, 8); pref[6] = pref[7] = 0; break;
	case 40: a4[0] = a6[5]; a4[1] = a6[6]; a4[2] = a6[7]; a4[3] = a6[9]; memcpy(pref, a6, 8); pref[6] = pref[7] = 0; pref[5] = 0; break;
	case 32: memcpy(a4, a6 + 4, 4); memcpy(pref, a6, 4); break;
	default: return 0;
	}
	return 1;
}

/* the static state tables (v6_state_map / v4_reversemap, nat64_kern.c:17-31) */
static const struct xdpgpu_nat64_map *find_v6(const struct xdpgpu_nat64_map *map,
					      uint32_t nmap, const uint8_t *v6)
{
	for (uint32_t i = 0; i < nmap; i++)
		if (!memcmp(map[i].v6, v6, 16))
			return &map[i];
	return NULL;
}

static const struct xdpgpu_nat64_map *find_v4(const struct xdpgpu_nat64_map *map,
					      uint32_t nmap, uint32_t v4)
{
	for (uint32_t i = 0; i < nmap; i++)
		if (map[i].v4 == v4)
			return &map[i];
	return NULL;
}

/* allowed_v6_src: an LPM trie with the one configured entry */
static int lpm_match(const uint8_t *addr, const uint8_t *pref, uint32_t plen)
{
	if (!plen)
		return 0;
	for (uint32_t b = 0; b < plen; b++) {
		int bit = 7 - (b & 7);
		if (((addr[b >> 3] >> bit) & 1) != ((pref[b >> 3] >> bit) & 1))
			return 0;
	}
	return 1;
}

/* parse_ethhdr (parsing_helpers.h:86-137): next EtherType, or -1 */
static int eth_type(const uint8_t *p, uint32_t len, uint32_t *off)
{
	if (len < 14)
		return -1;
	uint32_t pos = 14;
	uint16_t proto = be16(p + 12);
	for (int i = 0; i < 2; i++) {
		if (proto != 0x8100 && proto != 0x88A8)
			break;
		if (pos + 4 > len)
			break;
		proto = be16(p + pos + 2);
		pos += 4;
	}
	*off = pos;
	return proto;
}

/* skip_ip6hdrext (parsing_helpers.h:139-172) */
static int skip_ext(const uint8_t *p, uint32_t len, uint32_t *pos, int nh)
{
	for (int i = 0; i < 6; i++) {
		if (*pos + 2 > len)
			return -1;
		switch (nh) {
		case 0: case 60: case 43: case 135:
			nh = p[*pos];
			*pos += (p[*pos + 1] + 1) * 8;
			break;
		case 51:
			nh = p[*pos];
			*pos += (p[*pos + 1] + 2) * 4;
			break;
		case 44:
			nh = p[*pos];
			*pos += 8;
			break;
		default:
			return nh;
		}
	}
	return -1;
}

/* update_icmp_checksum (nat64_kern.c:120-158): pseudo header added or
 * removed, then the type/code word and the rest-of-header word */
static void icmp_csum(uint8_t *icmp_after, const uint8_t *before, const uint8_t *v6hdr,
		      int add)
{
	uint8_t ph[40];
	memcpy(ph, v6hdr + 8, 32);           /* saddr, daddr */
	/* .len = ip6h->payload_len: a __be16 stored in a __u32 */
	ph[32] = v6hdr[4]; ph[33] = v6hdr[5]; ph[34] = 0; ph[35] = 0;
	ph[36] = ph[37] = ph[38] = 0; ph[39] = 58;
	uint32_t d = add ? csum_diff_mod(NULL, 0, ph, 40) : csum_diff_mod(ph, 40, NULL, 0);
	uint8_t *c = icmp_after + 2;
	l4_csum_replace(c, d, 0);
	/* bpf_l4_csum_replace(skb, off, h_before, h_after, 2) */
	l4_csum_replace(c, csum_diff_mod(before, 2, icmp_after, 2), 0);
	if (memcmp(before + 4, icmp_after + 4, 4))
		l4_csum_replace(c, csum_diff_mod(before + 4, 4, icmp_after + 4, 4), 0);
}

/* rewrite_icmpv6 (nat64_kern.c:644-739): ICMPv6 header at h (8 bytes
 * present), translated in place; v6hdr is the original IPv6 header */
static int rewrite_icmpv6(uint8_t *h, const uint8_t *v6hdr)
{
	uint8_t old[8], n[8];
	memcpy(old, h, 8);
	memcpy(n, h, 8);
	uint32_t mtu, ptr;
	switch (old[0]) {
	case 128: n[0] = 8; break;
	case 129: n[0] = 0; break;
	case 1:
		n[0] = 3;
		switch (old[1]) {
		case 0: case 2: case 3: n[1] = 1; break;
		case 1: n[1] = 10; break;
		case 4: n[1] = 3; break;
		default: return -1;
		}
		break;
	case 2:
		n[0] = 3; n[1] = 4;
		mtu = be32(old + 4) - 20;
		if (mtu > 0xffff)
			return -1;
		put_be16(n + 6, (uint16_t)mtu);
		break;
	case 3: n[0] = 11; break;
	case 4:
		switch (old[1]) {
		case 0:
			n[0] = 12; n[1] = 0;
			ptr = be32(old + 4);
			if (ptr == 0 || ptr == 1) n[4] = (uint8_t)ptr;
			else if (ptr == 4 || ptr == 5) n[4] = 2;
			else if (ptr == 6) n[4] = 9;
			else if (ptr == 7) n[4] = 8;
			else if (ptr >= 8 && ptr <= 23) n[4] = 12;
			else if (ptr >= 24 && ptr <= 39) n[4] = 16;
			else return -1;
			break;
		case 1: n[0] = 3; n[1] = 2; break;
		default: return -1;
		}
		break;
	default: return -1;
	}
	memcpy(h, n, 8);
	icmp_csum(h, old, v6hdr, 0);
	return 0;
}

/* rewrite_icmp (nat64_kern.c:325-441); v6hdr is the new IPv6 header */
static int rewrite_icmp(uint8_t *h, const uint8_t *v6hdr)
{
	uint8_t old[8], n[8];
	memcpy(old, h, 8);
	memcpy(n, h, 8);
	uint32_t mtu;
	switch (old[0]) {
	case 8: n[0] = 128; break;
	case 0: n[0] = 129; break;
	case 3:
		n[0] = 1;
		switch (old[1]) {
		case 0: case 1: case 5: case 6: case 7: case 8: case 11: case 12:
			n[1] = 0; break;
		case 2: n[0] = 4; n[1] = 1; put_be32(n + 4, 6); break;
		case 3: n[1] = 4; break;
		case 4:
			n[0] = 2; n[1] = 0;
			mtu = be16(old + 6) + 20;
			if (mtu < 1280)
				mtu = 1280;
			put_be32(n + 4, mtu);
			break;
		case 9: case 10: case 13: case 15: n[1] = 1; break;
		default: return -1;
		}
		break;
	case 12:
		if (old[1] == 1)
			return -1;
		n[0] = 4; n[1] = 0;
		switch (old[4]) {
		case 0: put_be32(n + 4, 0); break;
		case 1: put_be32(n + 4, 1); break;
		case 2: case 3: put_be32(n + 4, 4); break;
		case 8: put_be32(n + 4, 7); break;
		case 9: put_be32(n + 4, 6); break;
		case 12: case 13: case 14: case 15: put_be32(n + 4, 8); break;
		case 16: case 17: case 18: case 19: put_be32(n + 4, 24); break;
		default: return -1;
		}
		break;
	default: return -1;
	}
	memcpy(h, n, 8);
	icmp_csum(h, old, v6hdr, 1);
	return 0;
}

/* update_l4_checksum (nat64_kern.c:83-118): the address part of the
 * pseudo header swapped; c is the checksum field */
static void l4_addr_update(uint8_t *c, int proto, const uint8_t *from, int fn,
			   const uint8_t *to, int tn)
{
	l4_csum_replace(c, csum_diff_mod(from, fn, to, tn), proto == 17);
}

/* nat64_handle_v6 (nat64_kern.c:741-873) on one frame */
static int handle_v6(uint8_t *umem, uint64_t eff, uint32_t len, uint32_t l3,
		     const struct xdpgpu_nat64_cfg *cfg,
		     const struct xdpgpu_nat64_map *map, uint32_t nmap,
		     struct xdpgpu_desc *out)
{
	uint8_t *p = umem + eff;
	if (l3 + 40 > len || (p[l3] >> 4) != 6)
		return XDPGPU_TC_ACT_OK;               /* parse_ip6hdr */
	uint32_t pos = l3 + 40;
	const int nexthdr = p[l3 + 6];
	const int ip_type = skip_ext(p, len, &pos, nexthdr);
	if (ip_type < 0)
		return XDPGPU_TC_ACT_OK;
	uint8_t a4[4], pref[16];
	if (!oracle_v6addr_to_v4(p + l3 + 24, (int)cfg->v6_plen, a4, pref))
		return XDPGPU_TC_ACT_OK;
	if (memcmp(pref, cfg->v6_prefix, 16))
		return XDPGPU_TC_ACT_OK;
	if (ip_type != nexthdr)
		return XDPGPU_TC_ACT_SHOT;
	const uint32_t d4 = be32(a4);
	if (!d4 || (d4 & 0xFF000000u) == 0x7F000000u || (d4 & 0xF0000000u) == 0xE0000000u)
		return XDPGPU_TC_ACT_SHOT;
	if (!lpm_match(p + l3 + 8, cfg->allow_prefix, cfg->allow_plen))
		return XDPGPU_TC_ACT_SHOT;
	const struct xdpgpu_nat64_map *st = find_v6(map, nmap, p + l3 + 8);
	if (!st)
		return XDPGPU_NAT64_NO_STATE;

	/* the new IPv4 header */
	uint8_t h4[20];
	memset(h4, 0, 20);
	h4[0] = 0x45;
	h4[1] = (uint8_t)(((p[l3] & 0x0f) << 4) | (p[l3 + 1] >> 4));
	put_be16(h4 + 2, (uint16_t)(be16(p + l3 + 4) + 20));
	put_be16(h4 + 6, 0x4000);
	h4[8] = p[l3 + 7];
	h4[9] = (uint8_t)nexthdr;
	put_be32(h4 + 12, st->v4);
	memcpy(h4 + 16, a4, 4);

	const uint32_t l4 = l3 + 40;
	switch (nexthdr) {
	case 58:
		if (l4 + 8 > len)
			return XDPGPU_TC_ACT_SHOT;
		{
			uint8_t h6[40];
			memcpy(h6, p + l3, 40);
			if (rewrite_icmpv6(p + l4, h6))
				return XDPGPU_TC_ACT_SHOT;
		}
		h4[9] = 1;
		break;
	case 6: case 17: {
		const uint32_t co = l4 + (nexthdr == 6 ? 16 : 6);
		/* bpf_l4_csum_replace fails (-EFAULT, ignored) past the end */
		if (co + 2 <= len)
			l4_addr_update(p + co, nexthdr, p + l3 + 8, 32, h4 + 12, 8);
		break;
	}
	default:
		break;
	}
	/* csum_fold_helper(bpf_csum_diff(0, 0, hdr, 20, 0)) */
	{
		uint64_t s = 0;
		for (int i = 0; i < 20; i += 2)
			s += le16(h4 + i);
		while (s >> 16)
			s = (s & 0xffff) + (s >> 16);
		put_le16(h4 + 10, (uint16_t)~s);
	}
	/* bpf_skb_change_proto: 20 bytes fewer in front of the network
	 * header; the L2 header moves, its h_proto becomes 0x0800 */
	uint8_t l2[22];
	memcpy(l2, p, l3);
	uint8_t *q = p + 20;
	memcpy(q, l2, l3);
	q[12] = 0x08; q[13] = 0x00;
	memcpy(q + l3, h4, 20);
	out->addr = eff + 20;
	out->len = len - 20;
	return XDPGPU_TC_ACT_REDIRECT;
}

/* nat64_handle_v4 (nat64_kern.c:443-541) on one frame */
static int handle_v4(uint8_t *umem, uint64_t eff, uint32_t len, uint32_t l3,
		     const struct xdpgpu_nat64_cfg *cfg,
		     const struct xdpgpu_nat64_map *map, uint32_t nmap,
		     struct xdpgpu_desc *out)
{
	uint8_t *p = umem + eff;
	if (l3 + 20 > len || (p[l3] >> 4) != 4)
		return XDPGPU_TC_ACT_OK;               /* parse_iphdr */
	const uint32_t ihl = (p[l3] & 0xf) * 4;
	if (ihl < 20 || l3 + ihl > len)
		return XDPGPU_TC_ACT_OK;
	const uint32_t d4 = be32(p + l3 + 16);
	if ((d4 & cfg->v4_mask) != cfg->v4_prefix)
		return XDPGPU_TC_ACT_OK;
	if (ihl != 20 || (be16(p + l3 + 6) & ~0x4000u))
		return XDPGPU_TC_ACT_SHOT;
	const struct xdpgpu_nat64_map *st = find_v4(map, nmap, d4);
	if (!st)
		return XDPGPU_TC_ACT_SHOT;
	uint8_t h6[40];
	memset(h6, 0, 40);
	if (!oracle_v4addr_to_v6(p + l3 + 12, h6 + 8, cfg->v6_prefix, (int)cfg->v6_plen))
		return XDPGPU_TC_ACT_SHOT;
	memcpy(h6 + 24, st->v6, 16);
	const uint8_t tos = p[l3 + 1], proto = p[l3 + 9];
	/* struct ipv6hdr on little-endian: priority:4 is the low nibble */
	h6[0] = (uint8_t)(6 << 4 | ((tos & 0x70) >> 4));
	h6[1] = (uint8_t)(tos << 4);
	put_be16(h6 + 4, (uint16_t)(be16(p + l3 + 2) - 20));
	h6[6] = proto;
	h6[7] = p[l3 + 8];
	if (eff < 20)
		return XDPGPU_TC_ACT_SHOT;             /* no headroom to grow */
	const uint32_t l4 = l3 + 20;
	switch (proto) {
	case 1:
		if (l4 + 8 > len)
			return XDPGPU_TC_ACT_SHOT;
		if (rewrite_icmp(p + l4, h6))
			return XDPGPU_TC_ACT_SHOT;
		h6[6] = 58;
		break;
	case 6: case 17: {
		const uint32_t co = l4 + (proto == 6 ? 16 : 6);
		if (co + 2 <= len)
			l4_addr_update(p + co, proto, p + l3 + 12, 8, h6 + 8, 32);
		break;
	}
	default:
		break;
	}
	uint8_t l2[22];
	memcpy(l2, p, l3);
	uint8_t *q = p - 20;
	memcpy(q, l2, l3);
	q[12] = 0x86; q[13] = 0xDD;
	memcpy(q + l3, h6, 40);
	out->addr = eff - 20;
	out->len = len + 20;
	return XDPGPU_TC_ACT_REDIRECT;
}

/* nat64_handler (nat64_kern.c:875-890) over a batch */
int oracle_nat64(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		 uint32_t n, const struct xdpgpu_nat64_cfg *cfg,
		 const struct xdpgpu_nat64_map *map, uint32_t nmap,
		 uint8_t *action, struct xdpgpu_desc *out)
{
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t addr = descs[i].addr;
		const uint32_t len = descs[i].len;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		out[i] = descs[i];
		if ((uint64_t)len > umem_size || eff > umem_size - len) {
			action[i] = XDPGPU_TC_ACT_SHOT;
			continue;
		}
		uint32_t l3 = 0;
		const int et = eth_type(umem + eff, len, &l3);
		int act = XDPGPU_TC_ACT_OK;
		if (cfg->direction == XDPGPU_NAT64_EGRESS && et == 0x0800)
			act = handle_v4(umem, eff, len, l3, cfg, map, nmap, &out[i]);
		else if (cfg->direction == XDPGPU_NAT64_INGRESS && et == 0x86DD)
			act = handle_v6(umem, eff, len, l3, cfg, map, nmap, &out[i]);
		if (act == XDPGPU_TC_ACT_REDIRECT)
			out[i].options = descs[i].options;
		action[i] = (uint8_t)act;
	}
	return 0;
}
