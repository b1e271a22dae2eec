// SPDX-License-Identifier: GPL-2.0
/*
 * xdp_oracle.c - TEST INFRASTRUCTURE ONLY: the parity oracle.
 *
 * A plain-C restatement of the reference algorithms on the AF_XDP receive
 * path, loop for loop where the reference has loops, so that every output of
 * the HIP kernels (bpf-examples_amd/csrc/) can be compared bit-exactly on the
 * same frames.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (as oracle/liboracle.so); the product never does.
 *
 * Pinning: the checksum and jhash primitives below are checked against the
 * reference headers themselves (oracle/_ref/libref.so built by
 * oracle/Makefile from AF_XDP-interaction/lib_checksum.h and
 * include/jhash.h) and against the golden vectors in tests/golden/.
 * include/xdp/parsing_helpers.h cannot be built here (it needs libbpf's
 * bpf/bpf_endian.h; lib/libbpf is an empty submodule), so the parse
 * restatement is pinned by the hand-built fixture frames of
 * tests/golden/make_golden.py, whose expected offsets/verdicts are written
 * independently of this file.  See DESIGN.md "Oracle".
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "oracle.h"

/* ------------------------------------------------------------------ */
/* byte access                                                         */

static inline uint16_t ld_be16(const uint8_t *p)
{
	return (uint16_t)((p[0] << 8) | p[1]);
}

static inline uint16_t ld_le16(const uint8_t *p)
{
	return (uint16_t)(p[0] | (p[1] << 8));
}

static inline uint32_t ld_le32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) |
	       ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline void st_le16(uint8_t *p, uint16_t v)
{
	p[0] = (uint8_t)v;
	p[1] = (uint8_t)(v >> 8);
}

/* ------------------------------------------------------------------ */
/* Checksums: AF_XDP-interaction/lib_checksum.h                        */

/* lib_checksum.h:27-34 */
static inline uint32_t fold_to_16(uint32_t x)
{
	x = (x & 0xffff) + (x >> 16);
	x = (x & 0xffff) + (x >> 16);
	return x;
}

/*
 * lib_checksum.h:40-95 (Linux lib/checksum.c do_csum), little-endian
 * branch.  The code path depends on the buffer's address (odd start, 2-byte
 * step, 32-bit carry loop); the result does not.  Kept path-faithful so the
 * CPU baseline does the reference's work.
 */
uint32_t oracle_do_csum(const uint8_t *buf, int len)
{
	uint32_t acc = 0;
	int odd_start;

	if (len <= 0)
		return 0;
	odd_start = (int)((uintptr_t)buf & 1);
	if (odd_start) {
		acc += (uint32_t)buf[0] << 8;   /* LE: first byte is a high byte */
		buf++;
		len--;
	}
	if (len >= 2) {
		if ((uintptr_t)buf & 2) {
			acc += ld_le16(buf);
			buf += 2;
			len -= 2;
		}
		if (len >= 4) {
			const uint8_t *stop = buf + ((unsigned int)len & ~3u);
			uint32_t cy = 0;

			while (buf < stop) {
				uint32_t w = ld_le32(buf);

				buf += 4;
				acc += cy;
				acc += w;
				cy = (w > acc);
			}
			acc += cy;
			acc = (acc & 0xffff) + (acc >> 16);
		}
		if (len & 2) {
			acc += ld_le16(buf);
			buf += 2;
		}
	}
	if (len & 1)
		acc += buf[0];                 /* LE: trailing byte is a low byte */
	acc = fold_to_16(acc);
	if (odd_start)
		acc = ((acc >> 8) & 0xff) | ((acc & 0xff) << 8);
	return acc;
}

/* lib_checksum.h:103-106 */
uint16_t oracle_ip_fast_csum(const uint8_t *iph, unsigned int ihl)
{
	return (uint16_t)~oracle_do_csum(iph, (int)(ihl * 4));
}

/* lib_checksum.h:113-120 */
uint16_t oracle_csum_fold(uint32_t csum)
{
	csum = (csum & 0xffff) + (csum >> 16);
	csum = (csum & 0xffff) + (csum >> 16);
	return (uint16_t)~csum;
}

/* lib_checksum.h:126-133 */
static inline uint32_t fold64_to_32(uint64_t x)
{
	x = (x & 0xffffffffull) + (x >> 32);
	x = (x & 0xffffffffull) + (x >> 32);
	return (uint32_t)x;
}

/* lib_checksum.h:142-155, little-endian branch (__BIG_ENDIAN__ unset) */
uint32_t oracle_csum_tcpudp_nofold(uint32_t saddr, uint32_t daddr, uint32_t len,
				   uint8_t proto, uint32_t sum)
{
	uint64_t s = sum;

	s += saddr;
	s += daddr;
	s += (uint64_t)((proto + len) << 8);
	return fold64_to_32(s);
}

/* lib_checksum.h:161-166 */
uint16_t oracle_csum_tcpudp_magic(uint32_t saddr, uint32_t daddr, uint32_t len,
				  uint8_t proto, uint32_t sum)
{
	return oracle_csum_fold(
		oracle_csum_tcpudp_nofold(saddr, daddr, len, proto, sum));
}

/* lib_checksum.h:168-179: 16-bit words into an unfolded u32.  For odd len
 * the last word takes one byte past the L4 end (caller provides it). */
uint16_t oracle_udp_csum(uint32_t saddr, uint32_t daddr, uint32_t len,
			 uint8_t proto, const uint8_t *l4)
{
	uint32_t csum = 0;
	uint32_t cnt;

	for (cnt = 0; cnt < len; cnt += 2)
		csum += ld_le16(l4 + cnt);
	return oracle_csum_tcpudp_magic(saddr, daddr, len, proto, csum);
}

/* xdp-synproxy/xdp_synproxy_kern.c:149-172: IPv6 pseudo header */
uint16_t oracle_csum_ipv6_magic(const uint8_t *saddr, const uint8_t *daddr,
				uint32_t len, uint8_t proto, uint32_t csum)
{
	uint64_t sum = csum;
	int i;

	for (i = 0; i < 4; i++)
		sum += ld_le32(saddr + 4 * i);
	for (i = 0; i < 4; i++)
		sum += ld_le32(daddr + 4 * i);
	sum += __builtin_bswap32(len);
	sum += __builtin_bswap32((uint32_t)proto);
	sum = (sum & 0xffffffffull) + (sum >> 32);
	sum = (sum & 0xffffffffull) + (sum >> 32);
	return oracle_csum_fold((uint32_t)sum);
}

/* af_xdp_user.c:590-606: RFC 1624 style 16-bit incremental update */
static inline uint16_t c16_add(uint16_t csum, uint16_t addend)
{
	uint16_t r = (uint16_t)(csum + addend);

	return (uint16_t)(r + (r < addend));
}

uint16_t oracle_csum_replace2(uint16_t sum, uint16_t old, uint16_t new_)
{
	uint16_t t = c16_add((uint16_t)~sum, (uint16_t)~old);

	return (uint16_t)~c16_add(t, new_);
}

/* ------------------------------------------------------------------ */
/* jhash: include/jhash.h (Bob Jenkins lookup3, Linux 4.18 copy)        */

#define JH_INIT 0xdeadbeefu   /* jhash.h:54 */

static inline uint32_t rotl32(uint32_t w, unsigned int s)
{
	return (w << s) | (w >> ((-s) & 31));          /* jhash.h:25-28 */
}

static inline void jh_mix(uint32_t *a, uint32_t *b, uint32_t *c)
{                                                   /* jhash.h:33-41 */
	*a -= *c; *a ^= rotl32(*c, 4);  *c += *b;
	*b -= *a; *b ^= rotl32(*a, 6);  *a += *c;
	*c -= *b; *c ^= rotl32(*b, 8);  *b += *a;
	*a -= *c; *a ^= rotl32(*c, 16); *c += *b;
	*b -= *a; *b ^= rotl32(*a, 19); *a += *c;
	*c -= *b; *c ^= rotl32(*b, 4);  *b += *a;
}

static inline void jh_final(uint32_t *a, uint32_t *b, uint32_t *c)
{                                                   /* jhash.h:43-52 */
	*c ^= *b; *c -= rotl32(*b, 14);
	*a ^= *c; *a -= rotl32(*c, 11);
	*b ^= *a; *b -= rotl32(*a, 25);
	*c ^= *b; *c -= rotl32(*b, 16);
	*a ^= *c; *a -= rotl32(*c, 4);
	*b ^= *a; *b -= rotl32(*a, 14);
	*c ^= *b; *c -= rotl32(*b, 24);
}

/* jhash.h:68-105: byte-key version, 12-byte blocks while more than 12
 * bytes remain, then a 1..12 byte tail; an empty tail skips the final. */
uint32_t oracle_jhash(const void *key, uint32_t length, uint32_t initval)
{
	const uint8_t *k = (const uint8_t *)key;
	uint32_t a, b, c;

	a = b = c = JH_INIT + length + initval;
	while (length > 12) {
		a += ld_le32(k);
		b += ld_le32(k + 4);
		c += ld_le32(k + 8);
		jh_mix(&a, &b, &c);
		length -= 12;
		k += 12;
	}
	if (length == 0)
		return c;
	/* tail bytes, each at its little-endian lane of a, b or c */
	{
		uint32_t t[3] = { 0, 0, 0 };
		uint32_t i;

		for (i = 0; i < length; i++)
			t[i >> 2] += (uint32_t)k[i] << (8 * (i & 3));
		a += t[0];
		b += t[1];
		c += t[2];
	}
	jh_final(&a, &b, &c);
	return c;
}

/* jhash.h:114-142 */
uint32_t oracle_jhash2(const uint32_t *k, uint32_t length, uint32_t initval)
{
	uint32_t a, b, c;

	a = b = c = JH_INIT + (length << 2) + initval;
	while (length > 3) {
		a += k[0];
		b += k[1];
		c += k[2];
		jh_mix(&a, &b, &c);
		length -= 3;
		k += 3;
	}
	if (length == 0)
		return c;
	if (length == 3)
		c += k[2];
	if (length >= 2)
		b += k[1];
	a += k[0];
	jh_final(&a, &b, &c);
	return c;
}

/* jhash.h:146-160 */
uint32_t oracle_jhash_3words(uint32_t a, uint32_t b, uint32_t c, uint32_t initval)
{
	uint32_t iv = initval + JH_INIT + (3 << 2);

	a += iv;
	b += iv;
	c += iv;
	jh_final(&a, &b, &c);
	return c;
}

/* ------------------------------------------------------------------ */
/* Header parsers: include/xdp/parsing_helpers.h, with a byte offset as
 * the cursor and `end` = desc.len as data_end.  Return -1 on failure.  */

#define P_8021Q  0x8100
#define P_8021AD 0x88A8
#define P_ARP    0x0806
#define P_IPV4   0x0800
#define P_IPV6   0x86DD

/* parsing_helpers.h:86-129, VLAN_MAX_DEPTH = 2 (:60-62).  Returns the
 * EtherType in host order (the reference returns it in network order and
 * compares against bpf_htons constants; same decision). */
static int parse_eth(const uint8_t *p, uint32_t end, uint32_t *cur,
		     int *nvlan, uint16_t *vid0)
{
	uint32_t c = 14;
	uint16_t proto;
	int i;

	if (end < 14)
		return -1;
	proto = ld_be16(p + 12);
	*nvlan = 0;
	for (i = 0; i < 2; i++) {
		if (proto != P_8021Q && proto != P_8021AD)  /* :75-79 */
			break;
		if (c + 4 > end)
			break;
		if (i == 0)
			*vid0 = ld_be16(p + c) & 0x0fff;
		proto = ld_be16(p + c + 2);
		c += 4;
		(*nvlan)++;
	}
	*cur = c;
	return proto;
}

/* parsing_helpers.h:174-194 + skip_ip6hdrext :139-172,
 * IPV6_EXT_MAX_CHAIN = 6 (:65-67).  Every iteration first requires the
 * 2-byte ipv6_opt_hdr to be inside the frame, even for the final
 * (non-extension) header; six extension headers exhaust the loop (-1). */
static int parse_ip6(const uint8_t *p, uint32_t end, uint32_t l3,
		     uint32_t *cur, int64_t *frag_at)
{
	uint32_t c;
	uint8_t nh;
	int i;

	if (l3 + 40 > end)
		return -1;
	if ((p[l3] >> 4) != 6)
		return -1;
	c = l3 + 40;
	nh = p[l3 + 6];
	for (i = 0; i < 6; i++) {
		if (c + 2 > end)
			return -1;
		switch (nh) {
		case 0:   /* IPPROTO_HOPOPTS */
		case 60:  /* IPPROTO_DSTOPTS */
		case 43:  /* IPPROTO_ROUTING */
		case 135: /* IPPROTO_MH */
			nh = p[c];
			c += ((uint32_t)p[c + 1] + 1) * 8;
			break;
		case 51:  /* IPPROTO_AH */
			nh = p[c];
			c += ((uint32_t)p[c + 1] + 2) * 4;
			break;
		case 44:  /* IPPROTO_FRAGMENT */
			*frag_at = c;
			nh = p[c];
			c += 8;
			break;
		default:
			*cur = c;
			return nh;
		}
	}
	return -1;
}

/* parsing_helpers.h:196-222 (tot_len, frag and checksum not checked) */
static int parse_ip4(const uint8_t *p, uint32_t end, uint32_t l3)
{
	uint32_t hl;

	if (l3 + 20 > end)
		return -1;
	if ((p[l3] >> 4) != 4)
		return -1;
	hl = (uint32_t)(p[l3] & 0x0f) * 4;
	if (hl < 20)
		return -1;
	if (l3 + hl > end)
		return -1;
	return p[l3 + 9];
}

/* parsing_helpers.h:224-252: icmphdr and icmp6hdr are both 8 bytes */
static int parse_icmp_any(const uint8_t *p, uint32_t end, uint32_t l4)
{
	if (l4 + 8 > end)
		return -1;
	return p[l4];
}

/* parsing_helpers.h:272-290 */
static int parse_udp(const uint8_t *p, uint32_t end, uint32_t l4)
{
	int len;

	if (l4 + 8 > end)
		return -1;
	len = (int)ld_be16(p + l4 + 4) - 8;
	if (len < 0)
		return -1;
	return len;
}

/* parsing_helpers.h:295-318 */
static int parse_tcp(const uint8_t *p, uint32_t end, uint32_t l4)
{
	uint32_t len;

	if (l4 + 20 > end)
		return -1;
	len = (uint32_t)(p[l4 + 12] >> 4) * 4;
	if (len < 20)
		return -1;
	if (l4 + len > end)
		return -1;
	return (int)len;
}

/* ------------------------------------------------------------------ */
/* The per-frame pipeline (verdict surface: SURVEY.md §8a a-V)          */

struct frame_out {
	uint8_t verdict;
	uint8_t l3_bad, l4_bad, l4_absent, frag;
	struct xdpgpu_result r;
	uint8_t key[44];           /* struct xdpgpu_network_tuple */
	uint16_t vid;
};

static void frame_pipeline(uint8_t *umem, uint64_t usize,
			   const struct xdpgpu_desc *d, uint32_t flags,
			   uint32_t initval, struct frame_out *o)
{
	uint64_t eff = (d->addr & ((1ull << 48) - 1)) + (d->addr >> 48);
	uint32_t end = d->len;
	uint8_t *p;
	uint32_t l3 = 0, l4 = 0, ip_end = 0, cl = 0, chk_off = 0;
	int nvlan = 0, ipv4, ipv6, nh = 0;
	int has_l4 = 0, has_csum = 0, nonfirst = 0, frag = 0;
	int l3_ok = 1, l4_ok = 0, absent = 0;
	int64_t frag_at = -1;
	uint16_t vid = 0;
	int et;

	memset(o, 0, sizeof(*o));
	o->verdict = XDPGPU_ABORTED;
	if ((uint64_t)end > usize || eff > usize - end)
		return;                           /* descriptor outside UMEM */
	p = umem + eff;

	et = parse_eth(p, end, &l3, &nvlan, &vid);
	if (et < 0)
		return;
	/* af_xdp_kern.c:114-148 parse_pkt__is_ARP_or_NDP, :178-183 */
	if (et == P_ARP) {
		o->verdict = XDPGPU_PASS;
		return;
	}
	ipv4 = (et == P_IPV4);
	ipv6 = (et == P_IPV6);
	if (ipv6) {
		nh = parse_ip6(p, end, l3, &l4, &frag_at);
		if (nh < 0)
			return;
		if (nh == 58) {
			int t = parse_icmp_any(p, end, l4);

			if (t < 0)
				return;
			if (t >= 133 && t <= 137) {        /* NDP */
				o->verdict = XDPGPU_PASS;
				return;
			}
		}
	}

	/* extended parse (build-defined): lengths, fragments, L4 */
	if (ipv6) {
		ip_end = l3 + 40 + ld_be16(p + l3 + 4);
		if (ip_end > end || l4 > ip_end)
			return;
		if (frag_at >= 0) {
			uint16_t fw = ld_be16(p + frag_at + 2);

			frag = 1;
			if (fw >> 3)
				nonfirst = 1;
		}
	} else if (ipv4) {
		uint32_t hl, tot;
		uint16_t fo;
		uint16_t chk3;

		nh = parse_ip4(p, end, l3);
		if (nh < 0)
			return;
		hl = (uint32_t)(p[l3] & 0x0f) * 4;
		tot = ld_be16(p + l3 + 2);
		if (tot < hl || l3 + tot > end)
			return;
		ip_end = l3 + tot;
		l4 = l3 + hl;
		fo = ld_be16(p + l3 + 6) & 0x3fff;
		if (fo) {
			frag = 1;
			if (fo & 0x1fff)
				nonfirst = 1;
		}
		/* recompute with the check word zeroed (af_xdp_user.c:664-665);
		 * verify = sum over the stored header (xdp_synproxy_kern.c:612) */
		l3_ok = (oracle_ip_fast_csum(p + l3, hl / 4) == 0);
		chk3 = ld_le16(p + l3 + 10);
		p[l3 + 10] = p[l3 + 11] = 0;
		o->r.l3_csum = oracle_ip_fast_csum(p + l3, hl / 4);
		st_le16(p + l3 + 10, chk3);
	}

	if ((ipv4 || ipv6) && !nonfirst) {
		if (nh == 17) {
			if (parse_udp(p, end, l4) < 0)
				return;
			has_l4 = 1;
			if (!frag) {
				cl = ld_be16(p + l4 + 4);
				if (l4 + cl > ip_end)
					return;
				chk_off = 6;
				has_csum = 1;
			}
		} else if (nh == 6) {
			int thl = parse_tcp(p, end, l4);

			if (thl < 0)
				return;
			has_l4 = 1;
			if (!frag) {
				cl = ip_end - l4;
				if (cl < (uint32_t)thl)
					return;
				chk_off = 16;
				has_csum = 1;
			}
		} else if ((nh == 1 && ipv4) || (nh == 58 && ipv6)) {
			if (parse_icmp_any(p, end, l4) < 0)
				return;
			has_l4 = 1;
			if (!frag) {
				cl = ip_end - l4;
				if (cl < 8)
					return;
				chk_off = 2;
				has_csum = 1;
			}
		}
	}

	if (has_csum) {
		/* Sum in place with the check word zeroed then restored (the
		 * generators' idiom, af_xdp_user.c:681-684); a copy only when the
		 * over-read byte would fall past the end of the UMEM. */
		static __thread uint8_t tmp[65536 + 4];
		uint32_t n_even = cl + (cl & 1);
		uint8_t *b = p + l4;
		uint16_t stored = ld_le16(p + l4 + chk_off);
		uint32_t i;

		if (eff + l4 + n_even > usize) {
			for (i = 0; i < n_even; i++) {
				uint64_t at = eff + l4 + i;

				tmp[i] = at < usize ? umem[at] : 0;
			}
			b = tmp;
		}
		if (ipv4 && nh != 1) {
			/* lib_checksum.h:168-179 (TCP uses proto 6) */
			uint32_t sa = ld_le32(p + l3 + 12), da = ld_le32(p + l3 + 16);

			l4_ok = (oracle_udp_csum(sa, da, cl, (uint8_t)nh, b) == 0);
			b[chk_off] = b[chk_off + 1] = 0;
			o->r.l4_csum = oracle_udp_csum(sa, da, cl, (uint8_t)nh, b);
			if (nh == 17 && stored == 0) {
				absent = 1;
				l4_ok = 1;
			}
		} else if (ipv4) {
			/* ICMP: ones-complement of the folded message sum */
			l4_ok = ((uint16_t)~oracle_do_csum(b, (int)cl) == 0);
			b[chk_off] = b[chk_off + 1] = 0;
			o->r.l4_csum = (uint16_t)~oracle_do_csum(b, (int)cl);
		} else {
			/* IPv6: csum_partial body (zero padded) + pseudo header,
			 * xdp_synproxy_kern.c:631-636 */
			const uint8_t *sa = p + l3 + 8, *da = p + l3 + 24;

			l4_ok = (oracle_csum_ipv6_magic(sa, da, cl, (uint8_t)nh,
					oracle_do_csum(b, (int)cl)) == 0);
			b[chk_off] = b[chk_off + 1] = 0;
			o->r.l4_csum = oracle_csum_ipv6_magic(sa, da, cl,
					(uint8_t)nh, oracle_do_csum(b, (int)cl));
		}
		st_le16(b + chk_off, stored);
	}

	/* result record */
	o->r.l3_off = (uint8_t)l3;
	o->r.nvlan = (uint8_t)nvlan;
	if (nvlan)
		o->r.flags |= XDPGPU_F_VLAN;
	o->vid = vid;
	if (ipv4 || ipv6) {
		o->r.flags |= XDPGPU_F_IP;
		if (ipv6)
			o->r.flags |= XDPGPU_F_IPV6;
		if (l3_ok)
			o->r.flags |= XDPGPU_F_L3_OK;
		if (frag)
			o->r.flags |= XDPGPU_F_FRAG;
		if (has_l4)
			o->r.flags |= XDPGPU_F_L4;
		if (has_csum && l4_ok)
			o->r.flags |= XDPGPU_F_L4_OK;
		if (absent)
			o->r.flags |= XDPGPU_F_L4_ABSENT;
		o->r.l4_proto = (uint8_t)nh;
		o->r.l4_off = (uint16_t)l4;
		o->r.l4_len = has_csum ? (uint16_t)cl : 0;

		/* flow key: pping.h:120-139 layout, v4 mapped per
		 * pping_kern.c:212-217 */
		if (ipv4) {
			o->key[10] = o->key[11] = 0xff;
			memcpy(o->key + 12, p + l3 + 12, 4);
			o->key[30] = o->key[31] = 0xff;
			memcpy(o->key + 32, p + l3 + 16, 4);
			o->key[42] = 2;      /* AF_INET */
		} else {
			memcpy(o->key, p + l3 + 8, 16);
			memcpy(o->key + 20, p + l3 + 24, 16);
			o->key[42] = 10;     /* AF_INET6 */
		}
		if (has_l4 && (nh == 6 || nh == 17)) {
			memcpy(o->key + 16, p + l4, 2);
			memcpy(o->key + 36, p + l4 + 2, 2);
		}
		o->key[40] = (uint8_t)nh;
	}
	o->r.hash = oracle_jhash(o->key, 44, initval);
	o->l3_bad = (ipv4 && !l3_ok);
	o->l4_bad = (has_csum && !l4_ok);
	o->l4_absent = (uint8_t)absent;
	o->frag = (uint8_t)frag;

	if ((flags & XDPGPU_CFG_VERIFY_CSUM) && (o->l3_bad || o->l4_bad)) {
		o->verdict = XDPGPU_DROP;
		return;
	}
	/* af_xdp_user.c:968-1040 process_packet: ICMPv6 echo -> reply */
	if ((flags & XDPGPU_CFG_ICMP6_ECHO) && nvlan == 0 && ipv6 &&
	    end >= 62 && p[20] == 58 && p[54] == 128) {
		uint8_t t[16];

		memcpy(t, p, 6);
		memcpy(p, p + 6, 6);
		memcpy(p + 6, t, 6);
		memcpy(t, p + 22, 16);
		memcpy(p + 22, p + 38, 16);
		memcpy(p + 38, t, 16);
		p[54] = 129;
		st_le16(p + 56, oracle_csum_replace2(ld_le16(p + 56),
						     0x0080, 0x0081));
		o->verdict = XDPGPU_TX;
		return;
	}
	o->verdict = XDPGPU_REDIRECT;
}

/* Multi-buffer packets (XDPGPU_CFG_FRAGS, include/xdpgpu.h): descriptors
 * [i, j] with XDPGPU_PKT_CONTD on all but d[j] (IS_EOP_DESC, xdpsock.c:67;
 * j == n when the batch ends inside the packet).  The fragments are
 * concatenated, with the byte after the last one as udp_csum's over-read
 * byte, and run through frame_pipeline as one frame; an echo rewrite is
 * copied back into the fragments.  *bytes: the packet's byte count. */
static void packet_pipeline(uint8_t *umem, uint64_t usize,
			    const struct xdpgpu_desc *d, uint32_t i, uint32_t j,
			    uint32_t n, uint32_t flags, uint32_t initval,
			    struct frame_out *o, uint64_t *bytes)
{
	const uint32_t last = j < n ? j : n - 1;
	uint64_t total = 0, at, end = 0;
	int ok = j < n;
	uint32_t k;
	uint8_t *buf;

	for (k = i; k <= last; k++) {
		const uint64_t eff = (d[k].addr & ((1ull << 48) - 1)) + (d[k].addr >> 48);

		total += d[k].len;
		if ((uint64_t)d[k].len > usize || eff > usize - d[k].len)
			ok = 0;
		end = eff + d[k].len;
	}
	*bytes = total;
	memset(o, 0, sizeof(*o));
	o->verdict = XDPGPU_ABORTED;
	if (!ok || total > 0xffffffffull)
		return;
	buf = malloc(total + 1);
	if (!buf)
		return;
	for (at = 0, k = i; k <= last; k++) {
		const uint64_t eff = (d[k].addr & ((1ull << 48) - 1)) + (d[k].addr >> 48);

		memcpy(buf + at, umem + eff, d[k].len);
		at += d[k].len;
	}
	buf[total] = end < usize ? umem[end] : 0;
	{
		const struct xdpgpu_desc pd = { 0, (uint32_t)total, 0 };

		frame_pipeline(buf, total + 1, &pd, flags, initval, o);
	}
	if (o->verdict == XDPGPU_TX) {
		for (at = 0, k = i; k <= last; k++) {
			const uint64_t eff = (d[k].addr & ((1ull << 48) - 1)) +
					     (d[k].addr >> 48);

			memcpy(umem + eff, buf + at, d[k].len);
			at += d[k].len;
		}
	}
	free(buf);
}

static void emit_tuple(const struct frame_out *o, uint32_t fmt, void *tuples,
		       uint32_t i)
{
	if (!tuples || fmt == XDPGPU_TUPLE_NONE)
		return;
	if (fmt == XDPGPU_TUPLE_NET) {
		memcpy((uint8_t *)tuples + (size_t)i * 44, o->key, 44);
	} else {
		struct xdpgpu_tuple4 t;

		memset(&t, 0, sizeof(t));
		if (o->verdict != XDPGPU_ABORTED && o->verdict != XDPGPU_PASS) {
			if (o->key[42] == 2) {
				memcpy(&t.saddr, o->key + 12, 4);
				memcpy(&t.daddr, o->key + 32, 4);
			}
			memcpy(&t.sport, o->key + 16, 2);
			memcpy(&t.dport, o->key + 36, 2);
			t.proto = o->key[40];
			t.ipv = o->key[42];
			t.vlan_id = o->vid;
		}
		memcpy((uint8_t *)tuples + (size_t)i * 16, &t, 16);
	}
}

/* One single-descriptor frame with oracle_process's outputs at index i (the
 * lean CPU leg's path for every frame outside its fast shape). */
void oracle_frame_one(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *d,
		      uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		      uint32_t i, uint8_t *verdict, struct xdpgpu_result *res,
		      void *tuples, struct xdpgpu_stats *stats)
{
	struct frame_out o;

	frame_pipeline(umem, umem_size, d, cfg_flags, initval, &o);
	if (o.verdict == XDPGPU_ABORTED || o.verdict == XDPGPU_PASS) {
		uint8_t v = o.verdict;

		memset(&o, 0, sizeof(o));
		o.verdict = v;
	}
	verdict[i] = o.verdict;
	if (res)
		res[i] = o.r;
	emit_tuple(&o, tuple_fmt, tuples, i);
	if (stats) {
		stats->frames++;
		stats->bytes += d->len;
		stats->verdict[o.verdict]++;
		stats->l3_bad += o.l3_bad;
		stats->l4_bad += o.l4_bad;
		stats->l4_absent += o.l4_absent;
		stats->frag += o.frag;
	}
}

int oracle_process(uint8_t *umem, uint64_t umem_size,
		   const struct xdpgpu_desc *descs, uint32_t n,
		   uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		   uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		   struct xdpgpu_stats *stats)
{
	struct frame_out zero;
	uint32_t i;

	if (!umem || !descs || !verdict)
		return -22;
	memset(&zero, 0, sizeof(zero));
	for (i = 0; i < n;) {
		struct frame_out o;
		uint64_t bytes;
		uint32_t j = i, last, k;

		/* a packet of several descriptors (XDPGPU_CFG_FRAGS) */
		if (cfg_flags & XDPGPU_CFG_FRAGS)
			while (j < n && (descs[j].options & XDPGPU_PKT_CONTD))
				j++;
		if (j == i) {
			frame_pipeline(umem, umem_size, &descs[i], cfg_flags, initval, &o);
			bytes = descs[i].len;
		} else {
			packet_pipeline(umem, umem_size, descs, i, j, n, cfg_flags,
					initval, &o, &bytes);
		}
		last = j < n ? j : n - 1;
		if (o.verdict == XDPGPU_ABORTED || o.verdict == XDPGPU_PASS) {
			/* not delivered to the application: zero records */
			uint8_t v = o.verdict;

			memset(&o, 0, sizeof(o));
			o.verdict = v;
		}
		/* every descriptor of a packet: its verdict; the first: its
		 * record and tuple, the others all-zero ones */
		for (k = i; k <= last; k++) {
			verdict[k] = o.verdict;
			if (res)
				res[k] = k == i ? o.r : zero.r;
			emit_tuple(k == i ? &o : &zero, tuple_fmt, tuples, k);
		}
		if (stats) {
			stats->frames++;
			stats->bytes += bytes;
			stats->verdict[o.verdict]++;
			stats->l3_bad += o.l3_bad;
			stats->l4_bad += o.l4_bad;
			stats->l4_absent += o.l4_absent;
			stats->frag += o.frag;
		}
		i = last + 1;
	}
	return 0;
}

/* XDP hints (af_xdp_user.c:813-829): the u32 before the frame is the BTF id
 * (xsk_umem__btf_id, lib_xsk_extend.c:16-27); a known id selects the struct
 * that ends at the frame (af_xdp_kern.c:42-51), read at its negative
 * offsets (xsk_btf__read, lib_xsk_extend.c:123-141). */
void oracle_hints(const uint8_t *umem, uint64_t umem_size,
		  const struct xdpgpu_desc *descs, uint32_t n, uint32_t rx_time_id,
		  uint32_t mark_id, struct xdpgpu_hints *out)
{
	uint32_t i;

	for (i = 0; i < n; i++) {
		const uint64_t eff = (descs[i].addr & ((1ull << 48) - 1)) +
				     (descs[i].addr >> 48);
		const uint8_t *p = umem + eff;

		memset(&out[i], 0, sizeof(out[i]));
		if (eff < 4 || eff > umem_size)
			continue;
		out[i].btf_id = ld_le32(p - 4);
		if (out[i].btf_id && out[i].btf_id == rx_time_id && eff >= 16) {
			out[i].rx_ktime = (uint64_t)ld_le32(p - 16) |
					  ((uint64_t)ld_le32(p - 12) << 32);
			out[i].value = ld_le32(p - 8);
		} else if (out[i].btf_id && out[i].btf_id == mark_id && eff >= 8) {
			out[i].value = ld_le32(p - 8);
		}
	}
}

/* ------------------------------------------------------------------ */
/* CPU baseline harness                                                */

struct bench_slice {
	uint8_t *umem;
	uint64_t umem_size;
	const struct xdpgpu_desc *descs;
	uint32_t n;
	uint32_t flags, initval, fmt, reps;
	uint8_t *verdict;
	struct xdpgpu_result *res;
	uint8_t *tuples;
};

static void *bench_worker(void *arg)
{
	struct bench_slice *s = (struct bench_slice *)arg;
	uint32_t r;

	for (r = 0; r < s->reps; r++)
		oracle_process(s->umem, s->umem_size, s->descs, s->n, s->flags,
			       s->initval, s->fmt, s->verdict, s->res,
			       s->tuples, NULL);
	return NULL;
}

double oracle_bench(uint8_t *umem, uint64_t umem_size,
		    const struct xdpgpu_desc *descs, uint32_t n,
		    uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		    uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		    uint32_t threads, uint32_t reps)
{
	struct bench_slice sl[256];
	pthread_t th[256];
	struct timespec t0, t1;
	uint32_t tsz = tuple_fmt == XDPGPU_TUPLE_NET ? 44 :
		       tuple_fmt == XDPGPU_TUPLE_V4 ? 16 : 0;
	uint32_t i, per;

	if (threads == 0)
		threads = 1;
	if (threads > 256)
		threads = 256;
	per = (n + threads - 1) / threads;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (i = 0; i < threads; i++) {
		uint32_t lo = i * per, hi = lo + per;

		if (lo > n)
			lo = n;
		if (hi > n)
			hi = n;
		sl[i].umem = umem;
		sl[i].umem_size = umem_size;
		sl[i].descs = descs + lo;
		sl[i].n = hi - lo;
		sl[i].flags = cfg_flags;
		sl[i].initval = initval;
		sl[i].fmt = tuple_fmt;
		sl[i].reps = reps;
		sl[i].verdict = verdict + lo;
		sl[i].res = res ? res + lo : NULL;
		sl[i].tuples = tuples ? (uint8_t *)tuples + (size_t)lo * tsz : NULL;
		if (threads == 1)
			bench_worker(&sl[i]);
		else
			pthread_create(&th[i], NULL, bench_worker, &sl[i]);
	}
	if (threads > 1)
		for (i = 0; i < threads; i++)
			pthread_join(th[i], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (double)(t1.tv_sec - t0.tv_sec) +
	       (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
}
