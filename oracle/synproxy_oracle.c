// SPDX-License-Identifier: GPL-2.0
/*
 * synproxy_oracle.c - TEST INFRASTRUCTURE ONLY: the parity oracle of the
 * SYN proxy transform (xdpgpu_synproxy_dev).
 *
 * A plain-C restatement of xdp-synproxy/xdp_synproxy_kern.c's XDP program
 * (syncookie_xdp, :803-819) on UMEM frames, function by function: nothing
 * of it is copied (it is BPF-C with libbpf headers, not buildable here).
 * Kernel pieces outside the reference are restated from their contracts:
 *   - bpf_csum_diff(0, 0, p, n, 0): the 32-bit ones' complement sum of the
 *     n (a multiple of 4) bytes at p;
 *   - bpf_xdp_adjust_tail(ctx, +k): the frame grows by k zeroed bytes when
 *     the buffer has the room, else the call fails.
 * Two kernel facilities are outside the transform: the
 * conntrack lookup (every frame taken as not established) and the kernel's
 * SYN cookie (a build-defined keyed cookie, include/xdpgpu.h).  Parity is
 * pinned by independent checks in tests/test_synproxy.py (checksums of the
 * SYN-ACK recomputed, option layouts written down from :480-531), not by a
 * reference build: "parity unpinned" at the reference level.
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

#define SP_PASS 2
#define SP_DROP 1
#define SP_TX 3
#define SP_ABORTED 0

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
static inline uint32_t le32(const uint8_t *p)
{
	return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

/* bpf_csum_diff(0, 0, p, n, 0) as a 64-bit accumulation of LE words */
static uint64_t sum32(const uint8_t *p, uint32_t n)
{
	uint64_t s = 0;
	for (uint32_t i = 0; i + 4 <= n; i += 4)
		s += le32(p + i);
	return s;
}

/* csum_fold (:121-126) of a 64-bit sum carried down to 32 bits */
static uint16_t fold(uint64_t s)
{
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffffffu) + (s >> 32);
	uint32_t c = (uint32_t)s;
	c = (c & 0xffff) + (c >> 16);
	c = (c & 0xffff) + (c >> 16);
	return (uint16_t)~c;
}

/* csum_tcpudp_magic (:128-147), little-endian: (proto + len) << 8 */
static uint16_t tcpudp_magic(const uint8_t *saddr, const uint8_t *daddr, uint32_t len,
			     uint64_t body)
{
	return fold(body + le32(saddr) + le32(daddr) + ((uint64_t)(6 + len) << 8));
}

/* csum_ipv6_magic (:149-172) */
static uint16_t ipv6_magic(const uint8_t *saddr, const uint8_t *daddr, uint32_t len,
			   uint64_t body)
{
	uint64_t s = body;
	for (int i = 0; i < 4; i++) {
		s += le32(saddr + 4 * i);
		s += le32(daddr + 4 * i);
	}
	s += __builtin_bswap32(len);
	s += __builtin_bswap32(6);
	return fold(s);
}

/* the build-defined SYN cookie (include/xdpgpu.h): jhash2 over the address
 * words (IPv4: one word each, the rest 0) and the ports, keyed by the key
 * and the minute */
static uint32_t cookie_hash(const uint8_t *p, uint32_t ip, int v6, uint32_t tcp,
			    uint32_t key, uint32_t count)
{
	uint32_t w[9];
	memset(w, 0, sizeof(w));
	if (v6) {
		for (int i = 0; i < 4; i++) {
			w[i] = le32(p + ip + 8 + 4 * i);
			w[4 + i] = le32(p + ip + 24 + 4 * i);
		}
	} else {
		w[0] = le32(p + ip + 12);
		w[4] = le32(p + ip + 16);
	}
	w[8] = (uint32_t)be16(p + tcp) << 16 | be16(p + tcp + 2);
	return oracle_jhash2(w, 9, key + count);
}

static int port_allowed(const struct xdpgpu_synproxy_cfg *c, uint16_t port)
{
	for (int i = 0; i < 8; i++) {
		if (c->ports[i] == 0)
			break;
		if (c->ports[i] == port)
			return 1;
	}
	return 0;
}

struct optctx {
	uint32_t off, end;          /* offsets in the frame; end = data_end */
	uint8_t wscale, ts, sack;
	uint8_t tsecr[4];
};

/* next() (:199-215): NULL when off + sz reaches data_end */
static int next(struct optctx *c, uint32_t sz, uint32_t *at)
{
	if (c->off > 0xffffu - sz)
		return 0;
	if (c->off + sz >= c->end)
		return 0;
	*at = c->off;
	c->off += sz;
	return 1;
}

/* tscookie_tcpopt_parse (:217-262): 1 ends the walk */
static int opt_parse(struct optctx *c, const uint8_t *p)
{
	uint32_t op, sz, v;
	const uint32_t off = c->off;

	if (!next(c, 1, &op))
		return 1;
	if (p[op] == 0)
		return 1;
	if (p[op] == 1)
		return 0;
	if (!next(c, 1, &sz) || p[sz] < 2)
		return 1;
	switch (p[op]) {
	case 3:
		if (!next(c, 1, &v))
			return 1;
		if (p[sz] == 3)
			c->wscale = p[v] < 14 ? p[v] : 14;
		break;
	case 8:
		if (!next(c, 4, &v))
			return 1;
		if (p[sz] == 10) {
			c->ts = 1;
			memcpy(c->tsecr, p + v, 4);
		}
		break;
	case 4:
		if (p[sz] == 2)
			c->sack = 1;
		break;
	}
	c->off = off + p[sz];
	return 0;
}

/* syncookie_handle_syn (:577-715) */
static int handle_syn(uint8_t *p, uint32_t *len, uint32_t ip, int v6, uint32_t tcp,
		      const struct xdpgpu_synproxy_cfg *cfg, uint64_t *synacks)
{
	uint32_t tcp_len = (p[tcp + 12] >> 4) * 4;
	const uint8_t fl = p[tcp + 13];
	uint32_t ip_len;

	if (fl & 0x05)                                  /* fin, rst */
		return SP_DROP;
	if (!v6) {
		const uint32_t ihl = (p[ip] & 15) * 4;
		if (fold(sum32(p + ip, ihl)) != 0)
			return SP_DROP;
		if (tcpudp_magic(p + ip + 12, p + ip + 16, tcp_len, sum32(p + tcp, tcp_len)))
			return SP_DROP;
		ip_len = 20;
	} else {
		if (ipv6_magic(p + ip + 8, p + ip + 24, tcp_len, sum32(p + tcp, tcp_len)))
			return SP_DROP;
		ip_len = 40;
	}
	const uint32_t count = (uint32_t)(cfg->now_ns / 60000000000ull);
	const uint32_t cookie = cookie_hash(p, ip, v6, tcp, cfg->cookie_key, count) +
				be32(p + tcp + 4);

	/* tscookie_init (:274-308): 6 x 7 option steps from the end of the
	 * fixed header, up to data_end */
	struct optctx oc = {tcp + 20, *len, 0xf, 0, 0, {0, 0, 0, 0}};
	int stop = 0;
	for (int i = 0; i < 42 && !stop; i++)
		stop = opt_parse(&oc, p);
	uint8_t tsopt[8];
	const int ts = oc.ts;
	if (ts) {
		uint32_t ck = (uint32_t)(cfg->now_ns / 1000000ull) & ~0x3fu;
		ck |= oc.wscale & 0xf;
		if (oc.sack)
			ck |= 1u << 4;
		if ((fl & 0x40) && (fl & 0x80))             /* ece, cwr */
			ck |= 1u << 5;
		put_be32(tsopt, ck);
		memcpy(tsopt + 4, oc.tsecr, 4);
	}
	if (14 + ip_len + 60 > *len)
		return SP_ABORTED;
	if (!v6 && (p[ip] & 15) * 4 > 20) {
		memmove(p + 14 + 20, p + tcp, 20);
		tcp = 14 + 20;
		p[ip] = (p[ip] & 0xf0) | 5;
	}

	/* values_get_tcpipopts (:310-330) */
	uint32_t mss, wscale, ttl;
	if (cfg->values) {
		mss = v6 ? (cfg->values >> 32) & 0xffff : cfg->values & 0xffff;
		wscale = (cfg->values >> 16) & 0xf;
		ttl = (cfg->values >> 24) & 0xff;
	} else {
		mss = v6 ? 1440 : 1460;
		wscale = 7;
		ttl = 64;
	}
	/* tcpv4/v6_gen_synack (:533-575) */
	uint8_t t6[6];
	memcpy(t6, p, 6);
	memcpy(p, p + 6, 6);
	memcpy(p + 6, t6, 6);
	uint8_t a[16];
	if (!v6) {
		memcpy(a, p + ip + 12, 4);
		memcpy(p + ip + 12, p + ip + 16, 4);
		memcpy(p + ip + 16, a, 4);
		p[ip + 10] = p[ip + 11] = 0;
		p[ip + 1] = 0;
		p[ip + 4] = p[ip + 5] = 0;
		p[ip + 8] = (uint8_t)ttl;
	} else {
		memcpy(a, p + ip + 8, 16);
		memcpy(p + ip + 8, p + ip + 24, 16);
		memcpy(p + ip + 24, a, 16);
		put_be32(p + ip, 0x60000000u);
		p[ip + 7] = (uint8_t)ttl;
	}
	/* tcp_gen_synack (:512-531): the flag word (bytes 12-15) = SYN | ACK
	 * (| ECE), doff 5, window 0 */
	uint8_t *t = p + tcp;
	t[12] = 0x50;
	t[13] = 0x12 | (ts && (tsopt[3] & (1u << 5)) ? 0x40 : 0);
	t[14] = t[15] = 0;
	uint8_t pt[2];
	memcpy(pt, t, 2);
	memcpy(t, t + 2, 2);
	memcpy(t + 2, pt, 2);
	put_be32(t + 8, be32(t + 4) + 1);
	put_be32(t + 4, cookie);
	t[16] = t[17] = t[18] = t[19] = 0;
	/* tcp_mkoptions (:480-510) */
	uint8_t *o = t + 20;
	uint32_t words = 0;
	put_be32(o + 4 * words++, 2u << 24 | 4u << 16 | (mss & 0xffff));
	if (ts) {
		if (tsopt[3] & (1u << 4))
			put_be32(o + 4 * words++, 4u << 24 | 2u << 16 | 8u << 8 | 10u);
		else
			put_be32(o + 4 * words++, 1u << 24 | 1u << 16 | 8u << 8 | 10u);
		memcpy(o + 4 * words++, tsopt, 4);
		memcpy(o + 4 * words++, tsopt + 4, 4);
		if ((tsopt[3] & 0xf) != 0xf)
			put_be32(o + 4 * words++, 1u << 24 | 3u << 16 | 3u << 8 | wscale);
	}
	t[12] = (uint8_t)((5 + words) << 4);
	tcp_len = (5 + words) * 4;
	if (!v6)
		put_be16(p + ip + 2, (uint16_t)(20 + tcp_len));
	else
		put_be16(p + ip + 4, (uint16_t)tcp_len);
	/* checksums (:679-704) */
	const uint64_t body = sum32(t, tcp_len);
	const uint16_t c = v6 ? ipv6_magic(p + ip + 8, p + ip + 24, tcp_len, body)
			      : tcpudp_magic(p + ip + 12, p + ip + 16, tcp_len, body);
	memcpy(t + 16, &c, 2);                          /* stored as computed */
	if (!v6) {
		const uint16_t h = fold(sum32(p + ip, 20));
		memcpy(p + ip + 10, &h, 2);
	}
	*len = 14 + ip_len + tcp_len;
	if (synacks)
		++*synacks;
	return SP_TX;
}

/* syncookie_handle_ack (:717-734) with the build-defined cookie check */
static int handle_ack(const uint8_t *p, uint32_t ip, int v6, uint32_t tcp,
		      const struct xdpgpu_synproxy_cfg *cfg)
{
	if (p[tcp + 13] & 0x04)
		return SP_DROP;
	const uint32_t count = (uint32_t)(cfg->now_ns / 60000000000ull);
	const uint32_t want = be32(p + tcp + 8) - 1, seq = be32(p + tcp + 4) - 1;
	for (uint32_t d = 0; d < 2; d++)
		if (cookie_hash(p, ip, v6, tcp, cfg->cookie_key, count - d) + seq == want)
			return SP_PASS;
	return SP_DROP;
}

/* syncookie_xdp (:803-819) on one frame: part1 (:736-767), part2 (:769-801) */
static int sp_frame(uint8_t *p, uint32_t *len, uint64_t room,
		    const struct xdpgpu_synproxy_cfg *cfg, uint64_t *synacks)
{
	/* tcp_dissect (:375-428) */
	if (*len < 14)
		return SP_DROP;
	const uint16_t proto = be16(p + 12);
	const uint32_t ip = 14;
	uint32_t tcp;
	int v6;
	if (proto == 0x0800) {
		v6 = 0;
		if (ip + 20 > *len)
			return SP_DROP;
		if ((p[ip] & 15) * 4 < 20 || (p[ip] >> 4) != 4)
			return SP_DROP;
		if (p[ip + 9] != 6)
			return SP_PASS;
		tcp = ip + (p[ip] & 15) * 4;
	} else if (proto == 0x86DD) {
		v6 = 1;
		if (ip + 40 > *len)
			return SP_DROP;
		if ((p[ip] >> 4) != 6)
			return SP_DROP;
		if (p[ip + 6] != 6)
			return SP_PASS;
		tcp = ip + 40;
	} else {
		return SP_PASS;
	}
	if (tcp + 20 > *len)
		return SP_DROP;
	uint32_t tcp_len = (p[tcp + 12] >> 4) * 4;
	if (tcp_len < 20)
		return SP_DROP;
	/* tcp_lookup (:430-478): fragments; conntrack outside the transform */
	if (!v6 && (be16(p + ip + 6) & 0x7fff) != 0x4000)       /* DF|MF|OFFSET */
		return SP_DROP;
	if (!port_allowed(cfg, be16(p + tcp + 2)))
		return SP_PASS;
	const int syn = (p[tcp + 13] >> 1) & 1, ack = (p[tcp + 13] >> 4) & 1;
	if ((syn ^ ack) != 1)
		return SP_DROP;
	/* bpf_xdp_adjust_tail(ctx, TCP_MAXLEN - tcp_len) */
	const uint32_t grow = 60 - tcp_len;
	if (grow > room)
		return SP_ABORTED;
	memset(p + *len, 0, grow);
	*len += grow;
	/* part2 */
	if (!v6) {
		if (ip + 60 > *len)
			return SP_ABORTED;
		tcp = ip + (p[ip] & 15) * 4;
	}
	if (tcp + 60 > *len)
		return SP_ABORTED;
	tcp_len = (p[tcp + 12] >> 4) * 4;
	if (tcp_len < 20)
		return SP_ABORTED;
	return syn ? handle_syn(p, len, ip, v6, tcp, cfg, synacks)
		   : handle_ack(p, ip, v6, tcp, cfg);
}

int oracle_synproxy(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		    uint32_t n, const struct xdpgpu_synproxy_cfg *cfg, uint8_t *verdict,
		    struct xdpgpu_desc *out, uint64_t *synacks)
{
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t addr = descs[i].addr;
		uint32_t len = descs[i].len;
		const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
		out[i] = descs[i];
		if ((uint64_t)len > umem_size || eff > umem_size - len) {
			verdict[i] = SP_ABORTED;
			continue;
		}
		/* the room to grow: the chunk's, inside the UMEM */
		uint64_t room = umem_size - eff - len;
		if (room > cfg->tailroom)
			room = cfg->tailroom;
		verdict[i] = (uint8_t)sp_frame(umem + eff, &len, room, cfg, synacks);
		out[i].len = len;
	}
	return 0;
}
