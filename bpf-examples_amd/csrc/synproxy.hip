// SPDX-License-Identifier: GPL-2.0
/*
 * synproxy.hip - the SYN proxy transform (xdpgpu_synproxy_dev): the XDP
 * program of xdp-synproxy/xdp_synproxy_kern.c (syncookie_xdp, :803-819)
 * over a batch of UMEM frames, one lane per frame.
 *
 * A lane stages its frame's first kRow bytes in an LDS row (the wave's
 * 16-byte aligned frames cooperatively, whole 16-byte chunks; others byte
 * by byte), runs the program on the row
 * (TCP option bytes past the row are read from the UMEM, bytes past the
 * frame's end as the zeros bpf_xdp_adjust_tail grows it with), and writes
 * back what changed: the SYN-ACK's headers (at most 14 + 40 + 40 bytes, all
 * in the row) or the zeroed growth of a frame the program grew and then
 * passed or dropped, as whole 16-byte chunks where the chunk lies in the
 * frame's buffer (the unchanged bytes from the lane's staged copy).  The
 * common SYN (untagged IPv4, 20-byte IP header, at most 20 option bytes)
 * runs in registers (handle_syn_fast); everything else byte-wise on the
 * row.  Semantics and what lies outside the transform (conntrack, the
 * kernel's cookie): include/xdpgpu.h.
 */
#include <hip/hip_runtime.h>

#include "xdpgpu.h"
#include "xdpgpu_internal.h"

namespace xdpgpu {
namespace {

/* staged bytes per frame (build knob for A/B): every byte the program
 * writes lies below 96 (an IPv6 SYN-ACK ends at 14 + 40 + 40); bytes past
 * the row are read from the UMEM.  SYN proxy leg, 8 M SYNs at a 128-byte
 * stride: 96 bytes 0.569 ms, 112 0.617, 128 0.640, 144 0.873 (with the
 * staging copy of 144 bytes reading into the next frame's line) */
#ifndef SP_ROW
#define SP_ROW 96
#endif
constexpr int kRow = SP_ROW;
constexpr int kRowDw = kRow / 4 + 1;      /* odd dword stride: no bank conflicts */
constexpr int kChunks = kRow / 16;
static_assert(kRow % 16 == 0 && kRow >= 96, "the row holds whole chunks, every write");
/* the cooperative write-back (build knob for A/B): 0 = the changed bytes
 * only (partial chunks by dwords and bytes), 1 = whole 16-byte chunks where
 * the chunk lies in the frame's buffer (its length plus the tail room it
 * may grow into), the unchanged bytes from the staged copy, 2 = also the
 * rest of every 64-byte sector written, so that HBM sees whole sectors.
 * SYN proxy leg (128-byte rows): 0.733 ms with 0, 0.637 with 1, 0.698
 * with 2 */
#ifndef SP_WB
#define SP_WB 1
#endif
constexpr int kWb = SP_WB;
/* cache policy (build knob for A/B): bit 0 the whole-chunk write-back
 * stores, bit 1 the verdict and output descriptor stores non-temporal.
 * No difference on the SYN proxy leg (0.560-0.570 ms either way) */
#ifndef SP_NT
#define SP_NT 0
#endif
/* 1: a grid of resident waves looping over the tiles, the next tile's
 * descriptors loaded before this tile's work (build knob for A/B): 1.63 vs
 * 0.57 ms with one tile per launched wave */
#ifndef SP_PERSIST
#define SP_PERSIST 0
#endif
constexpr int kBlockS = 64;      /* one wave: LDS rows bound the CU to 15 waves */

enum { SP_ABORTED = 0, SP_DROP = 1, SP_PASS = 2, SP_TX = 3 };

struct Frame {
	uint8_t *row;              /* LDS: bytes [0, kRow) */
	const uint8_t *g;          /* the frame in the UMEM */
	uint32_t len0;             /* the frame's length before any growth */
	/* the row holds the frame's bytes and zeros past its end (what the
	 * program writes goes to the row); past the row, the UMEM up to the
	 * frame's end, then the zeros of its growth */
	__device__ uint32_t b(uint32_t i) const
	{
		if (i < (uint32_t)kRow)
			return row[i];
		return i < len0 ? g[i] : 0u;
	}
	__device__ void put(uint32_t i, uint32_t v) const { row[i] = (uint8_t)v; }
	/* the LE word at byte i: two aligned LDS dwords and a byte align
	 * inside the row (the row's dword after the last is in the row's
	 * padding dword) */
	__device__ uint32_t le32(uint32_t i) const
	{
		if (i + 4 <= (uint32_t)kRow) {
			const uint32_t *w = reinterpret_cast<const uint32_t *>(row);
			const uint32_t lo = w[i >> 2], hi = w[(i >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, i & 3);
		}
		return b(i) | b(i + 1) << 8 | b(i + 2) << 16 | b(i + 3) << 24;
	}
	__device__ uint32_t be16(uint32_t i) const
	{
		const uint32_t v = le32(i);
		return (v & 0xff) << 8 | ((v >> 8) & 0xff);
	}
	__device__ uint32_t be32(uint32_t i) const { return __builtin_bswap32(le32(i)); }
	__device__ void put_be16(uint32_t i, uint32_t v) const
	{
		put(i, v >> 8);
		put(i + 1, v);
	}
	__device__ void put_be32(uint32_t i, uint32_t v) const
	{
		put_be16(i, v >> 16);
		put_be16(i + 2, v & 0xffff);
	}
};

/* bpf_csum_diff(0, 0, p, n, 0): LE words, 64-bit accumulation */
__device__ __forceinline__ uint64_t sum32(const Frame &F, uint32_t at, uint32_t n)
{
	uint64_t s = 0;
	for (uint32_t i = 0; i + 4 <= n; i += 4)
		s += F.le32(at + i);
	return s;
}

/* csum_fold (xdp_synproxy_kern.c:121-126) of a 64-bit sum */
__device__ __forceinline__ uint32_t fold(uint64_t s)
{
	s = (s & 0xffffffffu) + (s >> 32);
	s = (s & 0xffffffffu) + (s >> 32);
	uint32_t c = (uint32_t)s;
	c = (c & 0xffff) + (c >> 16);
	c = (c & 0xffff) + (c >> 16);
	return ~c & 0xffff;
}

/* csum_tcpudp_magic (:128-147, little-endian) / csum_ipv6_magic (:149-172) */
__device__ __forceinline__ uint32_t l4_magic(const Frame &F, uint32_t ip, bool v6, uint32_t len,
			     uint64_t body)
{
	uint64_t s = body;
	if (v6) {
		for (int i = 0; i < 8; i++)
			s += F.le32(ip + 8 + 4 * i);
		s += __builtin_bswap32(len);
		s += __builtin_bswap32(6u);
	} else {
		s += F.le32(ip + 12);
		s += F.le32(ip + 16);
		s += (uint64_t)(6 + len) << 8;
	}
	return fold(s);
}

/* the build-defined cookie (include/xdpgpu.h) */
__device__ __forceinline__ uint32_t cookie_hash(const Frame &F, uint32_t ip, bool v6, uint32_t tcp,
				uint32_t key, uint32_t count)
{
	uint32_t w[9];
	for (int i = 0; i < 9; i++)
		w[i] = 0;
	if (v6) {
		for (int i = 0; i < 4; i++) {
			w[i] = F.le32(ip + 8 + 4 * i);
			w[4 + i] = F.le32(ip + 24 + 4 * i);
		}
	} else {
		w[0] = F.le32(ip + 12);
		w[4] = F.le32(ip + 16);
	}
	w[8] = F.be16(tcp) << 16 | F.be16(tcp + 2);
	/* jhash2(w, 9, key + count), unrolled (include/jhash.h:114-142) */
	uint32_t a = 0xdeadbeefu + (9u << 2) + key + count, b = a, c = a;
	a += w[0];
	b += w[1];
	c += w[2];
	JH_MIX(a, b, c);
	a += w[3];
	b += w[4];
	c += w[5];
	JH_MIX(a, b, c);
	c += w[8];
	b += w[7];
	a += w[6];
	JH_FINAL(a, b, c);
	return c;
}

struct Opt {
	uint32_t off, end;
	uint32_t wscale, ts, sack, tsecr;   /* tsecr: the 4 bytes, LE word */
};

/* next() (:199-215) */
__device__ __forceinline__ bool next(Opt &c, uint32_t sz, uint32_t &at)
{
	if (c.off > 0xffffu - sz || c.off + sz >= c.end)
		return false;
	at = c.off;
	c.off += sz;
	return true;
}

/* tscookie_tcpopt_parse (:217-262): true ends the walk */
__device__ __forceinline__ bool opt_parse(Opt &c, const Frame &F)
{
	const uint32_t off = c.off;
	uint32_t op, sz, v;
	if (!next(c, 1, op))
		return true;
	const uint32_t code = F.b(op);
	if (code == 0)
		return true;
	if (code == 1)
		return false;
	if (!next(c, 1, sz))
		return true;
	const uint32_t osz = F.b(sz);
	if (osz < 2)
		return true;
	/* the fields are updated by value (a conditional store to one of
	 * them through a selected address would put the struct in scratch) */
	uint32_t wscale = c.wscale, ts = c.ts, sack = c.sack, tsecr = c.tsecr;
	if (code == 3) {
		if (!next(c, 1, v))
			return true;
		const uint32_t x = F.b(v);
		wscale = osz == 3 ? (x < 14 ? x : 14) : wscale;
	} else if (code == 8) {
		if (!next(c, 4, v))
			return true;
		const uint32_t x = F.le32(v);
		ts = osz == 10 ? 1u : ts;
		tsecr = osz == 10 ? x : tsecr;
	} else if (code == 4) {
		sack = osz == 2 ? 1u : sack;
	}
	c.wscale = wscale;
	c.ts = ts;
	c.sack = sack;
	c.tsecr = tsecr;
	c.off = off + osz;
	return false;
}

/* syncookie_handle_syn (:577-715); len is the grown length */
__device__ __forceinline__ uint32_t handle_syn(const Frame &F, uint32_t &len, uint32_t ip, bool v6,
			       uint32_t tcp, const xdpgpu_synproxy_cfg &cfg, bool &synack)
{
	uint32_t tcp_len = (F.b(tcp + 12) >> 4) * 4;
	const uint32_t fl = F.b(tcp + 13);
	if (fl & 0x05)
		return SP_DROP;
	if (!v6 && fold(sum32(F, ip, (F.b(ip) & 15) * 4)) != 0)
		return SP_DROP;
	if (l4_magic(F, ip, v6, tcp_len, sum32(F, tcp, tcp_len)) != 0)
		return SP_DROP;
	const uint32_t ip_len = v6 ? 40 : 20;
	const uint32_t count = (uint32_t)(cfg.now_ns / 60000000000ull);
	const uint32_t cookie = cookie_hash(F, ip, v6, tcp, cfg.cookie_key, count) +
				F.be32(tcp + 4);
	/* tscookie_init (:274-308) */
	Opt oc = {tcp + 20, len, 0xf, 0, 0, 0};
	for (int i = 0; i < 42; i++)
		if (opt_parse(oc, F))
			break;
	uint32_t tsval = 0;        /* the TS option's first word, host order */
	if (oc.ts) {
		tsval = (uint32_t)(cfg.now_ns / 1000000ull) & ~0x3fu;
		tsval |= oc.wscale & 0xf;
		if (oc.sack)
			tsval |= 1u << 4;
		if ((fl & 0x40) && (fl & 0x80))
			tsval |= 1u << 5;
	}
	if (14 + ip_len + 60 > len)
		return SP_ABORTED;
	if (!v6 && (F.b(ip) & 15) * 4 > 20) {
		/* the TCP header moves down to the end of a 20-byte IP header */
		for (uint32_t i = 0; i < 20; i++)
			F.put(34 + i, F.b(tcp + i));
		tcp = 34;
		F.put(ip, (F.b(ip) & 0xf0) | 5);
	}
	uint32_t mss, wscale, ttl;
	if (cfg.values) {
		mss = v6 ? (uint32_t)(cfg.values >> 32) & 0xffff : (uint32_t)cfg.values & 0xffff;
		wscale = (uint32_t)(cfg.values >> 16) & 0xf;
		ttl = (uint32_t)(cfg.values >> 24) & 0xff;
	} else {
		mss = v6 ? 1440 : 1460;
		wscale = 7;
		ttl = 64;
	}
	/* tcpv4/v6_gen_synack (:533-575) */
	for (uint32_t i = 0; i < 6; i++) {
		const uint32_t t = F.b(i);
		F.put(i, F.b(6 + i));
		F.put(6 + i, t);
	}
	const uint32_t sa = v6 ? ip + 8 : ip + 12, da = v6 ? ip + 24 : ip + 16;
	for (uint32_t i = 0; i < (v6 ? 16u : 4u); i++) {
		const uint32_t t = F.b(sa + i);
		F.put(sa + i, F.b(da + i));
		F.put(da + i, t);
	}
	if (!v6) {
		F.put(ip + 10, 0);
		F.put(ip + 11, 0);
		F.put(ip + 1, 0);
		F.put(ip + 4, 0);
		F.put(ip + 5, 0);
		F.put(ip + 8, ttl);
	} else {
		F.put_be32(ip, 0x60000000u);
		F.put(ip + 7, ttl);
	}
	/* tcp_gen_synack (:512-531) */
	const uint32_t seq = F.be32(tcp + 4);
	F.put(tcp + 12, 0x50);
	F.put(tcp + 13, 0x12 | ((oc.ts && (tsval & (1u << 5))) ? 0x40 : 0));
	F.put(tcp + 14, 0);
	F.put(tcp + 15, 0);
	const uint32_t sp = F.be16(tcp), dp = F.be16(tcp + 2);
	F.put_be16(tcp, dp);
	F.put_be16(tcp + 2, sp);
	F.put_be32(tcp + 8, seq + 1);
	F.put_be32(tcp + 4, cookie);
	for (uint32_t i = 16; i < 20; i++)
		F.put(tcp + i, 0);
	/* tcp_mkoptions (:480-510) */
	uint32_t o = tcp + 20;
	F.put_be32(o, 2u << 24 | 4u << 16 | (mss & 0xffff));
	o += 4;
	if (oc.ts) {
		F.put_be32(o, (tsval & (1u << 4)) ? (4u << 24 | 2u << 16 | 8u << 8 | 10u)
						  : (1u << 24 | 1u << 16 | 8u << 8 | 10u));
		F.put_be32(o + 4, tsval);
		F.put(o + 8, oc.tsecr);
		F.put(o + 9, oc.tsecr >> 8);
		F.put(o + 10, oc.tsecr >> 16);
		F.put(o + 11, oc.tsecr >> 24);
		o += 12;
		if ((tsval & 0xf) != 0xf) {
			F.put_be32(o, 1u << 24 | 3u << 16 | 3u << 8 | wscale);
			o += 4;
		}
	}
	tcp_len = o - tcp;
	F.put(tcp + 12, (tcp_len / 4) << 4);
	if (!v6)
		F.put_be16(ip + 2, 20 + tcp_len);
	else
		F.put_be16(ip + 4, tcp_len);
	/* checksums (:679-704), stored as computed (LE u16) */
	const uint32_t c = l4_magic(F, ip, v6, tcp_len, sum32(F, tcp, tcp_len));
	F.put(tcp + 16, c);
	F.put(tcp + 17, c >> 8);
	if (!v6) {
		const uint32_t h = fold(sum32(F, ip, 20));
		F.put(ip + 10, h);
		F.put(ip + 11, h >> 8);
	}
	len = 14 + ip_len + tcp_len;
	synack = true;
	return SP_TX;
}

/* syncookie_handle_ack (:717-734), the build-defined cookie check */
__device__ __forceinline__ uint32_t handle_ack(const Frame &F, uint32_t ip, bool v6, uint32_t tcp,
			       const xdpgpu_synproxy_cfg &cfg)
{
	if (F.b(tcp + 13) & 0x04)
		return SP_DROP;
	const uint32_t count = (uint32_t)(cfg.now_ns / 60000000000ull);
	const uint32_t want = F.be32(tcp + 8) - 1, seq = F.be32(tcp + 4) - 1;
	for (uint32_t d = 0; d < 2; d++)
		if (cookie_hash(F, ip, v6, tcp, cfg.cookie_key, count - d) + seq == want)
			return SP_PASS;
	return SP_DROP;
}

/* syncookie_xdp (:803-819): part1 (:736-767), part2 (:769-801) */
__device__ __forceinline__ uint32_t sp_frame(const Frame &F, uint32_t &len, uint64_t room,
			     const xdpgpu_synproxy_cfg &cfg, bool &synack, uint32_t &grow)
{
	grow = 0;
	if (len < 14)
		return SP_DROP;
	const uint32_t proto = F.be16(12), ip = 14;
	uint32_t tcp;
	bool v6;
	if (proto == 0x0800) {
		v6 = false;
		if (ip + 20 > len)
			return SP_DROP;
		if ((F.b(ip) & 15) * 4 < 20 || (F.b(ip) >> 4) != 4)
			return SP_DROP;
		if (F.b(ip + 9) != 6)
			return SP_PASS;
		tcp = ip + (F.b(ip) & 15) * 4;
	} else if (proto == 0x86DD) {
		v6 = true;
		if (ip + 40 > len)
			return SP_DROP;
		if ((F.b(ip) >> 4) != 6)
			return SP_DROP;
		if (F.b(ip + 6) != 6)
			return SP_PASS;
		tcp = ip + 40;
	} else {
		return SP_PASS;
	}
	if (tcp + 20 > len)
		return SP_DROP;
	uint32_t tcp_len = (F.b(tcp + 12) >> 4) * 4;
	if (tcp_len < 20)
		return SP_DROP;
	if (!v6 && (F.be16(ip + 6) & 0x7fff) != 0x4000)
		return SP_DROP;
	/* check_port_allowed (:342-365): the list up to its first 0 (constant
	 * indices: a loop with an early exit indexes the argument's array
	 * dynamically, which puts it in scratch memory) */
	bool allowed = false, live = true;
	const uint32_t port = F.be16(tcp + 2);
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const uint32_t pv = cfg.ports[i];
		live = live && pv != 0;
		allowed = allowed || (live && pv == port);
	}
	if (!allowed)
		return SP_PASS;
	const uint32_t fl = F.b(tcp + 13);
	const uint32_t syn = (fl >> 1) & 1, ack = (fl >> 4) & 1;
	if ((syn ^ ack) != 1)
		return SP_DROP;
	if (60 - tcp_len > room)
		return SP_ABORTED;
	grow = 60 - tcp_len;
	len += grow;
	if (!v6 && ip + 60 > len)
		return SP_ABORTED;
	if (tcp + 60 > len)
		return SP_ABORTED;
	return syn ? handle_syn(F, len, ip, v6, tcp, cfg, synack)
		   : handle_ack(F, ip, v6, tcp, cfg);
}

/* ------------------------------------------------------------------ */
/* The common SYN in registers: untagged IPv4 with a 20-byte header, a TCP
 * SYN to an allowed port with at most 20 option bytes, the growth inside
 * the row.  The row's first 96 bytes are taken into registers (W), the
 * checks, checksums, cookie and SYN-ACK of syncookie_handle_syn
 * (:577-715) are computed at fixed byte positions, and the new bytes go
 * back to the row as whole dwords; the option walk (tscookie_tcpopt_parse)
 * stays on the row.  Bit-exact with handle_syn on these frames, in a few
 * hundred instructions instead of a byte-wise pass over the row. */
constexpr int kW = 24;                    /* row dwords in registers */

__device__ __forceinline__ uint32_t wb8(const uint32_t (&W)[kW], int i)
{
	return (W[i >> 2] >> (8 * (i & 3))) & 0xff;
}

/* the LE word at byte i (i even) */
__device__ __forceinline__ uint32_t wle(const uint32_t (&W)[kW], int i)
{
	return (i & 3) ? __builtin_amdgcn_alignbyte(W[(i >> 2) + 1], W[i >> 2], i & 3)
		       : W[i >> 2];
}

__device__ __forceinline__ uint32_t wbe16(const uint32_t (&W)[kW], int i)
{
	return wb8(W, i) << 8 | wb8(W, i + 1);
}

__device__ __forceinline__ void wput(uint32_t (&O)[kW], int i, uint32_t v)
{
	const int s = 8 * (i & 3);
	O[i >> 2] = (O[i >> 2] & ~(0xffu << s)) | ((v & 0xff) << s);
}

__device__ __forceinline__ void wput_be16(uint32_t (&O)[kW], int i, uint32_t v)
{
	wput(O, i, v >> 8);
	wput(O, i + 1, v);
}

__device__ __forceinline__ void wput_be32(uint32_t (&O)[kW], int i, uint32_t v)
{
	wput_be16(O, i, v >> 16);
	wput_be16(O, i + 2, v & 0xffff);
}

/* is this lane's frame the common SYN (sp_frame's path to handle_syn
 * with tcp = 34 and nothing past the row)?  room: as sp_frame's */
__device__ __forceinline__ bool syn_fast_shape(const uint32_t (&W)[kW], uint32_t len0,
					       uint64_t room, const xdpgpu_synproxy_cfg &cfg)
{
	const uint32_t tcp_len = (wb8(W, 46) >> 4) * 4;
	bool allowed = false, live = true;
	const uint32_t port = wbe16(W, 36);
#pragma unroll
	for (int i = 0; i < 8; i++) {
		const uint32_t pv = cfg.ports[i];
		live = live && pv != 0;
		allowed = allowed || (live && pv == port);
	}
	const uint32_t fl = wb8(W, 47);
	return len0 >= 54 && wbe16(W, 12) == 0x0800 && wb8(W, 14) == 0x45 &&
	       wb8(W, 23) == 6 && tcp_len >= 20 && tcp_len <= 40 &&
	       len0 >= 34 + tcp_len && len0 + 60 - tcp_len <= (uint32_t)kRow &&
	       (wbe16(W, 20) & 0x7fff) == 0x4000 && allowed && (fl & 0x12) == 0x02 &&
	       60 - tcp_len <= room;
}

/* handle_syn on the common shape; len in: the grown length */
__device__ __forceinline__ uint32_t handle_syn_fast(const Frame &F, uint32_t (&W)[kW],
						    uint32_t &len,
						    const xdpgpu_synproxy_cfg &cfg,
						    bool &synack)
{
	const uint32_t tcp_len = (wb8(W, 46) >> 4) * 4;
	const uint32_t fl = wb8(W, 47);
	if (fl & 0x05)
		return SP_DROP;
	uint64_t s = 0;
#pragma unroll
	for (int k = 0; k < 5; k++)
		s += wle(W, 14 + 4 * k);
	if (fold(s) != 0)
		return SP_DROP;
	const uint32_t sa = wle(W, 26), da = wle(W, 30);
	s = (uint64_t)sa + da + ((uint64_t)(6 + tcp_len) << 8);
#pragma unroll
	for (int k = 0; k < 10; k++)
		s += 4 * k < (int)tcp_len ? wle(W, 34 + 4 * k) : 0u;
	if (fold(s) != 0)
		return SP_DROP;
	const uint32_t count = (uint32_t)(cfg.now_ns / 60000000000ull);
	const uint32_t seq = (uint32_t)wbe16(W, 38) << 16 | wbe16(W, 40);
	uint32_t cookie;
	{
		/* cookie_hash over (saddr, daddr, ports): jhash2(w, 9, key +
		 * count) with w[0] = saddr, w[4] = daddr, w[8] = the ports */
		uint32_t a = 0xdeadbeefu + (9u << 2) + cfg.cookie_key + count, b = a, c = a;
		a += sa;
		JH_MIX(a, b, c);
		b += da;
		JH_MIX(a, b, c);
		c += wbe16(W, 34) << 16 | wbe16(W, 36);
		JH_FINAL(a, b, c);
		cookie = c + seq;
	}
	/* tscookie_init (:274-308), on the row */
	Opt oc = {34 + 20, len, 0xf, 0, 0, 0};
	for (int i = 0; i < 42; i++)
		if (opt_parse(oc, F))
			break;
	uint32_t tsval = 0;
	if (oc.ts) {
		tsval = (uint32_t)(cfg.now_ns / 1000000ull) & ~0x3fu;
		tsval |= oc.wscale & 0xf;
		if (oc.sack)
			tsval |= 1u << 4;
		if ((fl & 0x40) && (fl & 0x80))
			tsval |= 1u << 5;
	}
	uint32_t mss, wscale, ttl;
	if (cfg.values) {
		mss = (uint32_t)cfg.values & 0xffff;
		wscale = (uint32_t)(cfg.values >> 16) & 0xf;
		ttl = (uint32_t)(cfg.values >> 24) & 0xff;
	} else {
		mss = 1460;
		wscale = 7;
		ttl = 64;
	}
	const bool ws = oc.ts && (tsval & 0xf) != 0xf;
	const uint32_t new_len = oc.ts ? (ws ? 40u : 36u) : 24u;

	/* tcpv4_gen_synack (:533-575), tcp_gen_synack (:512-531),
	 * tcp_mkoptions (:480-510) */
	uint32_t O[kW];
#pragma unroll
	for (int k = 0; k < kW; k++)
		O[k] = W[k];
#pragma unroll
	for (int i = 0; i < 6; i++) {
		wput(O, i, wb8(W, 6 + i));
		wput(O, 6 + i, wb8(W, i));
	}
	wput(O, 15, 0);
	wput_be16(O, 16, 20 + new_len);
	wput_be16(O, 18, 0);
	wput(O, 22, ttl);
	wput_be16(O, 24, 0);
	O[6] = (O[6] & 0x0000ffffu) | (da << 16);          /* bytes 26-29 */
	O[7] = (da >> 16) | (sa << 16);                     /* bytes 30-33 */
	O[8] = (O[8] & 0xffff0000u) | (sa >> 16);
	wput_be16(O, 34, wbe16(W, 36));
	wput_be16(O, 36, wbe16(W, 34));
	wput_be32(O, 38, cookie);
	wput_be32(O, 42, seq + 1);
	wput(O, 46, (new_len / 4) << 4);
	wput(O, 47, 0x12 | ((oc.ts && (tsval & (1u << 5))) ? 0x40 : 0));
	wput_be32(O, 48, 0);                                /* window, check */
	wput_be16(O, 52, 0);
	wput_be32(O, 54, 2u << 24 | 4u << 16 | (mss & 0xffff));
	if (oc.ts) {
		wput_be32(O, 58, (tsval & (1u << 4)) ? (4u << 24 | 2u << 16 | 8u << 8 | 10u)
						     : (1u << 24 | 1u << 16 | 8u << 8 | 10u));
		wput_be32(O, 62, tsval);
		wput(O, 66, oc.tsecr);
		wput(O, 67, oc.tsecr >> 8);
		wput(O, 68, oc.tsecr >> 16);
		wput(O, 69, oc.tsecr >> 24);
		if (ws)
			wput_be32(O, 70, 1u << 24 | 3u << 16 | 3u << 8 | wscale);
	}
	/* checksums (:679-704), stored as computed (LE u16) */
	s = (uint64_t)sa + da + ((uint64_t)(6 + new_len) << 8);
#pragma unroll
	for (int k = 0; k < 10; k++)
		s += 4 * k < (int)new_len ? wle(O, 34 + 4 * k) : 0u;
	const uint32_t c = fold(s);
	wput(O, 50, c);
	wput(O, 51, c >> 8);
	s = 0;
#pragma unroll
	for (int k = 0; k < 5; k++)
		s += wle(O, 14 + 4 * k);
	const uint32_t h = fold(s);
	wput(O, 24, h);
	wput(O, 25, h >> 8);
#pragma unroll
	for (int k = 0; k < kW; k++)
		W[k] = O[k];
	len = 34 + new_len;
	synack = true;
	return SP_TX;
}

__device__ __forceinline__ void put_verdict(uint8_t *v, uint32_t act)
{
	if constexpr ((SP_NT & 2) != 0)
		__builtin_nontemporal_store((uint8_t)act, v);
	else
		*v = (uint8_t)act;
}

/* one tile of kBlockS frames (one wave) from frame t0 on, dv this lane's
 * descriptor; true: this lane's frame was answered with a SYN-ACK */
__device__ __forceinline__ bool sp_tile(uint8_t *umem, uint64_t usize, uint4 dv,
					uint32_t n, const xdpgpu_synproxy_cfg &cfg,
					uint8_t *verdict, xdpgpu_desc *out, uint32_t *rows,
					uint64_t *dtab_all, uint2 *wtab_all, uint64_t t0)
{
	const uint64_t i = t0 + threadIdx.x;
	const bool active = i < n;
	uint8_t *row = reinterpret_cast<uint8_t *>(rows + threadIdx.x * kRowDw);
	const uint64_t addr = ((uint64_t)dv.y << 32) | dv.x;
	uint32_t len = dv.z;
	const uint64_t eff = (addr & ((1ull << 48) - 1)) + (addr >> 48);
	const bool valid = active && (uint64_t)len <= usize && eff <= usize - len;
	bool synack = false;
	uint32_t ws = 0, we = 0;   /* the byte range to write back (coop frames) */
	uint32_t own = 0;          /* the frame's buffer in the row */
	/* stage [0, kRow) of every lane's frame: 16-byte aligned frames whose
	 * row lies in the UMEM cooperatively (q = 64 k + lane: chunk q % kChunks
	 * of frame q / kChunks, kChunks lanes per frame reading its kRow bytes
	 * as whole chunks, each lane keeping the chunks it read for the
	 * write-back), the others byte by byte; zeros past each frame's end */
	uint64_t *dtab = dtab_all + (threadIdx.x & ~63u);
	const int lane = threadIdx.x & 63;
	const uint64_t us16 = usize & ~15ull;
	const bool coop = valid && !(eff & 15) && eff + kRow <= us16;
	dtab[lane] = coop ? eff : ~0ull;
	__builtin_amdgcn_wave_barrier();
	uint4 orig[kChunks];
#pragma unroll
	for (int k = 0; k < kChunks; k++) {
		const int q = 64 * k + lane;
		const int f = q / kChunks, c = q % kChunks;
		const uint64_t base = dtab[f];
		orig[k] = make_uint4(0, 0, 0, 0);
		if (base != ~0ull) {
			const uint4 v = *reinterpret_cast<const uint4 *>(umem + base + 16 * c);
			orig[k] = v;
			uint32_t *d = rows + ((threadIdx.x & ~63u) + f) * kRowDw + 4 * c;
			d[0] = v.x;
			d[1] = v.y;
			d[2] = v.z;
			d[3] = v.w;
		}
	}
	__builtin_amdgcn_wave_barrier();
	if (valid) {
		uint8_t *g = umem + eff;
		uint32_t *rw = rows + threadIdx.x * kRowDw;
		if (coop) {
			for (uint32_t w = 0; w < (uint32_t)kRow / 4; w++) {
				if (4 * w + 4 > len)
					rw[w] = 4 * w >= len ? 0u : rw[w] & (0xffffffffu >> (8 * (4 * w + 4 - len)));
			}
		} else {
			const uint32_t st = len < (uint32_t)kRow ? len : (uint32_t)kRow;
			for (uint32_t k = 0; k < (uint32_t)kRow; k++)
				row[k] = k < st ? g[k] : 0;
		}
		const Frame F = {row, g, len};
		uint64_t room = usize - eff - len;
		if (room > cfg.tailroom)
			room = cfg.tailroom;
		uint32_t grow = 0;
		const uint32_t len0 = len;
		uint32_t act;
		uint32_t W[kW];
#pragma unroll
		for (int k = 0; k < kW; k++)
			W[k] = rw[k];
		if (coop && syn_fast_shape(W, len0, room, cfg)) {
			/* sp_frame's growth (:389-404), then handle_syn */
			grow = 60 - (wb8(W, 46) >> 4) * 4;
			len += grow;
			act = handle_syn_fast(F, W, len, cfg, synack);
			if (act == SP_TX) {
#pragma unroll
				for (int k = 0; k < kW; k++)
					rw[k] = W[k];
			}
		} else {
			act = sp_frame(F, len, room, cfg, synack, grow);
		}
		/* the bytes to write back: the SYN-ACK and the rest of the growth
		 * (zeros), or the growth of a frame passed or dropped after it */
		ws = act == SP_TX ? 0u : len0;
		we = grow ? len0 + grow : 0u;
		if (act == SP_TX && len > we)
			we = len;
		if (we > (uint32_t)kRow) {
			/* past the row: zeros of the growth only */
			for (uint32_t k = len0 > (uint32_t)kRow ? len0 : (uint32_t)kRow; k < we; k++)
				g[k] = 0;
			we = kRow;
		}
		if (!coop) {
			for (uint32_t k = ws; k < we; k++)
				g[k] = row[k];
			ws = we = 0;
		}
		/* the frame's buffer: its bytes and the room it may grow into */
		own = (uint32_t)min((uint64_t)len0 + room, (uint64_t)kRow);
		put_verdict(verdict + i, act);
	} else if (active) {
		put_verdict(verdict + i, SP_ABORTED);
	}
	/* cooperative write-back of the 16-byte aligned frames' ranges
	 * [ws, we) from their rows: whole chunks as 16-byte stores (kWb >= 1:
	 * also a partial chunk inside the frame's buffer, its other bytes from
	 * the staged copy; kWb 2: the whole 64-byte sectors the range touches,
	 * inside the buffer), the other partial ones by dwords and bytes */
	uint2 *wtab = wtab_all + (threadIdx.x & ~63u);
	uint32_t *otab = reinterpret_cast<uint32_t *>(wtab + 64);
	wtab[lane] = make_uint2(ws, we);
	otab[lane] = own;
	__builtin_amdgcn_wave_barrier();
#pragma unroll
	for (int k = 0; k < kChunks; k++) {
		const int q = 64 * k + lane;
		const int f = q / kChunks, c = q % kChunks;
		const uint2 r = wtab[f];
		const uint32_t lo = 16 * c, hi = lo + 16;
		if (r.x >= r.y)
			continue;
		const uint32_t ob = otab[f] & ~15u;   /* whole chunks of the buffer */
		uint32_t x0 = r.x, x1 = r.y;          /* the chunks to store */
		if (kWb >= 2) {
			x0 = r.x & ~63u;
			x1 = min((r.y + 63) & ~63u, ob);
			x1 = x1 > r.y ? x1 : r.y;
		}
		if (x1 <= lo || x0 >= hi)
			continue;
		const uint64_t base = dtab[f];
		const uint32_t *src = rows + ((threadIdx.x & ~63u) + f) * kRowDw + 4 * c;
		uint8_t *dst = umem + base + lo;
		if (kWb >= 1 && hi <= ob && lo >= x0) {
			/* the changed bytes [r.x, r.y) from the row, the rest as
			 * staged */
			const uint32_t o4[4] = {orig[k].x, orig[k].y, orig[k].z, orig[k].w};
			uint32_t v[4];
#pragma unroll
			for (int d = 0; d < 4; d++) {
				uint32_t m = 0;
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const uint32_t b = lo + 4 * d + j;
					m |= (b >= r.x && b < r.y) ? 0xffu << (8 * j) : 0u;
				}
				v[d] = m == ~0u ? src[d] : (m ? (src[d] & m) | (o4[d] & ~m) : o4[d]);
			}
			if constexpr ((SP_NT & 1) != 0) {
				typedef uint32_t v4u __attribute__((ext_vector_type(4)));
				const v4u x = {v[0], v[1], v[2], v[3]};
				__builtin_nontemporal_store(x, reinterpret_cast<v4u *>(dst));
			} else {
				*reinterpret_cast<uint4 *>(dst) = make_uint4(v[0], v[1], v[2], v[3]);
			}
		} else if (r.y <= lo || r.x >= hi) {
			continue;
		} else if (r.x <= lo && r.y >= hi) {
			*reinterpret_cast<uint4 *>(dst) = make_uint4(src[0], src[1], src[2], src[3]);
		} else {
			const uint32_t a0 = r.x > lo ? r.x - lo : 0u;
			const uint32_t b0 = r.y < hi ? r.y - lo : 16u;
			for (uint32_t j = a0; j < b0; j++) {
				if (!(j & 3) && j + 4 <= b0) {
					*reinterpret_cast<uint32_t *>(dst + j) = src[j >> 2];
					j += 3;
				} else {
					dst[j] = (uint8_t)(src[j >> 2] >> (8 * (j & 3)));
				}
			}
		}
	}
	if (active) {
		uint4 od = dv;
		od.z = len;
		if constexpr ((SP_NT & 2) != 0) {
			typedef uint32_t v4u __attribute__((ext_vector_type(4)));
			const v4u x = {od.x, od.y, od.z, od.w};
			__builtin_nontemporal_store(x, reinterpret_cast<v4u *>(out + i));
		} else {
			*reinterpret_cast<uint4 *>(out + i) = od;
		}
	}
	__builtin_amdgcn_wave_barrier();
	return synack;
}

/* One wave per tile.  The SYN-ACK count (values[1], values_inc_synacks,
 * :332-340) goes to one of kSpread counters picked by the block index (one
 * atomic per wave on a single word serialised the launch: 1.7 ms per 8 M
 * SYNs), which synproxy_sum_kernel adds to the caller's counter. */
constexpr int kSpread = 256;
/* waves per SIMD the register allocation targets (build knob for A/B): 5
 * or more spill (122 VGPRs at 4) */
#ifndef SP_MINW
#define SP_MINW 1
#endif
__global__ __launch_bounds__(kBlockS, SP_MINW) void synproxy_kernel(uint8_t *umem, uint64_t usize,
							   const xdpgpu_desc *desc, uint32_t n,
							   xdpgpu_synproxy_cfg cfg, uint8_t *verdict,
							   xdpgpu_desc *out,
							   unsigned long long *spread)
{
	__shared__ uint32_t rows[kBlockS * kRowDw];
	__shared__ uint64_t dtab_all[kBlockS];
	__shared__ uint2 wtab_all[kBlockS + kBlockS / 2];   /* ranges, then buffers */
	const uint64_t ntiles = ((uint64_t)n + kBlockS - 1) / kBlockS;
	auto ld = [&](uint64_t t) -> uint4 {
		const uint64_t i = t * kBlockS + threadIdx.x;
		return t < ntiles && i < n ? *reinterpret_cast<const uint4 *>(desc + i)
					   : make_uint4(0, 0, 0, 0);
	};
	uint64_t cnt = 0;
	uint64_t t = blockIdx.x;
	uint4 dv = ld(t);
	while (t < ntiles) {
		const uint64_t tn = SP_PERSIST ? t + gridDim.x : ntiles;
		const uint4 dn = SP_PERSIST ? ld(tn) : make_uint4(0, 0, 0, 0);
		const bool synack = sp_tile(umem, usize, dv, n, cfg, verdict, out, rows, dtab_all,
					    wtab_all, t * kBlockS);
		cnt += __popcll(__ballot(synack));
		dv = dn;
		t = tn;
	}
	if (spread && cnt && threadIdx.x == 0)
		atomicAdd(spread + 16 * (blockIdx.x % kSpread), (unsigned long long)cnt);
}

/* the spread counters into the caller's, and cleared for the next launch */
__global__ void synproxy_sum_kernel(unsigned long long *spread, unsigned long long *synacks)
{
	unsigned long long v = spread[16 * threadIdx.x];
	spread[16 * threadIdx.x] = 0;
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o);
	__shared__ unsigned long long part[kSpread / 64];
	if ((threadIdx.x & 63) == 0)
		part[threadIdx.x / 64] = v;
	__syncthreads();
	if (threadIdx.x == 0) {
		unsigned long long t = 0;
		for (int k = 0; k < kSpread / 64; k++)
			t += part[k];
		*synacks += t;
	}
}

} // namespace

hipError_t launch_synproxy(uint8_t *umem, uint64_t usize, const xdpgpu_desc *desc,
			   uint32_t n, const xdpgpu_synproxy_cfg &cfg, uint8_t *verdict,
			   xdpgpu_desc *out, unsigned long long *synacks,
			   unsigned long long *spread, hipStream_t stream)
{
	uint32_t blocks = (n + kBlockS - 1) / kBlockS;
	if (!blocks)
		return hipSuccess;
	if (SP_PERSIST) {
		const uint32_t cap = resident_blocks_dev<synproxy_kernel, kBlockS>(8192);
		blocks = blocks < cap ? blocks : cap;
	}
	hipLaunchKernelGGL(synproxy_kernel, dim3(blocks), dim3(kBlockS), 0, stream, umem, usize,
			   desc, n, cfg, verdict, out, synacks ? spread : nullptr);
	hipError_t e = hipGetLastError();
	if (e != hipSuccess || !synacks)
		return e;
	hipLaunchKernelGGL(synproxy_sum_kernel, dim3(1), dim3(kSpread), 0, stream, spread,
			   synacks);
	return hipGetLastError();
}

uint32_t synproxy_spread_words()
{
	return 16 * kSpread;
}

} // namespace xdpgpu
