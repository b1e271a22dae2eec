// SPDX-License-Identifier: GPL-2.0
/*
 * ref_harness.c - TEST INFRASTRUCTURE ONLY.
 *
 * Thin exported wrappers around the reference's OWN header-only code, which
 * is compiled where it lies under /root/reference (see oracle/Makefile; the
 * output goes to oracle/_ref/libref.so and never into git).  No reference
 * source is copied here: the headers are #included from the reference tree.
 *   AF_XDP-interaction/lib_checksum.h   (do_csum, ip_fast_csum, udp_csum, ...)
 *   include/jhash.h                     (jhash, jhash2, jhash_3words)
 * Used only to pin oracle/xdp_oracle.c and to build tests/golden/.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <arpa/inet.h>
#include <linux/types.h>

#include "lib_checksum.h"
#include "jhash.h"

uint32_t ref_do_csum(const unsigned char *buf, int len) { return do_csum(buf, len); }
uint16_t ref_ip_fast_csum(const void *iph, unsigned int ihl) { return (uint16_t)ip_fast_csum(iph, ihl); }
uint16_t ref_csum_fold(uint32_t c) { return (uint16_t)csum_fold((__wsum)c); }
uint32_t ref_csum_tcpudp_nofold(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, uint32_t sum)
{ return (uint32_t)csum_tcpudp_nofold(s, d, len, proto, sum); }
uint16_t ref_csum_tcpudp_magic(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, uint32_t sum)
{ return (uint16_t)csum_tcpudp_magic(s, d, len, proto, sum); }
uint16_t ref_udp_csum(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, void *l4)
{ return udp_csum(s, d, len, proto, (__u16 *)l4); }
void ref_memset32_htonl(void *dest, uint32_t val, uint32_t size) { memset32_htonl(dest, val, size); }
uint32_t ref_jhash(const void *key, uint32_t len, uint32_t initval) { return jhash(key, len, initval); }
uint32_t ref_jhash2(const uint32_t *k, uint32_t len, uint32_t initval) { return jhash2(k, len, initval); }
uint32_t ref_jhash_3words(uint32_t a, uint32_t b, uint32_t c, uint32_t iv) { return jhash_3words(a, b, c, iv); }
uint32_t ref_jhash_2words(uint32_t a, uint32_t b, uint32_t iv) { return jhash_2words(a, b, iv); }
uint32_t ref_jhash_1word(uint32_t a, uint32_t iv) { return jhash_1word(a, iv); }

/* Calibration probe (SURVEY.md §5 "survey probe"): per frame a minimal
 * Ethernet/VLAN/IPv4/UDP parse, ip_fast_csum over the IPv4 header,
 * udp_csum over the UDP datagram and jhash of 13 bytes (addresses, ports,
 * protocol), all by the reference headers' own routines; the same work as
 * cpu_leg_probe (oracle/cpu_leg.c).  Returns wall seconds of reps passes on
 * the calling thread; *acc receives a value of the results (kept live). */
#include <string.h>
#include <time.h>

struct ref_desc { uint64_t addr; uint32_t len; uint32_t options; };

double ref_probe(const uint8_t *umem, uint64_t umem_size, const struct ref_desc *d,
		 uint32_t n, uint32_t reps, uint64_t *acc)
{
	struct timespec t0, t1;
	uint64_t x = 0;
	uint32_t r, i;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (r = 0; r < reps; r++) {
		for (i = 0; i < n; i++) {
			const uint64_t eff = (d[i].addr & ((1ull << 48) - 1)) + (d[i].addr >> 48);
			const uint32_t len = d[i].len;
			const uint8_t *p = umem + eff;
			uint32_t l3 = 14, cl, sa, da;
			uint16_t et;
			uint8_t key[13];

			if (len < 42 || eff > umem_size - len)
				continue;
			memcpy(&et, p + 12, 2);
			if (et == htons(0x8100))
				l3 = 18;
			memcpy(&et, p + l3 - 2, 2);
			if (et != htons(0x0800) || p[l3] != 0x45 || p[l3 + 9] != 17)
				continue;
			x += (uint16_t)ip_fast_csum(p + l3, 5);
			cl = ntohs(*(const uint16_t *)(p + l3 + 24));
			if (l3 + 20 + cl > len)
				continue;
			memcpy(&sa, p + l3 + 12, 4);
			memcpy(&da, p + l3 + 16, 4);
			x += udp_csum(sa, da, cl, 17, (__u16 *)(p + l3 + 20));
			memcpy(key, p + l3 + 12, 8);
			memcpy(key + 8, p + l3 + 20, 4);
			key[12] = 17;
			x += jhash(key, 13, 0);
		}
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	*acc = x;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------ */
/* The reference-routine leg of bench.py's cpu_baseline: the RX per-frame
 * work of oracle/cpu_leg.c (same shape test, same outputs) with every
 * checksum and hash computed by the reference headers' own routines, in
 * the reference's idiom: ip_fast_csum over the header as stored for the
 * verify and again with the check word zeroed for the recompute
 * (af_xdp_user.c:664-665), udp_csum the same way for the L4 checksum
 * (lib_checksum.h:168-179; verify = recompute over stored == 0), jhash
 * over the 44-byte network_tuple (jhash.h:68-105).  The check words are
 * zeroed in place and restored (each thread owns its slice of frames).
 * Parse is restated (parsing_helpers.h needs libbpf, absent).  Frames of
 * any other shape go through the oracle (liboracle.so). */
#include <pthread.h>
#include <sched.h>
#include "xdpgpu.h"

void oracle_frame_one(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *d,
		      uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		      uint32_t i, uint8_t *verdict, struct xdpgpu_result *res,
		      void *tuples, struct xdpgpu_stats *stats);

static inline uint16_t rl16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint32_t rl32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

static int ref_frame(uint8_t *umem, uint64_t usize, const struct xdpgpu_desc *d,
		     uint32_t flags, uint32_t iv, uint32_t fmt, uint32_t i,
		     uint8_t *verdict, struct xdpgpu_result *res, uint8_t *tup)
{
	const uint64_t eff = (d->addr & ((1ull << 48) - 1)) + (d->addr >> 48);
	const uint32_t len = d->len;
	uint32_t nv = 0, l3, l4, tot, proto, cl, chk, sa, da, ports;
	uint8_t *p;
	int udp;

	if (len < 42 || (uint64_t)len > usize || eff > usize - len)
		return 0;
	p = umem + eff;
	{
		uint16_t et = rl16(p + 12);

		if (et == htons(0x8100) || et == htons(0x88A8)) {
			nv = 1;
			et = rl16(p + 16);
			if (et == htons(0x8100) || et == htons(0x88A8)) {
				nv = 2;
				et = rl16(p + 20);
			}
		}
		if (et != htons(0x0800))
			return 0;
	}
	l3 = 14 + 4 * nv;
	l4 = l3 + 20;
	if (p[l3] != 0x45 || (rl16(p + l3 + 6) & htons(0x3fff)) != 0)
		return 0;
	proto = p[l3 + 9];
	udp = proto == 17;
	if (!udp && proto != 6)
		return 0;
	tot = ntohs(rl16(p + l3 + 2));
	if (tot < 20 || l3 + tot > len)
		return 0;
	if (udp) {
		if (len < l4 + 8)
			return 0;
		cl = ntohs(rl16(p + l4 + 4));
		if (cl < 8 || l4 + cl > l3 + tot)
			return 0;
		chk = 6;
	} else {
		uint32_t thl;

		if (len < l4 + 20)
			return 0;
		thl = (uint32_t)(p[l4 + 12] >> 4) * 4;
		cl = tot - 20;
		if (thl < 20 || l4 + thl > len || cl < thl)
			return 0;
		chk = 16;
	}
	/* udp_csum reads one byte past an odd length: inside the UMEM here
	 * (the oracle takes frames whose over-read byte is past the end) */
	if ((cl & 1) && eff + l4 + cl >= usize)
		return 0;
	sa = rl32(p + l3 + 12);
	da = rl32(p + l3 + 16);
	/* IPv4 header: verify as stored, recompute with the check zeroed */
	const int l3_ok = (uint16_t)ip_fast_csum(p + l3, 5) == 0;
	const uint16_t c3 = rl16(p + l3 + 10);
	memset(p + l3 + 10, 0, 2);
	const uint16_t l3c = (uint16_t)ip_fast_csum(p + l3, 5);
	memcpy(p + l3 + 10, &c3, 2);
	/* L4: udp_csum over the stored datagram (verify), then zeroed */
	const uint16_t c4 = rl16(p + l4 + chk);
	const int absent = udp && c4 == 0;
	const int l4_ok = absent || udp_csum(sa, da, cl, (uint8_t)proto, (__u16 *)(p + l4)) == 0;
	memset(p + l4 + chk, 0, 2);
	const uint16_t l4c = udp_csum(sa, da, cl, (uint8_t)proto, (__u16 *)(p + l4));
	memcpy(p + l4 + chk, &c4, 2);
	const int drop = (flags & XDPGPU_CFG_VERIFY_CSUM) && (!l3_ok || !l4_ok);
	ports = rl32(p + l4);
	const uint32_t key[11] = {0, 0, htonl(0xffff), sa, ports & 0xffff,
				  0, 0, htonl(0xffff), da, ports >> 16, proto | (2u << 16)};
	if (res) {
		uint32_t w[4];

		w[0] = jhash(key, 44, iv);
		w[1] = l3c | ((uint32_t)l4c << 16);
		w[2] = XDPGPU_F_IP | XDPGPU_F_L4 | (nv ? XDPGPU_F_VLAN : 0u) |
		       (l3_ok ? XDPGPU_F_L3_OK : 0u) | (l4_ok ? XDPGPU_F_L4_OK : 0u) |
		       (absent ? XDPGPU_F_L4_ABSENT : 0u) | (proto << 8) | (l3 << 16) | (nv << 24);
		w[3] = l4 | (cl << 16);
		memcpy(&res[i], w, 16);
	}
	if (tup && fmt == XDPGPU_TUPLE_V4) {
		const uint32_t vid = nv ? (ntohs(rl16(p + 14)) & 0x0fff) : 0u;
		const uint32_t t[4] = {sa, da, ports, proto | (2u << 8) | (vid << 16)};

		memcpy(tup + (size_t)i * 16, t, 16);
	} else if (tup && fmt == XDPGPU_TUPLE_NET) {
		memcpy(tup + (size_t)i * 44, key, 44);
	}
	verdict[i] = drop ? XDPGPU_DROP : XDPGPU_REDIRECT;
	return 1;
}

struct ref_slice {
	uint8_t *umem;
	uint64_t usize;
	const struct xdpgpu_desc *descs;
	uint32_t n, flags, iv, fmt, reps;
	int cpu;
	uint8_t *verdict;
	struct xdpgpu_result *res;
	uint8_t *tup;
};

static void *ref_worker(void *arg)
{
	struct ref_slice *s = (struct ref_slice *)arg;
	struct xdpgpu_stats st;
	uint32_t r, i;

	if (s->cpu >= 0) {
		cpu_set_t set;

		CPU_ZERO(&set);
		CPU_SET(s->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	for (r = 0; r < s->reps; r++)
		for (i = 0; i < s->n; i++)
			if (!ref_frame(s->umem, s->usize, &s->descs[i], s->flags, s->iv, s->fmt, i,
				       s->verdict, s->res, s->tup)) {
				memset(&st, 0, sizeof(st));
				oracle_frame_one(s->umem, s->usize, &s->descs[i], s->flags, s->iv,
						 s->fmt, i, s->verdict, s->res, s->tup, &st);
			}
	return NULL;
}

/* As cpu_leg_bench (oracle/cpu_leg.c): reps passes over descs on threads
 * threads, contiguous slices, pinned one per CPU of the affinity set.
 * Returns wall seconds; the outputs of the last pass are left in verdict,
 * res, tuples (bit-exact with the oracle: tests/test_oracle.py). */
double ref_leg_bench(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		     uint32_t n, uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		     uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		     uint32_t threads, uint32_t reps, int pin)
{
	enum { kMax = 1024 };
	static struct ref_slice sl[kMax];
	pthread_t th[kMax];
	int cpus[kMax];
	struct timespec t0, t1;
	const uint32_t tsz = tuple_fmt == XDPGPU_TUPLE_NET ? 44 :
			     tuple_fmt == XDPGPU_TUPLE_V4 ? 16 : 0;
	uint32_t i, per, ncpu = 0;
	cpu_set_t set;

	if (cfg_flags & (XDPGPU_CFG_FRAGS | XDPGPU_CFG_ICMP6_ECHO))
		return -1.0;
	if (threads == 0)
		threads = 1;
	if (threads > kMax)
		threads = kMax;
	if (sched_getaffinity(0, sizeof(set), &set) == 0)
		for (i = 0; i < CPU_SETSIZE && ncpu < kMax; i++)
			if (CPU_ISSET(i, &set))
				cpus[ncpu++] = (int)i;
	per = (n + threads - 1) / threads;
	for (i = 0; i < threads; i++) {
		uint32_t lo = i * per, hi = lo + per;

		if (lo > n)
			lo = n;
		if (hi > n)
			hi = n;
		memset(&sl[i], 0, sizeof(sl[i]));
		sl[i].umem = umem;
		sl[i].usize = umem_size;
		sl[i].descs = descs + lo;
		sl[i].n = hi - lo;
		sl[i].flags = cfg_flags;
		sl[i].iv = initval;
		sl[i].fmt = tuple_fmt;
		sl[i].reps = reps;
		sl[i].cpu = (pin && ncpu) ? cpus[i % ncpu] : -1;
		sl[i].verdict = verdict + lo;
		sl[i].res = res ? res + lo : NULL;
		sl[i].tup = tuples ? (uint8_t *)tuples + (size_t)lo * tsz : NULL;
	}
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (i = 0; i < threads; i++)
		pthread_create(&th[i], NULL, ref_worker, &sl[i]);
	for (i = 0; i < threads; i++)
		pthread_join(th[i], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
