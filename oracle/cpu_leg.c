// SPDX-License-Identifier: GPL-2.0
/*
 * cpu_leg.c - TEST INFRASTRUCTURE ONLY: the lean CPU baseline of bench.py.
 *
 * The RX per-frame path (parse, IPv4 header checksum, TCP/UDP checksum with
 * the pseudo header, jhash of the flow key, verdict) written for speed on a
 * CPU core, with the oracle's outputs: one pass over the bytes, the check
 * word left out of the sum instead of zeroed and restored, one fold per
 * checksum, unaligned little-endian loads.  Frames of the common shape
 * (Ethernet, at most two VLAN tags, IPv4 without options or fragmentation,
 * TCP or UDP with consistent lengths) take that path; every other frame goes
 * through the oracle's own pipeline (oracle_frame_one).  The outputs are
 * bit-exact with oracle_process on every frame (tests/test_cpu_leg.py), so
 * the timed baseline does the reference's work, not less.
 *
 * Why a second CPU path: oracle_process restates the reference loop for
 * loop (do_csum's alignment branches, the verify and the recompute as two
 * passes, lib_checksum.h:40-179) and ran ~7 Mpps per core, against ~55 Mpps
 * per core for the reference headers' own routines on this host (SURVEY.md
 * §5 probe): not the reference's speed.  The calibration of this leg
 * against the reference headers is cpu_leg_probe / ref_probe (same work as
 * the survey probe), DESIGN.md "CPU baseline".
 *
 * Arithmetic (one's complement, order-free): a 16-bit word at an even frame
 * offset is its little-endian value; a 32-bit little-endian load is the sum
 * of its two words mod 0xffff; fold16 maps a sum to 1..0xffff (0 only for
 * 0) like the reference's csum_fold input, so ~fold16 is the checksum
 * field and fold16(sum + stored) == 0xffff is the verify (RFC 1071).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

void oracle_frame_one(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *d,
		      uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		      uint32_t i, uint8_t *verdict, struct xdpgpu_result *res,
		      void *tuples, struct xdpgpu_stats *stats);

static inline uint32_t ld32(const uint8_t *p)
{
	uint32_t v;

	memcpy(&v, p, 4);
	return v;
}

static inline uint64_t ld64(const uint8_t *p)
{
	uint64_t v;

	memcpy(&v, p, 8);
	return v;
}

static inline uint16_t ld16(const uint8_t *p)
{
	uint16_t v;

	memcpy(&v, p, 2);
	return v;
}

static inline uint32_t bswap16(uint32_t v)
{
	return ((v & 0xff) << 8) | ((v >> 8) & 0xff);
}

static inline uint32_t fold16(uint64_t x)
{
	x = (x & 0xffffffffull) + (x >> 32);
	x = (x & 0xffffffffull) + (x >> 32);
	uint32_t y = (uint32_t)x;

	y = (y & 0xffff) + (y >> 16);
	y = (y & 0xffff) + (y >> 16);
	return y;
}

/* include/jhash.h:68-105 over the 11-word flow key (length 44) */
#define ROL32(w, s) (((w) << (s)) | ((w) >> (32 - (s))))
#define JMIX(a, b, c)                                                          \
	do {                                                                   \
		a -= c; a ^= ROL32(c, 4);  c += b;                             \
		b -= a; b ^= ROL32(a, 6);  a += c;                             \
		c -= b; c ^= ROL32(b, 8);  b += a;                             \
		a -= c; a ^= ROL32(c, 16); c += b;                             \
		b -= a; b ^= ROL32(a, 19); a += c;                             \
		c -= b; c ^= ROL32(b, 4);  b += a;                             \
	} while (0)
#define JFINAL(a, b, c)                                                        \
	do {                                                                   \
		c ^= b; c -= ROL32(b, 14);                                     \
		a ^= c; a -= ROL32(c, 11);                                     \
		b ^= a; b -= ROL32(a, 25);                                     \
		c ^= b; c -= ROL32(b, 16);                                     \
		a ^= c; a -= ROL32(c, 4);                                      \
		b ^= a; b -= ROL32(a, 14);                                     \
		c ^= b; c -= ROL32(b, 24);                                     \
	} while (0)

static inline uint32_t jhash_key44(const uint32_t k[11], uint32_t iv)
{
	uint32_t a, b, c;

	a = b = c = 0xdeadbeefu + 44u + iv;
	a += k[0]; b += k[1]; c += k[2];
	JMIX(a, b, c);
	a += k[3]; b += k[4]; c += k[5];
	JMIX(a, b, c);
	a += k[6]; b += k[7]; c += k[8];
	JMIX(a, b, c);
	a += k[9]; b += k[10];
	JFINAL(a, b, c);
	return c;
}

/* Sum of the bytes [0, n) of b as 16-bit little-endian words (n even),
 * 8 bytes a step. */
static inline uint64_t sum_bytes(const uint8_t *b, uint32_t n)
{
	uint64_t s = 0, t;
	uint32_t k = 0;

	for (; k + 8 <= n; k += 8) {
		t = ld64(b + k);
		s += (t & 0xffffffffull) + (t >> 32);
	}
	if (k + 4 <= n) {
		s += ld32(b + k);
		k += 4;
	}
	if (k + 2 <= n)
		s += ld16(b + k);
	return s;
}

struct leg_out {
	uint8_t *verdict;
	struct xdpgpu_result *res;
	uint8_t *tup;
	struct xdpgpu_stats *st;
};

/* One frame; returns 0 when it is not of the fast shape (nothing written). */
static inline int fast_frame(const uint8_t *umem, uint64_t usize,
			     const struct xdpgpu_desc *d, uint32_t flags,
			     uint32_t iv, uint32_t fmt, uint32_t i,
			     const struct leg_out *o)
{
	const uint64_t eff = (d->addr & ((1ull << 48) - 1)) + (d->addr >> 48);
	const uint32_t len = d->len;
	const uint8_t *p;
	uint32_t nv = 0, l3, l4, tot, proto, cl, c3, c4, chk, sa, da, ports;
	uint64_t s3, s4;
	int udp, l3_ok, l4_ok, absent, drop;

	if (len < 42 || (uint64_t)len > usize || eff > usize - len)
		return 0;
	p = umem + eff;
	{
		uint32_t et = ld16(p + 12);

		if (et == 0x0081 || et == 0xa888) {
			nv = 1;
			et = ld16(p + 16);
			if (et == 0x0081 || et == 0xa888) {
				nv = 2;
				et = ld16(p + 20);
			}
		}
		if (et != 0x0008)
			return 0;
	}
	l3 = 14 + 4 * nv;
	l4 = l3 + 20;
	/* version 4, ihl 5; no fragment bits; TCP or UDP */
	if (p[l3] != 0x45 || (ld16(p + l3 + 6) & 0xff3f) != 0)
		return 0;
	proto = p[l3 + 9];
	udp = proto == 17;
	if (!udp && proto != 6)
		return 0;
	tot = bswap16(ld16(p + l3 + 2));
	if (tot < 20 || l3 + tot > len)
		return 0;
	if (udp) {
		if (len < l4 + 8)
			return 0;
		cl = bswap16(ld16(p + l4 + 4));
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

	/* IPv4 header: 10 words, the check word (l3 + 10) left out */
	c3 = ld16(p + l3 + 10);
	{
		const uint64_t h0 = ld64(p + l3), h1 = ld64(p + l3 + 12);

		s3 = (h0 & 0xffffffffull) + (h0 >> 32) + ld16(p + l3 + 8) +
		     (h1 & 0xffffffffull) + (h1 >> 32);
	}
	l3_ok = fold16(s3 + c3) == 0xffff;

	/* L4: pseudo header (saddr, daddr, proto, length) + [l4, l4 + cl)
	 * with udp_csum's odd over-read byte (0 past the UMEM,
	 * lib_checksum.h:142-179), the check word left out */
	sa = ld32(p + l3 + 12);
	da = ld32(p + l3 + 16);
	c4 = ld16(p + l4 + chk);
	s4 = (uint64_t)sa + da + ((uint64_t)(proto + cl) << 8) +
	     sum_bytes(p + l4, cl & ~1u) - c4;
	if (cl & 1) {
		const uint64_t at = eff + l4 + cl;

		s4 += (uint64_t)p[l4 + cl - 1] | ((uint64_t)(at < usize ? umem[at] : 0) << 8);
	}
	/* s4 > 0: the words summed include c4, and the pseudo header is
	 * not 0; so fold16 of s4 and of the masked sum agree */
	absent = udp && c4 == 0;
	{
		const uint32_t sum4 = fold16(s4);

		l4_ok = absent || (~fold16((uint64_t)sum4 + c4) & 0xffff) == 0;
		drop = (flags & XDPGPU_CFG_VERIFY_CSUM) && (!l3_ok || !l4_ok);
		ports = ld32(p + l4);
		if (o->res) {
			uint32_t key[11] = {0, 0, 0xffff0000u, sa, ports & 0xffff,
					    0, 0, 0xffff0000u, da, ports >> 16,
					    proto | (2u << 16)};
			uint32_t w[4];

			w[0] = jhash_key44(key, iv);
			w[1] = (~fold16(s3) & 0xffff) | ((~sum4 & 0xffff) << 16);
			w[2] = XDPGPU_F_IP | XDPGPU_F_L4 | (nv ? XDPGPU_F_VLAN : 0u) |
			       (l3_ok ? XDPGPU_F_L3_OK : 0u) | (l4_ok ? XDPGPU_F_L4_OK : 0u) |
			       (absent ? XDPGPU_F_L4_ABSENT : 0u) | (proto << 8) |
			       (l3 << 16) | (nv << 24);
			w[3] = l4 | (cl << 16);
			memcpy(&o->res[i], w, 16);
		}
		if (o->tup && fmt == XDPGPU_TUPLE_V4) {
			const uint32_t vid = nv ? (bswap16(ld16(p + 14)) & 0x0fff) : 0u;
			const uint32_t t[4] = {sa, da, ports, proto | (2u << 8) | (vid << 16)};

			memcpy(o->tup + (size_t)i * 16, t, 16);
		} else if (o->tup && fmt == XDPGPU_TUPLE_NET) {
			const uint32_t key[11] = {0, 0, 0xffff0000u, sa, ports & 0xffff,
						  0, 0, 0xffff0000u, da, ports >> 16,
						  proto | (2u << 16)};

			memcpy(o->tup + (size_t)i * 44, key, 44);
		}
	}
	o->verdict[i] = drop ? XDPGPU_DROP : XDPGPU_REDIRECT;
	if (o->st) {
		o->st->frames++;
		o->st->bytes += len;
		o->st->verdict[drop ? XDPGPU_DROP : XDPGPU_REDIRECT]++;
		o->st->l3_bad += !l3_ok;
		o->st->l4_bad += !l4_ok;
		o->st->l4_absent += absent;
	}
	return 1;
}

/* xdpgpu_process_dev's outputs for a batch of single-descriptor frames
 * (no XDPGPU_CFG_FRAGS, no XDPGPU_CFG_ICMP6_ECHO: those go to the oracle
 * whole).  Returns the number of frames of the fast shape. */
uint32_t cpu_leg_process(uint8_t *umem, uint64_t umem_size,
			 const struct xdpgpu_desc *descs, uint32_t n,
			 uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
			 uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
			 struct xdpgpu_stats *stats)
{
	const struct leg_out o = {verdict, res, (uint8_t *)tuples, stats};
	uint32_t i, nfast = 0;

	if (cfg_flags & (XDPGPU_CFG_FRAGS | XDPGPU_CFG_ICMP6_ECHO)) {
		oracle_process(umem, umem_size, descs, n, cfg_flags, initval, tuple_fmt,
			       verdict, res, tuples, stats);
		return 0;
	}
	for (i = 0; i < n; i++) {
		if (fast_frame(umem, umem_size, &descs[i], cfg_flags, initval, tuple_fmt,
			       i, &o)) {
			nfast++;
			continue;
		}
		oracle_frame_one(umem, umem_size, &descs[i], cfg_flags, initval, tuple_fmt,
				 i, verdict, res, tuples, stats);
	}
	return nfast;
}

/* ------------------------------------------------------------------ */
/* timing harness                                                      */

struct leg_slice {
	uint8_t *umem;
	uint64_t usize;
	const struct xdpgpu_desc *descs;
	uint32_t n, flags, iv, fmt, reps;
	int cpu;                      /* pin to this CPU, -1: no pinning */
	uint8_t *verdict;
	struct xdpgpu_result *res;
	uint8_t *tup;
	struct xdpgpu_stats st;
};

static void *leg_worker(void *arg)
{
	struct leg_slice *s = (struct leg_slice *)arg;
	uint32_t r;

	if (s->cpu >= 0) {
		cpu_set_t set;

		CPU_ZERO(&set);
		CPU_SET(s->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	for (r = 0; r < s->reps; r++)
		cpu_leg_process(s->umem, s->usize, s->descs, s->n, s->flags, s->iv,
				s->fmt, s->verdict, s->res, s->tup, &s->st);
	return NULL;
}

/* `reps` passes over descs on `threads` threads, each a contiguous slice
 * and (pin) pinned to the i-th CPU of the process's affinity set.  Returns
 * wall seconds. */
double cpu_leg_bench(uint8_t *umem, uint64_t umem_size,
		     const struct xdpgpu_desc *descs, uint32_t n,
		     uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		     uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		     uint32_t threads, uint32_t reps, int pin)
{
	enum { kMax = 1024 };
	static struct leg_slice sl[kMax];
	pthread_t th[kMax];
	int cpus[kMax];
	struct timespec t0, t1;
	const uint32_t tsz = tuple_fmt == XDPGPU_TUPLE_NET ? 44 :
			     tuple_fmt == XDPGPU_TUPLE_V4 ? 16 : 0;
	uint32_t i, per, ncpu = 0;
	cpu_set_t set;

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
		pthread_create(&th[i], NULL, leg_worker, &sl[i]);
	for (i = 0; i < threads; i++)
		pthread_join(th[i], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------ */
/* calibration: the survey probe's work (parse, IPv4 header
 * checksum, UDP checksum, jhash of 13 bytes) in this leg's arithmetic, to
 * set beside ref_probe (oracle/ref_harness.c, the reference headers' own
 * routines) on the same frames.  Returns wall seconds of reps passes on one
 * thread; *acc receives a value of the results (kept live). */
static inline uint32_t jhash_13(const uint8_t *k, uint32_t iv)
{
	uint32_t a, b, c;

	a = b = c = 0xdeadbeefu + 13u + iv;
	a += ld32(k);
	b += ld32(k + 4);
	c += ld32(k + 8);
	JMIX(a, b, c);
	a += k[12];
	JFINAL(a, b, c);
	return c;
}

double cpu_leg_probe(const uint8_t *umem, uint64_t umem_size,
		     const struct xdpgpu_desc *descs, uint32_t n, uint32_t reps,
		     uint64_t *acc)
{
	struct timespec t0, t1;
	uint64_t x = 0;
	uint32_t r, i;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (r = 0; r < reps; r++) {
		for (i = 0; i < n; i++) {
			const uint64_t eff = (descs[i].addr & ((1ull << 48) - 1)) +
					     (descs[i].addr >> 48);
			const uint32_t len = descs[i].len;
			const uint8_t *p = umem + eff;
			uint32_t l3 = 14, cl;
			uint64_t s;
			uint8_t key[13];

			if (len < 42 || eff > umem_size - len)
				continue;
			if (ld16(p + 12) == 0x0081)
				l3 = 18;
			if (ld16(p + l3 - 2) != 0x0008 || p[l3] != 0x45 || p[l3 + 9] != 17)
				continue;
			{
				const uint64_t h0 = ld64(p + l3), h1 = ld64(p + l3 + 8);

				s = (h0 & 0xffffffffull) + (h0 >> 32) + (h1 & 0xffffffffull) +
				    (h1 >> 32) + ld32(p + l3 + 16);
			}
			x += (~fold16(s)) & 0xffff;
			cl = bswap16(ld16(p + l3 + 24));
			if (l3 + 20 + cl > len)
				continue;
			s = (uint64_t)ld32(p + l3 + 12) + ld32(p + l3 + 16) + ((17u + cl) << 8) +
			    sum_bytes(p + l3 + 20, cl & ~1u);
			if (cl & 1)
				s += p[l3 + 20 + cl - 1];
			x += (~fold16(s)) & 0xffff;
			memcpy(key, p + l3 + 12, 8);
			memcpy(key + 8, p + l3 + 20, 4);
			key[12] = 17;
			x += jhash_13(key, 0);
		}
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	*acc = x;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
