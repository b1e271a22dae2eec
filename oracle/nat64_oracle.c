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
#include <stdlib.h>
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
/* ------------------------------------------------------------------ */
/* Dynamic state (nat64_kern.c:543-622): v6_state_map, v4_reversemap and
 * reclaimed_addrs as plain arrays, searched linearly (test sizes).  The
 * reference walks v6_state_map in its kernel hash order when it reclaims;
 * this restatement (and the build) walk insertion order. */
struct ent6 {
	uint8_t v6[16];
	uint32_t v4, static_conf, alive;
	uint64_t last_seen;
};
struct ent4 {
	uint32_t v4, alive;
	uint8_t v6[16];
};
struct oracle_nat64_state {
	uint64_t timeout_ns, next_addr;
	uint32_t v4_prefix, v4_mask, cap;
	uint32_t n6, n4, max6, max4, count;   /* count: live v6 entries */
	struct ent6 *e6;
	struct ent4 *e4;
	uint32_t *queue, qhead, qlen;          /* ring of cap entries */
};

static struct ent6 *st_find6(struct oracle_nat64_state *st, const uint8_t *v6)
{
	for (uint32_t i = 0; i < st->n6; i++)
		if (st->e6[i].alive && !memcmp(st->e6[i].v6, v6, 16))
			return &st->e6[i];
	return NULL;
}

static struct ent4 *st_find4(struct oracle_nat64_state *st, uint32_t v4)
{
	for (uint32_t i = 0; i < st->n4; i++)
		if (st->e4[i].alive && st->e4[i].v4 == v4)
			return &st->e4[i];
	return NULL;
}

static int st_grow(void **p, uint32_t *max, uint32_t need, size_t sz)
{
	if (need <= *max)
		return 0;
	uint32_t m = *max ? *max : 64;
	while (m < need)
		m *= 2;
	void *q = realloc(*p, (size_t)m * sz);
	if (!q)
		return -1;
	*p = q;
	*max = m;
	return 0;
}

/* a map update: an existing key keeps its place and takes the value */
static struct ent6 *st_put6(struct oracle_nat64_state *st, const uint8_t *v6, uint32_t v4,
			    uint32_t stat, uint64_t ls)
{
	struct ent6 *e = st_find6(st, v6);
	if (!e) {
		if (st_grow((void **)&st->e6, &st->max6, st->n6 + 1, sizeof(*e)))
			return NULL;
		e = &st->e6[st->n6++];
		memcpy(e->v6, v6, 16);
		e->alive = 1;
		st->count++;
	}
	e->v4 = v4;
	e->static_conf = stat;
	e->last_seen = ls;
	return e;
}

static void st_put4(struct oracle_nat64_state *st, uint32_t v4, const uint8_t *v6)
{
	struct ent4 *e = st_find4(st, v4);
	if (!e) {
		if (st_grow((void **)&st->e4, &st->max4, st->n4 + 1, sizeof(*e)))
			return;
		e = &st->e4[st->n4++];
		e->v4 = v4;
		e->alive = 1;
	}
	memcpy(e->v6, v6, 16);
}

static void st_del6(struct oracle_nat64_state *st, struct ent6 *e)
{
	e->alive = 0;
	st->count--;
}

/* bpf_map_push_elem / pop_elem on the BPF_MAP_TYPE_QUEUE of num_addr */
static void st_push(struct oracle_nat64_state *st, uint32_t v4)
{
	if (st->qlen < st->cap)
		st->queue[(st->qhead + st->qlen++) % st->cap] = v4;
}

static int st_pop(struct oracle_nat64_state *st, uint32_t *v4)
{
	if (!st->qlen)
		return -1;
	*v4 = st->queue[st->qhead];
	st->qhead = (st->qhead + 1) % st->cap;
	st->qlen--;
	return 0;
}

/* reclaim_v4_addr + check_item (nat64_kern.c:543-574) */
static uint32_t st_reclaim(struct oracle_nat64_state *st, uint64_t now)
{
	const uint64_t timeout = now - st->timeout_ns;
	uint32_t v4;

	if (st_pop(st, &v4) == 0)
		return v4;
	for (uint32_t i = 0; i < st->n6; i++) {
		struct ent6 *e = &st->e6[i];
		if (e->alive && e->last_seen < timeout && !e->static_conf) {
			const uint32_t a = e->v4;
			struct ent4 *r = st_find4(st, a);
			st_del6(st, e);
			if (r)
				r->alive = 0;
			st_push(st, a);
			break;          /* one address at a time */
		}
	}
	return st_pop(st, &v4) ? 0 : v4;
}

/* alloc_new_state (nat64_kern.c:576-622), one thread: the CAS loop's first
 * round decides */
static struct ent6 *st_alloc(struct oracle_nat64_state *st, const uint8_t *v6, uint64_t now)
{
	const uint32_t max_v4 = (st->v4_prefix | ~st->v4_mask) - 1;
	const uint32_t next_v4 = st->v4_prefix + (uint32_t)st->next_addr;
	uint32_t src_v4;

	if (next_v4 >= max_v4) {
		src_v4 = st_reclaim(st, now);
	} else {
		st->next_addr++;
		src_v4 = next_v4;
	}
	if (!src_v4)
		return NULL;
	if (st->count >= st->cap) {          /* v6_state_map full: -E2BIG */
		st_push(st, src_v4);
		return NULL;
	}
	struct ent6 *e = st_put6(st, v6, src_v4, 0, now);
	if (!e)
		return NULL;
	if (st_find4(st, src_v4)) {          /* v4_reversemap NOEXIST fails */
		st_del6(st, e);
		st_push(st, src_v4);
		return NULL;
	}
	st_put4(st, src_v4, v6);
	return e;
}

struct oracle_nat64_state *oracle_nat64_state_new(const struct xdpgpu_nat64_cfg *cfg,
						  const struct xdpgpu_nat64_map *map,
						  uint32_t nmap, uint64_t timeout_ns,
						  uint64_t next_addr)
{
	struct oracle_nat64_state *st = calloc(1, sizeof(*st));
	if (!st)
		return NULL;
	st->timeout_ns = timeout_ns;
	st->next_addr = next_addr;
	st->v4_prefix = cfg->v4_prefix;
	st->v4_mask = cfg->v4_mask;
	/* num_addr (nat64.c:396) */
	st->cap = (cfg->v4_prefix | ~cfg->v4_mask) - cfg->v4_prefix - 2;
	st->queue = calloc(st->cap ? st->cap : 1, sizeof(uint32_t));
	for (uint32_t i = 0; i < nmap; i++) {
		st_put6(st, map[i].v6, map[i].v4, 1, 0);
		st_put4(st, map[i].v4, map[i].v6);
	}
	return st;
}

void oracle_nat64_state_free(struct oracle_nat64_state *st)
{
	if (!st)
		return;
	free(st->e6);
	free(st->e4);
	free(st->queue);
	free(st);
}

int oracle_nat64_state_read(const struct oracle_nat64_state *st,
			    struct xdpgpu_nat64_entry *out, uint32_t max, uint32_t *n,
			    uint64_t *next_addr, uint32_t *queue, uint32_t qmax, uint32_t *nq)
{
	uint32_t k = 0;
	for (uint32_t i = 0; i < st->n6; i++) {
		const struct ent6 *e = &st->e6[i];
		if (!e->alive)
			continue;
		if (k < max) {
			memset(&out[k], 0, sizeof(out[k]));
			memcpy(out[k].v6, e->v6, 16);
			out[k].v4 = e->v4;
			out[k].static_conf = e->static_conf;
			out[k].last_seen = e->last_seen;
		}
		k++;
	}
	*n = k;
	*next_addr = st->next_addr;
	for (uint32_t i = 0; i < st->qlen && i < qmax; i++)
		queue[i] = st->queue[(st->qhead + i) % st->cap];
	*nq = st->qlen;
	return 0;
}

/* the tables one call sees: the static map, or the dynamic state; for a
 * static map, open-addressed indices by v6 and by v4 (entry + 1, 0 empty)
 * built per call, each holding a key's first entry as find_v6 / find_v4
 * return it (a lookup tool of the test infrastructure: the map's semantics
 * are the linear search's) */
struct tabs {
	const struct xdpgpu_nat64_map *map;
	uint32_t nmap;
	struct oracle_nat64_state *st;
	uint64_t now;
	uint32_t *ix6, *ix4, mask;
};

static uint32_t hash_bytes(const uint8_t *p, uint32_t n)
{
	uint32_t h = 2166136261u;                 /* FNV-1a */
	for (uint32_t i = 0; i < n; i++)
		h = (h ^ p[i]) * 16777619u;
	return h;
}

static void tabs_index(struct tabs *T)
{
	uint32_t cap = 64;
	while (cap < 2 * T->nmap)
		cap <<= 1;
	T->ix6 = calloc(cap, sizeof(uint32_t));
	T->ix4 = calloc(cap, sizeof(uint32_t));
	if (!T->ix6 || !T->ix4) {
		free(T->ix6);
		free(T->ix4);
		T->ix6 = T->ix4 = NULL;
		return;
	}
	T->mask = cap - 1;
	for (uint32_t k = 0; k < T->nmap; k++) {
		const struct xdpgpu_nat64_map *m = &T->map[k];
		uint32_t h = hash_bytes(m->v6, 16) & T->mask;
		while (T->ix6[h] && memcmp(T->map[T->ix6[h] - 1].v6, m->v6, 16))
			h = (h + 1) & T->mask;
		if (!T->ix6[h])
			T->ix6[h] = k + 1;
		h = hash_bytes((const uint8_t *)&m->v4, 4) & T->mask;
		while (T->ix4[h] && T->map[T->ix4[h] - 1].v4 != m->v4)
			h = (h + 1) & T->mask;
		if (!T->ix4[h])
			T->ix4[h] = k + 1;
	}
}

static const struct xdpgpu_nat64_map *tabs_find_v6(const struct tabs *T, const uint8_t *v6)
{
	if (!T->ix6)
		return find_v6(T->map, T->nmap, v6);
	for (uint32_t h = hash_bytes(v6, 16) & T->mask; T->ix6[h]; h = (h + 1) & T->mask)
		if (!memcmp(T->map[T->ix6[h] - 1].v6, v6, 16))
			return &T->map[T->ix6[h] - 1];
	return NULL;
}

static const struct xdpgpu_nat64_map *tabs_find_v4(const struct tabs *T, uint32_t v4)
{
	if (!T->ix4)
		return find_v4(T->map, T->nmap, v4);
	for (uint32_t h = hash_bytes((const uint8_t *)&v4, 4) & T->mask; T->ix4[h];
	     h = (h + 1) & T->mask)
		if (T->map[T->ix4[h] - 1].v4 == v4)
			return &T->map[T->ix4[h] - 1];
	return NULL;
}

/* v6_state_map for nat64_handle_v6 (:809-828): 1 and the address, 0 no
 * entry (static tables: NO_STATE), -1 allocation failed */
static int tab_v6(const struct tabs *T, const uint8_t *v6, uint32_t *v4)
{
	if (!T->st) {
		const struct xdpgpu_nat64_map *m = tabs_find_v6(T, v6);
		if (!m)
			return 0;
		*v4 = m->v4;
		return 1;
	}
	struct ent6 *e = st_find6(T->st, v6);
	if (e) {
		e->last_seen = T->now;
	} else {
		e = st_alloc(T->st, v6, T->now);
		if (!e)
			return -1;
	}
	*v4 = e->v4;
	return 1;
}

/* v4_reversemap for nat64_handle_v4 (:491) */
static int tab_v4(const struct tabs *T, uint32_t v4, uint8_t v6[16])
{
	if (!T->st) {
		const struct xdpgpu_nat64_map *m = tabs_find_v4(T, v4);
		if (!m)
			return 0;
		memcpy(v6, m->v6, 16);
		return 1;
	}
	const struct ent4 *r = st_find4(T->st, v4);
	if (!r)
		return 0;
	memcpy(v6, r->v6, 16);
	return 1;
}

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

/* Opt-in (XDPGPU_NAT64_F_ICMP_INNER, include/xdpgpu.h): the header
 * embedded in an ICMPv6 error at p + ii, as a new IPv4 header h4i (the
 * outer construction of nat64_handle_v6, nat64_kern.c:830-850).  outer_src
 * is the error's own IPv6 source, src4 its IPv4 address.  0 ok, -1 not
 * translatable.  Not in the reference (FIXME at nat64_kern.c:736). */
static int inner_v6_to_v4(const uint8_t *p, uint32_t len, uint32_t ii, uint32_t outer_plen,
			  const uint8_t *outer_src, uint32_t src4,
			  const struct xdpgpu_nat64_cfg *cfg, const struct tabs *T,
			  uint8_t h4i[20])
{
	if (ii + 40 > len || outer_plen < 48 || (p[ii] >> 4) != 6)
		return -1;
	const uint8_t nh = p[ii + 6];
	if (nh == 0 || nh == 43 || nh == 44 || nh == 51 || nh == 60 || nh == 135)
		return -1;                 /* an extension header: not handled */
	uint8_t a4[4], pref[16];
	if (!oracle_v6addr_to_v4(p + ii + 8, (int)cfg->v6_plen, a4, pref) ||
	    memcmp(pref, cfg->v6_prefix, 16))
		return -1;
	uint32_t d4;
	if (!memcmp(p + ii + 24, outer_src, 16)) {
		d4 = src4;
	} else {
		/* static state only: a dynamic entry is the error's own source */
		const struct xdpgpu_nat64_map *m = T->st ? NULL :
			find_v6(T->map, T->nmap, p + ii + 24);
		if (!m)
			return -1;
		d4 = m->v4;
	}
	memset(h4i, 0, 20);
	h4i[0] = 0x45;
	h4i[1] = (uint8_t)(((p[ii] & 0x0f) << 4) | (p[ii + 1] >> 4));
	put_be16(h4i + 2, (uint16_t)(be16(p + ii + 4) + 20));
	put_be16(h4i + 6, 0x4000);
	h4i[8] = p[ii + 7];
	h4i[9] = nh == 58 ? 1 : nh;
	memcpy(h4i + 12, a4, 4);
	put_be32(h4i + 16, d4);
	uint64_t s = 0;
	for (int i = 0; i < 20; i += 2)
		s += le16(h4i + i);
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	put_le16(h4i + 10, (uint16_t)~s);
	return 0;
}

/* The same for an ICMPv4 error (FIXME at nat64_kern.c:438): the embedded
 * IPv4 header at p + ii (IHL *ihl) as a new IPv6 header h6i (the outer
 * construction of nat64_handle_v4, :497-519). */
static int inner_v4_to_v6(const uint8_t *p, uint32_t len, uint32_t ii, uint32_t outer_tot,
			  const struct xdpgpu_nat64_cfg *cfg, const struct tabs *T,
			  uint8_t h6i[40], uint32_t *ihl)
{
	if (ii + 20 > len || (p[ii] >> 4) != 4)
		return -1;
	*ihl = (p[ii] & 0xf) * 4;
	if (*ihl < 20 || ii + *ihl > len || outer_tot < 28 + *ihl)
		return -1;
	if (be16(p + ii + 6) & ~0x4000u)
		return -1;                 /* a fragment: not handled */
	memset(h6i, 0, 40);
	if (!tab_v4(T, be32(p + ii + 12), h6i + 8))
		return -1;
	if (!oracle_v4addr_to_v6(p + ii + 16, h6i + 24, cfg->v6_prefix, (int)cfg->v6_plen))
		return -1;
	const uint8_t tos = p[ii + 1], proto = p[ii + 9];
	h6i[0] = (uint8_t)(6 << 4 | ((tos & 0x70) >> 4));
	h6i[1] = (uint8_t)(tos << 4);
	put_be16(h6i + 4, (uint16_t)(be16(p + ii + 2) - *ihl));
	h6i[6] = proto == 1 ? 58 : proto;
	h6i[7] = p[ii + 8];
	return 0;
}

/* nat64_handle_v6 (nat64_kern.c:741-873) on one frame */
static int handle_v6(uint8_t *umem, uint64_t eff, uint32_t len, uint32_t l3,
		     const struct xdpgpu_nat64_cfg *cfg, const struct tabs *T,
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
	uint32_t src4 = 0;
	const int got = tab_v6(T, p + l3 + 8, &src4);
	if (got == 0)
		return XDPGPU_NAT64_NO_STATE;
	if (got < 0)
		return XDPGPU_TC_ACT_SHOT;     /* alloc_new_state failed */

	/* the new IPv4 header */
	uint8_t h4[20];
	memset(h4, 0, 20);
	h4[0] = 0x45;
	h4[1] = (uint8_t)(((p[l3] & 0x0f) << 4) | (p[l3 + 1] >> 4));
	put_be16(h4 + 2, (uint16_t)(be16(p + l3 + 4) + 20));
	put_be16(h4 + 6, 0x4000);
	h4[8] = p[l3 + 7];
	h4[9] = (uint8_t)nexthdr;
	put_be32(h4 + 12, src4);
	memcpy(h4 + 16, a4, 4);

	const uint32_t l4 = l3 + 40;
	int inner = 0;
	uint8_t h4i[20];
	switch (nexthdr) {
	case 58:
		if (l4 + 8 > len)
			return XDPGPU_TC_ACT_SHOT;
		inner = (cfg->flags & XDPGPU_NAT64_F_ICMP_INNER) && p[l4] >= 1 && p[l4] <= 4;
		if (inner && inner_v6_to_v4(p, len, l4 + 8, be16(p + l3 + 4), p + l3 + 8, src4,
					    cfg, T, h4i))
			return XDPGPU_TC_ACT_SHOT;
		{
			uint8_t h6[40];
			memcpy(h6, p + l3, 40);
			if (rewrite_icmpv6(p + l4, h6))
				return XDPGPU_TC_ACT_SHOT;
		}
		h4[9] = 1;
		if (inner) {
			/* 40 header bytes out, 20 in; the ICMPv4 message
			 * is the IPv6 payload less 20 bytes */
			l4_csum_replace(p + l4 + 2, csum_diff_mod(p + l4 + 8, 40, h4i, 20), 0);
			put_be16(h4 + 2, be16(p + l3 + 4));
		}
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
	if (inner) {
		/* [L2][IPv4][ICMP][inner IPv4] end where the inner IPv6
		 * header did: the frame starts 40 bytes later */
		uint8_t l2[22], icmp[8];
		memcpy(l2, p, l3);
		memcpy(icmp, p + l4, 8);
		uint8_t *q = p + 40;
		memcpy(q + l3 + 28, h4i, 20);
		memcpy(q + l3 + 20, icmp, 8);
		memcpy(q + l3, h4, 20);
		memcpy(q, l2, l3);
		q[12] = 0x08; q[13] = 0x00;
		out->addr = eff + 40;
		out->len = len - 40;
		return XDPGPU_TC_ACT_REDIRECT;
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
		     const struct xdpgpu_nat64_cfg *cfg, const struct tabs *T,
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
	uint8_t dst6[16];
	if (!tab_v4(T, d4, dst6))
		return XDPGPU_TC_ACT_SHOT;
	uint8_t h6[40];
	memset(h6, 0, 40);
	if (!oracle_v4addr_to_v6(p + l3 + 12, h6 + 8, cfg->v6_prefix, (int)cfg->v6_plen))
		return XDPGPU_TC_ACT_SHOT;
	memcpy(h6 + 24, dst6, 16);
	const uint8_t tos = p[l3 + 1], proto = p[l3 + 9];
	/* struct ipv6hdr on little-endian: priority:4 is the low nibble */
	h6[0] = (uint8_t)(6 << 4 | ((tos & 0x70) >> 4));
	h6[1] = (uint8_t)(tos << 4);
	put_be16(h6 + 4, (uint16_t)(be16(p + l3 + 2) - 20));
	h6[6] = proto;
	h6[7] = p[l3 + 8];
	/* the bytes in front the frame may grow into (cfg->headroom) */
	const uint64_t room = cfg->headroom && cfg->headroom < eff ? cfg->headroom : eff;
	if (room < 20)
		return XDPGPU_TC_ACT_SHOT;             /* no headroom to grow */
	const uint32_t l4 = l3 + 20;
	int inner = 0;
	uint8_t h6i[40];
	uint32_t ihl_i = 0, grow = 0;
	switch (proto) {
	case 1:
		if (l4 + 8 > len)
			return XDPGPU_TC_ACT_SHOT;
		inner = (cfg->flags & XDPGPU_NAT64_F_ICMP_INNER) &&
			(p[l4] == 3 || p[l4] == 11 || p[l4] == 12);
		if (inner) {
			if (inner_v4_to_v6(p, len, l4 + 8, be16(p + l3 + 2), cfg, T, h6i, &ihl_i))
				return XDPGPU_TC_ACT_SHOT;
			grow = 40 - ihl_i;
			if (room < 20 + grow)
				return XDPGPU_TC_ACT_SHOT;     /* headroom */
			/* the pseudo header's length is the new payload_len */
			put_be16(h6 + 4, (uint16_t)(be16(h6 + 4) + grow));
		}
		if (rewrite_icmp(p + l4, h6))
			return XDPGPU_TC_ACT_SHOT;
		h6[6] = 58;
		if (inner) {
			l4_csum_replace(p + l4 + 2,
					csum_diff_mod(p + l4 + 8, (int)ihl_i, h6i, 40), 0);
			/* [L2][IPv6][ICMPv6][inner IPv6] end where the inner
			 * IPv4 header did: the frame starts 20 + grow earlier */
			const uint32_t sh = 20 + grow;
			uint8_t l2[22], icmp[8];
			memcpy(l2, p, l3);
			memcpy(icmp, p + l4, 8);
			uint8_t *q = p - sh;
			memcpy(q, l2, l3);
			q[12] = 0x86; q[13] = 0xDD;
			memcpy(q + l3, h6, 40);
			memcpy(q + l3 + 40, icmp, 8);
			memcpy(q + l3 + 48, h6i, 40);
			out->addr = eff - sh;
			out->len = len + sh;
			return XDPGPU_TC_ACT_REDIRECT;
		}
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
static int run_batch(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		     uint32_t n, const struct xdpgpu_nat64_cfg *cfg, const struct tabs *T,
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
			act = handle_v4(umem, eff, len, l3, cfg, T, &out[i]);
		else if (cfg->direction == XDPGPU_NAT64_INGRESS && et == 0x86DD)
			act = handle_v6(umem, eff, len, l3, cfg, T, &out[i]);
		if (act == XDPGPU_TC_ACT_REDIRECT)
			out[i].options = descs[i].options;
		action[i] = (uint8_t)act;
	}
	return 0;
}

int oracle_nat64(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		 uint32_t n, const struct xdpgpu_nat64_cfg *cfg,
		 const struct xdpgpu_nat64_map *map, uint32_t nmap,
		 uint8_t *action, struct xdpgpu_desc *out)
{
	struct tabs T = {map, nmap, NULL, 0, NULL, NULL, 0};
	if (nmap > 64)
		tabs_index(&T);
	const int rc = run_batch(umem, umem_size, descs, n, cfg, &T, action, out);
	free(T.ix6);
	free(T.ix4);
	return rc;
}

int oracle_nat64_dyn(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		     uint32_t n, const struct xdpgpu_nat64_cfg *cfg,
		     struct oracle_nat64_state *st, uint64_t now, uint8_t *action,
		     struct xdpgpu_desc *out)
{
	const struct tabs T = {NULL, 0, st, now, NULL, NULL, 0};
	return run_batch(umem, umem_size, descs, n, cfg, &T, action, out);
}
