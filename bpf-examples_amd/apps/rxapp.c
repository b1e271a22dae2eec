// SPDX-License-Identifier: GPL-2.0
/*
 * rxapp.c - frame sources, the batched RX loop and the statistics of the
 * drop-in front-ends (rxapp.h).  Everything per frame happens on the GPU
 * behind the C ABI; this file only moves descriptors and applies verdicts,
 * as the reference's RX loops do with the per-packet results
 * (af_xdp_user.c:1079-1113, xdpsock.c:1462-1506 and 1718-1784).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <locale.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rxapp.h"
#include "xsk.h"

#include <pthread.h>
#include <unistd.h>
#include <linux/if_link.h>

static volatile sig_atomic_t rx_done;

static void on_signal(int sig)
{
	(void)sig;
	rx_done = 1;
}

static uint64_t now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static uint64_t desc_off(const struct xdpgpu_desc *d)
{
	/* XSK_UNALIGNED_BUF_OFFSET_SHIFT, headers/linux/if_xdp.h:104-106 */
	return (d->addr & ((1ull << 48) - 1)) + (d->addr >> 48);
}

bool rx_parse_mac(const char *s, uint8_t mac[6])
{
	unsigned int v[6];
	char tail;

	if (sscanf(s, "%x:%x:%x:%x:%x:%x%c", &v[0], &v[1], &v[2], &v[3], &v[4],
		   &v[5], &tail) != 6)
		return false;
	for (int i = 0; i < 6; i++) {
		if (v[i] > 0xff)
			return false;
		mac[i] = (uint8_t)v[i];
	}
	return true;
}

/* ------------------------------------------------------------------ */
/* sources                                                             */

static void *umem_alloc(uint64_t size)
{
	void *p = NULL;

	/* page aligned (posix_memalign, af_xdp_user.c:1574), +64: the GPU
	 * loads 16-byte chunks of a frame's last line */
	if (posix_memalign(&p, 4096, (size + 64 + 4095) & ~4095ull))
		return NULL;
	memset(p, 0, (size + 64 + 4095) & ~4095ull);
	return p;
}

int rx_source_pool(struct rx_source *src, const struct xdpgpu_pool_spec *spec,
		   uint32_t n)
{
	memset(src, 0, sizeof(*src));
	if (!n)
		return -EINVAL;
	uint64_t size = (xdpgpu_pool_size(spec, n) + 63) & ~63ull;

	src->umem = umem_alloc(size);
	src->descs = calloc(n, sizeof(*src->descs));
	if (!src->umem || !src->descs) {
		rx_source_free(src);
		return -ENOMEM;
	}
	src->umem_size = size;
	src->n = n;
	src->packets = n;
	src->headroom = spec->headroom;
	int rc = xdpgpu_pool_generate(spec, src->umem, size, src->descs, n, NULL);
	if (rc)
		rx_source_free(src);
	return rc;
}

static uint32_t rd32(const uint8_t *p, bool swap)
{
	uint32_t v;

	memcpy(&v, p, 4);
	return swap ? __builtin_bswap32(v) : v;
}

int rx_source_pcap(struct rx_source *src, const char *path, uint32_t chunk_size,
		   uint32_t headroom, bool unaligned, bool frags, uint32_t max_frames)
{
	memset(src, 0, sizeof(*src));
	FILE *f = fopen(path, "rb");
	if (!f)
		return -errno;
	uint8_t gh[24];
	if (fread(gh, 1, 24, f) != 24) {
		fclose(f);
		return -EPROTO;
	}
	uint32_t magic;
	memcpy(&magic, gh, 4);
	bool swap;
	if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du)
		swap = false;
	else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u)
		swap = true;
	else {
		fclose(f);
		return -EPROTO;
	}
	if ((rd32(gh + 20, swap) & 0x0fffffff) != 1) { /* LINKTYPE_ETHERNET */
		fclose(f);
		return -EPROTO;
	}
	if (!unaligned && (chunk_size < 128 || (chunk_size & (chunk_size - 1)) ||
			   headroom >= chunk_size)) {
		fclose(f);
		return -EINVAL;
	}

	/* pass 1: sizes (a record split over nch chunks with frags) */
	const uint32_t room = unaligned ? 0 : chunk_size - headroom;
	uint64_t n = 0, size = 0, packets = 0;
	long body = ftell(f);
	uint8_t rh[16];
	while (fread(rh, 1, 16, f) == 16) {
		uint32_t incl = rd32(rh + 8, swap);
		if (incl > 262144 || fseek(f, incl, SEEK_CUR)) {
			fclose(f);
			return -EPROTO;
		}
		if (max_frames && n >= max_frames)
			break;
		if ((!unaligned && incl > room && !frags) || incl > 65535) {
			src->skipped++;
			continue;
		}
		const uint64_t nch = unaligned ? 1 : incl > room ? (incl + room - 1) / room : 1;
		size += unaligned ? ((headroom + incl + 63) & ~63ull) : nch * chunk_size;
		n += nch;
		packets++;
	}
	if (!n || n > 0xffffffffull) {
		fclose(f);
		return n ? -E2BIG : -ENODATA;
	}
	uint64_t skipped = src->skipped;
	src->umem = umem_alloc(size);
	src->descs = calloc(n, sizeof(*src->descs));
	if (!src->umem || !src->descs) {
		fclose(f);
		rx_source_free(src);
		return -ENOMEM;
	}
	src->umem_size = size;
	src->n = (uint32_t)n;
	src->packets = (uint32_t)packets;
	src->skipped = skipped;
	src->chunk_size = unaligned ? 0 : chunk_size;
	src->headroom = headroom;
	src->umem_flags = unaligned ? XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG : 0;

	/* pass 2: frames */
	fseek(f, body, SEEK_SET);
	uint64_t off = 0;
	uint32_t k = 0;
	while (k < n && fread(rh, 1, 16, f) == 16) {
		uint32_t incl = rd32(rh + 8, swap);
		if ((!unaligned && incl > room && !frags) || incl > 65535) {
			fseek(f, incl, SEEK_CUR);
			continue;
		}
		/* the record's bytes over one chunk, or several (fragments) */
		uint32_t left = incl;
		do {
			const uint32_t piece = unaligned || left <= room ? left : room;
			if (k >= n || fread(src->umem + off + headroom, 1, piece, f) != piece) {
				fclose(f);
				rx_source_free(src);
				return -EPROTO;
			}
			left -= piece;
			src->descs[k].addr = off + headroom;
			src->descs[k].len = piece;
			src->descs[k].options = left ? XDPGPU_PKT_CONTD : 0;
			off += unaligned ? ((headroom + piece + 63) & ~63ull) : chunk_size;
			k++;
		} while (left);
	}
	fclose(f);
	return 0;
}

int rx_source_write_pcap(const struct rx_source *src, const uint8_t *select,
			 uint8_t want, const char *path)
{
	FILE *f = fopen(path, "wb");
	if (!f)
		return -errno;
	const uint32_t gh[6] = { 0xa1b2c3d4u, 0x00040002u, 0, 0, 65535, 1 };
	int rc = fwrite(gh, 4, 6, f) == 6 ? 0 : -EIO;
	for (uint32_t i = 0; i < src->n && !rc; i++) {
		if (select && select[i] != want)
			continue;
		const uint32_t rh[4] = { i, 0, src->descs[i].len, src->descs[i].len };
		if (fwrite(rh, 4, 4, f) != 4 ||
		    fwrite(src->umem + desc_off(&src->descs[i]), 1, src->descs[i].len, f) !=
			    src->descs[i].len)
			rc = -EIO;
	}
	if (fclose(f) && !rc)
		rc = -EIO;
	return rc;
}

void rx_source_free(struct rx_source *src)
{
	free(src->umem);
	free(src->descs);
	src->umem = NULL;
	src->descs = NULL;
	src->n = 0;
}

void rx_source_describe(const struct rx_source *src, const char *what)
{
	uint64_t bytes = 0;
	uint32_t lo = UINT32_MAX, hi = 0;

	for (uint32_t i = 0; i < src->n; i++) {
		uint32_t l = src->descs[i].len;
		bytes += l;
		lo = l < lo ? l : lo;
		hi = l > hi ? l : hi;
	}
	printf("%s: %u frames, %llu bytes (len %u..%u), UMEM %llu bytes, "
	       "chunk %u, headroom %u%s",
	       what, src->n, (unsigned long long)bytes, src->n ? lo : 0, hi,
	       (unsigned long long)src->umem_size, src->chunk_size, src->headroom,
	       src->umem_flags & XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG ? ", unaligned" : "");
	if (src->packets != src->n)
		printf(", %u packets", src->packets);
	if (src->skipped)
		printf(", %llu records skipped (larger than a chunk)",
		       (unsigned long long)src->skipped);
	printf("\n");
}

/* ------------------------------------------------------------------ */
/* statistics                                                          */

struct rx_stats_state {
	uint64_t t_prev;
	uint64_t rx_prev, tx_prev, rxb_prev, txb_prev, rxf_prev, txf_prev;
};

static void print_stats(const struct rx_opts *o, const struct rx_totals *t,
			struct rx_stats_state *st, const char *label, uint64_t now)
{
	const double dt = (double)(now - st->t_prev) / 1e9;
	const double period = dt > 0 ? dt : 1;

	if (o->stats_fmt == RX_STATS_XDPSOCK) {
		/* dump_stats, xdpsock.c:478-582 */
		const char *fmt = "%-18s %'-14.0f %'-14lu\n";
		printf("\n sock0@%s\n", label);
		if (o->frags) {
			/* the --frags table, xdpsock.c:500-514 */
			const char *ffmt = "%-18s %'-14.0f %'-14lu %'-14.0f %'-14lu\n";
			printf("%-18s %-14s %-14s %-14s %-14s %-14.2f\n", "", "pps", "pkts",
			       "fps", "frags", dt);
			printf(ffmt, "rx", (double)(t->rx_pkts - st->rx_prev) / period,
			       (unsigned long)t->rx_pkts,
			       (double)(t->rx_frags - st->rxf_prev) / period,
			       (unsigned long)t->rx_frags);
			printf(ffmt, "tx", (double)(t->tx_pkts - st->tx_prev) / period,
			       (unsigned long)t->tx_pkts,
			       (double)(t->tx_frags - st->txf_prev) / period,
			       (unsigned long)t->tx_frags);
		} else {
			printf("%-18s %-14s %-14s %-14.2f\n", "", "pps", "pkts", dt);
			printf(fmt, "rx", (double)(t->rx_pkts - st->rx_prev) / period,
			       (unsigned long)t->rx_pkts);
			printf(fmt, "tx", (double)(t->tx_pkts - st->tx_prev) / period,
			       (unsigned long)t->tx_pkts);
		}
		if (o->cfg_flags & XDPGPU_CFG_STATS) {
			/* extra: the GPU verdict histogram (enum xdp_action) */
			printf(fmt, "gpu aborted", 0.0, (unsigned long)t->verdict[XDPGPU_ABORTED]);
			printf(fmt, "gpu drop", 0.0, (unsigned long)t->verdict[XDPGPU_DROP]);
			printf(fmt, "gpu pass", 0.0, (unsigned long)t->verdict[XDPGPU_PASS]);
			printf(fmt, "gpu tx", 0.0, (unsigned long)t->verdict[XDPGPU_TX]);
			printf(fmt, "gpu redirect", 0.0,
			       (unsigned long)t->verdict[XDPGPU_REDIRECT]);
		}
	} else {
		/* stats_print, af_xdp_user.c:1360-1397 */
		const char *fmt = "%-12s %'11lld pkts (%'10.0f pps) %'11lld Kbytes "
				  "(%'6.0f Mbits/s) period:%f\n";
		printf(fmt, "AF_XDP RX:", (long long)t->rx_pkts,
		       (double)(t->rx_pkts - st->rx_prev) / period,
		       (long long)(t->rx_bytes / 1000),
		       (double)(t->rx_bytes - st->rxb_prev) * 8 / period / 1e6, period);
		printf(fmt, "       TX:", (long long)t->tx_pkts,
		       (double)(t->tx_pkts - st->tx_prev) / period,
		       (long long)(t->tx_bytes / 1000),
		       (double)(t->tx_bytes - st->txb_prev) * 8 / period / 1e6, period);
		printf("\n");
	}
	fflush(stdout);
	st->t_prev = now;
	st->rx_prev = t->rx_pkts;
	st->tx_prev = t->tx_pkts;
	st->rxb_prev = t->rx_bytes;
	st->txb_prev = t->tx_bytes;
	st->rxf_prev = t->rx_frags;
	st->txf_prev = t->tx_frags;
}

/* ------------------------------------------------------------------ */
/* the RX loop                                                          */

struct rx_slot {
	struct xdpgpu_desc *d;
	uint8_t *v;
	uint32_t n;
	uint64_t first;     /* ring position of d[0] */
	bool busy;
};

/* swap_mac_addresses, xdpsock.c:1700-1716 */
static void swap_macs(uint8_t *p)
{
	uint8_t t[6];

	memcpy(t, p, 6);
	memcpy(p, p + 6, 6);
	memcpy(p + 6, t, 6);
}

/* Apply a batch's verdicts as the reference bodies do (rx_drop, l2fwd:
 * xdpsock.c:1462-1506, 1718-1784; process_packet's TX, af_xdp_user.c:
 * 1023-1036).  With fragments (IS_EOP_DESC, xdpsock.c:67) packets count on
 * their last descriptor and the MAC swap touches a packet's first. */
static void apply(const struct rx_source *src, const struct rx_opts *o,
		  const struct rx_slot *s, struct rx_totals *t, uint8_t *first_pass)
{
	for (uint32_t i = 0; i < s->n; i++) {
		const uint8_t v = s->v[i];
		const uint32_t len = s->d[i].len;
		const bool eop = !o->frags || !(s->d[i].options & XDPGPU_PKT_CONTD);
		const bool first = t->open_frags++ == 0;
		t->rx_frags++;
		t->rx_bytes += len;
		if (first_pass && s->first + i < src->n)
			first_pass[s->first + i] = v;
		bool tx = false;
		if (o->mode == RX_MODE_L2FWD && v == XDPGPU_REDIRECT) {
			if (first)
				swap_macs(src->umem + desc_off(&s->d[i]));
			tx = true;
		} else if (v == XDPGPU_TX) {
			/* process_packet returned true: the reply goes out
			 * (af_xdp_user.c:1023-1036) */
			tx = o->mode != RX_MODE_DROP;
		}
		if (tx) {
			t->tx_frags++;
			t->tx_bytes += len;
		}
		if (eop) {
			t->rx_pkts++;
			if (v < XDPGPU_NUM_VERDICTS)
				t->verdict[v]++;
			if (tx)
				t->tx_pkts++;
			t->open_frags = 0;
		}
	}
}

int rx_run(const struct rx_source *src, const struct rx_opts *o,
	   struct rx_totals *out)
{
	struct xdpgpu_cfg cfg = {
		.device = o->device,
		.flags = o->cfg_flags,
		.max_batch = o->batch,
		.jhash_initval = o->initval,
		.tuple_fmt = o->tuple_fmt,
		.window = 64,
	};
	struct xdpgpu_ctx *ctx = NULL;
	struct rx_slot slot[2];
	uint8_t *first_pass = NULL;
	int rc;

	memset(out, 0, sizeof(*out));
	memset(slot, 0, sizeof(slot));
	if (!o->batch || !src->n)
		return -EINVAL;
	if (o->frags) {
		/* a batch ends on a packet's last fragment: every packet must
		 * fit one batch */
		uint32_t run = 0, most = 0;
		for (uint32_t i = 0; i < src->n; i++) {
			run++;
			if (!(src->descs[i].options & XDPGPU_PKT_CONTD)) {
				most = run > most ? run : most;
				run = 0;
			}
		}
		most = run > most ? run : most;
		if (most > o->batch) {
			fprintf(stderr, "%s: a packet of %u fragments does not fit a batch of %u "
				"(-b)\n", o->prog, most, o->batch);
			return -EINVAL;
		}
	}
	rc = xdpgpu_init(&cfg, &ctx);
	if (rc) {
		fprintf(stderr, "%s: xdpgpu_init: %s%s\n", o->prog, strerror(-rc),
			rc == -ENODEV ? " (no GPU: this build has no CPU fallback)" : "");
		return rc;
	}
	rc = xdpgpu_register_umem(ctx, src->umem, src->umem_size, src->chunk_size,
				  src->headroom, src->umem_flags);
	if (rc) {
		fprintf(stderr, "%s: xdpgpu_register_umem: %s %s\n", o->prog,
			strerror(-rc), xdpgpu_last_error(ctx));
		xdpgpu_fini(ctx);
		return rc;
	}
	/* page-locked batch arrays: xdpgpu_submit copies them unstaged */
	for (int k = 0; k < 2; k++) {
		slot[k].d = xdpgpu_host_alloc((uint64_t)o->batch * sizeof(*slot[k].d));
		slot[k].v = xdpgpu_host_alloc(o->batch);
		if (!slot[k].d || !slot[k].v)
			rc = -ENOMEM;
	}
	if (!rc && (o->verdict_out || o->tx_pcap)) {
		first_pass = malloc(src->n);
		if (!first_pass)
			rc = -ENOMEM;
		else
			memset(first_pass, 0xff, src->n);
	}

	rx_done = 0;
	signal(SIGINT, on_signal);
	signal(SIGTERM, on_signal);
	setlocale(LC_NUMERIC, "en_US");

	const uint64_t limit = o->count ? o->count :
			       o->duration_ns ? UINT64_MAX : (uint64_t)src->n;
	const uint64_t t0 = now_ns();
	struct rx_stats_state st = { .t_prev = t0 };
	uint64_t pos = 0;           /* frames peeked from the ring */
	uint32_t k = 0;
	const char *label = o->label ? o->label : o->prog;

	while (!rc) {
		struct rx_slot *s = &slot[k & 1];
		/* peek the next batch (xsk_ring_cons__peek) */
		uint64_t want = limit - pos;
		const bool stop = rx_done || !want ||
				  (o->duration_ns && now_ns() - t0 >= o->duration_ns);
		if (!stop) {
			s->n = (uint32_t)(want < o->batch ? want : o->batch);
			s->first = pos;
			for (uint32_t i = 0; i < s->n; i++)
				s->d[i] = src->descs[(pos + i) % src->n];
			/* fragments: release whole packets only (l2fwd's
			 * frags_done, xdpsock.c:1764-1775); the rest is peeked
			 * again with the next batch */
			if (o->frags && (s->d[s->n - 1].options & XDPGPU_PKT_CONTD)) {
				uint32_t e = s->n - 1;
				while (e && (s->d[e - 1].options & XDPGPU_PKT_CONTD))
					e--;
				if (e) {
					s->n = e;
				} else if (s->n == o->batch) {
					/* one packet fills the whole batch and goes on:
					 * it cannot be cut (its verdict needs all of it) */
					fprintf(stderr, "%s: a packet has more than -b %u fragments\n",
						o->prog, o->batch);
					rc = -E2BIG;
					break;
				}
				/* else the count (-C) ends inside the packet: its
				 * fragments go as they are (ABORTED, frags.hip) */
			}
			rc = xdpgpu_submit(ctx, k & 1, s->d, s->n, s->v, NULL, NULL);
			if (rc)
				break;
			s->busy = true;
			pos += s->n;
		}
		/* the previous batch: wait, apply its verdicts, release */
		struct rx_slot *p = &slot[(k + 1) & 1];
		if (p->busy) {
			rc = xdpgpu_wait(ctx, (k + 1) & 1);
			if (rc)
				break;
			p->busy = false;
			apply(src, o, p, out, first_pass);
			out->batches++;
		}
		if (stop)
			break;
		k++;
		if (o->interval_s && !o->quiet) {
			const uint64_t t = now_ns();
			if (t - st.t_prev >= (uint64_t)o->interval_s * 1000000000ull)
				print_stats(o, out, &st, label, t);
		}
	}
	for (int j = 0; j < 2 && rc; j++)
		if (slot[j].busy)
			(void)xdpgpu_wait(ctx, j);
	const uint64_t t1 = now_ns();
	out->seconds = (double)(t1 - t0) / 1e9;
	if (rc)
		fprintf(stderr, "%s: GPU batch failed: %s %s\n", o->prog, strerror(-rc),
			xdpgpu_last_error(ctx));
	else if (!o->quiet)
		print_stats(o, out, &st, label, t1);   /* xdpsock_cleanup */

	if (!rc && o->verdict_out) {
		FILE *f = fopen(o->verdict_out, "wb");
		if (!f || fwrite(first_pass, 1, src->n, f) != src->n)
			rc = -EIO;
		if (f && fclose(f))
			rc = -EIO;
	}
	if (!rc && o->tx_pcap)
		rc = rx_source_write_pcap(src, first_pass,
					  o->mode == RX_MODE_L2FWD ? XDPGPU_REDIRECT : XDPGPU_TX,
					  o->tx_pcap);
	if (!rc && o->json) {
		const double mpps = out->seconds > 0 ? out->rx_pkts / out->seconds / 1e6 : 0;
		printf("{\"prog\": \"%s\", \"frames\": %llu, \"seconds\": %.6f, \"mpps\": %.3f, "
		       "\"rx_pkts\": %llu, \"rx_frags\": %llu, \"rx_bytes\": %llu, "
		       "\"tx_pkts\": %llu, "
		       "\"tx_bytes\": %llu, \"batch\": %u, \"batches\": %llu, "
		       "\"verdict\": {\"ABORTED\": %llu, \"DROP\": %llu, \"PASS\": %llu, "
		       "\"TX\": %llu, \"REDIRECT\": %llu}}\n",
		       o->prog, (unsigned long long)out->rx_pkts, out->seconds, mpps,
		       (unsigned long long)out->rx_pkts, (unsigned long long)out->rx_frags,
		       (unsigned long long)out->rx_bytes,
		       (unsigned long long)out->tx_pkts, (unsigned long long)out->tx_bytes,
		       o->batch, (unsigned long long)out->batches,
		       (unsigned long long)out->verdict[0], (unsigned long long)out->verdict[1],
		       (unsigned long long)out->verdict[2], (unsigned long long)out->verdict[3],
		       (unsigned long long)out->verdict[4]);
		fflush(stdout);
	}
	for (int j = 0; j < 2; j++) {
		xdpgpu_host_free(slot[j].d);
		xdpgpu_host_free(slot[j].v);
	}
	free(first_pass);
	xdpgpu_fini(ctx);
	return rc;
}

/* ------------------------------------------------------------------ */
/* live mode                                                            */

struct injector {
	const struct rx_live *lv;
	const struct xsk_sock *x;    /* the receiving socket (its counters) */
	const char *ifname;
	volatile uint64_t received;  /* frames the RX loop has taken */
	volatile uint64_t sent;
	volatile uint64_t lost;      /* frames the kernel dropped (no fill
				      * buffer, RX ring full), or given up on */
	volatile int stop;
	volatile int done;           /* every frame sent and accounted for,
				      * or the injector failed (rc)         */
	int rc;
	int64_t drops0;              /* XDP_STATISTICS drops at the start  */
	uint64_t given_up;           /* frames of stalled windows          */
};

/* Frames lost so far: the kernel's drops since the start, or the frames
 * given up on in stalled windows, whichever is more (a window given up on
 * may be the kernel's drops, reported later: not counted twice). */
static uint64_t inject_lost(struct injector *in)
{
	const int64_t dr = xsk_rx_drops(in->x);
	const uint64_t kdrop = dr >= 0 && in->drops0 >= 0 && dr > in->drops0 ?
				       (uint64_t)(dr - in->drops0) : 0;
	const uint64_t lost = kdrop > in->given_up ? kdrop : in->given_up;
	in->lost = lost;
	return lost;
}

/* Frames given up on when the window has not moved for this long and the
 * kernel reports no drop: far longer than any batch, the first one's code
 * object load and buffer allocation included. */
#define INJECT_STALL_NS 5000000000ull
/* After the last send: how long the loss of the final window is waited
 * for (the receive loop stops 200 ms after its last frame anyway). */
#define INJECT_DRAIN_NS 1000000000ull

/* Sends the source's frames into the peer, cycling it, keeping at most
 * ring_size / 2 frames ahead of the receiver (no RX-ring overflow: every
 * frame sent is received, so verdicts line up with the source).  `received`
 * moves when the RX loop takes frames off the RX ring, before it hands them
 * to the GPU.  Frames the kernel dropped (a frame finds no fill buffer when
 * the receiver holds them all; XDP_STATISTICS) count as lost, and so do the
 * frames of a window that has not moved for INJECT_STALL_NS; any loss is
 * reported and the per-frame verdict file is then not written. */
static void *inject_main(void *arg)
{
	struct injector *in = arg;
	const struct rx_source *src = in->lv->inject;
	const uint64_t window = in->lv->ring_size / 2;
	uint64_t k = 0;
	const int fd = xsk_packet_socket(in->ifname);

	if (fd < 0) {
		in->rc = fd;
		in->done = 1;
		return NULL;
	}

	in->drops0 = xsk_rx_drops(in->x);
	in->given_up = 0;
	uint64_t last_rx = 0, t_stall = 0;
	while (!in->stop && k < in->lv->inject_count) {
		uint64_t m = in->lv->inject_count - k;
		const uint64_t lost = inject_lost(in);
		const uint64_t got = in->received + lost;
		const uint64_t ahead = k > got ? k - got : 0;
		if (ahead >= window) {
			const uint64_t t = now_ns();
			if (in->received != last_rx || !t_stall) {
				last_rx = in->received;
				t_stall = t;
			} else if (t - t_stall > INJECT_STALL_NS) {
				in->given_up += ahead;
				t_stall = 0;
			}
			usleep(20);
			continue;
		}
		t_stall = 0;
		const uint64_t room = window - ahead;
		m = m < room ? m : room;
		m = m < 256 ? m : 256;
		const uint32_t at = (uint32_t)(k % src->n);
		if (m > src->n - at)
			m = src->n - at;
		const int r = xsk_inject_fd(fd, src->umem,
					    (const struct xdp_desc *)(src->descs + at), (uint32_t)m);
		if (r < 0) {
			in->rc = r;
			break;
		}
		k += (uint64_t)r;
		in->sent = k;
	}
	close(fd);
	/* the last window (up to ring_size / 2 frames): the kernel counts its
	 * drops after the last send, so the loss is read until every frame
	 * sent is received or dropped, for at most INJECT_DRAIN_NS */
	const uint64_t t_end = now_ns();
	while (!in->stop && !in->rc) {
		if (in->received + inject_lost(in) >= k || now_ns() - t_end > INJECT_DRAIN_NS)
			break;
		usleep(100);
	}
	in->done = 1;
	return NULL;
}

/* Give n frames back to the fill ring.  The kernel publishes the fill
 * ring's consumer index lazily (it can deliver a frame to the RX ring
 * before its fill entry reads as consumed), so a full fill ring is waited
 * out, as xdpsock's reserve loop does (rx_drop, xdpsock.c:1472-1482: wake
 * the kernel and retry).  0 or -errno (-ETIMEDOUT after 5 s). */
static int fill_all(struct xsk_sock *x, const uint64_t *a, uint32_t n)
{
	const uint64_t t0 = now_ns();
	for (uint32_t spin = 0;; spin++) {
		const int r = xsk_fill(x, a, n);
		if (r != -ENOSPC)
			return r;
		xsk_wakeup_rx(x, 0);
		if (spin > 64) {
			if (now_ns() - t0 > 5000000000ull)
				return -ETIMEDOUT;
			usleep(10);
		}
	}
}

/* Queue n TX descriptors whatever the ring's state: while the TX ring has
 * no room, recycle what the kernel has sent (completion ring -> fill ring)
 * and kick it, as l2fwd's reserve loop does (complete_tx_l2fwd + kick_tx,
 * xdpsock.c:1736-1746).  scratch holds cap addresses.  0 or -errno
 * (-ETIMEDOUT when the kernel sends nothing for 5 s). */
static int tx_all(struct xsk_sock *x, const struct xdp_desc *d, uint32_t n,
		  uint64_t *scratch, uint32_t cap)
{
	const uint64_t t0 = now_ns();
	for (uint32_t spin = 0;; spin++) {
		int r = xsk_tx(x, d, n);
		if (r != -ENOSPC)
			return r;
		const uint32_t c = xsk_complete(x, scratch, cap);
		if (c && (r = fill_all(x, scratch, c)))
			return r;
		if ((r = xsk_kick_tx(x)))
			return r;
		if (!c && spin > 64) {
			if (now_ns() - t0 > 5000000000ull)
				return -ETIMEDOUT;
			usleep(10);
		}
	}
}

int rx_run_live(const struct rx_live *lv, const struct rx_opts *o, struct rx_totals *out)
{
	struct xdpgpu_cfg cfg = {
		.device = o->device,
		.flags = o->cfg_flags,
		.max_batch = o->batch,
		.jhash_initval = o->initval,
		.tuple_fmt = o->tuple_fmt,
		.window = 64,
		.queue_id = lv->queue,
	};
	struct xdpgpu_ctx *ctx = NULL;
	struct rx_slot slot[2];
	struct xsk_sock x;
	struct injector in;
	pthread_t th;
	bool th_up = false, veth = false;
	uint8_t *verdicts = NULL;
	uint64_t *fill = NULL;
	struct xdp_desc *txd = NULL;
	int rc;

	memset(out, 0, sizeof(*out));
	memset(slot, 0, sizeof(slot));
	memset(&in, 0, sizeof(in));
	memset(&x, 0, sizeof(x));
	x.fd = x.map_fd = x.prog_fd = x.link_fd = -1;
	if (!o->batch || o->batch > lv->ring_size || lv->nframes < 2 * lv->ring_size)
		return -EINVAL;
	if (lv->veth_peer) {
		(void)xsk_link_delete(lv->ifname);
		rc = xsk_veth_create(lv->ifname, lv->veth_peer);
		if (rc) {
			fprintf(stderr, "%s: veth %s <-> %s: %s\n", o->prog, lv->ifname,
				lv->veth_peer, strerror(-rc));
			return rc == -EPERM || rc == -EACCES ? 1 : rc;
		}
		veth = true;
	}
	const struct xsk_cfg xc = {
		.ifname = lv->ifname, .queue = lv->queue, .nframes = lv->nframes,
		.frame_size = lv->frame_size, .headroom = 0, .ring_size = lv->ring_size,
		.bind_flags = lv->bind_flags, .xdp_flags = lv->xdp_flags, .attach_prog = true,
	};
	rc = xsk_open(&x, &xc);
	if (rc) {
		fprintf(stderr, "%s: AF_XDP on %s:%u: %s\n", o->prog, lv->ifname, lv->queue, x.err);
		rc = (rc == -EPERM || rc == -EACCES || rc == -EAFNOSUPPORT) ? 1 : rc;
		goto out;
	}
	if (!o->plumbing) {
		rc = xdpgpu_init(&cfg, &ctx);
		if (rc) {
			fprintf(stderr, "%s: xdpgpu_init: %s%s\n", o->prog, strerror(-rc),
				rc == -ENODEV ? " (no GPU: this build has no CPU fallback)" : "");
			goto out;
		}
		rc = xdpgpu_register_umem(ctx, x.umem, x.umem_size, lv->frame_size, 0, 0);
		if (rc) {
			fprintf(stderr, "%s: xdpgpu_register_umem: %s %s\n", o->prog,
				strerror(-rc), xdpgpu_last_error(ctx));
			goto out;
		}
	}
	for (int k = 0; k < 2; k++) {
		/* plumbing: no GPU, plain host memory */
		const uint64_t db = (uint64_t)o->batch * sizeof(*slot[k].d);
		slot[k].d = o->plumbing ? malloc(db) : xdpgpu_host_alloc(db);
		slot[k].v = o->plumbing ? malloc(o->batch) : xdpgpu_host_alloc(o->batch);
		if (!slot[k].d || !slot[k].v)
			rc = -ENOMEM;
	}
	fill = malloc((size_t)lv->nframes * sizeof(*fill));
	txd = malloc((size_t)o->batch * sizeof(*txd));
	if (o->verdict_out && o->count)
		verdicts = calloc(o->count, 1);
	if (rc || !fill || !txd || (o->verdict_out && o->count && !verdicts)) {
		rc = -ENOMEM;
		goto out;
	}
	/* the fill ring takes the first ring_size frames, the rest wait in a
	 * free list (xsk_populate_fill_ring, xdpsock.c:1081-1098) */
	uint32_t nfree = 0;
	for (uint32_t i = 0; i < lv->nframes; i++)
		fill[nfree++] = (uint64_t)i * lv->frame_size;
	nfree -= lv->ring_size;
	rc = xsk_fill(&x, fill + nfree, lv->ring_size);
	if (rc)
		goto out;

	if (lv->inject) {
		in.lv = lv;
		in.x = &x;
		in.ifname = lv->veth_peer ? lv->veth_peer : lv->ifname;
		if (pthread_create(&th, NULL, inject_main, &in)) {
			rc = -errno;
			goto out;
		}
		th_up = true;
	}

	rx_done = 0;
	signal(SIGINT, on_signal);
	signal(SIGTERM, on_signal);
	setlocale(LC_NUMERIC, "en_US");
	const uint64_t t0 = now_ns();
	struct rx_stats_state st = { .t_prev = t0 };
	const char *label = o->label ? o->label : o->prog;
	uint64_t seen = 0, t_last = t0;    /* last frame received */
	uint32_t k = 0, idle = 0;

	while (!rc) {
		struct rx_slot *s = &slot[k & 1];
		const bool stop = rx_done || (o->count && seen >= o->count) ||
				  (o->duration_ns && now_ns() - t0 >= o->duration_ns) ||
				  (lv->inject && !o->count && !o->duration_ns && in.done &&
				   (seen >= in.sent - in.lost || now_ns() - t_last > 200000000ull));
		s->n = 0;
		if (!stop) {
			uint32_t want = o->batch;
			if (o->count && o->count - seen < want)
				want = (uint32_t)(o->count - seen);
			s->n = xsk_rx(&x, (struct xdp_desc *)s->d, want);
			if (s->n) {
				/* plumbing: every frame is the application's, as
				 * in xdpsock's own loop (no verdict compute) */
				if (o->plumbing)
					memset(s->v, XDPGPU_REDIRECT, s->n);
				s->first = seen;
				seen += s->n;
				/* off the RX ring: the injector's window moves now,
				 * however long the GPU batch takes */
				in.received = seen;
				t_last = now_ns();
				if (!o->plumbing)
					rc = xdpgpu_submit(ctx, k & 1, s->d, s->n, s->v, NULL, NULL);
				if (rc)
					break;
				s->busy = true;
			}
		}
		/* the previous batch: wait, apply its verdicts to the rings */
		struct rx_slot *p = &slot[(k + 1) & 1];
		if (p->busy) {
			rc = o->plumbing ? 0 : xdpgpu_wait(ctx, (k + 1) & 1);
			if (rc)
				break;
			p->busy = false;
			uint32_t ntx = 0, nfill = 0;
			for (uint32_t i = 0; i < p->n; i++) {
				const uint8_t v = p->v[i];
				const uint64_t a = p->d[i].addr;
				bool tx = false;

				out->rx_frags++;
				out->rx_pkts++;
				out->rx_bytes += p->d[i].len;
				if (v < XDPGPU_NUM_VERDICTS && !o->plumbing)
					out->verdict[v]++;
				if (verdicts && p->first + i < o->count)
					verdicts[p->first + i] = v;
				if (o->mode == RX_MODE_L2FWD && v == XDPGPU_REDIRECT) {
					swap_macs(x.umem + a);
					tx = true;
				} else if (v == XDPGPU_TX && o->mode != RX_MODE_DROP) {
					tx = true;     /* the reply the GPU wrote */
				}
				if (tx) {
					txd[ntx].addr = a;
					txd[ntx].len = p->d[i].len;
					txd[ntx].options = 0;
					ntx++;
					out->tx_pkts++;
					out->tx_frags++;
					out->tx_bytes += p->d[i].len;
				} else {
					fill[nfree + nfill++] = a - a % lv->frame_size;
				}
			}
			/* the fill ring first: tx_all uses the same scratch */
			if (nfill)
				rc = fill_all(&x, fill + nfree, nfill);
			if (!rc && ntx)
				rc = tx_all(&x, txd, ntx, fill + nfree, lv->ring_size);
			out->batches++;
		}
		/* sent frames back to the fill ring (complete_tx_l2fwd) */
		if (!rc) {
			uint32_t c = xsk_complete(&x, fill + nfree, lv->ring_size);
			if (c)
				rc = fill_all(&x, fill + nfree, c);
			else if (x.tx.cached_prod != x.tx.cached_cons)
				(void)xsk_kick_tx(&x);
		}
		if (stop && !slot[0].busy && !slot[1].busy)
			break;
		if (!s->n && !p->n) {
			if (++idle > 64)
				xsk_wakeup_rx(&x, 1);
		} else {
			idle = 0;
		}
		p->n = 0;
		k++;
		if (o->interval_s && !o->quiet) {
			const uint64_t t = now_ns();
			if (t - st.t_prev >= (uint64_t)o->interval_s * 1000000000ull)
				print_stats(o, out, &st, label, t);
		}
	}
	for (int j = 0; j < 2 && ctx; j++)
		if (slot[j].busy)
			(void)xdpgpu_wait(ctx, j);
	const uint64_t t1 = now_ns();
	if (th_up) {
		/* the injector's counts are final before they are printed */
		in.stop = 1;
		pthread_join(th, NULL);
		th_up = false;
		if (!rc && in.rc)
			rc = in.rc;
		/* drops the kernel counted after the injector's last look */
		(void)inject_lost(&in);
	}
	out->seconds = (double)(t1 - t0) / 1e9;
	if (rc)
		fprintf(stderr, "%s: live RX failed: %s %s\n", o->prog, strerror(-rc),
			ctx ? xdpgpu_last_error(ctx) : "");
	else if (!o->quiet)
		print_stats(o, out, &st, label, t1);
	const bool aligned = !in.lost;
	if (!rc && verdicts && !aligned)
		fprintf(stderr, "%s: %llu injected frames lost: verdicts no longer line up "
			"with the source, %s not written\n", o->prog,
			(unsigned long long)in.lost, o->verdict_out);
	if (!rc && verdicts && aligned) {
		FILE *f = fopen(o->verdict_out, "wb");
		const size_t nv = seen < o->count ? (size_t)seen : (size_t)o->count;
		if (!f || fwrite(verdicts, 1, nv, f) != nv)
			rc = -EIO;
		if (f && fclose(f))
			rc = -EIO;
	}
	if (!rc && o->json) {
		const double mpps = out->seconds > 0 ? out->rx_pkts / out->seconds / 1e6 : 0;
		printf("{\"prog\": \"%s\", \"live\": \"%s:%u\", \"plumbing\": %s, "
		       "\"mode\": \"%s\", \"frames\": %llu, \"seconds\": %.6f, "
		       "\"mpps\": %.3f, \"rx_pkts\": %llu, \"rx_bytes\": %llu, \"tx_pkts\": %llu, "
		       "\"injected\": %llu, \"lost\": %llu, \"verdicts_aligned\": %s, "
		       "\"batch\": %u, \"batches\": %llu, "
		       "\"verdict\": {\"ABORTED\": %llu, \"DROP\": %llu, \"PASS\": %llu, "
		       "\"TX\": %llu, \"REDIRECT\": %llu}}\n",
		       o->prog, lv->ifname, lv->queue, o->plumbing ? "true" : "false",
		       o->mode == RX_MODE_L2FWD ? "l2fwd" : o->mode == RX_MODE_ECHO ? "echo" : "rxdrop",
		       (unsigned long long)out->rx_pkts,
		       out->seconds, mpps, (unsigned long long)out->rx_pkts,
		       (unsigned long long)out->rx_bytes, (unsigned long long)out->tx_pkts,
		       (unsigned long long)in.sent, (unsigned long long)in.lost,
		       aligned ? "true" : "false", o->batch,
		       (unsigned long long)out->batches,
		       (unsigned long long)out->verdict[0], (unsigned long long)out->verdict[1],
		       (unsigned long long)out->verdict[2], (unsigned long long)out->verdict[3],
		       (unsigned long long)out->verdict[4]);
		fflush(stdout);
	}
out:
	if (th_up) {
		in.stop = 1;
		pthread_join(th, NULL);
		if (!rc && in.rc)
			rc = in.rc;
	}
	for (int j = 0; j < 2; j++) {
		if (o->plumbing) {
			free(slot[j].d);
			free(slot[j].v);
		} else {
			xdpgpu_host_free(slot[j].d);
			xdpgpu_host_free(slot[j].v);
		}
	}
	free(fill);
	free(txd);
	free(verdicts);
	if (ctx)
		xdpgpu_fini(ctx);
	xsk_close(&x);
	if (veth)
		(void)xsk_link_delete(lv->ifname);
	return rc;
}
