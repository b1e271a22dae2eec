// SPDX-License-Identifier: GPL-2.0
/*
 * xsk_probe - the live AF_XDP plumbing without a GPU: make a veth pair,
 * bind an AF_XDP socket (copy mode, generic XDP redirect program) to one
 * end, send frames into the other with AF_PACKET and check that each comes
 * out of the socket's RX ring byte for byte; then send them back out of
 * the TX ring and check the completions.  Prints one JSON line; exit 0
 * when every step worked, 2 when the host refuses AF_XDP / bpf / netlink
 * (the "live" column of DESIGN.md records which).
 *
 *   xsk_probe [--frames N] [--ifa NAME] [--ifb NAME] [--size BYTES]
 *             [--inject-file F] [--capture F]
 *   xsk_probe --caps      which live steps the host allows
 *
 * --inject-file: the frames to send instead of the built-in ones ("XGPI",
 * u32 count, then per frame u32 length and its bytes); --capture: what the
 * RX ring delivered, in order ("XGPC", u32 count, u32 chunk size, then per
 * descriptor the struct xdp_desc and the frame's bytes) - the live
 * fixture of tests/test_live.py (tools/live_capture.py).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <getopt.h>
#include <net/if.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <sys/socket.h>
#include <linux/if_link.h>

#include "xsk.h"

#ifndef AF_XDP
#define AF_XDP 44
#endif

static uint64_t now_ns(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

/* frame k: Ethernet (ff.. dst, 02:00:00:00:00:01 src), IPv4/UDP, the
 * payload bytes a function of k */
static uint32_t make_frame(uint8_t *p, uint32_t k, uint32_t size)
{
	memset(p, 0xff, 6);
	const uint8_t src[6] = {2, 0, 0, 0, 0, 1};
	memcpy(p + 6, src, 6);
	p[12] = 0x08;
	p[13] = 0x00;
	p[14] = 0x45;
	p[15] = 0;
	const uint32_t tot = size - 14;
	p[16] = (uint8_t)(tot >> 8);
	p[17] = (uint8_t)tot;
	memset(p + 18, 0, 4);
	p[22] = 64;
	p[23] = 17;
	p[24] = p[25] = 0;
	const uint8_t sa[4] = {10, 0, 0, 1}, da[4] = {10, 0, 0, 2};
	memcpy(p + 26, sa, 4);
	memcpy(p + 30, da, 4);
	p[34] = (uint8_t)(1000 + k % 64) >> 8;
	p[35] = (uint8_t)(1000 + k % 64);
	p[36] = 0x12;
	p[37] = 0x34;
	p[38] = (uint8_t)((tot - 20) >> 8);
	p[39] = (uint8_t)(tot - 20);
	p[40] = p[41] = 0;
	for (uint32_t j = 42; j < size; j++)
		p[j] = (uint8_t)(k * 31 + j);
	return size;
}

/* --caps: which of the live steps this host allows, one by one */
static int caps(void)
{
	const int s = socket(AF_XDP, SOCK_RAW, 0);
	const int e_sock = s < 0 ? errno : 0;
	if (s >= 0)
		close(s);
	int rc = xsk_veth_create("xgcap0", "xgcap1");
	if (!rc)
		xsk_link_delete("xgcap0");
	/* an AF_XDP socket on lo (no program: the bind alone) */
	struct xsk_cfg cfg = {
		.ifname = "lo", .queue = 0, .nframes = 1024, .frame_size = 2048,
		.ring_size = 512, .bind_flags = XDP_COPY, .attach_prog = false,
	};
	struct xsk_sock x;
	const int rb = xsk_open(&x, &cfg);
	char err[160];
	snprintf(err, sizeof(err), "%s", rb ? x.err : "");
	xsk_close(&x);
	/* the redirect program (BPF_PROG_LOAD + BPF_LINK_CREATE on lo) */
	cfg.attach_prog = true;
	const int rp = xsk_open(&x, &cfg);
	char perr[160];
	snprintf(perr, sizeof(perr), "%s", rp ? x.err : "");
	xsk_close(&x);
	printf("{\"uid\": %u, \"af_xdp_socket\": \"%s\", \"veth_netlink\": \"%s\", "
	       "\"xsk_bind_lo\": \"%s\", \"xdp_program\": \"%s\"}\n", (unsigned)getuid(),
	       e_sock ? strerror(e_sock) : "ok", rc ? strerror(-rc) : "ok", rb ? err : "ok",
	       rp ? perr : "ok");
	return 0;
}

int main(int argc, char **argv)
{
	uint32_t nframes = 4096, size = 128;
	if (argc > 1 && !strcmp(argv[1], "--caps"))
		return caps();
	const char *ifa = "xgpa0", *ifb = "xgpb0", *inject_file = NULL, *capture = NULL;
	static const struct option opts[] = {
		{"frames", required_argument, 0, 'n'}, {"size", required_argument, 0, 's'},
		{"ifa", required_argument, 0, 'a'}, {"ifb", required_argument, 0, 'b'},
		{"inject-file", required_argument, 0, 'i'}, {"capture", required_argument, 0, 'c'},
		{0, 0, 0, 0}};
	int c;

	while ((c = getopt_long(argc, argv, "n:s:a:b:i:c:", opts, NULL)) != -1) {
		switch (c) {
		case 'n': nframes = (uint32_t)atoi(optarg); break;
		case 's': size = (uint32_t)atoi(optarg); break;
		case 'a': ifa = optarg; break;
		case 'b': ifb = optarg; break;
		case 'i': inject_file = optarg; break;
		case 'c': capture = optarg; break;
		default: return 1;
		}
	}
	uint8_t *ibuf = NULL;
	uint32_t *ilen = NULL;
	if (inject_file) {
		FILE *f = fopen(inject_file, "rb");
		char magic[4];
		uint32_t n = 0;
		if (!f || fread(magic, 1, 4, f) != 4 || memcmp(magic, "XGPI", 4) ||
		    fread(&n, 4, 1, f) != 1 || !n || n > 65536) {
			fprintf(stderr, "xsk_probe: bad inject file\n");
			return 1;
		}
		nframes = n;
		ibuf = calloc(n, 2048);
		ilen = calloc(n, 4);
		for (uint32_t k = 0; k < n; k++)
			if (fread(&ilen[k], 4, 1, f) != 1 || ilen[k] > 2048 ||
			    fread(ibuf + (size_t)k * 2048, 1, ilen[k], f) != ilen[k]) {
				fprintf(stderr, "xsk_probe: short inject file\n");
				return 1;
			}
		fclose(f);
	}
	if (size < 60 || size > 1514 || !nframes || nframes > 65536)
		return 1;

	(void)xsk_link_delete(ifa);
	int rc = xsk_veth_create(ifa, ifb);
	if (rc) {
		printf("{\"ok\": false, \"step\": \"veth\", \"error\": \"%s\"}\n", strerror(-rc));
		return 2;
	}
	/* a UMEM of 2x the frames: the fill ring holds one half */
	struct xsk_cfg cfg = {
		.ifname = ifa, .queue = 0, .nframes = 2 * 4096, .frame_size = 2048,
		.headroom = 0, .ring_size = 4096, .bind_flags = XDP_COPY,
		.xdp_flags = XDP_FLAGS_SKB_MODE, .attach_prog = true,
	};
	struct xsk_sock x;
	rc = xsk_open(&x, &cfg);
	if (rc) {
		printf("{\"ok\": false, \"step\": \"xsk_open\", \"error\": \"%s\"}\n", x.err);
		xsk_close(&x);
		xsk_link_delete(ifa);
		return 2;
	}
	uint64_t addrs[4096];
	for (uint32_t i = 0; i < 4096; i++)
		addrs[i] = (uint64_t)i * cfg.frame_size;
	rc = xsk_fill(&x, addrs, 4096);

	/* the frames to send, in a buffer of their own */
	uint8_t *src = calloc(nframes, 2048);
	struct xdp_desc *sd = calloc(nframes, sizeof(*sd));
	struct xdp_desc *rd = calloc(nframes, sizeof(*rd));
	for (uint32_t k = 0; k < nframes; k++) {
		sd[k].addr = (uint64_t)k * 2048;
		if (ibuf) {
			memcpy(src + sd[k].addr, ibuf + (size_t)k * 2048, ilen[k]);
			sd[k].len = ilen[k];
		} else {
			sd[k].len = make_frame(src + sd[k].addr, k, size - (k % 7));
		}
	}
	FILE *cap = NULL;
	if (capture) {
		cap = fopen(capture, "wb");
		const uint32_t hdr[2] = {nframes, cfg.frame_size};
		if (!cap || fwrite("XGPC", 1, 4, cap) != 4 || fwrite(hdr, 4, 2, cap) != 2) {
			fprintf(stderr, "xsk_probe: cannot write %s\n", capture);
			return 1;
		}
	}
	uint32_t got = 0, bad = 0, sent_total = 0;
	const uint64_t t0 = now_ns();
	/* in waves that the fill ring can absorb */
	for (uint32_t lo = 0; lo < nframes && !rc;) {
		const uint32_t m = nframes - lo < 2048 ? nframes - lo : 2048;
		const int s = xsk_inject(ifb, src, sd + lo, m);
		if (s < 0) {
			rc = s;
			break;
		}
		sent_total += (uint32_t)s;
		const uint64_t deadline = now_ns() + 2000000000ull;
		uint32_t want = got + (uint32_t)s;
		while (got < want && now_ns() < deadline) {
			const uint32_t r = xsk_rx(&x, rd + got, want - got);
			if (!r) {
				xsk_wakeup_rx(&x, 10);
				continue;
			}
			/* recycle the received frames' chunks to the fill ring */
			for (uint32_t j = 0; j < r; j++) {
				const struct xdp_desc *d = &rd[got + j];
				const uint32_t k = got + j;

				if (d->len != sd[k].len ||
				    memcmp(x.umem + d->addr, src + sd[k].addr, d->len))
					bad++;
				if (cap && (fwrite(d, sizeof(*d), 1, cap) != 1 ||
					    fwrite(x.umem + d->addr, 1, d->len, cap) != d->len))
					rc = -EIO;
				uint64_t a = d->addr - (d->addr % cfg.frame_size);
				(void)xsk_fill(&x, &a, 1);
			}
			got += r;
		}
		lo += m;
	}
	const double rx_s = (now_ns() - t0) / 1e9;

	/* TX: send the first min(got, 1024) received frames back out */
	uint32_t ntx = got < 1024 ? got : 1024, done = 0;
	if (!rc && ntx) {
		/* TX frames from the second half of the UMEM */
		struct xdp_desc *td = calloc(ntx, sizeof(*td));
		for (uint32_t j = 0; j < ntx; j++) {
			td[j].addr = (uint64_t)(4096 + j) * cfg.frame_size;
			td[j].len = sd[j].len;
			memcpy(x.umem + td[j].addr, src + sd[j].addr, sd[j].len);
		}
		rc = xsk_tx(&x, td, ntx);
		const uint64_t deadline = now_ns() + 2000000000ull;
		uint64_t ca[1024];
		while (!rc && done < ntx && now_ns() < deadline) {
			const uint32_t r = xsk_complete(&x, ca, ntx - done);
			done += r;
			if (!r)
				(void)xsk_kick_tx(&x);
		}
		free(td);
	}
	printf("{\"ok\": %s, \"frames\": %u, \"sent\": %u, \"received\": %u, \"mismatched\": %u, "
	       "\"tx\": %u, \"tx_completed\": %u, \"rx_seconds\": %.4f, \"ifindex\": %d, "
	       "\"mode\": \"copy, generic XDP\"%s%s%s}\n",
	       (!rc && got == nframes && !bad && done == ntx) ? "true" : "false", nframes,
	       sent_total, got, bad, ntx, done, rx_s, x.ifindex,
	       rc ? ", \"error\": \"" : "", rc ? strerror(-rc) : "", rc ? "\"" : "");
	if (cap && fclose(cap))
		rc = -EIO;
	xsk_close(&x);
	xsk_link_delete(ifa);
	free(ibuf);
	free(ilen);
	free(src);
	free(sd);
	free(rd);
	return (!rc && got == nframes && !bad && done == ntx) ? 0 : 1;
}
