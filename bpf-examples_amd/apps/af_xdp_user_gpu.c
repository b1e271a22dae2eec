// SPDX-License-Identifier: GPL-2.0
/*
 * af_xdp_user-gpu - the af_xdp_user command line
 * (AF_XDP-interaction/af_xdp_user.c:225-309 and common_params.c:103-284)
 * with process_packet (af_xdp_user.c:968-1040) on an MI355X: every frame
 * is parsed and checked on the GPU; ICMPv6 echo requests are rewritten in
 * place into replies (csum_replace2, af_xdp_user.c:590-606) and counted as
 * sent, every other frame is recycled, as handle_receive_packets does
 * (af_xdp_user.c:1079-1113).  Statistics are stats_print's
 * (af_xdp_user.c:1360-1397), every 2 seconds as stats_poll prints them.
 *
 * process_packet does not verify checksums, so neither does this program
 * by default (--verify turns the DROP verdict on).  The reference's
 * options are parsed with its short-option string; the ones that act on a
 * kernel socket or XDP program (-S -N -A -F -c -z -Q -p -w -s -U -B
 * --filename --progsec --offload-mode) have no effect on a pool or pcap
 * source, -d labels the statistics, --src-ip/--dst-ip/-G/-H set the
 * generated frames (gen_base_pkt, af_xdp_user.c:688-700).  Frames come from
 * --pool N or --pcap FILE, or, with -d IF and neither, from a live AF_XDP
 * socket on IF (apps/xsk.c; -S / -N, -c / -z, -Q queue as the reference
 * uses them; --veth PEER, --inject N, --inject-pcap FILE as xdpsock-gpu's),
 * the echo replies sent on its TX ring.
 *
 * Exit status as common_defines.h:50-54: 0, 1 (EXIT_FAIL), 2
 * (EXIT_FAIL_OPTION).
 */
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <errno.h>
#include <getopt.h>
#include <libgen.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <linux/if_link.h>

#include "rxapp.h"
#include "xsk.h"

#define EXIT_OK 0
#define EXIT_FAIL 1
#define EXIT_FAIL_OPTION 2

enum {
	OPT_GPU = 256, OPT_POOL, OPT_POOL_KIND, OPT_SEED, OPT_PCAP, OPT_VERIFY,
	OPT_COUNT, OPT_DURATION, OPT_JSON, OPT_VERDICTS, OPT_TX_PCAP, OPT_DRY_RUN,
	OPT_ECHO_PPM, OPT_SIZE, OPT_BATCH, OPT_VETH, OPT_INJECT, OPT_INJECT_PCAP,
};

struct opt_help {
	struct option option;
	const char *help;
	const char *metavar;
};

/* af_xdp_user.c:225-309, plus this build's options */
static const struct opt_help opts[] = {
	{ { "help", no_argument, NULL, 'h' }, "Show help", NULL },
	{ { "dev", required_argument, NULL, 'd' }, "Live AF_XDP on <ifname> (no --pool/--pcap), else a label", "<ifname>" },
	{ { "skb-mode", no_argument, NULL, 'S' }, "Generic XDP (live; default)", NULL },
	{ { "native-mode", no_argument, NULL, 'N' }, "Native XDP (live)", NULL },
	{ { "auto-mode", no_argument, NULL, 'A' }, "(no effect)", NULL },
	{ { "force", no_argument, NULL, 'F' }, "(no effect)", NULL },
	{ { "copy", no_argument, NULL, 'c' }, "Copy mode (live; default)", NULL },
	{ { "zero-copy", no_argument, NULL, 'z' }, "Zero-copy mode (live)", NULL },
	{ { "queue", required_argument, NULL, 'Q' }, "Receive queue", NULL },
	{ { "priority", required_argument, NULL, 'p' }, "(no effect)", NULL },
	{ { "wakeup-mode", no_argument, NULL, 'w' }, "(no effect)", NULL },
	{ { "spin-mode", no_argument, NULL, 's' }, "(no effect)", NULL },
	{ { "unload", no_argument, NULL, 'U' }, "(no effect)", NULL },
	{ { "quiet", no_argument, NULL, 'q' }, "Quiet mode (no output)", NULL },
	{ { "pktinfo", no_argument, NULL, 'P' }, "(no effect)", NULL },
	{ { "metainfo", no_argument, NULL, 'm' }, "(no effect)", NULL },
	{ { "timedebug", no_argument, NULL, 't' }, "(no effect)", NULL },
	{ { "debug", no_argument, NULL, 'D' }, "(no effect)", NULL },
	{ { "filename", required_argument, NULL, 1 }, "(no effect)", "<file>" },
	{ { "progsec", required_argument, NULL, 2 }, "(no effect)", "<section>" },
	{ { "offload-mode", no_argument, NULL, 3 }, "(no effect)", NULL },
	{ { "src-ip", required_argument, NULL, 4 }, "IPv4 source address of generated frames", "<ip>" },
	{ { "dst-ip", required_argument, NULL, 5 }, "IPv4 destination address of generated frames", "<ip>" },
	{ { "busy-poll", no_argument, NULL, 'B' }, "(no effect)", NULL },
	{ { "tx-dmac", required_argument, NULL, 'G' }, "Dest MAC of generated frames", "aa:bb:cc:dd:ee:ff" },
	{ { "tx-smac", required_argument, NULL, 'H' }, "Src MAC of generated frames", "aa:bb:cc:dd:ee:ff" },
	{ { "interval", required_argument, NULL, 'i' }, "(no effect: no cyclic TX)", "<usec>" },
	{ { "batch-pkts", required_argument, NULL, 'b' }, "Descriptors per GPU batch (default 64)", "<pkts>" },
	{ { "gpu", required_argument, NULL, OPT_GPU }, "HIP device (default 0)", "<n>" },
	{ { "pool", required_argument, NULL, OPT_POOL }, "Synthetic UMEM pool of <n> frames", "<n>" },
	{ { "pool-kind", required_argument, NULL, OPT_POOL_KIND }, "afxdp (default) | udp4 | imix | xdpsock", "<k>" },
	{ { "pool-size", required_argument, NULL, OPT_SIZE }, "Pool frame size (default 64)", "<bytes>" },
	{ { "echo-ppm", required_argument, NULL, OPT_ECHO_PPM }, "ICMPv6 echo requests per million (udp4/imix pools)", "<n>" },
	{ { "seed", required_argument, NULL, OPT_SEED }, "Pool seed", "<s>" },
	{ { "pcap", required_argument, NULL, OPT_PCAP }, "Frames of a pcap file (Ethernet)", "<file>" },
	{ { "verify", no_argument, NULL, OPT_VERIFY }, "Drop frames with bad checksums", NULL },
	{ { "count", required_argument, NULL, OPT_COUNT }, "Frames to receive (default: one pass)", "<n>" },
	{ { "duration", required_argument, NULL, OPT_DURATION }, "Seconds to run", "<s>" },
	{ { "json", no_argument, NULL, OPT_JSON }, "One JSON summary line at the end", NULL },
	{ { "verdicts", required_argument, NULL, OPT_VERDICTS }, "Per-frame verdicts of the first pass", "<file>" },
	{ { "tx-pcap", required_argument, NULL, OPT_TX_PCAP }, "The echo replies of the first pass, as pcap", "<file>" },
	{ { "dry-run", no_argument, NULL, OPT_DRY_RUN }, "Build the UMEM, describe it, no GPU", NULL },
	{ { "veth", required_argument, NULL, OPT_VETH }, "Live: make the veth pair <ifname> <-> <peer>", "<peer>" },
	{ { "inject", required_argument, NULL, OPT_INJECT }, "Live: send <n> frames of the pool into the peer", "<n>" },
	{ { "inject-pcap", required_argument, NULL, OPT_INJECT_PCAP }, "Live: send a pcap file's frames into the peer", "<file>" },
	{ { NULL, 0, NULL, 0 }, NULL, NULL },
};

static void usage(const char *prog, bool full)
{
	printf("Usage: %s [options]\n", prog);
	if (!full) {
		printf("Use --help (or -h) to see full option list.\n");
		return;
	}
	printf("\nDOCUMENTATION:\n AF_XDP kernel bypass example, per-packet work on the GPU\n\n");
	printf("Options:\n");
	for (int i = 0; opts[i].option.name; i++) {
		char buf[40];
		int pos;
		if (opts[i].option.val > 64 && opts[i].option.val < 128)
			printf(" -%c,", opts[i].option.val);
		else
			printf("    ");
		pos = snprintf(buf, sizeof(buf), " --%s", opts[i].option.name);
		if (opts[i].metavar)
			snprintf(buf + pos, sizeof(buf) - pos, " %s", opts[i].metavar);
		printf("%-22s  %s\n", buf, opts[i].help);
	}
	printf("\n");
}

/* parse_cmdline_args' error path, common_params.c:276-281 */
static int opt_error(const char *prog)
{
	usage(prog, false);
	return EXIT_FAIL_OPTION;
}

static int pool_kind(const char *s)
{
	if (!strcmp(s, "afxdp"))
		return XDPGPU_POOL_AFXDP_USER;
	if (!strcmp(s, "udp4"))
		return XDPGPU_POOL_UDP4;
	if (!strcmp(s, "imix"))
		return XDPGPU_POOL_IMIX;
	if (!strcmp(s, "xdpsock"))
		return XDPGPU_POOL_XDPSOCK;
	return -1;
}

int main(int argc, char **argv)
{
	const char *prog = basename(argv[0]);
	const char *ifname = "pool", *pcap = NULL, *veth = NULL, *inject_pcap = NULL;
	int queue = 0, kind = XDPGPU_POOL_AFXDP_USER, dry = 0;
	bool dev_set = false, native = false, zerocopy = false;
	uint64_t inject_n = 0;
	uint32_t pool_n = 0, size = 64, echo_ppm = 0, saddr = 0, daddr = 0;
	bool have_echo = false, have_dmac = false, have_smac = false;
	uint64_t seed = 0x5EED0003;
	uint8_t dmac[6], smac[6];
	struct option lo[sizeof(opts) / sizeof(opts[0])];
	struct rx_opts o = {
		.cfg_flags = XDPGPU_CFG_ICMP6_ECHO | XDPGPU_CFG_STATS,
		.tuple_fmt = XDPGPU_TUPLE_NONE,
		.batch = 64,              /* RX_BATCH_SIZE, af_xdp_user.c:58 */
		.interval_s = 2,          /* stats_poll, af_xdp_user.c:1401 */
		.mode = RX_MODE_ECHO,
		.stats_fmt = RX_STATS_AFXDP,
		.prog = prog,
	};
	int c, idx;

	for (size_t i = 0; i < sizeof(opts) / sizeof(opts[0]); i++)
		lo[i] = opts[i].option;
	/* common_params.c:121 */
	while ((c = getopt_long(argc, argv, "hd:r:L:R:BASNFUMQ:G:H:czqp:ti:b:", lo,
				&idx)) != -1) {
		switch (c) {
		case 'd':
			if (strlen(optarg) >= 16) {
				fprintf(stderr, "ERR: --dev name too long\n");
				return opt_error(prog);
			}
			ifname = optarg;
			dev_set = true;
			break;
		case 'Q': queue = atoi(optarg); break;
		case 'q': o.quiet = true; break;
		case 'b': o.batch = (uint32_t)atoi(optarg); break;
		case 'G':
			if (!rx_parse_mac(optarg, dmac)) {
				fprintf(stderr, "Invalid dest MAC address:%s\n", optarg);
				return opt_error(prog);
			}
			have_dmac = true;
			break;
		case 'H':
			if (!rx_parse_mac(optarg, smac)) {
				fprintf(stderr, "Invalid src MAC address:%s\n", optarg);
				return opt_error(prog);
			}
			have_smac = true;
			break;
		case 4:
		case 5: {
			uint32_t a;
			if (inet_pton(AF_INET, optarg, &a) != 1) {
				fprintf(stderr, "ERROR: IPv4 \"%s\" not in presentation format\n",
					optarg);
				return opt_error(prog);
			}
			if (c == 4)
				saddr = a;
			else
				daddr = a;
			break;
		}
		case 'N': native = true; break;
		case 'S': native = false; break;
		case 'z': zerocopy = true; break;
		case 'c': zerocopy = false; break;
		case OPT_VETH: veth = optarg; break;
		case OPT_INJECT: inject_n = strtoull(optarg, NULL, 0); break;
		case OPT_INJECT_PCAP: inject_pcap = optarg; break;
		case 'r': case 'L': case 'R': case 'B': case 'A':
		case 'F': case 'U': case 'M': case 'p': case 't':
		case 'i': case 'w': case 's': case 'P': case 'm': case 'D':
		case 1: case 2: case 3:
			break;    /* kernel socket / XDP program / debug options */
		case OPT_GPU: o.device = atoi(optarg); break;
		case OPT_POOL: pool_n = (uint32_t)strtoul(optarg, NULL, 0); break;
		case OPT_POOL_KIND:
			kind = pool_kind(optarg);
			if (kind < 0) {
				fprintf(stderr, "ERR: unknown pool kind %s\n", optarg);
				return opt_error(prog);
			}
			break;
		case OPT_SIZE: size = (uint32_t)atoi(optarg); break;
		case OPT_ECHO_PPM:
			echo_ppm = (uint32_t)strtoul(optarg, NULL, 0);
			have_echo = true;
			break;
		case OPT_SEED: seed = strtoull(optarg, NULL, 0); break;
		case OPT_PCAP: pcap = optarg; break;
		case OPT_VERIFY: o.cfg_flags |= XDPGPU_CFG_VERIFY_CSUM; break;
		case OPT_COUNT: o.count = strtoull(optarg, NULL, 0); break;
		case OPT_DURATION: o.duration_ns = strtoull(optarg, NULL, 0) * 1000000000ull; break;
		case OPT_JSON: o.json = true; break;
		case OPT_VERDICTS: o.verdict_out = optarg; break;
		case OPT_TX_PCAP: o.tx_pcap = optarg; break;
		case OPT_DRY_RUN: dry = 1; break;
		case 'h':
			usage(prog, true);
			return EXIT_FAIL_OPTION;
		default:
			return opt_error(prog);
		}
	}
	if (optind < argc)
		return opt_error(prog);
	const bool live = !pool_n && !pcap && dev_set;
	if (!live && !pool_n == !pcap) {
		fprintf(stderr, "ERR: give one of -d IF (live AF_XDP), --pool N or --pcap FILE\n");
		return opt_error(prog);
	}
	if (!live && (veth || inject_n || inject_pcap)) {
		fprintf(stderr, "ERR: --veth / --inject need a live socket (-d IF)\n");
		return opt_error(prog);
	}
	if (!o.batch) {
		fprintf(stderr, "ERR: batch must be positive\n");
		return opt_error(prog);
	}

	struct rx_source src;
	int rc;
	if (live) {
		/* af_xdp_user's geometry: NUM_FRAMES 4096 of FRAME_SIZE,
		 * af_xdp_user.c:55-56; default rings */
		struct rx_source inj;
		bool have_inj = false;
		if (inject_n || inject_pcap) {
			if (inject_pcap) {
				rc = rx_source_pcap(&inj, inject_pcap, 2048, 0, true, false, 0);
			} else {
				struct xdpgpu_pool_spec spec;
				xdpgpu_pool_spec_default(&spec, (uint32_t)kind, size, seed);
				if (have_echo)
					spec.ppm_echo6 = echo_ppm;
				rc = rx_source_pool(&inj, &spec,
						    (uint32_t)(inject_n < 1048576 ? inject_n : 1048576));
			}
			if (rc) {
				fprintf(stderr, "ERR: inject source: %s\n", strerror(-rc));
				return EXIT_FAIL;
			}
			have_inj = true;
			if (!inject_n)
				inject_n = inj.n;
		}
		struct rx_live lv = {
			.ifname = ifname, .queue = (uint32_t)queue, .frame_size = 4096,
			.nframes = 4096, .ring_size = 2048,
			.bind_flags = (zerocopy ? XDP_ZEROCOPY : XDP_COPY) | XDP_USE_NEED_WAKEUP,
			.xdp_flags = native ? XDP_FLAGS_DRV_MODE : XDP_FLAGS_SKB_MODE,
			.veth_peer = veth, .inject = have_inj ? &inj : NULL,
			.inject_count = inject_n,
		};
		char label[64];
		snprintf(label, sizeof(label), "%s:%d", ifname, queue);
		o.label = label;
		struct rx_totals t;
		rc = rx_run_live(&lv, &o, &t);
		if (have_inj)
			rx_source_free(&inj);
		return rc ? EXIT_FAIL : EXIT_OK;
	}
	if (pcap) {
		/* af_xdp_user's UMEM: FRAME_SIZE chunks, af_xdp_user.c:56 */
		rc = rx_source_pcap(&src, pcap, 4096, 0, false, false, 0);
		if (rc) {
			fprintf(stderr, "ERR: %s: %s\n", pcap, strerror(-rc));
			return EXIT_FAIL;
		}
	} else {
		struct xdpgpu_pool_spec spec;
		xdpgpu_pool_spec_default(&spec, (uint32_t)kind, size, seed);
		if (have_echo)
			spec.ppm_echo6 = echo_ppm;
		spec.saddr = saddr;
		spec.daddr = daddr;
		if (have_dmac)
			memcpy(spec.dmac, dmac, 6);
		if (have_smac)
			memcpy(spec.smac, smac, 6);
		rc = rx_source_pool(&src, &spec, pool_n);
		if (rc) {
			fprintf(stderr, "ERR: pool: %s\n", strerror(-rc));
			return EXIT_FAIL;
		}
	}
	if (dry) {
		rx_source_describe(&src, pcap ? pcap : "pool");
		rx_source_free(&src);
		return EXIT_OK;
	}
	char label[64];
	snprintf(label, sizeof(label), "%s:%d", ifname, queue);
	o.label = label;
	struct rx_totals t;
	rc = rx_run(&src, &o, &t);
	rx_source_free(&src);
	return rc ? EXIT_FAIL : EXIT_OK;
}
