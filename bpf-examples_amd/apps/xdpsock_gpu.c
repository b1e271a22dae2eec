// SPDX-License-Identifier: GPL-2.0
/*
 * xdpsock-gpu - the xdpsock command line (AF_XDP-example/xdpsock.c) with
 * the per-packet work on an MI355X through the C ABI (include/xdpgpu.h).
 *
 * Every xdpsock option is accepted with its meaning where it has one
 * without a kernel socket: -r/-l (rx_drop / l2fwd bodies,
 * xdpsock.c:1462-1506, 1718-1784), -b batch, -C count, -d duration, -n
 * interval, -Q, -x, -f frame size and -u unaligned chunks (UMEM geometry),
 * and the generator's -s/-P/-V/-J/-K/-G/-H (gen_eth_hdr_data,
 * xdpsock.c:893-971) for pool mode.  Socket and scheduling options (-i, -q,
 * -p, -S, -N, -z, -c, -m, -M, -B, -R, -w, -W, -U, -I, -O, -T, -y, -a)
 * are parsed as xdpsock parses them and only label the statistics.  -F
 * (--frags) splits pcap records longer than a chunk into multi-buffer
 * packets (XDPGPU_CFG_FRAGS) and counts packets and fragments.  Frames
 * come from a UMEM this program fills, either a synthetic pool (--pool N)
 * or a pcap file (--pcap FILE), or, with -i IF and neither, from a live
 * AF_XDP socket on IF:queue (apps/xsk.c; -S generic / -N native XDP, -c
 * copy / -z zero-copy, -m no need_wakeup, -f chunk size): config 1.
 *
 * Added options: --gpu N, --pool N, --pool-kind xdpsock|udp4|imix|afxdp,
 * --seed S, --pcap FILE, --no-verify, --initval N, --json, --verdicts FILE,
 * --tx-pcap FILE, --dry-run; live mode: --veth PEER (make the veth pair
 * IF <-> PEER, as testenv.sh does), --inject N (send N frames of the pool
 * the pool options describe into PEER), --inject-pcap FILE, --plumbing
 * (xdpsock's own rx_drop / l2fwd bodies with no GPU: config 1 as the
 * reference runs it, for its xdpsock-format pps).  Exit status:
 * 0, 1 on a failure (live: also when the host refuses AF_XDP), 2 on a bad
 * option (xdpsock's usage() exits with EXIT_FAILURE).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <getopt.h>
#include <libgen.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <linux/if_link.h>

#include "rxapp.h"
#include "xsk.h"

#define MIN_PKT_SIZE 64            /* xdpsock.c:65 */
#define MAX_PKT_SIZE 9728          /* xdpsock.c:66 */
#define DEFAULT_FRAME_SIZE 4096    /* XSK_UMEM__DEFAULT_FRAME_SIZE */
#define DEFAULT_PATTERN 0x12345678 /* opt_pkt_fill_pattern */

enum {
	OPT_GPU = 256, OPT_POOL, OPT_POOL_KIND, OPT_SEED, OPT_PCAP, OPT_NO_VERIFY,
	OPT_INITVAL, OPT_JSON, OPT_VERDICTS, OPT_TX_PCAP, OPT_DRY_RUN, OPT_HELP,
	OPT_VETH, OPT_INJECT, OPT_INJECT_PCAP, OPT_PLUMBING,
};

static struct option long_options[] = {
	{ "rxdrop", no_argument, 0, 'r' },
	{ "txonly", no_argument, 0, 't' },
	{ "l2fwd", no_argument, 0, 'l' },
	{ "interface", required_argument, 0, 'i' },
	{ "queue", required_argument, 0, 'q' },
	{ "poll", no_argument, 0, 'p' },
	{ "xdp-skb", no_argument, 0, 'S' },
	{ "xdp-native", no_argument, 0, 'N' },
	{ "interval", required_argument, 0, 'n' },
	{ "retries", required_argument, 0, 'O' },
	{ "zero-copy", no_argument, 0, 'z' },
	{ "copy", no_argument, 0, 'c' },
	{ "frame-size", required_argument, 0, 'f' },
	{ "no-need-wakeup", no_argument, 0, 'm' },
	{ "unaligned", no_argument, 0, 'u' },
	{ "shared-umem", no_argument, 0, 'M' },
	{ "frags", no_argument, 0, 'F' },
	{ "duration", required_argument, 0, 'd' },
	{ "clock", required_argument, 0, 'w' },
	{ "batch-size", required_argument, 0, 'b' },
	{ "tx-pkt-count", required_argument, 0, 'C' },
	{ "tx-pkt-size", required_argument, 0, 's' },
	{ "tx-pkt-pattern", required_argument, 0, 'P' },
	{ "tx-vlan", no_argument, 0, 'V' },
	{ "tx-vlan-id", required_argument, 0, 'J' },
	{ "tx-vlan-pri", required_argument, 0, 'K' },
	{ "tx-dmac", required_argument, 0, 'G' },
	{ "tx-smac", required_argument, 0, 'H' },
	{ "tx-cycle", required_argument, 0, 'T' },
	{ "tstamp", no_argument, 0, 'y' },
	{ "policy", required_argument, 0, 'W' },
	{ "schpri", required_argument, 0, 'U' },
	{ "extra-stats", no_argument, 0, 'x' },
	{ "quiet", no_argument, 0, 'Q' },
	{ "app-stats", no_argument, 0, 'a' },
	{ "irq-string", required_argument, 0, 'I' },
	{ "busy-poll", no_argument, 0, 'B' },
	{ "reduce-cap", no_argument, 0, 'R' },
	/* this build */
	{ "gpu", required_argument, 0, OPT_GPU },
	{ "pool", required_argument, 0, OPT_POOL },
	{ "pool-kind", required_argument, 0, OPT_POOL_KIND },
	{ "seed", required_argument, 0, OPT_SEED },
	{ "pcap", required_argument, 0, OPT_PCAP },
	{ "no-verify", no_argument, 0, OPT_NO_VERIFY },
	{ "initval", required_argument, 0, OPT_INITVAL },
	{ "json", no_argument, 0, OPT_JSON },
	{ "verdicts", required_argument, 0, OPT_VERDICTS },
	{ "tx-pcap", required_argument, 0, OPT_TX_PCAP },
	{ "dry-run", no_argument, 0, OPT_DRY_RUN },
	{ "veth", required_argument, 0, OPT_VETH },
	{ "inject", required_argument, 0, OPT_INJECT },
	{ "inject-pcap", required_argument, 0, OPT_INJECT_PCAP },
	{ "plumbing", no_argument, 0, OPT_PLUMBING },
	{ "help", no_argument, 0, OPT_HELP },
	{ 0, 0, 0, 0 }
};

static void usage(const char *prog)
{
	fprintf(stderr,
		"  Usage: %s [OPTIONS]\n"
		"  Options (xdpsock):\n"
		"  -r, --rxdrop		Discard all incoming packets (default)\n"
		"  -l, --l2fwd		MAC swap L2 forwarding\n"
		"  -t, --txonly		(not available: no receive path)\n"
		"  -i, --interface=n	Live AF_XDP socket on n (no --pool/--pcap), else a label\n"
		"  -q, --queue=n	Queue (default 0)\n"
		"  -S, --xdp-skb	Generic XDP (live; the default on veth)\n"
		"  -N, --xdp-native	Native XDP (live)\n"
		"  -c, --copy		Copy mode (live, default)\n"
		"  -z, --zero-copy	Zero-copy mode (live)\n"
		"  -m, --no-need-wakeup	No need_wakeup flag (live)\n"
		"  -n, --interval=n	Statistics update interval (default 1 sec)\n"
		"  -f, --frame-size=n   UMEM chunk size for --pcap (power of two unless -u, default %d)\n"
		"  -u, --unaligned	Unaligned (packed) chunk placement\n"
		"  -d, --duration=n	Duration in secs (default: one pass over the source)\n"
		"  -b, --batch-size=n	Descriptors per GPU batch (default %d)\n"
		"  -C, --tx-pkt-count=n	Frames to receive (replaying the source)\n"
		"  -s, --tx-pkt-size=n	Pool frame size, %d..%d (default %d)\n"
		"  -P, --tx-pkt-pattern=n Pool fill pattern (default 0x%x)\n"
		"  -V, --tx-vlan        VLAN-tagged pool frames\n"
		"  -J, --tx-vlan-id=n   VLAN ID [1-4095] (default 1)\n"
		"  -K, --tx-vlan-pri=n  VLAN priority [0-7] (default 0)\n"
		"  -G, --tx-dmac=<MAC>  Pool destination MAC\n"
		"  -H, --tx-smac=<MAC>  Pool source MAC\n"
		"  -x, --extra-stats	GPU verdict counters in the statistics\n"
		"  -Q, --quiet          Do not display any stats\n"
		"  -F, --frags          Multi-buffer packets: pcap records longer than a chunk span\n"
		"                       several chunks (XDP_PKT_CONTD); packets and frags counted\n"
		"  -p -M -B -R -w -W -U -I -O -T -y -a: accepted, no effect\n"
		"  Options (this build):\n"
		"      --gpu=n          HIP device (default 0)\n"
		"      --pool=n         Synthetic UMEM pool of n frames\n"
		"      --pool-kind=k    xdpsock (default) | udp4 | imix | afxdp\n"
		"      --seed=s         Pool seed\n"
		"      --pcap=file      Frames of a pcap file (Ethernet)\n"
		"      --no-verify      Do not drop frames with bad checksums\n"
		"      --initval=n      jhash initval (default 0)\n"
		"      --json           One JSON summary line at the end\n"
		"      --verdicts=file  Per-frame verdicts (u8, enum xdp_action) of the first pass\n"
		"      --tx-pcap=file   The frames sent (l2fwd) in the first pass, as pcap\n"
		"      --dry-run        Build the UMEM, describe it, no GPU\n"
		"      --veth=peer      Live: make the veth pair IF <-> peer (removed at exit)\n"
		"      --inject=n       Live: send n frames of the pool (pool options) into peer\n"
		"      --inject-pcap=f  Live: send the frames of a pcap file into peer\n"
		"      --plumbing       Live: xdpsock's own rx_drop / l2fwd bodies, no GPU\n"
		"                       (config 1: the reference's CPU-only run on a veth)\n",
		prog, DEFAULT_FRAME_SIZE, 64, MIN_PKT_SIZE, MAX_PKT_SIZE, MIN_PKT_SIZE,
		DEFAULT_PATTERN);
	exit(2);
}

static int pool_kind(const char *s)
{
	if (!strcmp(s, "xdpsock"))
		return XDPGPU_POOL_XDPSOCK;
	if (!strcmp(s, "udp4"))
		return XDPGPU_POOL_UDP4;
	if (!strcmp(s, "imix"))
		return XDPGPU_POOL_IMIX;
	if (!strcmp(s, "afxdp"))
		return XDPGPU_POOL_AFXDP_USER;
	return -1;
}

/* config 1: a live socket, frames from the wire (or the injected source) */
static int run_live(const char *prog, const char *ifname, uint32_t queue, struct rx_opts *o,
		    uint32_t frame_size, bool skb, bool zerocopy, bool no_wakeup,
		    const char *veth, uint64_t inject_n, const char *inject_pcap, int kind,
		    uint32_t pkt_size, uint64_t seed)
{
	struct rx_source inj;
	bool have_inj = false;
	int rc;

	if (inject_n || inject_pcap) {
		if (inject_pcap) {
			rc = rx_source_pcap(&inj, inject_pcap, 2048, 0, true, false, 0);
		} else {
			struct xdpgpu_pool_spec spec;
			xdpgpu_pool_spec_default(&spec, (uint32_t)kind, pkt_size, seed);
			rc = rx_source_pool(&inj, &spec,
					    (uint32_t)(inject_n < 1048576 ? inject_n : 1048576));
		}
		if (rc) {
			fprintf(stderr, "%s: inject source: %s\n", prog, strerror(-rc));
			return 1;
		}
		have_inj = true;
		if (!inject_n)
			inject_n = inj.n;
	}
	/* xdpsock's defaults: NUM_FRAMES 4096, 2048-entry rings
	 * (XSK_RING_*__DEFAULT_NUM_DESCS), 4096-byte frames */
	struct rx_live lv = {
		.ifname = ifname, .queue = queue, .frame_size = frame_size,
		.nframes = 4096, .ring_size = 2048,
		.bind_flags = (zerocopy ? XDP_ZEROCOPY : XDP_COPY) |
			      (no_wakeup ? 0 : XDP_USE_NEED_WAKEUP),
		.xdp_flags = skb ? XDP_FLAGS_SKB_MODE : XDP_FLAGS_DRV_MODE,
		.veth_peer = veth, .inject = have_inj ? &inj : NULL, .inject_count = inject_n,
	};
	char label[128];
	snprintf(label, sizeof(label), "%s:%u %s %s", ifname, queue,
		 o->mode == RX_MODE_L2FWD ? "l2fwd" : "rxdrop", skb ? "xdp-skb" : "xdp-drv");
	o->label = label;
	struct rx_totals t;
	rc = rx_run_live(&lv, o, &t);
	if (have_inj)
		rx_source_free(&inj);
	return rc ? 1 : 0;
}

int main(int argc, char **argv)
{
	const char *prog = basename(argv[0]);
	const char *ifname = "pool", *pcap = NULL;
	int queue = 0, kind = XDPGPU_POOL_XDPSOCK, vlan = 0, dry = 0, extra = 0;
	uint32_t pool_n = 0, pkt_size = MIN_PKT_SIZE, frame_size = DEFAULT_FRAME_SIZE;
	uint32_t pattern = DEFAULT_PATTERN, vlan_id = 1, vlan_pri = 0, unaligned = 0;
	uint64_t seed = 0x5EED0002, inject_n = 0;
	const char *veth = NULL, *inject_pcap = NULL;
	bool live_native = false, zerocopy = false, no_wakeup = false, iface_set = false;
	uint8_t dmac[6], smac[6];
	bool have_dmac = false, have_smac = false, have_pattern = false, skb = false;
	struct rx_opts o = {
		.cfg_flags = XDPGPU_CFG_DEFAULT,
		.tuple_fmt = XDPGPU_TUPLE_NONE,
		.batch = 64,              /* opt_batch_size, xdpsock.c:108 */
		.interval_s = 1,          /* opt_interval, xdpsock.c:127 */
		.mode = RX_MODE_DROP,
		.stats_fmt = RX_STATS_XDPSOCK,
		.prog = prog,
	};
	int c, idx;

	opterr = 0;
	while ((c = getopt_long(argc, argv,
				"rtli:q:pSNn:w:O:czf:muMd:b:C:s:P:VJ:K:G:H:T:yW:U:xQaI:BRF",
				long_options, &idx)) != -1) {
		switch (c) {
		case 'r': o.mode = RX_MODE_DROP; break;
		case 'l': o.mode = RX_MODE_L2FWD; break;
		case 't':
			fprintf(stderr, "%s: -t/--txonly has no receive path; use xdpsock\n",
				prog);
			return 2;
		case 'i': ifname = optarg; iface_set = true; break;
		case 'q': queue = atoi(optarg); break;
		case 'S': skb = true; break;
		case 'N': live_native = true; break;
		case 'z': zerocopy = true; break;
		case 'c': zerocopy = false; break;
		case 'm': no_wakeup = true; break;
		case 'n': o.interval_s = (uint32_t)atoi(optarg); break;
		case 'f': frame_size = (uint32_t)atoi(optarg); break;
		case 'u': unaligned = 1; break;
		case 'd': o.duration_ns = (uint64_t)atoi(optarg) * 1000000000ull; break;
		case 'b': o.batch = (uint32_t)atoi(optarg); break;
		case 'C': o.count = strtoull(optarg, NULL, 0); break;
		case 's':
			pkt_size = (uint32_t)atoi(optarg);
			if (pkt_size > MAX_PKT_SIZE || pkt_size < MIN_PKT_SIZE) {
				fprintf(stderr, "ERROR: Invalid frame size %d\n", (int)pkt_size);
				usage(prog);
			}
			break;
		case 'P':
			pattern = (uint32_t)strtol(optarg, NULL, 16);
			have_pattern = true;
			break;
		case 'V': vlan = 1; break;
		case 'J': vlan_id = (uint32_t)atoi(optarg); break;
		case 'K': vlan_pri = (uint32_t)atoi(optarg); break;
		case 'G':
			if (!rx_parse_mac(optarg, dmac)) {
				fprintf(stderr, "Invalid dmac address:%s\n", optarg);
				usage(prog);
			}
			have_dmac = true;
			break;
		case 'H':
			if (!rx_parse_mac(optarg, smac)) {
				fprintf(stderr, "Invalid smac address:%s\n", optarg);
				usage(prog);
			}
			have_smac = true;
			break;
		case 'x': extra = 1; break;
		case 'Q': o.quiet = true; break;
		case 'p': case 'w': case 'O':
		case 'M': case 'T': case 'y': case 'W': case 'U': case 'a': case 'I':
		case 'B': case 'R':
			break;    /* scheduling options: no effect */
		case 'F':
			/* opt_frags (xdpsock.c:1349): multi-buffer packets */
			o.frags = true;
			o.cfg_flags |= XDPGPU_CFG_FRAGS;
			break;
		case OPT_GPU: o.device = atoi(optarg); break;
		case OPT_POOL: pool_n = (uint32_t)strtoul(optarg, NULL, 0); break;
		case OPT_POOL_KIND:
			kind = pool_kind(optarg);
			if (kind < 0) {
				fprintf(stderr, "%s: unknown pool kind %s\n", prog, optarg);
				usage(prog);
			}
			break;
		case OPT_SEED: seed = strtoull(optarg, NULL, 0); break;
		case OPT_PCAP: pcap = optarg; break;
		case OPT_NO_VERIFY: o.cfg_flags &= ~XDPGPU_CFG_VERIFY_CSUM; break;
		case OPT_INITVAL: o.initval = (uint32_t)strtoul(optarg, NULL, 0); break;
		case OPT_JSON: o.json = true; break;
		case OPT_VERDICTS: o.verdict_out = optarg; break;
		case OPT_TX_PCAP: o.tx_pcap = optarg; break;
		case OPT_DRY_RUN: dry = 1; break;
		case OPT_VETH: veth = optarg; break;
		case OPT_INJECT: inject_n = strtoull(optarg, NULL, 0); break;
		case OPT_INJECT_PCAP: inject_pcap = optarg; break;
		case OPT_PLUMBING: o.plumbing = true; break;
		default:
			usage(prog);
		}
	}
	if (optind < argc)
		usage(prog);
	const bool live = !pool_n && !pcap;
	if (live && !iface_set) {
		fprintf(stderr, "%s: give -i IF (live AF_XDP), --pool N or --pcap FILE\n", prog);
		usage(prog);
	}
	if (!live && (veth || inject_n || inject_pcap || o.plumbing)) {
		fprintf(stderr, "%s: --veth / --inject / --plumbing are live-mode options (-i IF)\n",
			prog);
		usage(prog);
	}
	if (pool_n && pcap) {
		fprintf(stderr, "%s: --pool and --pcap are exclusive\n", prog);
		usage(prog);
	}
	if ((frame_size & (frame_size - 1)) && !unaligned) {
		/* xdpsock.c:1363-1368 */
		fprintf(stderr, "--frame-size=%d is not a power of two\n", (int)frame_size);
		usage(prog);
	}
	if (!o.batch) {
		fprintf(stderr, "%s: batch size must be positive\n", prog);
		usage(prog);
	}
	if (!extra)
		o.cfg_flags &= ~XDPGPU_CFG_STATS;
	if (live)
		return run_live(prog, ifname, (uint32_t)queue, &o, frame_size, skb || !live_native,
				zerocopy, no_wakeup, veth, inject_n, inject_pcap, kind, pkt_size,
				seed);

	struct rx_source src;
	int rc;
	if (pcap) {
		rc = rx_source_pcap(&src, pcap, frame_size, 0, unaligned, o.frags, 0);
		if (rc) {
			fprintf(stderr, "%s: %s: %s\n", prog, pcap, strerror(-rc));
			return 1;
		}
	} else {
		struct xdpgpu_pool_spec spec;
		xdpgpu_pool_spec_default(&spec, (uint32_t)kind, pkt_size, seed);
		if (kind == XDPGPU_POOL_XDPSOCK || kind == XDPGPU_POOL_AFXDP_USER) {
			spec.vlan = (uint32_t)vlan;
			spec.vlan_id = (uint16_t)vlan_id;
			spec.vlan_pri = (uint16_t)vlan_pri;
			if (have_pattern)
				spec.fill_pattern = pattern;
			if (have_dmac)
				memcpy(spec.dmac, dmac, 6);
			if (have_smac)
				memcpy(spec.smac, smac, 6);
		}
		rc = rx_source_pool(&src, &spec, pool_n);
		if (rc) {
			fprintf(stderr, "%s: pool: %s\n", prog, strerror(-rc));
			return 1;
		}
	}
	if (dry) {
		rx_source_describe(&src, pcap ? pcap : "pool");
		rx_source_free(&src);
		return 0;
	}

	/* print_benchmark, xdpsock.c:284-310 */
	char label[128];
	snprintf(label, sizeof(label), "%s:%d %s %s", ifname, queue,
		 o.mode == RX_MODE_L2FWD ? "l2fwd" : "rxdrop", skb ? "xdp-skb" : "xdp-drv");
	o.label = label;
	struct rx_totals t;
	rc = rx_run(&src, &o, &t);
	rx_source_free(&src);
	return rc ? 1 : 0;
}
