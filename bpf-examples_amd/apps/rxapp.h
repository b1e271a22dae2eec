/* SPDX-License-Identifier: GPL-2.0 */
/*
 * rxapp.h - shared host side of the drop-in front-ends xdpsock-gpu and
 * af_xdp_user-gpu: frame sources that fill a UMEM (synthetic pools, pcap
 * files), the batched RX loop over the C ABI (include/xdpgpu.h) and the
 * reference programs' statistics output.
 *
 * The RX ring of the reference (xsk_ring_cons__peek / __release,
 * AF_XDP-interaction/af_xdp_user.c:1079-1113, AF_XDP-example/xdpsock.c:
 * 1462-1506) is modelled by replaying the source's descriptor array: each
 * batch "peeks" the next -b descriptors, hands them to the GPU with
 * xdpgpu_submit on one of two slots and applies the verdicts of the batch
 * before it (double buffering).  Plain C.
 */
#ifndef RXAPP_H
#define RXAPP_H

#include <stdbool.h>
#include <stdint.h>

#include "xdpgpu.h"

/* A UMEM and the descriptors of the frames in it. */
struct rx_source {
	uint8_t *umem;
	uint64_t umem_size;
	struct xdpgpu_desc *descs;
	uint32_t n;
	uint32_t chunk_size;     /* registration: 0 for a packed pool      */
	uint32_t headroom;
	uint32_t umem_flags;     /* XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG       */
	uint64_t skipped;        /* pcap records that did not fit a chunk */
	uint32_t packets;        /* packets: n, or fewer when split into
				  * fragments (XDPGPU_PKT_CONTD)           */
};

/* Synthetic pool (xdpgpu_pool_generate) of n frames.  0 or -errno. */
int rx_source_pool(struct rx_source *src, const struct xdpgpu_pool_spec *spec,
		   uint32_t n);

/* Frames of a classic pcap file (LINKTYPE_ETHERNET; either byte order,
 * micro- or nanosecond timestamps), at most max_frames (0: all).  Aligned
 * mode: one chunk of chunk_size bytes per frame, the frame at headroom
 * (xdpsock's UMEM geometry, xdpsock.c:2062); a record longer than a chunk
 * is skipped, or with frags split over consecutive chunks as a multi-buffer
 * packet (XDPGPU_PKT_CONTD on all but the last, xdpsock --frags).
 * Unaligned: packed at 64-byte rounded strides.  0 or -errno (-EPROTO: not
 * a usable pcap). */
int rx_source_pcap(struct rx_source *src, const char *path, uint32_t chunk_size,
		   uint32_t headroom, bool unaligned, bool frags, uint32_t max_frames);

void rx_source_free(struct rx_source *src);

/* Write the frames of a source as a classic pcap file (LINKTYPE_ETHERNET,
 * microseconds), e.g. the echo replies an af_xdp_user-gpu run sent. */
int rx_source_write_pcap(const struct rx_source *src, const uint8_t *select,
			 uint8_t want, const char *path);

/* What the application does with the frames the GPU delivers. */
enum rx_mode {
	RX_MODE_DROP = 0,   /* xdpsock rx_drop: count and recycle           */
	RX_MODE_L2FWD = 1,  /* xdpsock l2fwd: MAC swap, back out (TX count)   */
	RX_MODE_ECHO = 2,   /* af_xdp_user process_packet: ICMPv6 echo -> TX  */
};

enum rx_stats_fmt {
	RX_STATS_XDPSOCK = 0,   /* dump_stats, xdpsock.c:478-582        */
	RX_STATS_AFXDP = 1,     /* stats_print, af_xdp_user.c:1360-1397 */
};

struct rx_opts {
	int device;
	uint32_t cfg_flags;      /* XDPGPU_CFG_*                              */
	uint32_t tuple_fmt;
	uint32_t initval;
	uint32_t batch;          /* descriptors per GPU batch (-b)            */
	uint64_t count;          /* frames to receive, 0: by duration         */
	uint64_t duration_ns;    /* 0 with count 0: one pass over the source  */
	uint32_t interval_s;     /* stats period, 0: none                     */
	enum rx_mode mode;
	enum rx_stats_fmt stats_fmt;
	bool quiet;
	bool json;               /* final JSON summary line on stdout         */
	bool frags;              /* multi-buffer packets (XDPGPU_CFG_FRAGS):
				  * batches end on a packet's last fragment,
				  * packets and fragments counted apart    */
	bool plumbing;           /* live mode without the GPU: the reference's
				  * own bodies only (rx_drop recycles, l2fwd
				  * swaps MACs and sends everything), config 1
				  * as xdpsock runs it on a veth            */
	const char *verdict_out; /* per-frame verdicts of the first pass      */
	const char *tx_pcap;     /* frames sent on TX in the first pass       */
	const char *prog;        /* program name for messages                 */
	const char *label;       /* socket label of the stats ("if:q bench")  */
};

struct rx_totals {
	uint64_t rx_pkts, rx_bytes, tx_pkts, tx_bytes;
	uint64_t rx_frags, tx_frags;  /* descriptors (xdpsock ring_stats)   */
	uint32_t open_frags;          /* fragments of the packet in progress */
	uint64_t verdict[XDPGPU_NUM_VERDICTS];
	uint64_t batches;
	double seconds;
};

/* The RX loop: runs until opts.count frames, opts.duration_ns, one pass,
 * or SIGINT / SIGTERM, printing statistics.  0 or -errno (the ABI's). */
int rx_run(const struct rx_source *src, const struct rx_opts *opts,
	   struct rx_totals *out);

/* Live mode: an AF_XDP socket on ifname:queue
 * (apps/xsk.c), its RX ring feeding the GPU batches, the verdicts applied
 * to the fill and TX rings as the reference loops do (rx_drop / l2fwd,
 * xdpsock.c:1462-1506, 1718-1784; af_xdp_user.c:1042-1113).  With
 * veth_peer the program makes the veth pair ifname <-> veth_peer and
 * removes it at the end (testenv.sh:214-307); with inject, a thread sends
 * the source's frames into the peer (cycling it, inject_count frames,
 * paced so that the RX ring never overflows). */
struct rx_live {
	const char *ifname;
	uint32_t queue;
	uint32_t frame_size;     /* chunk size (XSK_UMEM__DEFAULT_FRAME_SIZE) */
	uint32_t nframes;        /* UMEM frames (NUM_FRAMES)                  */
	uint32_t ring_size;      /* each ring (XSK_RING_*__DEFAULT_NUM_DESCS)  */
	uint32_t bind_flags;     /* XDP_COPY / XDP_ZEROCOPY | NEED_WAKEUP      */
	uint32_t xdp_flags;      /* XDP_FLAGS_SKB_MODE / DRV_MODE              */
	const char *veth_peer;
	const struct rx_source *inject;
	uint64_t inject_count;
};

/* 0, -errno, or 1 when the host refuses AF_XDP / bpf / netlink (printed). */
int rx_run_live(const struct rx_live *lv, const struct rx_opts *opts,
		struct rx_totals *out);

/* Parse "aa:bb:cc:dd:ee:ff". */
bool rx_parse_mac(const char *s, uint8_t mac[6]);

/* Print the frames of a source (count, bytes, sizes) without a GPU. */
void rx_source_describe(const struct rx_source *src, const char *what);

#endif /* RXAPP_H */
