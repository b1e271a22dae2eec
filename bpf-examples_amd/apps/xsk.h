/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xsk.h - a live AF_XDP socket without libxdp/libbpf, for the drop-in
 * front-ends' live mode (xdpsock-gpu -i IF): the UMEM and its fill and
 * completion rings, the RX and TX rings (linux/if_xdp.h UAPI), the XDP
 * program that redirects a queue's frames to the socket (an XSKMAP and a
 * 5-instruction program loaded with bpf(2), attached by a BPF link), and
 * the netlink calls that make a veth pair for a self-contained run
 * (lib/testenv/testenv.sh:214-307 makes one with ip(8)).
 *
 * What it replaces in the reference: xsk_configure_socket / xsk_umem__create
 * (AF_XDP-example/xdpsock.c:985-1100, AF_XDP-interaction/af_xdp_user.c:
 * 360-470 through libxdp's xsk.c), the ring accessors of <xdp/xsk.h>
 * (xsk_ring_prod__reserve / submit, xsk_ring_cons__peek / release) and
 * xdp_program__attach of the default redirect program.
 */
#ifndef XSK_H
#define XSK_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include <linux/if_xdp.h>

/* One of the four rings (producer/consumer indices free-running u32). */
struct xsk_ring {
	uint32_t *producer;
	uint32_t *consumer;
	uint32_t *flags;
	void *desc;              /* u64 addresses (fill, completion) or
				  * struct xdp_desc (rx, tx)                 */
	uint32_t size, mask;
	uint32_t cached_prod, cached_cons;
	void *map;
	size_t map_len;
};

struct xsk_sock {
	int fd;
	int ifindex;
	uint32_t queue;
	uint8_t *umem;           /* nframes * frame_size, page aligned        */
	uint64_t umem_size;
	uint32_t frame_size, headroom, nframes;
	struct xsk_ring fill, comp, rx, tx;
	int map_fd, prog_fd, link_fd;
	uint32_t bind_flags;     /* XDP_COPY / XDP_ZEROCOPY | NEED_WAKEUP  */
	char err[160];
};

struct xsk_cfg {
	const char *ifname;
	uint32_t queue;
	uint32_t nframes;        /* UMEM frames (power of two)                */
	uint32_t frame_size;     /* 2048 or 4096 (XSK_UMEM__DEFAULT_FRAME_SIZE)*/
	uint32_t headroom;
	uint32_t ring_size;      /* each ring (power of two)                  */
	uint32_t bind_flags;     /* XDP_COPY, XDP_ZEROCOPY, XDP_USE_NEED_WAKEUP */
	uint32_t xdp_flags;      /* XDP_FLAGS_SKB_MODE / DRV_MODE (if_link.h) */
	bool attach_prog;        /* load and attach the redirect program     */
};

/* Open, map and bind; 0 or -errno (x->err says which step). */
int xsk_open(struct xsk_sock *x, const struct xsk_cfg *c);
void xsk_close(struct xsk_sock *x);

/* Fill ring: give n frame addresses to the kernel (all or none). */
int xsk_fill(struct xsk_sock *x, const uint64_t *addrs, uint32_t n);
/* RX ring: up to max received descriptors copied to out and released. */
uint32_t xsk_rx(struct xsk_sock *x, struct xdp_desc *out, uint32_t max);
/* TX ring: queue n descriptors (all or none) and kick the kernel. */
int xsk_tx(struct xsk_sock *x, const struct xdp_desc *d, uint32_t n);
/* Kick the kernel to send what the TX ring holds (copy mode sends at most
 * 32 frames a call). */
int xsk_kick_tx(struct xsk_sock *x);
/* Completion ring: up to max sent frame addresses. */
uint32_t xsk_complete(struct xsk_sock *x, uint64_t *out, uint32_t max);
/* Wake the kernel for RX (poll) when the fill ring asks for it. */
void xsk_wakeup_rx(struct xsk_sock *x, int timeout_ms);
/* Frames the kernel dropped on their way to the RX ring (XDP_STATISTICS:
 * no fill buffer, rx_dropped; RX ring full, rx_ring_full), or -errno. */
int64_t xsk_rx_drops(const struct xsk_sock *x);

/* Netlink: a veth pair a <-> b, both up.  0 or -errno. */
int xsk_veth_create(const char *a, const char *b);
int xsk_link_delete(const char *name);
int xsk_link_up(const char *name);

/* Send frames on an interface through an AF_PACKET socket.  Returns frames
 * sent or -errno. */
int xsk_inject(const char *ifname, const uint8_t *umem,
	       const struct xdp_desc *d, uint32_t n);
/* The same over a send-only AF_PACKET socket kept open (sendmmsg, 64
 * frames a call): xsk_packet_socket returns its fd or -errno. */
int xsk_packet_socket(const char *ifname);
int xsk_inject_fd(int fd, const uint8_t *umem, const struct xdp_desc *d, uint32_t n);

#endif /* XSK_H */
