// SPDX-License-Identifier: GPL-2.0
/*
 * xsk.c - live AF_XDP socket, XDP redirect program and veth plumbing for
 * the front-ends (see xsk.h).  Plain C over the kernel UAPI: socket(2),
 * setsockopt(2) / mmap(2) of the rings, bpf(2), rtnetlink.
 */
#define _GNU_SOURCE
#include "xsk.h"

#include <errno.h>
#include <stddef.h>
#include <net/if.h>
#include <poll.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <arpa/inet.h>
#include <linux/bpf.h>
#include <linux/if_ether.h>
#include <linux/if_link.h>
#include <linux/if_packet.h>
#include <linux/netlink.h>
#include <linux/rtnetlink.h>
#include <linux/veth.h>

#ifndef SOL_XDP
#define SOL_XDP 283
#endif
#ifndef AF_XDP
#define AF_XDP 44
#endif

static int fail(struct xsk_sock *x, int rc, const char *fmt, ...)
{
	va_list ap;

	va_start(ap, fmt);
	vsnprintf(x->err, sizeof(x->err), fmt, ap);
	va_end(ap);
	return rc;
}

/* ------------------------------------------------------------------ */
/* rings: indices are published with release and read with acquire, as
 * the kernel side does (net/xdp/xsk_queue.h) */

static inline uint32_t ld_acq(const uint32_t *p)
{
	return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

static inline void st_rel(uint32_t *p, uint32_t v)
{
	__atomic_store_n(p, v, __ATOMIC_RELEASE);
}

/* free entries of a producer ring (fill, tx) */
static uint32_t prod_free(struct xsk_ring *r, uint32_t want)
{
	uint32_t fr = r->size - (r->cached_prod - r->cached_cons);

	if (fr < want) {
		r->cached_cons = ld_acq(r->consumer);
		fr = r->size - (r->cached_prod - r->cached_cons);
	}
	return fr;
}

/* available entries of a consumer ring (rx, completion) */
static uint32_t cons_avail(struct xsk_ring *r, uint32_t want)
{
	uint32_t av = r->cached_prod - r->cached_cons;

	if (av < want) {
		r->cached_prod = ld_acq(r->producer);
		av = r->cached_prod - r->cached_cons;
	}
	return av;
}

int xsk_fill(struct xsk_sock *x, const uint64_t *addrs, uint32_t n)
{
	struct xsk_ring *r = &x->fill;
	uint64_t *ring = (uint64_t *)r->desc;

	if (prod_free(r, n) < n)
		return -ENOSPC;
	for (uint32_t i = 0; i < n; i++)
		ring[(r->cached_prod + i) & r->mask] = addrs[i];
	r->cached_prod += n;
	st_rel(r->producer, r->cached_prod);
	return 0;
}

uint32_t xsk_rx(struct xsk_sock *x, struct xdp_desc *out, uint32_t max)
{
	struct xsk_ring *r = &x->rx;
	const struct xdp_desc *ring = (const struct xdp_desc *)r->desc;
	uint32_t n = cons_avail(r, max);

	if (n > max)
		n = max;
	for (uint32_t i = 0; i < n; i++)
		out[i] = ring[(r->cached_cons + i) & r->mask];
	r->cached_cons += n;
	if (n)
		st_rel(r->consumer, r->cached_cons);
	return n;
}

int xsk_tx(struct xsk_sock *x, const struct xdp_desc *d, uint32_t n)
{
	struct xsk_ring *r = &x->tx;
	struct xdp_desc *ring = (struct xdp_desc *)r->desc;

	if (n) {
		if (prod_free(r, n) < n)
			return -ENOSPC;
		for (uint32_t i = 0; i < n; i++)
			ring[(r->cached_prod + i) & r->mask] = d[i];
		r->cached_prod += n;
		st_rel(r->producer, r->cached_prod);
	}
	return xsk_kick_tx(x);
}

int xsk_kick_tx(struct xsk_sock *x)
{
	/* copy mode sends in the sendto (at most 32 frames a call); with
	 * need_wakeup only when asked (kick_tx, xdpsock.c:1356-1369) */
	if (!(x->bind_flags & XDP_USE_NEED_WAKEUP) ||
	    (ld_acq(x->tx.flags) & XDP_RING_NEED_WAKEUP)) {
		if (sendto(x->fd, NULL, 0, MSG_DONTWAIT, NULL, 0) < 0 &&
		    errno != ENOBUFS && errno != EAGAIN && errno != EBUSY &&
		    errno != ENETDOWN)
			return -errno;
	}
	return 0;
}

int64_t xsk_rx_drops(const struct xsk_sock *x)
{
	struct xdp_statistics st;
	socklen_t len = sizeof(st);

	memset(&st, 0, sizeof(st));
	if (getsockopt(x->fd, SOL_XDP, XDP_STATISTICS, &st, &len))
		return -errno;
	/* rx_ring_full is reported since Linux 5.9 (len says whether it is) */
	const uint64_t full = len >= offsetof(struct xdp_statistics, rx_ring_full) +
				     sizeof(st.rx_ring_full) ? st.rx_ring_full : 0;
	return (int64_t)(st.rx_dropped + full);
}

uint32_t xsk_complete(struct xsk_sock *x, uint64_t *out, uint32_t max)
{
	struct xsk_ring *r = &x->comp;
	const uint64_t *ring = (const uint64_t *)r->desc;
	uint32_t n = cons_avail(r, max);

	if (n > max)
		n = max;
	for (uint32_t i = 0; i < n; i++)
		out[i] = ring[(r->cached_cons + i) & r->mask];
	r->cached_cons += n;
	if (n)
		st_rel(r->consumer, r->cached_cons);
	return n;
}

void xsk_wakeup_rx(struct xsk_sock *x, int timeout_ms)
{
	if ((x->bind_flags & XDP_USE_NEED_WAKEUP) &&
	    !(ld_acq(x->fill.flags) & XDP_RING_NEED_WAKEUP) && timeout_ms == 0)
		return;
	struct pollfd p = { .fd = x->fd, .events = POLLIN };

	(void)poll(&p, 1, timeout_ms);
}

static int map_ring(struct xsk_sock *x, struct xsk_ring *r, const struct xdp_ring_offset *o,
		    uint32_t size, size_t esz, off_t pgoff)
{
	r->map_len = o->desc + (size_t)size * esz;
	r->map = mmap(NULL, r->map_len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE,
		      x->fd, pgoff);
	if (r->map == MAP_FAILED) {
		r->map = NULL;
		return -errno;
	}
	r->producer = (uint32_t *)((uint8_t *)r->map + o->producer);
	r->consumer = (uint32_t *)((uint8_t *)r->map + o->consumer);
	r->flags = (uint32_t *)((uint8_t *)r->map + o->flags);
	r->desc = (uint8_t *)r->map + o->desc;
	r->size = size;
	r->mask = size - 1;
	r->cached_prod = ld_acq(r->producer);
	r->cached_cons = ld_acq(r->consumer);
	return 0;
}

/* ------------------------------------------------------------------ */
/* bpf(2): the XSKMAP and the redirect program                          */

static long sys_bpf(int cmd, union bpf_attr *attr)
{
	return syscall(__NR_bpf, cmd, attr, sizeof(*attr));
}

/* xdp_sock_prog's redirect (af_xdp_kern.c:185-189):
 *   return bpf_redirect_map(&xsks_map, ctx->rx_queue_index, XDP_PASS);
 * the lower bits of the flags are the action when the queue has no socket
 * (kernel 5.3+), the same XDP_PASS as the reference's fall-through. */
static int load_prog(struct xsk_sock *x, int map_fd)
{
	struct bpf_insn insn[] = {
		/* r2 = ctx->rx_queue_index */
		{ .code = BPF_LDX | BPF_MEM | BPF_W, .dst_reg = BPF_REG_2, .src_reg = BPF_REG_1,
		  .off = offsetof(struct xdp_md, rx_queue_index) },
		/* r1 = &xsks_map */
		{ .code = BPF_LD | BPF_DW | BPF_IMM, .dst_reg = BPF_REG_1,
		  .src_reg = BPF_PSEUDO_MAP_FD, .imm = map_fd },
		{ 0 },
		/* r3 = XDP_PASS */
		{ .code = BPF_ALU64 | BPF_MOV | BPF_K, .dst_reg = BPF_REG_3, .imm = XDP_PASS },
		{ .code = BPF_JMP | BPF_CALL, .imm = BPF_FUNC_redirect_map },
		{ .code = BPF_JMP | BPF_EXIT },
	};
	static char log[4096];
	union bpf_attr a;

	memset(&a, 0, sizeof(a));
	a.prog_type = BPF_PROG_TYPE_XDP;
	a.insns = (uint64_t)(uintptr_t)insn;
	a.insn_cnt = sizeof(insn) / sizeof(insn[0]);
	a.license = (uint64_t)(uintptr_t)"GPL";
	a.expected_attach_type = BPF_XDP;
	a.log_buf = (uint64_t)(uintptr_t)log;
	a.log_size = sizeof(log);
	a.log_level = 1;
	strncpy(a.prog_name, "xdpgpu_redir", sizeof(a.prog_name) - 1);
	const long fd = sys_bpf(BPF_PROG_LOAD, &a);
	if (fd < 0)
		return fail(x, -errno, "BPF_PROG_LOAD: %s (%.80s)", strerror(errno), log);
	return (int)fd;
}

static int setup_prog(struct xsk_sock *x, uint32_t xdp_flags)
{
	union bpf_attr a;

	memset(&a, 0, sizeof(a));
	a.map_type = BPF_MAP_TYPE_XSKMAP;
	a.key_size = 4;
	a.value_size = 4;
	a.max_entries = 64;
	strncpy(a.map_name, "xsks_map", sizeof(a.map_name) - 1);
	long fd = sys_bpf(BPF_MAP_CREATE, &a);
	if (fd < 0)
		return fail(x, -errno, "BPF_MAP_CREATE(XSKMAP): %s", strerror(errno));
	x->map_fd = (int)fd;
	const int pfd = load_prog(x, x->map_fd);
	if (pfd < 0)
		return pfd;
	x->prog_fd = pfd;
	memset(&a, 0, sizeof(a));
	a.link_create.prog_fd = (uint32_t)x->prog_fd;
	a.link_create.target_ifindex = (uint32_t)x->ifindex;
	a.link_create.attach_type = BPF_XDP;
	a.link_create.flags = xdp_flags;
	fd = sys_bpf(BPF_LINK_CREATE, &a);
	if (fd < 0)
		return fail(x, -errno, "BPF_LINK_CREATE(XDP, ifindex %d): %s", x->ifindex,
			    strerror(errno));
	x->link_fd = (int)fd;
	return 0;
}

static int map_insert(struct xsk_sock *x)
{
	union bpf_attr a;
	uint32_t key = x->queue, val = (uint32_t)x->fd;

	memset(&a, 0, sizeof(a));
	a.map_fd = (uint32_t)x->map_fd;
	a.key = (uint64_t)(uintptr_t)&key;
	a.value = (uint64_t)(uintptr_t)&val;
	a.flags = BPF_ANY;
	if (sys_bpf(BPF_MAP_UPDATE_ELEM, &a) < 0)
		return fail(x, -errno, "xsks_map[%u] = socket: %s", x->queue, strerror(errno));
	return 0;
}

/* ------------------------------------------------------------------ */

int xsk_open(struct xsk_sock *x, const struct xsk_cfg *c)
{
	int rc;

	memset(x, 0, sizeof(*x));
	x->fd = x->map_fd = x->prog_fd = x->link_fd = -1;
	if (!c->ifname || !c->nframes || !c->frame_size || !c->ring_size ||
	    (c->ring_size & (c->ring_size - 1)))
		return fail(x, -EINVAL, "bad configuration");
	x->ifindex = (int)if_nametoindex(c->ifname);
	if (!x->ifindex)
		return fail(x, -ENODEV, "no interface %s", c->ifname);
	x->queue = c->queue;
	x->nframes = c->nframes;
	x->frame_size = c->frame_size;
	x->headroom = c->headroom;
	x->bind_flags = c->bind_flags;
	x->umem_size = (uint64_t)c->nframes * c->frame_size;
	x->umem = mmap(NULL, x->umem_size, PROT_READ | PROT_WRITE,
		       MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
	if (x->umem == MAP_FAILED) {
		x->umem = NULL;
		return fail(x, -errno, "UMEM mmap: %s", strerror(errno));
	}
	x->fd = socket(AF_XDP, SOCK_RAW | SOCK_CLOEXEC, 0);
	if (x->fd < 0)
		return fail(x, -errno, "socket(AF_XDP): %s", strerror(errno));

	struct xdp_umem_reg mr;
	memset(&mr, 0, sizeof(mr));
	mr.addr = (uint64_t)(uintptr_t)x->umem;
	mr.len = x->umem_size;
	mr.chunk_size = c->frame_size;
	mr.headroom = c->headroom;
	if (setsockopt(x->fd, SOL_XDP, XDP_UMEM_REG, &mr, sizeof(mr)))
		return fail(x, -errno, "XDP_UMEM_REG: %s", strerror(errno));
	uint32_t sz = c->ring_size;
	if (setsockopt(x->fd, SOL_XDP, XDP_UMEM_FILL_RING, &sz, sizeof(sz)) ||
	    setsockopt(x->fd, SOL_XDP, XDP_UMEM_COMPLETION_RING, &sz, sizeof(sz)) ||
	    setsockopt(x->fd, SOL_XDP, XDP_RX_RING, &sz, sizeof(sz)) ||
	    setsockopt(x->fd, SOL_XDP, XDP_TX_RING, &sz, sizeof(sz)))
		return fail(x, -errno, "ring sizes: %s", strerror(errno));
	struct xdp_mmap_offsets off;
	socklen_t ol = sizeof(off);
	if (getsockopt(x->fd, SOL_XDP, XDP_MMAP_OFFSETS, &off, &ol))
		return fail(x, -errno, "XDP_MMAP_OFFSETS: %s", strerror(errno));
	if ((rc = map_ring(x, &x->fill, &off.fr, sz, sizeof(uint64_t),
			   XDP_UMEM_PGOFF_FILL_RING)) ||
	    (rc = map_ring(x, &x->comp, &off.cr, sz, sizeof(uint64_t),
			   XDP_UMEM_PGOFF_COMPLETION_RING)) ||
	    (rc = map_ring(x, &x->rx, &off.rx, sz, sizeof(struct xdp_desc),
			   XDP_PGOFF_RX_RING)) ||
	    (rc = map_ring(x, &x->tx, &off.tx, sz, sizeof(struct xdp_desc),
			   XDP_PGOFF_TX_RING)))
		return fail(x, rc, "ring mmap: %s", strerror(-rc));

	if (c->attach_prog && (rc = setup_prog(x, c->xdp_flags)))
		return rc;

	struct sockaddr_xdp sa;
	memset(&sa, 0, sizeof(sa));
	sa.sxdp_family = AF_XDP;
	sa.sxdp_ifindex = (uint32_t)x->ifindex;
	sa.sxdp_queue_id = c->queue;
	sa.sxdp_flags = (uint16_t)c->bind_flags;
	if (bind(x->fd, (struct sockaddr *)&sa, sizeof(sa)))
		return fail(x, -errno, "bind(%s queue %u, flags %#x): %s", c->ifname, c->queue,
			    c->bind_flags, strerror(errno));
	if (c->attach_prog && (rc = map_insert(x)))
		return rc;
	return 0;
}

void xsk_close(struct xsk_sock *x)
{
	struct xsk_ring *rings[] = { &x->fill, &x->comp, &x->rx, &x->tx };

	for (int i = 0; i < 4; i++)
		if (rings[i]->map)
			munmap(rings[i]->map, rings[i]->map_len);
	if (x->link_fd >= 0)
		close(x->link_fd);          /* detaches the program */
	if (x->prog_fd >= 0)
		close(x->prog_fd);
	if (x->map_fd >= 0)
		close(x->map_fd);
	if (x->fd >= 0)
		close(x->fd);
	if (x->umem)
		munmap(x->umem, x->umem_size);
	x->fd = x->link_fd = x->prog_fd = x->map_fd = -1;
	x->umem = NULL;
}

/* ------------------------------------------------------------------ */
/* rtnetlink                                                            */

struct nlreq {
	struct nlmsghdr h;
	struct ifinfomsg i;
	char buf[512];
};

static struct rtattr *nla_put(struct nlmsghdr *h, int type, const void *data, int len)
{
	struct rtattr *a = (struct rtattr *)((char *)h + NLMSG_ALIGN(h->nlmsg_len));

	a->rta_type = (unsigned short)type;
	a->rta_len = (unsigned short)RTA_LENGTH(len);
	if (len)
		memcpy(RTA_DATA(a), data, (size_t)len);
	h->nlmsg_len = NLMSG_ALIGN(h->nlmsg_len) + RTA_ALIGN(a->rta_len);
	return a;
}

static void nla_end(struct nlmsghdr *h, struct rtattr *a)
{
	a->rta_len = (unsigned short)((char *)h + h->nlmsg_len - (char *)a);
}

static int nl_talk(struct nlmsghdr *h)
{
	int fd = socket(AF_NETLINK, SOCK_RAW | SOCK_CLOEXEC, NETLINK_ROUTE);
	char reply[4096];
	int rc = 0;

	if (fd < 0)
		return -errno;
	h->nlmsg_flags |= NLM_F_REQUEST | NLM_F_ACK;
	h->nlmsg_seq = 1;
	if (send(fd, h, h->nlmsg_len, 0) < 0) {
		rc = -errno;
	} else {
		const ssize_t n = recv(fd, reply, sizeof(reply), 0);
		const struct nlmsghdr *r = (const struct nlmsghdr *)reply;

		if (n < 0)
			rc = -errno;
		else if (r->nlmsg_type == NLMSG_ERROR)
			rc = ((const struct nlmsgerr *)NLMSG_DATA(r))->error;
	}
	close(fd);
	return rc;
}

static void no_ipv6(const char *ifname)
{
	char path[128];
	FILE *f;

	snprintf(path, sizeof(path), "/proc/sys/net/ipv6/conf/%s/disable_ipv6", ifname);
	f = fopen(path, "w");
	if (f) {
		fputs("1\n", f);
		fclose(f);
	}
}

int xsk_veth_create(const char *a, const char *b)
{
	struct nlreq q;
	int rc;

	memset(&q, 0, sizeof(q));
	q.h.nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
	q.h.nlmsg_type = RTM_NEWLINK;
	q.h.nlmsg_flags = NLM_F_CREATE | NLM_F_EXCL;
	q.i.ifi_family = AF_UNSPEC;
	nla_put(&q.h, IFLA_IFNAME, a, (int)strlen(a) + 1);
	struct rtattr *li = nla_put(&q.h, IFLA_LINKINFO, NULL, 0);
	nla_put(&q.h, IFLA_INFO_KIND, "veth", 5);
	struct rtattr *data = nla_put(&q.h, IFLA_INFO_DATA, NULL, 0);
	struct rtattr *peer = nla_put(&q.h, VETH_INFO_PEER, NULL, 0);
	/* the peer's ifinfomsg, then its attributes */
	struct ifinfomsg pi;
	memset(&pi, 0, sizeof(pi));
	memcpy((char *)&q + q.h.nlmsg_len, &pi, sizeof(pi));
	q.h.nlmsg_len += NLMSG_ALIGN(sizeof(pi));
	nla_put(&q.h, IFLA_IFNAME, b, (int)strlen(b) + 1);
	nla_end(&q.h, peer);
	nla_end(&q.h, data);
	nla_end(&q.h, li);
	rc = nl_talk(&q.h);
	if (rc)
		return rc;
	/* no IPv6 on the pair: a new link's router solicitations, MLD
	 * reports and DAD probes would otherwise arrive in the socket among
	 * the test's frames (best effort: the sysctl may be absent) */
	no_ipv6(a);
	no_ipv6(b);
	if ((rc = xsk_link_up(a)) || (rc = xsk_link_up(b)))
		return rc;
	return 0;
}

int xsk_link_up(const char *name)
{
	struct nlreq q;

	memset(&q, 0, sizeof(q));
	q.h.nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
	q.h.nlmsg_type = RTM_NEWLINK;
	q.i.ifi_family = AF_UNSPEC;
	q.i.ifi_index = (int)if_nametoindex(name);
	if (!q.i.ifi_index)
		return -ENODEV;
	q.i.ifi_flags = IFF_UP;
	q.i.ifi_change = IFF_UP;
	return nl_talk(&q.h);
}

int xsk_link_delete(const char *name)
{
	struct nlreq q;

	memset(&q, 0, sizeof(q));
	q.h.nlmsg_len = NLMSG_LENGTH(sizeof(struct ifinfomsg));
	q.h.nlmsg_type = RTM_DELLINK;
	q.i.ifi_family = AF_UNSPEC;
	q.i.ifi_index = (int)if_nametoindex(name);
	if (!q.i.ifi_index)
		return -ENODEV;
	return nl_talk(&q.h);
}

/* ------------------------------------------------------------------ */

int xsk_packet_socket(const char *ifname)
{
	const int ifindex = (int)if_nametoindex(ifname);
	int fd;

	if (!ifindex)
		return -ENODEV;
	fd = socket(AF_PACKET, SOCK_RAW | SOCK_CLOEXEC, 0);
	if (fd < 0)
		return -errno;
	/* protocol 0: a send-only socket (no copy of every frame the
	 * interface receives is queued to it) */
	struct sockaddr_ll ll;
	memset(&ll, 0, sizeof(ll));
	ll.sll_family = AF_PACKET;
	ll.sll_ifindex = ifindex;
	if (bind(fd, (struct sockaddr *)&ll, sizeof(ll))) {
		const int e = -errno;

		close(fd);
		return e;
	}
	return fd;
}

int xsk_inject_fd(int fd, const uint8_t *umem, const struct xdp_desc *d, uint32_t n)
{
	enum { kBatch = 64 };
	struct mmsghdr mm[kBatch];
	struct iovec iov[kBatch];
	uint32_t sent = 0;

	while (sent < n) {
		const uint32_t m = n - sent < kBatch ? n - sent : kBatch;
		for (uint32_t i = 0; i < m; i++) {
			const struct xdp_desc *x = &d[sent + i];
			const uint64_t eff = (x->addr & ((1ull << XSK_UNALIGNED_BUF_OFFSET_SHIFT) - 1)) +
					     (x->addr >> XSK_UNALIGNED_BUF_OFFSET_SHIFT);

			iov[i].iov_base = (void *)(umem + eff);
			iov[i].iov_len = x->len;
			memset(&mm[i], 0, sizeof(mm[i]));
			mm[i].msg_hdr.msg_iov = &iov[i];
			mm[i].msg_hdr.msg_iovlen = 1;
		}
		const int r = sendmmsg(fd, mm, m, 0);
		if (r > 0) {
			sent += (uint32_t)r;
			continue;
		}
		if (r < 0 && errno != ENOBUFS && errno != EAGAIN)
			return sent ? (int)sent : -errno;
		usleep(50);
	}
	return (int)sent;
}

int xsk_inject(const char *ifname, const uint8_t *umem, const struct xdp_desc *d,
	       uint32_t n)
{
	const int fd = xsk_packet_socket(ifname);

	if (fd < 0)
		return fd;
	const int r = xsk_inject_fd(fd, umem, d, n);
	close(fd);
	return r;
}
