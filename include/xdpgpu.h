/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xdpgpu.h - C ABI of the MI355X (gfx950) AF_XDP receive-path transform.
 *
 * This is the drop-in boundary for the per-packet hot path of
 * xdp-project/bpf-examples: Ethernet/VLAN/IPv4/IPv6/L4 parse
 * (include/xdp/parsing_helpers.h), Internet one's-complement checksum
 * verify/recompute (AF_XDP-interaction/lib_checksum.h) and jhash flow-key
 * hashing (include/jhash.h), with the per-packet XDP verdict of
 * AF_XDP-interaction/af_xdp_kern.c.
 *
 * Plain C: pointers, sizes and fixed-layout structs only.  Every entry point
 * returns 0 or a negative errno (-EINVAL, -ENOMEM, -EIO for a HIP failure,
 * -E2BIG for a batch above cfg.max_batch, -ENODEV when no GPU is present).
 * Per-frame problems are never errors: they are verdicts (XDPGPU_ABORTED).
 *
 * Which reference interface each entry point replaces is noted on the entry
 * point (file:line into the reference tree).  See INTEGRATION.md for the
 * binding a maintainer adds on the reference side.
 */
#ifndef XDPGPU_H
#define XDPGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XDPGPU_ABI_VERSION 1

/* Per-frame verdicts: the numeric values of enum xdp_action
 * (headers/linux/bpf.h:6283-6289). */
enum xdpgpu_verdict {
	XDPGPU_ABORTED  = 0, /* parse error / truncated / bad descriptor    */
	XDPGPU_DROP     = 1, /* bad IPv4 header or L4 checksum              */
	XDPGPU_PASS     = 2, /* ARP or IPv6 NDP: left to the kernel stack   */
	XDPGPU_TX       = 3, /* ICMPv6 echo request rewritten into a reply  */
	XDPGPU_REDIRECT = 4, /* delivered to the application (XSK)          */
};
#define XDPGPU_NUM_VERDICTS 5

/* Descriptor: identical layout to struct xdp_desc
 * (headers/linux/if_xdp.h:109-113).  In unaligned-chunk mode the frame
 * offset lives in bits 63..48 (XSK_UNALIGNED_BUF_OFFSET_SHIFT,
 * headers/linux/if_xdp.h:104-106); the effective UMEM offset is always
 * (addr & ((1<<48)-1)) + (addr >> 48), which equals addr in aligned mode. */
struct xdpgpu_desc {
	uint64_t addr;
	uint32_t len;
	uint32_t options;
};

/* Result flags */
#define XDPGPU_F_L3_OK     0x01 /* IPv4 header checksum verifies (or IPv6)  */
#define XDPGPU_F_L4_OK     0x02 /* L4 checksum verifies (or is absent)      */
#define XDPGPU_F_VLAN      0x04 /* at least one 802.1Q/802.1ad tag consumed */
#define XDPGPU_F_IPV6      0x08
#define XDPGPU_F_FRAG      0x10 /* IPv4 MF/offset or IPv6 fragment header    */
#define XDPGPU_F_L4_ABSENT 0x20 /* IPv4/UDP with stored checksum 0          */
#define XDPGPU_F_IP        0x40 /* an IPv4 or IPv6 header was parsed        */
#define XDPGPU_F_L4        0x80 /* a TCP/UDP/ICMP/ICMPv6 header was parsed  */

/* Per-frame result record, 16 bytes.  Checksum words are u16 values as
 * stored in memory on little-endian (the two bytes are the wire bytes).
 * Frames with verdict ABORTED or PASS carry an all-zero record: they are
 * not delivered to the application (af_xdp_kern.c:178-183). */
struct xdpgpu_result {
	uint32_t hash;     /* jhash(network_tuple, 44, initval)  jhash.h:68  */
	uint16_t l3_csum;  /* recomputed IPv4 header checksum (check as 0)   */
	uint16_t l4_csum;  /* recomputed TCP/UDP/ICMP(v6) checksum            */
	uint8_t  flags;    /* XDPGPU_F_*                                      */
	uint8_t  l4_proto; /* IPv4 protocol / final IPv6 next header          */
	uint8_t  l3_off;   /* offset of the L3 header (14 + 4 * vlans)        */
	uint8_t  nvlan;    /* VLAN tags consumed (0..2)                       */
	uint16_t l4_off;   /* offset of the L4 header                         */
	uint16_t l4_len;   /* L4 bytes covered by the checksum                */
};

/* Tuple formats */
#define XDPGPU_TUPLE_NONE 0
#define XDPGPU_TUPLE_V4   1 /* struct xdpgpu_tuple4, 16 B               */
#define XDPGPU_TUPLE_NET  2 /* struct xdpgpu_network_tuple, 44 B        */

/* IPv4-compact 5-tuple.  Addresses and ports in wire order. */
struct xdpgpu_tuple4 {
	uint32_t saddr;
	uint32_t daddr;
	uint16_t sport;
	uint16_t dport;
	uint8_t  proto;
	uint8_t  ipv;      /* 2 (AF_INET), 10 (AF_INET6) or 0 (not IP)  */
	uint16_t vlan_id;  /* outer VID (TCI & 0x0fff), host order       */
};

/* Flow key hashed by jhash: the layout of pping's struct network_tuple
 * (pping/pping.h:120-139); IPv4 addresses mapped to ::ffff:a.b.c.d
 * (pping/pping_kern.c:212-217).  Ports in wire order, 0 for non-TCP/UDP. */
struct xdpgpu_network_tuple {
	uint8_t  saddr[16];
	uint16_t sport;
	uint16_t rsvd0;
	uint8_t  daddr[16];
	uint16_t dport;
	uint16_t rsvd1;
	uint16_t proto;
	uint8_t  ipv;
	uint8_t  rsvd2;
};

/* cfg.flags */
#define XDPGPU_CFG_VERIFY_CSUM 0x1 /* bad checksum -> XDP_DROP (xdp_synproxy_kern.c:610-623) */
#define XDPGPU_CFG_ICMP6_ECHO  0x2 /* process_packet echo responder (af_xdp_user.c:968-1040)  */
#define XDPGPU_CFG_STATS       0x4 /* keep per-verdict counters (xdpgpu_stats)                */
#define XDPGPU_CFG_TIMING      0x8 /* record HIP events around each RX kernel (diagnostic)     */
/* Multi-buffer packets (xdpsock --frags, xdpsock.c:67,1349; the XDP_USE_SG
 * socket): a packet is a run of descriptors whose options carry
 * XDPGPU_PKT_CONTD on all but the last (headers/linux/if_xdp.h:122).  The
 * packet is processed as one frame: the concatenation of its fragments,
 * with udp_csum's over-read byte the byte after the last fragment.  Every
 * descriptor of the packet gets the packet's verdict; the first carries its
 * result record and tuple, the others all-zero ones; an ICMPv6 echo reply
 * is written back into the fragments.  A packet the batch ends inside of,
 * or with a fragment outside the UMEM, is ABORTED.  The counters count
 * packets (and their bytes).  Without this flag options are ignored and
 * every descriptor is a frame, as process_packet does. */
#define XDPGPU_CFG_FRAGS       0x10
#define XDPGPU_PKT_CONTD       0x1 /* xdp_desc.options: the packet continues  */
/* Host path on a chunked UMEM (register_umem's chunk_size): a batch's
 * frame bytes reach the slot's device mirror through a gather kernel that
 * reads the registered UMEM through its GPU mapping (plain 16-byte loads,
 * read only, the frames' own bytes), instead of the copy engine's pitched
 * copies of one window per chunk.  About twice the rows per second for
 * small frames in 4 KiB chunks.  Ignored (the copies
 * are used) for a UMEM registered without chunk_size or one the GPU cannot
 * map. */
#define XDPGPU_CFG_UMEM_GATHER 0x20
/* Host path: the context's host threads copy each frame's bytes (the same
 * 16-byte pieces the gather reads, udp_csum's over-read byte included) out
 * of the registered UMEM into one page-locked staging buffer per slot, one
 * transfer brings the batch over, and a device kernel puts each piece at
 * its UMEM offset of the slot's mirror.  No kernel touches host memory; the
 * copy engine moves one contiguous buffer instead of one row per chunk.
 * For sparse frames (the reference's 4 KiB chunks, aligned or unaligned
 * mode); a packed UMEM's span copies need no host pass.
 * xdpgpu_host_threads sets the thread count.  Takes precedence over
 * XDPGPU_CFG_UMEM_GATHER. */
#define XDPGPU_CFG_HOST_COMPACT 0x40
#define XDPGPU_CFG_DEFAULT     (XDPGPU_CFG_VERIFY_CSUM | XDPGPU_CFG_STATS)

struct xdpgpu_cfg {
	int32_t  device;        /* HIP device ordinal                          */
	uint32_t flags;         /* XDPGPU_CFG_*                                */
	uint32_t max_batch;     /* max descriptors per host-path call (0: 2^20) */
	uint32_t jhash_initval; /* initval of jhash (CLI option, default 0)    */
	uint32_t tuple_fmt;     /* XDPGPU_TUPLE_*                              */
	uint32_t window;        /* header bytes staged per frame: 64, or 128
				 * (a frame longer than 64 bytes that starts
				 * a 128-byte line has its whole first line
				 * staged, so the payload pass does not read
				 * it again); 0: per batch, 128 when its frames
				 * average at least 128 bytes (the host path:
				 * their mean length; the device path: the
				 * UMEM size over the frame count), else 64;
				 * any other value is -EINVAL.  Outputs are
				 * the same whatever the window. */
	uint32_t tune;          /* kernel variant (diagnostic, 0 = default):
				 * bit 8 the exception pass keeps its payload
				 * sums, bit 9 every frame through the
				 * exception pass, bits 16-17 no-compute / no-store
				 * timing variants, bit 18 no IPv6 in the
				 * fast shape, bit 21 no shared tiles, bit 28
				 * no partner head; nat64: bits 12-13 no map
				 * probe / no frame stores, bit 14 no shared
				 * tiles */
	uint32_t queue_id;      /* the RX queue this context serves (the XDP
				 * program's ctx->rx_queue_index): its
				 * counters add into that queue's
				 * (xdpgpu_queue_stats)                      */
};

/* UMEM registration flags (headers/linux/if_xdp.h:31) */
#define XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG (1u << 0)

struct xdpgpu_stats {
	uint64_t frames;
	uint64_t bytes;
	uint64_t verdict[XDPGPU_NUM_VERDICTS];
	uint64_t l3_bad;
	uint64_t l4_bad;
	uint64_t l4_absent;
	uint64_t frag;
	uint64_t rsvd[5];
};

struct xdpgpu_ctx;

/* Create a context bound to one GPU and one HIP stream pair.  A context is
 * the GPU analogue of one xsk_socket_info (af_xdp_user.c:85-98): one per RX
 * thread/queue, not re-entrant. */
int xdpgpu_init(const struct xdpgpu_cfg *cfg, struct xdpgpu_ctx **out);
void xdpgpu_fini(struct xdpgpu_ctx *ctx);

/* Register the host UMEM (replaces xsk_umem__create's buffer argument,
 * af_xdp_user.c:433 / xdpsock.c:1013).  The memory stays owned by the caller;
 * it is pinned (hipHostRegister: for the copy engines, and with
 * XDPGPU_CFG_UMEM_GATHER for the gather kernel's reads) and each in-flight
 * slot keeps a device mirror of it.  chunk_size (aligned mode, a
 * power of two, 0: none) lets the host path copy only each chunk's window
 * of frame bytes (xdpgpu_host_stats).  -EBUSY while a slot is in flight. */
int xdpgpu_register_umem(struct xdpgpu_ctx *ctx, void *base, uint64_t size,
			 uint32_t chunk_size, uint32_t headroom, uint32_t flags);

/* Batch replacement of the per-descriptor loop
 *   for each desc: process_packet(xsk, addr, len)   (af_xdp_user.c:1092-1100)
 * and of the kernel-side verdict xdp_sock_prog() (af_xdp_kern.c:150-191).
 * Host buffers: descs[n] in, verdict[n] out (required), res[n] and
 * tuples[n] (format cfg.tuple_fmt) out, both nullable.  Synchronous.
 * The UMEM is only read, except that with XDPGPU_CFG_ICMP6_ECHO the TX
 * frames' first min(len, 64) bytes are rewritten in place (the reply of
 * process_packet, af_xdp_user.c:990-1037); no other UMEM byte is written.
 * Buffers from xdpgpu_host_alloc (pinned) are copied asynchronously;
 * pageable ones are staged by the HIP runtime. */
int xdpgpu_process(struct xdpgpu_ctx *ctx, const struct xdpgpu_desc *descs,
		   uint32_t n, uint8_t *verdict, struct xdpgpu_result *res,
		   void *tuples);

/* Asynchronous form of xdpgpu_process on one of two in-flight slots
 * (double buffering of the RX batches).  The descriptor array and the
 * output buffers must stay valid until xdpgpu_wait(ctx, slot) returns
 * (page-locked ones are read and written by the copies and, with
 * XDPGPU_CFG_UMEM_GATHER, the gather kernel after xdpgpu_submit has
 * returned), and the batch's frames must not be
 * handed back to the kernel (fill or TX ring) before it returns.  The two
 * slots are independent: their batches may name the same UMEM frames
 * (each slot reads its own device mirror), and each writes back only its
 * own TX frames. */
int xdpgpu_submit(struct xdpgpu_ctx *ctx, uint32_t slot,
		  const struct xdpgpu_desc *descs, uint32_t n, uint8_t *verdict,
		  struct xdpgpu_result *res, void *tuples);
int xdpgpu_wait(struct xdpgpu_ctx *ctx, uint32_t slot);

/* Page-locked host memory for descriptor and output arrays (the RX loop's
 * per-batch buffers): xdpgpu_submit copies them without staging.  NULL on
 * failure. */
void *xdpgpu_host_alloc(uint64_t size);
void xdpgpu_host_free(void *p);

/* What the host path moved over PCIe since the context was made (a
 * diagnostic beside xdpsock's rx/tx counts, xdpsock.c:dump_stats): UMEM
 * bytes copied host to device, in how many copies, descriptor bytes in and
 * output bytes (verdict, record, tuple) back.  With a chunk size given to
 * xdpgpu_register_umem (aligned mode), a batch moves one window of each
 * chunk it names, the same offsets in every chunk (rows of a pitched
 * copy); otherwise spans of nearby frames.  With XDPGPU_CFG_UMEM_GATHER the
 * batches a gather kernel moved count in umem_gathers (their bytes, the
 * 16-byte pieces read, in umem_h2d_bytes, counted on the device: a batch
 * still in flight may be missing; umem_copies counts one a batch). */
struct xdpgpu_host_stats {
	uint64_t batches;
	uint64_t frames;
	uint64_t umem_h2d_bytes;
	uint64_t umem_copies;
	uint64_t desc_h2d_bytes;
	uint64_t out_d2h_bytes;
	uint64_t umem_gathers;
	uint64_t umem_compacted;   /* batches packed by the host threads
				    * (XDPGPU_CFG_HOST_COMPACT); their
				    * staging bytes count in umem_h2d_bytes,
				    * the 4-byte piece offsets in
				    * desc_h2d_bytes */
	uint64_t compact_ns;       /* host time those batches' packing took */
};
int xdpgpu_host_stats(struct xdpgpu_ctx *ctx, struct xdpgpu_host_stats *out);

/* XDPGPU_CFG_HOST_COMPACT: the number of host threads that pack a batch
 * (the calling thread is one of them); 0 picks the CPUs this process may
 * run on (its affinity set and cgroup CPU quota), at most 16.  Returns the
 * count now in effect, or a negative errno (-EBUSY while a slot is in
 * flight). */
int xdpgpu_host_threads(struct xdpgpu_ctx *ctx, uint32_t n);

/* Diagnostic: how many contexts hold the library's page-locking of the
 * host memory at p (several RX queues registering one UMEM share one
 * registration, released by the last of them; 0: the library pins none,
 * e.g. memory the caller page-locked itself). */
int xdpgpu_host_pin_refs(const void *p);

/* Device-resident form: every pointer is device memory (d_umem is written
 * only for ICMPv6 echo rewrites; a d_umem in host memory, pinned or not, is
 * refused with -EINVAL: no kernel of the library dereferences host
 * memory but XDPGPU_CFG_UMEM_GATHER's reads).  stream is a hipStream_t (NULL: the
 * context's stream).  Returns after the launch is enqueued, also with
 * XDPGPU_CFG_FRAGS (no host round trip).  d_umem must be readable up to
 * round_up(umem_size, 16) (the kernel loads 16-byte aligned chunks and
 * masks what lies past umem_size).  Launches of one context on different
 * streams are ordered by the context (they share its scratch); launches
 * on one stream run back to back (on the context's own stream with no
 * event between them: back-to-back launches on one caller stream each
 * record one, as the caller's stream may not outlive the next call).
 * Scratch per context slot: deferral
 * lists of 3 n + 5.2 M entries (24 bytes each; about 1.3 GB at n = 16 M),
 * grown on first use of a larger n. */
int xdpgpu_process_dev(struct xdpgpu_ctx *ctx, void *d_umem,
		       uint64_t umem_size, const struct xdpgpu_desc *d_descs,
		       uint32_t n, uint8_t *d_verdict,
		       struct xdpgpu_result *d_res, void *d_tuples,
		       void *stream);

/* Double-buffered form of xdpgpu_process_dev: the device-resident RX loop
 * with two batches in flight, as xdpgpu_submit is for host buffers (the
 * reference's loop takes batch after batch off one RX ring,
 * af_xdp_user.c:1079-1113 handle_receive_packets under rx_and_process).
 * The launch goes to slot `slot`'s own stream with that slot's scratch, so
 * a launch on the other slot can start on the CUs this one leaves while its
 * last tiles finish; launches on one slot run in order.  Returns after the
 * launch is enqueued (no host round trip); xdpgpu_wait(ctx, slot) or
 * xdpgpu_sync(ctx, NULL) waits.  Batches in flight on the two slots must
 * not write the same outputs or (with XDPGPU_CFG_ICMP6_ECHO) the same
 * frames.  -EBUSY while the slot has a host batch (xdpgpu_submit) in
 * flight.  Pointers and sizes as xdpgpu_process_dev. */
int xdpgpu_submit_dev(struct xdpgpu_ctx *ctx, uint32_t slot, void *d_umem,
		      uint64_t umem_size, const struct xdpgpu_desc *d_descs,
		      uint32_t n, uint8_t *d_verdict, struct xdpgpu_result *d_res,
		      void *d_tuples);

/* The hipStream_t of a slot (NULL for a bad slot): a caller orders its own
 * work (events, copies) with the slot's launches on it. */
void *xdpgpu_slot_stream(struct xdpgpu_ctx *ctx, uint32_t slot);

/* Counters accumulated over every launch of this context (synchronises). */
int xdpgpu_stats(struct xdpgpu_ctx *ctx, struct xdpgpu_stats *out);
int xdpgpu_stats_reset(struct xdpgpu_ctx *ctx);

/* Per-queue counters (AF_XDP-interaction/af_xdp_kern.c:19-24 xdp_stats_map,
 * indexed by rx_queue_index, :157-160): the sum of the counters of every
 * context of this process with cfg.queue_id == queue_id, live or finished
 * (a finished context's counters are kept).  frames is the map's packet
 * count; the other fields split it as xdpgpu_stats does. */
int xdpgpu_queue_stats(uint32_t queue_id, struct xdpgpu_stats *out);

/* Device primitives, one lane per item (device pointers, stream as above).
 * jhash over n keys of key_len bytes at key_stride   (include/jhash.h:68-105)
 * ip_fast_csum over n IPv4 headers at hdr_stride      (lib_checksum.h:103-106) */
int xdpgpu_jhash_dev(struct xdpgpu_ctx *ctx, const void *d_keys,
		     uint32_t key_len, uint32_t key_stride, uint32_t n,
		     uint32_t initval, uint32_t *d_out, void *stream);
/* jhash2 over n keys of nwords u32 at word_stride words
 *   (include/jhash.h:114-142: jhash2(k, length, initval));
 * jhash_1word / jhash_2words / jhash_3words for nwords = 1..3 over n items
 *   of nwords u32 at word_stride words (jhash.h:157-170; the flow-key
 *   hash of the IPv4 fast variant, jhash_3words(saddr, daddr, ports, iv)). */
int xdpgpu_jhash2_dev(struct xdpgpu_ctx *ctx, const uint32_t *d_words,
		      uint32_t nwords, uint32_t word_stride, uint32_t n,
		      uint32_t initval, uint32_t *d_out, void *stream);
int xdpgpu_jhash_nwords_dev(struct xdpgpu_ctx *ctx, const uint32_t *d_words,
			    uint32_t nwords, uint32_t word_stride, uint32_t n,
			    uint32_t initval, uint32_t *d_out, void *stream);
int xdpgpu_ip_fast_csum_dev(struct xdpgpu_ctx *ctx, const void *d_hdrs,
			    uint32_t hdr_stride, uint32_t n, uint16_t *d_out,
			    void *stream);

/* XDP hints (AF_XDP-interaction/af_xdp_kern.c:42-105): the metadata an XDP
 * program writes in front of a frame (bpf_xdp_adjust_meta), the struct's
 * BTF id in its last 4 bytes, read per frame as print_meta_info_via_btf
 * does (af_xdp_user.c:813-829, xsk_umem__btf_id lib_xsk_extend.c:16-27):
 * btf_id = the u32 before the frame; rx_time_btf_id selects struct
 * xdp_hints_rx_time {u64 rx_ktime; u32 xdp_rx_cpu; u32 btf_id} (packed, 16
 * bytes), mark_btf_id struct xdp_hints_mark {u32 mark; u32 btf_id}.  Ids
 * of 0 never match.  A frame with fewer bytes in front of it than its
 * struct, or outside the UMEM, reads as no hints (all zero). */
struct xdpgpu_hints {
	uint64_t rx_ktime;   /* xdp_hints_rx_time.rx_ktime, else 0        */
	uint32_t value;      /* xdp_rx_cpu (rx_time) or mark (mark), else 0 */
	uint32_t btf_id;     /* the id in front of the frame (0: none)     */
};

int xdpgpu_hints_dev(struct xdpgpu_ctx *ctx, const void *d_umem,
		     uint64_t umem_size, const struct xdpgpu_desc *d_descs,
		     uint32_t n, uint32_t rx_time_btf_id, uint32_t mark_btf_id,
		     struct xdpgpu_hints *d_out, void *stream);

/* Diagnostic: the RX kernel's memory traffic (descriptor, 64-byte header
 * window, 16 B result + 16 B tuple + verdict stores) with no parse, to
 * measure the achievable bandwidth ceiling of that access pattern.  Outputs
 * are meaningless. */
int xdpgpu_ceiling_dev(struct xdpgpu_ctx *ctx, const void *d_umem,
		       uint64_t umem_size, const struct xdpgpu_desc *d_descs,
		       uint32_t n, uint8_t *d_verdict, void *d_res,
		       void *d_tuples, void *stream);

/* Diagnostic (XDPGPU_CFG_TIMING): RX launches recorded since the last call
 * and their summed durations from HIP events on the launch stream.  An RX
 * launch is one kernel (xdp_rx_db_kernel) between two events: fast_ms and
 * total_ms are that pair's span; exception_ms and bulk_ms stay in the
 * struct for its layout and read 0.  Waits for the recorded work; resets
 * the record.  At most
 * XDPGPU_TIMING_MAX launches are kept between calls (later ones are not
 * recorded). */
#define XDPGPU_TIMING_MAX 1024
struct xdpgpu_ktimes {
	uint64_t launches;
	double fast_ms;
	double bulk_ms;
	double exception_ms;
	double total_ms;     /* the launches' event pairs, summed */
};
int xdpgpu_kernel_times(struct xdpgpu_ctx *ctx, struct xdpgpu_ktimes *out);

/* Wait for all work of the context (or of stream if non-NULL). */
int xdpgpu_sync(struct xdpgpu_ctx *ctx, void *stream);

int xdpgpu_device_count(void);
const char *xdpgpu_last_error(struct xdpgpu_ctx *ctx);
int xdpgpu_abi_version(void);

/* ------------------------------------------------------------------ */
/* nat64 (nat64-bpf/nat64_kern.c): the stateful NAT64 translator as a batch
 * transform over UMEM frames, BASELINE config 4.                      */

#define XDPGPU_NAT64_INGRESS 0 /* IPv6 -> IPv4: nat64_handle_v6 (nat64_kern.c:741-873) */
#define XDPGPU_NAT64_EGRESS  1 /* IPv4 -> IPv6: nat64_handle_v4 (nat64_kern.c:443-541) */

/* Per-frame result: the reference program's TC action (linux/pkt_cls.h),
 * plus one build-defined value. */
#define XDPGPU_TC_ACT_OK       0  /* not for the translator: untouched   */
#define XDPGPU_TC_ACT_SHOT     2  /* in the prefix but not translatable  */
#define XDPGPU_TC_ACT_REDIRECT 7  /* translated                          */
/* An allowed IPv6 source with no mapping in the state table, when dynamic
 * state is off (the frame is untouched; xdpgpu_nat64_dynamic turns on the
 * reference's allocation, alloc_new_state, nat64_kern.c:576-622). */
#define XDPGPU_NAT64_NO_STATE  0x80

/* struct nat64_config (nat64.h:6-12) plus the allowed_v6_src entry. */
struct xdpgpu_nat64_cfg {
	uint8_t  v6_prefix[16];    /* pref64; nat64.c default 64:ff9b::/96   */
	uint32_t v6_plen;          /* 32, 40, 48, 56, 64 or 96               */
	uint32_t v4_prefix;        /* host byte order (nat64.c:155-158)      */
	uint32_t v4_mask;          /* host byte order                        */
	uint32_t allow_plen;       /* allowed_v6_src LPM entry, 0: none      */
	uint8_t  allow_prefix[16];
	uint32_t direction;        /* XDPGPU_NAT64_*                         */
	uint32_t flags;            /* XDPGPU_NAT64_F_*, 0: the reference     */
	uint32_t headroom;         /* bytes in front of each frame that are
				    * its own (its chunk's headroom), which
				    * egress may grow into; 0: up to the
				    * UMEM's start (below)                   */
	uint32_t rsvd;
};

/* Opt-in extension (not in the reference, whose rewrite_icmp /
 * rewrite_icmpv6 leave the embedded header alone: the FIXMEs at
 * nat64_kern.c:438 and :736).  With this flag an ICMP error (ICMPv6 types
 * 1-4, ICMPv4 types 3, 11, 12) also has its embedded IP header translated,
 * RFC 7915 sections 4.3/5.3, with the same field rules the outer header
 * gets from nat64_handle_v6/_v4:
 *   ingress: the embedded IPv6 header (no extension header; its source
 *     inside the pref64, its destination the error's own source or, with
 *     static state, a v6_state_map entry) becomes a 20-byte IPv4 header;
 *     the frame starts 40 bytes later and the outer tot_len is the IPv6
 *     payload_len.
 *   egress: the embedded IPv4 header (any IHL, not a fragment; its source
 *     in v4_reversemap) becomes a 40-byte IPv6 header; the frame starts
 *     60 - IHL bytes earlier (40 for IHL 20: that much headroom) and
 *     the outer payload_len grows by 40 - IHL.
 * Egress writes in front of the frame (20 bytes; 60 - IHL with this flag).
 * With headroom 0 the only bound is the UMEM's start, as in the reference,
 * where the kernel guarantees the skb's headroom; in a packed UMEM that
 * overwrites the previous frame, so a caller with packed frames sets
 * headroom to what each frame owns, and a frame that would grow further
 * is TC_ACT_SHOT.
 * The ICMP checksum is updated incrementally for the swapped header (a
 * frame that arrived with a valid checksum leaves with one); the embedded
 * transport header and its checksum are left as they are (RFC 7915 allows
 * it).  An error whose embedded header cannot be translated is
 * TC_ACT_SHOT. */
#define XDPGPU_NAT64_F_ICMP_INNER 0x1

/* A static v6_state_map entry (struct v6_addr_state with static_conf,
 * nat64.h:15-19); v4_reversemap is its inverse. */
struct xdpgpu_nat64_map {
	uint8_t  v6[16];
	uint32_t v4;               /* host byte order, inside the v4 prefix  */
	uint32_t rsvd;
};

/* Configure the translator of a context and upload its static tables
 * (replaces nat64.c's map setup, nat64.c:396-420). */
int xdpgpu_nat64_setup(struct xdpgpu_ctx *ctx,
		       const struct xdpgpu_nat64_cfg *cfg,
		       const struct xdpgpu_nat64_map *map, uint32_t nmap);

/* Translate frames in place (device pointers, stream as above).  Replaces
 * the per-packet TC programs nat64_ingress / nat64_egress
 * (nat64_kern.c:875-902).  d_action[i] gets the action; d_out[i] the
 * translated frame: an IPv6->IPv4 frame starts 20 bytes later, an
 * IPv4->IPv6 frame 20 bytes earlier (it needs 20 bytes of headroom: cfg
 * headroom, or of UMEM when that is 0),
 * both as a plain UMEM offset.  Other frames keep their descriptor.  The
 * L2 header moves with the frame; only headers and the L4 checksum (ICMP:
 * type, code and rest-of-header) are written. */
int xdpgpu_nat64_dev(struct xdpgpu_ctx *ctx, void *d_umem, uint64_t umem_size,
		     const struct xdpgpu_desc *d_descs, uint32_t n,
		     uint8_t *d_action, struct xdpgpu_desc *d_out, void *stream);

/* Dynamic state: v6_state_map entries made on first sight of an allowed
 * source (alloc_new_state, nat64_kern.c:576-622): the next address of the
 * v4 pool (config.next_addr) while prefix + next_addr < (prefix | ~mask) - 1,
 * then reclaimed addresses (reclaim_v4_addr, :563-574: the reclaimed_addrs
 * queue, else one entry whose last_seen is older than now - timeout_ns and
 * not static, found in insertion order: which timed-out entry is taken is
 * implementation-defined, the kernel walks its hash order), within num_addr = (prefix | ~mask)
 * - prefix - 2 entries (nat64.c:396-401); a hit refreshes last_seen
 * (:821-823).  A failed allocation is TC_ACT_SHOT.  Frames are taken in
 * descriptor order, one batch at one instant: `now_ns`, or CLOCK_MONOTONIC
 * read once per xdpgpu_nat64_dev call when 0 (bpf_ktime_get_ns()).  With
 * dynamic state xdpgpu_nat64_dev returns after the batch has completed: the
 * frames that need a new or timed-out entry are committed in order on the
 * host and translated in a second pass. */
struct xdpgpu_nat64_dyn {
	uint64_t timeout_ns;       /* config.timeout_ns; nat64.c: 7200 s     */
	uint64_t next_addr;        /* config.next_addr; nat64.c: 1           */
	uint64_t now_ns;           /* the batch clock, 0: CLOCK_MONOTONIC    */
	uint64_t rsvd;
};

/* One v6_state_map entry (struct v6_addr_state, nat64.h:15-19, with its key). */
struct xdpgpu_nat64_entry {
	uint8_t  v6[16];
	uint32_t v4;               /* host byte order                        */
	uint32_t static_conf;
	uint64_t last_seen;
};

/* Turn dynamic state on (dyn) or off (NULL), after xdpgpu_nat64_setup: the
 * tables are rebuilt from the static entries, sized for num_addr entries,
 * and the reclaim queue is emptied. */
int xdpgpu_nat64_dynamic(struct xdpgpu_ctx *ctx, const struct xdpgpu_nat64_dyn *dyn);
/* Set the batch clock for the following calls (0: CLOCK_MONOTONIC). */
int xdpgpu_nat64_clock(struct xdpgpu_ctx *ctx, uint64_t now_ns);
/* Switch the direction of the following calls, keeping the tables: the
 * reference's nat64_ingress and nat64_egress programs share their maps
 * (nat64_kern.c:875-902); egress reads v4_reversemap only. */
int xdpgpu_nat64_direction(struct xdpgpu_ctx *ctx, uint32_t direction);
/* Read the state: up to max entries in insertion order (*n: how many there
 * are), the dynamic configuration with the current next_addr (dyn, may be
 * NULL) and up to qmax reclaim-queue addresses, oldest first (*nq: how
 * many there are; queue may be NULL). */
int xdpgpu_nat64_state(struct xdpgpu_ctx *ctx, struct xdpgpu_nat64_entry *out,
		       uint32_t max, uint32_t *n, struct xdpgpu_nat64_dyn *dyn,
		       uint32_t *queue, uint32_t qmax, uint32_t *nq);

/* ------------------------------------------------------------------ */
/* SYN proxy (xdp-synproxy/xdp_synproxy_kern.c, syncookie_xdp): a SYN to an
 * allowed port is answered in place with a SYN-ACK carrying a cookie (the
 * TCP checksum verify and recompute path), an ACK is
 * checked against the cookie, other traffic passes.                     */

/* The reference program's maps and clock.  Two things it takes from the
 * kernel are outside this transform (xdp-synproxy row):
 * the conntrack lookup (bpf_xdp_ct_lookup, :430-478; every frame is taken
 * as not established, the answer for a new connection) and the kernel's
 * SYN cookie (bpf_tcp_raw_gen/check_syncookie_*, :627-641, :717-734),
 * replaced by a build-defined keyed cookie: jhash2 over the source and
 * destination address words and the ports, with initval cookie_key +
 * now_ns / 60 s, plus the client's sequence number; an ACK passes when its
 * ack_seq - 1 matches that cookie for the current or the previous minute. */
struct xdpgpu_synproxy_cfg {
	uint64_t values;           /* values[0] (:76-81, :310-330): 0 = the
				    * defaults, else mss4 | wscale << 16 |
				    * ttl << 24 | mss6 << 32                */
	uint16_t ports[8];         /* allowed_ports (:83-88), 0 terminates   */
	uint64_t now_ns;           /* bpf_ktime_get_ns() for the batch       */
	uint32_t tailroom;         /* bytes each frame may grow past its end
				    * (the chunk's room, bpf_xdp_adjust_tail) */
	uint32_t cookie_key;
	uint32_t rsvd[4];
};

/* Process frames in place (device pointers): d_verdict[i] the XDP action
 * (XDP_TX: a SYN-ACK was written over the frame), d_out[i] the frame's
 * descriptor after the program's bpf_xdp_adjust_tail calls.  d_synacks
 * (device u64, may be NULL) is incremented per SYN-ACK (values[1]). */
int xdpgpu_synproxy_dev(struct xdpgpu_ctx *ctx, void *d_umem, uint64_t umem_size,
			const struct xdpgpu_desc *d_descs, uint32_t n,
			const struct xdpgpu_synproxy_cfg *cfg, uint8_t *d_verdict,
			struct xdpgpu_desc *d_out, uint64_t *d_synacks, void *stream);

/* ------------------------------------------------------------------ */
/* Synthetic UMEM pool generator (host).  Replaces the reference's packet
 * generators gen_eth_hdr_data (xdpsock.c:893-971) and gen_base_pkt
 * (af_xdp_user.c:688-700) for pool mode.                              */

enum xdpgpu_pool_kind {
	XDPGPU_POOL_UDP4       = 0, /* fixed-size IPv4/UDP from a flow table   */
	XDPGPU_POOL_IMIX       = 1, /* 64/570/1500 7:4:1, VLAN/QinQ, v4/v6, ... */
	XDPGPU_POOL_XDPSOCK    = 2, /* xdpsock txonly base frame, replicated    */
	XDPGPU_POOL_AFXDP_USER = 3, /* af_xdp_user base frame, replicated       */
	XDPGPU_POOL_NAT64      = 4, /* config 4: IPv6 toward 64:ff9b::/96       */
	XDPGPU_POOL_NAT64_V4   = 5, /* IPv4 toward the nat64 v4 pool (egress)   */
};

struct xdpgpu_pool_spec {
	uint32_t kind;         /* enum xdpgpu_pool_kind                       */
	uint32_t frame_size;   /* declared size S (L2 = S-4 + 4 B FCS slot)   */
	uint32_t stride;       /* bytes between frames (0: round_up(S, 64))   */
	uint32_t headroom;     /* bytes before each frame inside its stride   */
	uint64_t seed;
	uint32_t flow_bits;    /* log2 of the flow table (0: 20)              */
	uint32_t ppm_bad_l3;   /* per-million corrupt IPv4 header checksums    */
	uint32_t ppm_bad_l4;   /* per-million corrupt L4 checksums             */
	uint32_t ppm_malformed;/* per-million truncated / malformed frames     */
	uint32_t ppm_arp;
	uint32_t ppm_ndp;
	uint32_t ppm_echo6;    /* per-million ICMPv6 echo requests             */
	uint32_t vlan;         /* xdpsock -V: tag frames with vlan_id/pri      */
	uint16_t vlan_id;
	uint16_t vlan_pri;
	uint32_t fill_pattern; /* xdpsock -P / af_xdp_user opt_pkt_fill_pattern */
	uint8_t  dmac[6];
	uint8_t  smac[6];
	uint32_t saddr;        /* wire order; 0 = the generator's default     */
	uint32_t daddr;
	uint32_t threads;      /* 0: hardware concurrency                     */
	uint32_t ppm_v6;       /* IMIX: per-million IPv6 frames over the whole
				* pool (300000); the 64 B class
				* is IPv4-only, so the 570/1500 B classes carry
				* all of them.  0 in a default spec = 300000  */
	uint32_t rsvd[2];
};

/* Bytes of UMEM needed for n frames of this spec. */
uint64_t xdpgpu_pool_size(const struct xdpgpu_pool_spec *spec, uint32_t n);

/* Fill umem (>= xdpgpu_pool_size bytes) and descs[n]; expect[n] (nullable)
 * receives the verdict the generator intended for each frame under
 * XDPGPU_CFG_VERIFY_CSUM without ICMP6_ECHO. */
int xdpgpu_pool_generate(const struct xdpgpu_pool_spec *spec, uint8_t *umem,
			 uint64_t umem_size, struct xdpgpu_desc *descs,
			 uint32_t n, uint8_t *expect);

/* Set a spec to the defaults of BASELINE config kind (frame size S). */
/* The translator configuration and static map the NAT64 pools are drawn
 * from: pref64 64:ff9b::/96, v4 pool 10.99.0.0/16, allowed sources
 * 2001:db8:1:2::/64, source k (1..nmap) = 2001:db8:1:2::k mapped to
 * 10.99.0.0 + k.  map must hold nmap entries (at most 65533). */
int xdpgpu_nat64_pool_config(uint32_t direction, struct xdpgpu_nat64_cfg *cfg,
			     struct xdpgpu_nat64_map *map, uint32_t nmap);

void xdpgpu_pool_spec_default(struct xdpgpu_pool_spec *spec, uint32_t kind,
			      uint32_t frame_size, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif /* XDPGPU_H */
