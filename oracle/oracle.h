/* SPDX-License-Identifier: GPL-2.0 */
/*
 * oracle.h - TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference algorithms on the hot path, used as the
 * parity checker by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  Nothing in the product (bpf-examples_amd/) links,
 * loads or calls this code.
 */
#ifndef XDP_ORACLE_H
#define XDP_ORACLE_H

#include <stdint.h>
#include "xdpgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* primitives (see xdp_oracle.c for the reference file:line of each) */
uint32_t oracle_do_csum(const uint8_t *buf, int len);
uint16_t oracle_ip_fast_csum(const uint8_t *iph, unsigned int ihl);
uint16_t oracle_csum_fold(uint32_t csum);
uint32_t oracle_csum_tcpudp_nofold(uint32_t saddr, uint32_t daddr, uint32_t len,
				   uint8_t proto, uint32_t sum);
uint16_t oracle_csum_tcpudp_magic(uint32_t saddr, uint32_t daddr, uint32_t len,
				  uint8_t proto, uint32_t sum);
uint16_t oracle_udp_csum(uint32_t saddr, uint32_t daddr, uint32_t len,
			 uint8_t proto, const uint8_t *l4);
uint16_t oracle_csum_ipv6_magic(const uint8_t *saddr, const uint8_t *daddr,
				uint32_t len, uint8_t proto, uint32_t csum);
uint16_t oracle_csum_replace2(uint16_t sum, uint16_t old, uint16_t new_);
uint32_t oracle_jhash(const void *key, uint32_t length, uint32_t initval);
uint32_t oracle_jhash2(const uint32_t *k, uint32_t length, uint32_t initval);
uint32_t oracle_jhash_3words(uint32_t a, uint32_t b, uint32_t c, uint32_t initval);

/* Whole per-frame pipeline over a batch: same inputs and outputs as
 * xdpgpu_process_dev.  umem is written only for ICMPv6 echo rewrites. */
int oracle_process(uint8_t *umem, uint64_t umem_size,
		   const struct xdpgpu_desc *descs, uint32_t n,
		   uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		   uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		   struct xdpgpu_stats *stats);

/* nat64 (nat64_oracle.c): same inputs and outputs as xdpgpu_nat64_dev;
 * umem is translated in place. */
/* XDP hints in front of each frame (xdpgpu_hints_dev semantics) */
void oracle_hints(const uint8_t *umem, uint64_t umem_size,
		  const struct xdpgpu_desc *descs, uint32_t n, uint32_t rx_time_id,
		  uint32_t mark_id, struct xdpgpu_hints *out);
int oracle_nat64(uint8_t *umem, uint64_t umem_size,
		 const struct xdpgpu_desc *descs, uint32_t n,
		 const struct xdpgpu_nat64_cfg *cfg,
		 const struct xdpgpu_nat64_map *map, uint32_t nmap,
		 uint8_t *action, struct xdpgpu_desc *out);
/* nat64 with dynamic state (alloc_new_state): the tables live in an opaque
 * object made from the configuration and the static entries; one call is
 * one batch at time `now`, frames in order. */
struct oracle_nat64_state;
struct oracle_nat64_state *oracle_nat64_state_new(const struct xdpgpu_nat64_cfg *cfg,
						  const struct xdpgpu_nat64_map *map,
						  uint32_t nmap, uint64_t timeout_ns,
						  uint64_t next_addr);
void oracle_nat64_state_free(struct oracle_nat64_state *st);
int oracle_nat64_dyn(uint8_t *umem, uint64_t umem_size,
		     const struct xdpgpu_desc *descs, uint32_t n,
		     const struct xdpgpu_nat64_cfg *cfg, struct oracle_nat64_state *st,
		     uint64_t now, uint8_t *action, struct xdpgpu_desc *out);
/* entries in insertion order, next_addr, reclaim queue oldest first (the
 * counts are returned whatever max / qmax allow to be copied) */
int oracle_nat64_state_read(const struct oracle_nat64_state *st,
			    struct xdpgpu_nat64_entry *out, uint32_t max, uint32_t *n,
			    uint64_t *next_addr, uint32_t *queue, uint32_t qmax, uint32_t *nq);
/* SYN proxy (synproxy_oracle.c): same inputs and outputs as
 * xdpgpu_synproxy_dev, frames rewritten in place */
int oracle_synproxy(uint8_t *umem, uint64_t umem_size, const struct xdpgpu_desc *descs,
		    uint32_t n, const struct xdpgpu_synproxy_cfg *cfg, uint8_t *verdict,
		    struct xdpgpu_desc *out, uint64_t *synacks);
int oracle_v4addr_to_v6(const uint8_t a4[4], uint8_t a6[16],
			const uint8_t pref[16], int plen);
int oracle_v6addr_to_v4(const uint8_t a6[16], int plen, uint8_t a4[4],
			uint8_t pref[16]);

/* CPU baseline: run oracle_process over descs[0..n) `reps` times on
 * `threads` threads, each on a contiguous slice.  Returns wall seconds. */
double oracle_bench(uint8_t *umem, uint64_t umem_size,
		    const struct xdpgpu_desc *descs, uint32_t n,
		    uint32_t cfg_flags, uint32_t initval, uint32_t tuple_fmt,
		    uint8_t *verdict, struct xdpgpu_result *res, void *tuples,
		    uint32_t threads, uint32_t reps);

#ifdef __cplusplus
}
#endif

#endif
