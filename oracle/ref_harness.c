// SPDX-License-Identifier: GPL-2.0
/*
 * ref_harness.c - TEST INFRASTRUCTURE ONLY.
 *
 * Thin exported wrappers around the reference's OWN header-only code, which
 * is compiled where it lies under /root/reference (see oracle/Makefile; the
 * output goes to oracle/_ref/libref.so and never into git).  No reference
 * source is copied here: the headers are #included from the reference tree.
 *   AF_XDP-interaction/lib_checksum.h   (do_csum, ip_fast_csum, udp_csum, ...)
 *   include/jhash.h                     (jhash, jhash2, jhash_3words)
 * Used only to pin oracle/xdp_oracle.c and to build tests/golden/.
 */
#include <stdint.h>
#include <arpa/inet.h>
#include <linux/types.h>

#include "lib_checksum.h"
#include "jhash.h"

uint32_t ref_do_csum(const unsigned char *buf, int len) { return do_csum(buf, len); }
uint16_t ref_ip_fast_csum(const void *iph, unsigned int ihl) { return (uint16_t)ip_fast_csum(iph, ihl); }
uint16_t ref_csum_fold(uint32_t c) { return (uint16_t)csum_fold((__wsum)c); }
uint32_t ref_csum_tcpudp_nofold(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, uint32_t sum)
{ return (uint32_t)csum_tcpudp_nofold(s, d, len, proto, sum); }
uint16_t ref_csum_tcpudp_magic(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, uint32_t sum)
{ return (uint16_t)csum_tcpudp_magic(s, d, len, proto, sum); }
uint16_t ref_udp_csum(uint32_t s, uint32_t d, uint32_t len, uint8_t proto, void *l4)
{ return udp_csum(s, d, len, proto, (__u16 *)l4); }
void ref_memset32_htonl(void *dest, uint32_t val, uint32_t size) { memset32_htonl(dest, val, size); }
uint32_t ref_jhash(const void *key, uint32_t len, uint32_t initval) { return jhash(key, len, initval); }
uint32_t ref_jhash2(const uint32_t *k, uint32_t len, uint32_t initval) { return jhash2(k, len, initval); }
uint32_t ref_jhash_3words(uint32_t a, uint32_t b, uint32_t c, uint32_t iv) { return jhash_3words(a, b, c, iv); }
uint32_t ref_jhash_2words(uint32_t a, uint32_t b, uint32_t iv) { return jhash_2words(a, b, iv); }
uint32_t ref_jhash_1word(uint32_t a, uint32_t iv) { return jhash_1word(a, iv); }
