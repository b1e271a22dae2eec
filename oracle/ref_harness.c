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

/* Calibration probe (SURVEY.md §5 "survey probe"): per frame a minimal
 * Ethernet/VLAN/IPv4/UDP parse, ip_fast_csum over the IPv4 header,
 * udp_csum over the UDP datagram and jhash of 13 bytes (addresses, ports,
 * protocol), all by the reference headers' own routines; the same work as
 * cpu_leg_probe (oracle/cpu_leg.c).  Returns wall seconds of reps passes on
 * the calling thread; *acc receives a value of the results (kept live). */
#include <string.h>
#include <time.h>

struct ref_desc { uint64_t addr; uint32_t len; uint32_t options; };

double ref_probe(const uint8_t *umem, uint64_t umem_size, const struct ref_desc *d,
		 uint32_t n, uint32_t reps, uint64_t *acc)
{
	struct timespec t0, t1;
	uint64_t x = 0;
	uint32_t r, i;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (r = 0; r < reps; r++) {
		for (i = 0; i < n; i++) {
			const uint64_t eff = (d[i].addr & ((1ull << 48) - 1)) + (d[i].addr >> 48);
			const uint32_t len = d[i].len;
			const uint8_t *p = umem + eff;
			uint32_t l3 = 14, cl, sa, da;
			uint16_t et;
			uint8_t key[13];

			if (len < 42 || eff > umem_size - len)
				continue;
			memcpy(&et, p + 12, 2);
			if (et == htons(0x8100))
				l3 = 18;
			memcpy(&et, p + l3 - 2, 2);
			if (et != htons(0x0800) || p[l3] != 0x45 || p[l3 + 9] != 17)
				continue;
			x += (uint16_t)ip_fast_csum(p + l3, 5);
			cl = ntohs(*(const uint16_t *)(p + l3 + 24));
			if (l3 + 20 + cl > len)
				continue;
			memcpy(&sa, p + l3 + 12, 4);
			memcpy(&da, p + l3 + 16, 4);
			x += udp_csum(sa, da, cl, 17, (__u16 *)(p + l3 + 20));
			memcpy(key, p + l3 + 12, 8);
			memcpy(key + 8, p + l3 + 20, 4);
			key[12] = 17;
			x += jhash(key, 13, 0);
		}
	}
	clock_gettime(CLOCK_MONOTONIC, &t1);
	*acc = x;
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
