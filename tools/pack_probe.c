// SPDX-License-Identifier: GPL-2.0
/*
 * pack_probe.c - diagnostic (not a test): the host side of
 * XDPGPU_CFG_HOST_COMPACT alone, on this machine's CPUs.  A UMEM of 1 M
 * 4 KiB chunks (af_xdp_user.c:56-57), one 64-byte frame at each chunk's
 * headroom 256; batches of 512 K consecutive descriptors; T threads copy
 * each frame's 16-byte pieces into a packed buffer as compact_batch does
 * (csrc/xdpgpu.cpp).  Prints M frames/s per (threads, prefetch distance,
 * page kind): the UMEM in 4 KiB pages, or madvise(MADV_HUGEPAGE).
 *
 *   gcc -O2 -o tools/pack_probe tools/pack_probe.c -lpthread
 *   tools/pack_probe [maxthreads]
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

struct desc {
	uint64_t addr;
	uint32_t len, options;
};

static uint8_t *umem, *dst;
static struct desc *d;
static uint32_t *poff;
static uint64_t base[65], usize;
static uint32_t n;
static int T, PF;

static double now(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec + t.tv_nsec * 1e-9;
}

static void *work(void *p)
{
	const long t = (long)p;
	const uint32_t i0 = (uint64_t)n * t / T, i1 = (uint64_t)n * (t + 1) / T;
	uint64_t o = base[t];
	for (uint32_t i = i0; i < i1; i++) {
		if (PF && i + PF < i1) {
			__builtin_prefetch(umem + d[i + PF].addr);
			__builtin_prefetch(umem + d[i + PF].addr + 64);
		}
		const uint64_t eff = d[i].addr, lo = eff & ~15ull;
		uint64_t hi = (eff + d[i].len + (d[i].len & 1) + 15) & ~15ull;
		if (hi > usize)
			hi = usize;
		memcpy(dst + o, umem + lo, hi - lo);
		poff[i] = (uint32_t)(o >> 4);
		o += (hi - lo + 15) & ~15ull;
	}
	return NULL;
}

static double run(int threads, int pf, int reps)
{
	pthread_t th[64];
	double best = 0;
	T = threads;
	PF = pf;
	for (int rep = 0; rep < reps; rep++) {
		const uint64_t c0 = (uint64_t)(rep & 1) * n;
		for (uint32_t i = 0; i < n; i++) {
			d[i].addr = (c0 + i) * 4096 + 256;
			d[i].len = 64;
		}
		for (int t = 0; t <= T; t++)
			base[t] = (uint64_t)t * (n / T + 1) * 80;
		const double t0 = now();
		for (long t = 1; t < T; t++)
			pthread_create(&th[t], NULL, work, (void *)t);
		work(0);
		for (int t = 1; t < T; t++)
			pthread_join(th[t], NULL);
		const double r = n / (now() - t0) / 1e6;
		if (rep && r > best)
			best = r;
	}
	return best;
}

int main(int argc, char **argv)
{
	const int maxt = argc > 1 ? atoi(argv[1]) : 16;
	const uint64_t nc = 1ull << 20;
	usize = nc * 4096;
	n = 1u << 19;
	d = malloc(n * sizeof(*d));
	dst = malloc((uint64_t)n * 96);
	poff = malloc(n * 4);
	memset(dst, 0, (uint64_t)n * 96);
	for (int huge = 0; huge < 2; huge++) {
		umem = mmap(NULL, usize, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
		if (umem == MAP_FAILED)
			return 1;
		if (huge)
			madvise(umem, usize, MADV_HUGEPAGE);
		for (uint64_t c = 0; c < nc; c++)
			memset(umem + c * 4096, (int)c, 4096);
		for (int t = 1; t <= maxt; t *= 2)
			for (int pf = 0; pf <= 16; pf += 8)
				printf("{\"threads\": %d, \"prefetch\": %d, \"pages\": \"%s\", "
				       "\"mframes_s\": %.1f}\n", t, pf, huge ? "madvise-huge" : "4k",
				       run(t, pf, 5));
		munmap(umem, usize);
	}
	return 0;
}
