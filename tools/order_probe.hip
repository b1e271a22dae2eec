// SPDX-License-Identifier: GPL-2.0
/*
 * order_probe.hip - does a counted `s_waitcnt vmcnt(K)` retire an LDS-DMA
 * (global_load_lds) that was issued before K younger vector-memory ops?
 * Diagnostic, not part of the product; it tests the assumption the round-2
 * RX tile loop rested on ("vmcnt counts loads, stores and LDS-DMA together
 * in issue order", xdp_rx.hip read_tile_db) and the one its replacement
 * rests on (LDS-DMA loads retire in issue order among themselves).
 *
 * Per trial, each wave:
 *   1. writes a poison value over its 1 KiB LDS buffer (ds_write, lgkmcnt(0));
 *   2. issues one global_load_lds_dwordx4 of 1 KiB from a cold HBM address
 *      (a new 1 MiB-strided address per trial, 4 GiB buffer: no L2/MALL hit),
 *      plain or non-temporal;
 *   3. issues K younger vector-memory ops of one kind;
 *   4. s_waitcnt vmcnt(K), then ds_read of its own 16 bytes: still poison =
 *      the DMA had not landed although the count said it had ("stale").
 *
 * Kinds of the K younger ops:
 *   0 control: K = 0 (vmcnt(0): must never be stale)
 *   1 buffer stores out of the resource's range (dropped by the hardware)
 *   2 buffer stores, plain, to a cold 1 MiB-strided address
 *   3 buffer stores, non-temporal
 *   4 buffer loads into VGPRs of a hot (L2-resident) line
 *   5 LDS-DMA of a hot line into a second buffer, plain
 *   6 LDS-DMA of a cold line into a second buffer, the other cache policy
 *   7 positive control: 5 dropped stores and vmcnt(6), a count that does
 *     not cover the DMA (stale reads must show up: the probe can see them)
 *
 * Build: hipcc --offload-arch=gfx950 -O3 -o tools/order_probe tools/order_probe.hip
 * Run:   tools/order_probe            (prints one line per case)
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(3))) uint4 lds_uint4_t;

constexpr int kWaves = 8;                  /* waves per block */
constexpr uint32_t kPoison = 0x5bd1e995u;
constexpr uint64_t kSrcBytes = 4ull << 30;
constexpr uint64_t kStride = 1ull << 20;

template <int KIND, int K, bool NT>
__global__ __launch_bounds__(64 * kWaves) void probe(const uint8_t *src, uint8_t *dst,
						      int iters, unsigned long long *stale)
{
	__shared__ uint4 buf[kWaves][64];
	__shared__ uint4 aux[kWaves][64];
	const int lane = threadIdx.x & 63;
	const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
	const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wid;
	const uint64_t nw = (uint64_t)gridDim.x * kWaves;
	const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 1 << 30, 0x00020000);
	uint32_t n_stale = 0, sink = 0;
	const uint32_t a_buf = (uint32_t)(uintptr_t)((lds_uint4_t *)&buf[wid][0] + lane);
	for (int it = 0; it < iters; it++) {
		/* 1. poison */
		asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
			     :: "v"(a_buf), "v"((v4u){kPoison, kPoison, kPoison, kPoison}) : "memory");
		/* 2. the DMA under test: cold */
		const uint64_t slot = (gw + (uint64_t)it * nw) % (kSrcBytes / kStride);
		const uint8_t *p = src + slot * kStride + ((gw * 4096) % (kStride - 1024)) + 16 * lane;
		__builtin_amdgcn_global_load_lds((const void *)p, (lds_void_t *)&buf[wid][0], 16, 0,
						 NT ? 2 : 0);
		asm volatile("" ::: "memory");
		/* 3. K younger ops (kind 4 in asm: its results are used only after
		 * the final vmcnt(0), so the compiler adds no wait for them) */
		uint32_t l0 = 0, l1 = 0, l2 = 0, l3 = 0, l4 = 0;
		if constexpr (KIND == 4) {
			const uint8_t *h = src + 4 * lane;
			asm volatile("global_load_dword %0, %5, off\n\t"
				     "global_load_dword %1, %5, off offset:1024\n\t"
				     "global_load_dword %2, %5, off offset:2048\n\t"
				     "global_load_dword %3, %5, off offset:3072\n\t"
				     "global_load_dword %4, %5, off offset:4064"
				     : "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3), "=&v"(l4)
				     : "v"(h) : "memory");
		}
#pragma unroll
		for (int k = 0; k < K; k++) {
			const uint32_t so = (uint32_t)(((gw * 131 + it * 7 + k) % 1000) * 1048576u) & 0x3fffffc0u;
			if constexpr (KIND == 1 || KIND == 7)
				__builtin_amdgcn_raw_buffer_store_b32(it + k, rs, 0x80000000u + 4096u * k, 0, 0);
			else if constexpr (KIND == 2)
				__builtin_amdgcn_raw_buffer_store_b32(it, rs, so + 4 * lane, 0, 0);
			else if constexpr (KIND == 3)
				__builtin_amdgcn_raw_buffer_store_b32(it, rs, so + 4 * lane, 0, 2);
			else if constexpr (KIND == 5)
				__builtin_amdgcn_global_load_lds((const void *)(src + 16 * lane),
								 (lds_void_t *)&aux[wid][0], 16, 0, 0);
			else if constexpr (KIND == 6)
				__builtin_amdgcn_global_load_lds(
					(const void *)(src + ((slot + 1 + k) % (kSrcBytes / kStride)) * kStride +
						       16 * lane),
					(lds_void_t *)&aux[wid][0], 16, 0, NT ? 0 : 2);
		}
		/* 4. the counted wait and the read */
		v4u v;
#define RD(N) asm volatile("s_waitcnt vmcnt(" #N ")\n\tds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" \
			   : "=v"(v) : "v"(a_buf) : "memory")
		if constexpr (KIND == 7) RD(6);
		else if constexpr (K == 0) RD(0);
		else if constexpr (K == 1) RD(1);
		else if constexpr (K == 2) RD(2);
		else if constexpr (K == 5) RD(5);
		else RD(10);
#undef RD
		n_stale += (v.x == kPoison) | (v.y == kPoison) | (v.z == kPoison) | (v.w == kPoison);
		asm volatile("s_waitcnt vmcnt(0)"
			     : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3), "+v"(l4) :: "memory");
		sink += l0 + l1 + l2 + l3 + l4;
	}
	if (n_stale)
		atomicAdd(stale, (unsigned long long)n_stale);
	if (sink == 0x12345678u)
		stale[1] = sink;
}

template <int KIND, int K, bool NT>
static void run(const char *name, const uint8_t *src, uint8_t *dst, unsigned long long *d_st,
		int blocks, int iters)
{
	CK(hipMemset(d_st, 0, 16));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	CK(hipEventRecord(e0));
	probe<KIND, K, NT><<<blocks, 64 * kWaves>>>(src, dst, iters, d_st);
	CK(hipEventRecord(e1));
	CK(hipEventSynchronize(e1));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, e0, e1));
	unsigned long long h[2];
	CK(hipMemcpy(h, d_st, 16, hipMemcpyDeviceToHost));
	const double trials = (double)blocks * kWaves * 64 * iters;
	printf("{\"case\": \"%s\", \"kind\": %d, \"K\": %d, \"dma_nt\": %d, \"lane_trials\": %.0f, "
	       "\"stale_lanes\": %llu, \"ms\": %.3f}\n",
	       name, KIND, K, (int)NT, trials, h[0], ms);
	fflush(stdout);
}

int main(int argc, char **argv)
{
	const int iters = argc > 1 ? atoi(argv[1]) : 64;
	const int blocks = 1024;
	uint8_t *src, *dst;
	unsigned long long *d_st;
	CK(hipMalloc(&src, kSrcBytes));
	CK(hipMalloc(&dst, 1ull << 30));
	CK(hipMalloc(&d_st, 16));
	CK(hipMemset(src, 0x11, kSrcBytes));
	CK(hipDeviceSynchronize());
#define R(KIND, K, NT, NAME) run<KIND, K, NT>(NAME, src, dst, d_st, blocks, iters)
	R(7, 5, false, "positive control: vmcnt(6) after 5 dropped stores, plain DMA");
	R(7, 5, true, "positive control: vmcnt(6) after 5 dropped stores, nt DMA");
	R(0, 0, false, "control vmcnt(0), plain DMA");
	R(0, 0, true, "control vmcnt(0), nt DMA");
	R(1, 5, false, "5 dropped stores, plain DMA");
	R(1, 5, true, "5 dropped stores, nt DMA");
	R(1, 10, true, "10 dropped stores, nt DMA");
	R(2, 5, false, "5 plain stores, plain DMA");
	R(2, 5, true, "5 plain stores, nt DMA");
	R(3, 5, false, "5 nt stores, plain DMA");
	R(3, 5, true, "5 nt stores, nt DMA");
	R(4, 5, false, "5 hot VGPR loads, plain DMA");
	R(4, 5, true, "5 hot VGPR loads, nt DMA");
	R(5, 5, false, "5 hot LDS-DMAs, plain DMA");
	R(5, 5, true, "5 hot LDS-DMAs, nt DMA");
	R(6, 1, false, "1 cold nt LDS-DMA, plain DMA");
	R(6, 1, true, "1 cold plain LDS-DMA, nt DMA");
	R(6, 5, false, "5 cold nt LDS-DMAs, plain DMA");
	R(6, 5, true, "5 cold plain LDS-DMAs, nt DMA");
#undef R
	CK(hipFree(src));
	CK(hipFree(dst));
	CK(hipFree(d_st));
	return 0;
}
