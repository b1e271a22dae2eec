// SPDX-License-Identifier: GPL-2.0
/*
 * hbm_probe.hip - achievable HBM bandwidth on this MI355X for the access
 * shapes of the RX kernel (diagnostic; not part of the product).
 *
 *   read      : dwordx4 streaming reads, grid-stride
 *   read_nt   : the same with non-temporal loads
 *   write     : dwordx4 streaming stores
 *   copy      : read + write of equal size
 *   rx_mix    : 80 B read + 33 B written per 64-B frame, as the RX kernel
 *               (16 B descriptor + 64 B frame; 16 B + 16 B + 1 B stores)
 *   rx_mix_nt : the same with non-temporal loads and stores
 *   syn       : the SYN proxy leg's in-place shape (argument "syn")
 *   imix      : config 3's two read patterns and the tile loop's head+outputs
 *               shape (argument "imix")
 *   rec       : the bulk pass's 16-byte record stores (argument "rec")
 *
 * Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ntl(const uint4 *p)
{
	v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p));
	return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nts(uint4 r, uint4 *p)
{
	v4u v = {r.x, r.y, r.z, r.w};
	__builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const uint4 *p, size_t n, uint32_t *out)
{
	uint32_t x = 0;
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		uint4 v = NT ? ntl(p + i) : p[i];
		x ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (x == 0x12345678u)
		out[0] = x;
}

__global__ __launch_bounds__(256) void k_write(uint4 *p, size_t n)
{
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
		p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ __launch_bounds__(256) void k_copy(const uint4 *s, uint4 *d, size_t n)
{
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
		d[i] = s[i];
}

/* per frame: desc (16 B) + frame (64 B) read, 16 + 16 + 1 B written */
template <bool NT, int UNROLL>
__global__ __launch_bounds__(256) void k_rxmix(const uint4 *desc, const uint4 *frames,
					       uint4 *res, uint4 *tup, uint8_t *verd,
					       size_t nframes)
{
	const size_t tiles = nframes / 64;
	const int lane = threadIdx.x & 63;
	const size_t wave = blockIdx.x * 4ull + (threadIdx.x >> 6);
	const size_t nw = (size_t)gridDim.x * 4;
	for (size_t t = wave * UNROLL; t < tiles; t += nw * UNROLL) {
		uint4 d[UNROLL], f[UNROLL][4];
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const size_t i = (t + u) * 64 + lane;
			d[u] = NT ? ntl(desc + i) : desc[i];
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const size_t c = (t + u) * 256 + k * 64 + lane;  /* transposed */
				f[u][k] = NT ? ntl(frames + c) : frames[c];
			}
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const size_t i = (t + u) * 64 + lane;
			uint32_t x = d[u].x ^ d[u].z;
#pragma unroll
			for (int k = 0; k < 4; k++)
				x ^= f[u][k].x ^ f[u][k].y ^ f[u][k].z ^ f[u][k].w;
			const uint4 r = make_uint4(x, x + 1, x + 2, x + 3);
			if (NT) {
				nts(r, res + i);
				nts(r, tup + i);
			} else {
				res[i] = r;
				tup[i] = r;
			}
			verd[i] = (uint8_t)x;
		}
	}
}

/* the same traffic, but each lane loads its own frame's four 16-B chunks
 * (stride 64 B across lanes) straight into registers */
template <bool NT, int UNROLL>
__global__ __launch_bounds__(256) void k_rxdirect(const uint4 *desc, const uint4 *frames,
						  uint4 *res, uint4 *tup, uint8_t *verd,
						  size_t nframes)
{
	const size_t tiles = nframes / 64;
	const int lane = threadIdx.x & 63;
	const size_t wave = blockIdx.x * 4ull + (threadIdx.x >> 6);
	const size_t nw = (size_t)gridDim.x * 4;
	for (size_t t = wave * UNROLL; t < tiles; t += nw * UNROLL) {
		uint4 d[UNROLL], f[UNROLL][4];
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const size_t i = (t + u) * 64 + lane;
			d[u] = NT ? ntl(desc + i) : desc[i];
			const uint4 *fp = frames + (d[u].x & 0) + i * 4;
#pragma unroll
			for (int k = 0; k < 4; k++)
				f[u][k] = NT ? ntl(fp + k) : fp[k];
		}
#pragma unroll
		for (int u = 0; u < UNROLL; u++) {
			const size_t i = (t + u) * 64 + lane;
			uint32_t x = d[u].x ^ d[u].z;
#pragma unroll
			for (int k = 0; k < 4; k++)
				x ^= f[u][k].x ^ f[u][k].y ^ f[u][k].z ^ f[u][k].w;
			const uint4 r = make_uint4(x, x + 1, x + 2, x + 3);
			if (NT) {
				nts(r, res + i);
				nts(r, tup + i);
			} else {
				res[i] = r;
				tup[i] = r;
			}
			verd[i] = (uint8_t)x;
		}
	}
}

/* LDS-DMA staging: the transposed 16-B chunks of a tile go straight into
 * LDS (global_load_lds_dwordx4 nt), slot(f, c) = 4f + (c ^ ((f >> 2) & 3))
 * so that each lane's four ds_read_b128 of its own frame are conflict-free;
 * the DMA of tile t+1 is in flight while tile t is processed. */
typedef __attribute__((address_space(3))) void lds_void;
__global__ __launch_bounds__(256) void k_rxlds(const uint4 *desc, const uint8_t *frames,
					       uint4 *res, uint4 *tup, uint8_t *verd,
					       size_t nframes)
{
	__shared__ uint4 buf_all[4 * 256];
	__shared__ uint64_t dtab_all[4 * 64];
	const int lane = threadIdx.x & 63;
	const int wid = threadIdx.x >> 6;
	uint4 *buf = buf_all + wid * 256;
	uint64_t *dtab = dtab_all + wid * 64;
	const size_t tiles = nframes / 64;
	const size_t nw = (size_t)gridDim.x * 4;
	size_t t = blockIdx.x * 4ull + wid;
	auto issue = [&](uint4 dv) {
		dtab[lane] = ((uint64_t)dv.y << 32) | dv.x;
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int k = 0; k < 4; k++) {
			const int f = 16 * k + (lane >> 2);
			const int c = (lane & 3) ^ ((f >> 2) & 3);
			const uint8_t *src = frames + dtab[f] + 16 * c;
			__builtin_amdgcn_global_load_lds((const void *)src,
				(lds_void *)(buf + 64 * k), 16, 0, 2);
		}
	};
	if (t >= tiles)
		return;
	uint4 dcur = desc[t * 64 + lane];
	issue(dcur);
	auto ld = [&](size_t tt) { return desc[(tt < tiles ? tt : tiles - 1) * 64 + lane]; };
	uint4 dnext = ld(t + nw);
	for (; t < tiles; t += nw) {
		const size_t i = t * 64 + lane;
		uint4 f[4];
#pragma unroll
		for (int c = 0; c < 4; c++)
			f[c] = buf[4 * lane + (c ^ ((lane >> 2) & 3))];
		__builtin_amdgcn_s_waitcnt(0xc07f);   /* lgkmcnt(0) */
		__builtin_amdgcn_wave_barrier();
		const uint4 dv = dcur;
		if (t + nw < tiles) {
			dcur = dnext;
			issue(dcur);
			dnext = ld(t + 2 * nw);
		}
		uint32_t x = dv.x ^ dv.z;
#pragma unroll
		for (int k = 0; k < 4; k++)
			x ^= f[k].x ^ f[k].y ^ f[k].z ^ f[k].w;
		const uint4 r = make_uint4(x, x + 1, x + 2, x + 3);
		nts(r, res + i);
		nts(r, tup + i);
		verd[i] = (uint8_t)x;
	}
}

/* Verdict store shapes (round 2): VS 0 = one byte per lane (64 B per
 * wave-instruction, a half line; the neighbouring tile's wave writes the
 * other half), 1 = no verdict store, 2 = two tiles' verdicts as one 128-B
 * line per wave (lane l stores the u16 of frames 2l, 2l+1 of the tile
 * pair), 3 = as 0 but tiles dealt to waves in contiguous runs (each 128-B
 * verdict line has one writer).  Plain loads, nt stores, one tile pair per
 * iteration. */
template <int VS>
__global__ __launch_bounds__(256) void k_rxpair(const uint4 *desc, const uint4 *frames,
						uint4 *res, uint4 *tup, uint8_t *verd,
						size_t nframes)
{
	const size_t pairs = nframes / 128;
	const int lane = threadIdx.x & 63;
	const size_t wave = blockIdx.x * 4ull + (threadIdx.x >> 6);
	const size_t nw = (size_t)gridDim.x * 4;
	size_t p0 = wave, pstep = nw, pend = pairs;
	if (VS == 3) {
		const size_t per = (pairs + nw - 1) / nw;
		p0 = wave * per;
		pstep = 1;
		pend = p0 + per < pairs ? p0 + per : pairs;
	}
	for (size_t p = p0; p < pend; p += pstep) {
		uint32_t xv[2];
#pragma unroll
		for (int u = 0; u < 2; u++) {
			const size_t t = 2 * p + u;
			const size_t i = t * 64 + lane;
			const uint4 d = desc[i];
			uint4 f[4];
#pragma unroll
			for (int k = 0; k < 4; k++)
				f[k] = frames[t * 256 + k * 64 + lane];
			uint32_t x = d.x ^ d.z;
#pragma unroll
			for (int k = 0; k < 4; k++)
				x ^= f[k].x ^ f[k].y ^ f[k].z ^ f[k].w;
			const uint4 r = make_uint4(x, x + 1, x + 2, x + 3);
			nts(r, res + i);
			nts(r, tup + i);
			xv[u] = x & 0xff;
			if (VS == 0 || VS == 3)
				verd[i] = (uint8_t)x;
		}
		if (VS == 2) {
			/* frames 2l, 2l+1 of the pair: tile (l >= 32), lanes 2l mod 64, +1 */
			const int s0 = (2 * lane) & 63, s1 = (2 * lane + 1) & 63;
			const uint32_t a0 = __shfl(xv[0], s0), a1 = __shfl(xv[0], s1);
			const uint32_t b0 = __shfl(xv[1], s0), b1 = __shfl(xv[1], s1);
			const uint32_t v = lane < 32 ? (a0 | (a1 << 8)) : (b0 | (b1 << 8));
			reinterpret_cast<uint16_t *>(verd + p * 128)[lane] = (uint16_t)v;
		}
	}
}

static float time_it(void (*fn)(void *), void *arg, int reps)
{
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	fn(arg);
	CK(hipDeviceSynchronize());
	CK(hipEventRecord(a, 0));
	for (int r = 0; r < reps; r++)
		fn(arg);
	CK(hipEventRecord(b, 0));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	return ms / reps;
}

struct Ctx {
	uint4 *a, *b, *desc, *res, *tup;
	uint8_t *verd;
	uint32_t *out;
	size_t n16, frames;
	int grid;
};

static Ctx C;
static void run_read(void *) { hipLaunchKernelGGL(k_read<false>, dim3(C.grid), dim3(256), 0, 0, C.a, C.n16, C.out); }
static void run_read_nt(void *) { hipLaunchKernelGGL(k_read<true>, dim3(C.grid), dim3(256), 0, 0, C.a, C.n16, C.out); }
static void run_write(void *) { hipLaunchKernelGGL(k_write, dim3(C.grid), dim3(256), 0, 0, C.b, C.n16); }
static void run_copy(void *) { hipLaunchKernelGGL(k_copy, dim3(C.grid), dim3(256), 0, 0, C.a, C.b, C.n16 / 2); }
static uint4 *descs_real;
static void run_lds(void *) { hipLaunchKernelGGL(k_rxlds, dim3(C.grid), dim3(256), 0, 0, descs_real, (const uint8_t *)C.a, C.res, C.tup, C.verd, C.frames); }
template <bool NT, int U>
static void run_direct(void *) { hipLaunchKernelGGL((k_rxdirect<NT, U>), dim3(C.grid), dim3(256), 0, 0, C.desc, C.a, C.res, C.tup, C.verd, C.frames); }
template <bool NT, int U>
static void run_mix(void *) { hipLaunchKernelGGL((k_rxmix<NT, U>), dim3(C.grid), dim3(256), 0, 0, C.desc, C.a, C.res, C.tup, C.verd, C.frames); }

template <int VS>
static void run_pair(void *) { hipLaunchKernelGGL((k_rxpair<VS>), dim3(C.grid), dim3(256), 0, 0, C.desc, C.a, C.res, C.tup, C.verd, C.frames); }

/* bulk payload probes: bytes [64, 1500) of frames at stride 1536 */
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_bulkq(const uint8_t *fr, size_t nframes,
					       uint32_t *out)
{
	const int lane = threadIdx.x & 63, q = lane >> 4, sub = lane & 15;
	const size_t nw = (size_t)gridDim.x * 4;
	uint32_t x = 0;
	for (size_t t = blockIdx.x * 4ull + (threadIdx.x >> 6); t < nframes / 64; t += nw) {
		for (int j = 0; j < 16; j++) {
			const uint8_t *f = fr + (t * 64 + 4 * j + q) * 1536ull + 64;
			for (uint32_t o = 0; o < 1436; o += 256 * U) {
				uint4 v[U];
#pragma unroll
				for (int u = 0; u < U; u++) {
					const uint32_t ou = o + 256 * u + 16 * sub;
					v[u] = make_uint4(0, 0, 0, 0);
					if (ou < 1436)
						v[u] = NT ? ntl((const uint4 *)(f + ou)) : *(const uint4 *)(f + ou);
				}
#pragma unroll
				for (int u = 0; u < U; u++)
					x += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
			}
		}
	}
	if (x == 0x12345678u)
		out[0] = x;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_bulkw(const uint8_t *fr, size_t nframes,
					       uint32_t *out)
{
	const int lane = threadIdx.x & 63;
	const size_t nw = (size_t)gridDim.x * 4;
	uint32_t x = 0;
	for (size_t t = blockIdx.x * 4ull + (threadIdx.x >> 6); t < nframes / U; t += nw) {
		uint4 v[2 * U];
#pragma unroll
		for (int u = 0; u < U; u++) {
			const uint8_t *f = fr + (t * U + u) * 1536ull + 64;
#pragma unroll
			for (int h = 0; h < 2; h++) {
				const uint32_t ou = 1024 * h + 16 * lane;
				v[2 * u + h] = make_uint4(0, 0, 0, 0);
				if (ou < 1436)
					v[2 * u + h] = NT ? ntl((const uint4 *)(f + ou)) : *(const uint4 *)(f + ou);
			}
		}
#pragma unroll
		for (int u = 0; u < 2 * U; u++)
			x += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	if (x == 0x12345678u)
		out[0] = x;
}

/* the same quarter-wave streaming over IMIX's middle class: bytes [64, 570)
 * of 570-byte frames at a 576-byte stride (every frame), or of every other
 * frame (SKIP 2: the frames between are not read, as 64-byte frames
 * between bulk frames are not) */
template <int U, int SKIP>
__global__ __launch_bounds__(256) void k_bulk570(const uint8_t *fr, size_t nframes,
						 uint32_t *out)
{
	const int lane = threadIdx.x & 63, q = lane >> 4, sub = lane & 15;
	const size_t nw = (size_t)gridDim.x * 4;
	const size_t nb = nframes / SKIP;
	uint32_t x = 0;
	for (size_t t = blockIdx.x * 4ull + (threadIdx.x >> 6); t < nb / 64; t += nw) {
		for (int j = 0; j < 16; j++) {
			const uint8_t *f = fr + (t * 64 + 4 * j + q) * SKIP * 576ull + 64;
			uint4 v[U];
#pragma unroll
			for (int u = 0; u < U; u++) {
				const uint32_t ou = 256 * u + 16 * sub;
				v[u] = make_uint4(0, 0, 0, 0);
				if (ou < 506)
					v[u] = ntl((const uint4 *)(f + ou));
			}
#pragma unroll
			for (int u = 0; u < U; u++)
				x += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
		}
	}
	if (x == 0x12345678u)
		out[0] = x;
}

static uint8_t *bulk_buf;
static size_t bulk_frames = 2ull << 20;
template <int U, bool NT>
static void run_bulkq(void *) { hipLaunchKernelGGL((k_bulkq<U, NT>), dim3(C.grid), dim3(256), 0, 0, bulk_buf, bulk_frames, C.out); }
template <int U, bool NT>
static void run_bulkw(void *) { hipLaunchKernelGGL((k_bulkw<U, NT>), dim3(C.grid), dim3(256), 0, 0, bulk_buf, bulk_frames, C.out); }
template <bool NT>
static void run_bulkflat(void *) { hipLaunchKernelGGL((k_read<NT>), dim3(C.grid), dim3(256), 0, 0, (const uint4 *)bulk_buf, bulk_frames * 1536 / 16, C.out); }

template <int SKIP>
static void run_bulk570(void *) { hipLaunchKernelGGL((k_bulk570<4, SKIP>), dim3(C.grid), dim3(256), 0, 0, bulk_buf, bulk_frames * 1536 / 576, C.out); }

static int bulk_main()
{
	CK(hipMalloc(&bulk_buf, bulk_frames * 1536));
	CK(hipMemset(bulk_buf, 3, bulk_frames * 1536));
	CK(hipMalloc(&C.out, 64));
	{
		const size_t n570 = bulk_frames * 1536 / 576;
		for (int grid : {1024, 2048, 4096}) {
			C.grid = grid;
			float t = time_it(run_bulk570<1>, 0, 20);
			printf("grid %5d b570 all   %7.1f GB/s (of 506 B/frame) %.4f ms\n", grid,
			       n570 * 506.0 / 1e9 / t * 1e3, t);
			t = time_it(run_bulk570<2>, 0, 20);
			printf("grid %5d b570 every2 %7.1f GB/s (of 506 B/frame) %.4f ms\n", grid,
			       n570 / 2 * 506.0 / 1e9 / t * 1e3, t);
		}
	}
	const double gb = bulk_frames * 1436.0 / 1e9;
	const int grids[] = {1024, 1536, 2048, 4096};
	for (int gi = 0; gi < 4; gi++) {
		C.grid = grids[gi];
		float t;
		t = time_it(run_bulkflat<false>, 0, 20);
		printf("grid %5d flat       %7.1f GB/s (of 1436 B/frame) %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkflat<true>, 0, 20);
		printf("grid %5d flat_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkq<2, false>, 0, 20);
		printf("grid %5d q_u2       %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkq<2, true>, 0, 20);
		printf("grid %5d q_u2_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkq<4, true>, 0, 20);
		printf("grid %5d q_u4_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkq<6, true>, 0, 20);
		printf("grid %5d q_u6_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkw<1, true>, 0, 20);
		printf("grid %5d w_u1_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkw<2, true>, 0, 20);
		printf("grid %5d w_u2_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
		t = time_it(run_bulkw<4, true>, 0, 20);
		printf("grid %5d w_u4_nt    %7.1f GB/s  %.4f ms\n", C.grid, gb / t * 1e3, t);
	}
	return 0;
}

/* "stride": the first CH chunks of 16 B of each 128-B frame, read (R),
 * written (W) or both in place, as the nat64 header rewrite touches them */
template <int CH, bool R, bool W, bool NT>
__global__ __launch_bounds__(256) void k_stride(uint4 *p, size_t nframes, uint32_t *out)
{
	uint32_t x = 0;
	const size_t n = nframes * CH;
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		uint4 *q = p + (i / CH) * 8 + (i % CH);
		uint4 v = make_uint4((uint32_t)i, 1, 2, 3);
		if (R)
			v = NT ? ntl(q) : *q;
		if (W) {
			v.x += 1;
			if (NT)
				nts(v, q);
			else
				*q = v;
		} else {
			x ^= v.x ^ v.y ^ v.z ^ v.w;
		}
	}
	if (x == 0x12345678u)
		out[0] = x;
}

/* nat64 egress's shape (config-4 egress pool: 128-byte frames at a
 * 192-byte stride behind 64 bytes of headroom): per frame, read its first
 * 64 bytes and write them back with the 20 bytes in front of the frame (a
 * dword and a 16-byte chunk of the headroom's last sector, FRONT 1), or
 * with that whole headroom sector (FRONT 2: a measurement of what a
 * partial sector costs; the translator may not write bytes outside the
 * frame's -20), or nothing in front (FRONT 0). */
template <int FRONT>
__global__ __launch_bounds__(256) void k_egress(uint8_t *p, size_t nframes, uint32_t *out)
{
	const size_t n = nframes * 4;
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		uint8_t *f = p + (i / 4) * 192 + 64;
		const uint32_t c = i % 4;
		uint4 *q = reinterpret_cast<uint4 *>(f) + c;
		uint4 v = *q;
		v.x += 1;
		*q = v;
		if (FRONT == 1 && c == 3) {
			*reinterpret_cast<uint32_t *>(f - 20) = v.y;
			*reinterpret_cast<uint4 *>(f - 16) = v;
		} else if (FRONT == 2) {
			reinterpret_cast<uint4 *>(f - 64)[c] = v;
		}
	}
}

/* the SYN proxy leg's shape (8 M frames at a 128-byte stride): per frame
 * its first 96 bytes read and 80 written back in place (a 74-byte SYN-ACK
 * as whole 16-byte chunks), and with DESC the 16-byte descriptor read, the
 * 16-byte output descriptor and the verdict byte written */
template <bool DESC>
__global__ __launch_bounds__(256) void k_syn(uint4 *p, const uint4 *desc, uint4 *odesc,
					     uint8_t *verdict, size_t nframes)
{
	const size_t n = nframes * 6;
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
		const size_t f = i / 6;
		const uint32_t c = i % 6;
		uint4 *q = p + f * 8 + c;
		uint4 v = *q;
		if (c < 5) {
			v.x += 1;
			*q = v;
		}
		if (DESC && c == 0) {
			uint4 d = desc[f];
			d.z = 74;
			odesc[f] = d;
			verdict[f] = (uint8_t)(v.y | 3);
		}
	}
}

static int syn_main()
{
	const size_t frames = 8ull << 20;
	uint4 *p, *d, *od;
	uint8_t *vd;
	CK(hipMalloc(&p, frames * 128));
	CK(hipMalloc(&d, frames * 16));
	CK(hipMalloc(&od, frames * 16));
	CK(hipMalloc(&vd, frames));
	CK(hipMemset(p, 1, frames * 128));
	CK(hipMemset(d, 2, frames * 16));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	for (int rep = 0; rep < 2; rep++)
		for (int desc = 0; desc < 2; desc++)
			for (int grid : {2048, 8192}) {
				auto k = desc ? k_syn<true> : k_syn<false>;
				for (int w = 0; w < 2; w++)
					hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, p, d, od, vd, frames);
				CK(hipEventRecord(e0, 0));
				for (int r = 0; r < 10; r++)
					hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, p, d, od, vd, frames);
				CK(hipEventRecord(e1, 0));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				printf("syn %s grid %5d  %.4f ms / 8 M frames\n",
				       desc ? "frame+desc+out" : "frame rw96/80", grid, ms / 10);
			}
	return 0;
}

static int stride_main()
{
	const size_t frames = 16ull << 20;
	uint4 *p;
	uint32_t *o;
	CK(hipMalloc(&p, frames * 128));
	CK(hipMalloc(&o, 64));
	CK(hipMemset(p, 1, frames * 128));
	hipEvent_t e0, e1;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	struct V { const char *name; void (*k)(uint4 *, size_t, uint32_t *); double bytes; };
	const V vs[] = {
		{"read64   ", k_stride<4, true, false, false>, 64.0},
		{"write64  ", k_stride<4, false, true, false>, 64.0},
		{"write64nt", k_stride<4, false, true, true>, 64.0},
		{"rw64     ", k_stride<4, true, true, false>, 128.0},
		{"rw64nt   ", k_stride<4, true, true, true>, 128.0},
		{"read128  ", k_stride<8, true, false, false>, 128.0},
		{"write128 ", k_stride<8, false, true, false>, 128.0},
		{"rw128    ", k_stride<8, true, true, false>, 256.0},
	};
	/* egress shape: 16 M frames at a 192-byte stride (3 GiB) */
	uint8_t *pe;
	CK(hipMalloc(&pe, frames * 192 + 64));
	CK(hipMemset(pe, 1, frames * 192 + 64));
	struct E { const char *name; void (*k)(uint8_t *, size_t, uint32_t *); };
	const E es[] = {{"egress rw64          ", k_egress<0>},
			{"egress rw64+front20  ", k_egress<1>},
			{"egress rw64+sector64 ", k_egress<2>}};
	for (int rep = 0; rep < 2; rep++)
		for (const E &v : es)
			for (int grid : {2048, 8192}) {
				for (int w = 0; w < 2; w++)
					hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, pe, frames, o);
				CK(hipEventRecord(e0, 0));
				for (int r = 0; r < 10; r++)
					hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, pe, frames, o);
				CK(hipEventRecord(e1, 0));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				printf("stride %s grid %5d  %.4f ms / 16 M frames\n", v.name, grid, ms / 10);
			}
	CK(hipFree(pe));
	for (int rep = 0; rep < 2; rep++)
		for (const V &v : vs)
			for (int grid : {2048, 8192}) {
				for (int w = 0; w < 2; w++)
					hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, p, frames, o);
				CK(hipEventRecord(e0, 0));
				for (int r = 0; r < 10; r++)
					hipLaunchKernelGGL(v.k, dim3(grid), dim3(256), 0, 0, p, frames, o);
				CK(hipEventRecord(e1, 0));
				CK(hipEventSynchronize(e1));
				float ms;
				CK(hipEventElapsedTime(&ms, e0, e1));
				ms /= 10;
				printf("stride %s grid %5d  %.4f ms  %7.1f GB/s of bytes touched\n", v.name,
				       grid, ms, frames * v.bytes / ms / 1e6);
			}
	return 0;
}

/*
 * IMIX's two read patterns (argument "imix"): a pool of 16 M frames of
 * 64/570/1500 bytes (7:4:1, seeded order) packed at a 64-byte-rounded
 * stride, as config 3's.  Set A is every frame's first 128 bytes (the
 * lines the RX tile loop's windows read), set B the lines after them (the
 * bulk pass's); each is read from a list of 64-byte line numbers, four
 * lanes a line, U lines a lane-quad in flight.  "split" runs A on even
 * workgroups and B on odd ones at once (the two passes overlapped).
 */
template <int U>
__global__ __launch_bounds__(256) void k_lines(const uint4 *pool, const uint32_t *l0, size_t n0,
					       const uint32_t *l1, size_t n1, int split, uint32_t *out)
{
	const uint32_t *l = l0;
	size_t n = n0, b = blockIdx.x, g = gridDim.x;
	if (split) {
		g >>= 1;
		if (b & 1) { l = l1; n = n1; }
		b >>= 1;
	}
	const size_t q = b * 64 + (threadIdx.x >> 2), nq = g * 64;
	const uint32_t sub = threadIdx.x & 3;
	uint32_t x = 0;
	size_t i = q;
	for (; i + (U - 1) * nq < n; i += U * nq) {
		uint4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = pool[(size_t)l[i + u * nq] * 4 + sub];
#pragma unroll
		for (int u = 0; u < U; u++)
			x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
	}
	for (; i < n; i += nq) {
		uint4 v = pool[(size_t)l[i] * 4 + sub];
		x ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (x == 0x12345678u)
		out[0] = x;
}

/* set A as the tile loop moves it: a lane quad per frame reads the frame's
 * first two lines (a 64-byte frame's second is its neighbour's first) and
 * writes the frame's outputs, 16 B result + 44 B tuple + 1 B verdict, into
 * packed per-frame arrays */
__global__ __launch_bounds__(256) void k_headw(const uint4 *pool, const uint32_t *first,
					       size_t nframes, uint4 *res, uint32_t *tup,
					       uint8_t *verd, int write)
{
	const size_t nq = (size_t)gridDim.x * 64;
	const uint32_t sub = threadIdx.x & 3;
	for (size_t f = blockIdx.x * 64ull + (threadIdx.x >> 2); f < nframes; f += 2 * nq) {
		const size_t f2 = f + nq < nframes ? f + nq : f;
		const uint4 *p = pool + (size_t)first[f] * 4, *p2 = pool + (size_t)first[f2] * 4;
		uint4 v0 = p[sub], v1 = p[4 + sub], v2 = p2[sub], v3 = p2[4 + sub];
		uint32_t x = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
		uint32_t y = v2.x ^ v2.y ^ v2.z ^ v2.w ^ v3.x ^ v3.y ^ v3.z ^ v3.w;
		if (!write) {
			if ((x ^ y) == 0x12345678u)
				verd[0] = 1;
			continue;
		}
		for (int k = 0; k < 2; k++) {
			const size_t g = k ? f2 : f;
			const uint32_t z = k ? y : x;
			if (sub == 0) {
				res[g] = make_uint4(z, z, z, z);
				verd[g] = (uint8_t)z;
			}
			for (uint32_t d = sub; d < 11; d += 4)
				tup[g * 11 + d] = z + d;
		}
	}
}

static struct {
	uint4 *pool, *res;
	uint32_t *a, *b, *all, *first, *tup;
	uint8_t *verd;
	size_t na, nb, nall, n16, frames;
} IM;
static int headw_write;
static void run_headw(void *) { hipLaunchKernelGGL(k_headw, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.first, IM.frames, IM.res, IM.tup, IM.verd, headw_write); }
template <int U>
static void run_la(void *) { hipLaunchKernelGGL(k_lines<U>, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.a, IM.na, IM.a, 0, 0, C.out); }
template <int U>
static void run_lb(void *) { hipLaunchKernelGGL(k_lines<U>, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.b, IM.nb, IM.b, 0, 0, C.out); }
template <int U>
static void run_lall(void *) { hipLaunchKernelGGL(k_lines<U>, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.all, IM.nall, IM.all, 0, 0, C.out); }
template <int U>
static void run_lsplit(void *) { hipLaunchKernelGGL(k_lines<U>, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.a, IM.na, IM.b, IM.nb, 1, C.out); }
static void run_pool(void *) { hipLaunchKernelGGL(k_read<false>, dim3(C.grid), dim3(256), 0, 0, IM.pool, IM.n16, C.out); }

static int imix_main()
{
	const size_t frames = 16ull << 20;
	uint64_t s = 0x5EED0003ull, lines = 0;
	std::vector<uint32_t> a, b, all, first;
	first.reserve(frames);
	a.reserve(frames * 3 / 2);
	b.reserve(frames * 9 / 2);
	for (size_t f = 0; f < frames; f++) {
		s ^= s << 13; s ^= s >> 7; s ^= s << 17;
		const uint32_t r = (uint32_t)(s >> 32) % 12;
		const uint32_t len = r < 7 ? 64 : r < 11 ? 570 : 1500;
		const uint32_t nl = (len + 63) / 64;
		first.push_back((uint32_t)lines);
		for (uint32_t k = 0; k < nl; k++) {
			(k < 2 ? a : b).push_back((uint32_t)(lines + k));
			all.push_back((uint32_t)(lines + k));
		}
		lines += nl;
	}
	IM.na = a.size(); IM.nb = b.size(); IM.nall = all.size();
	IM.n16 = lines * 4;
	CK(hipMalloc(&IM.pool, lines * 64));
	CK(hipMemset(IM.pool, 1, lines * 64));
	CK(hipMalloc(&IM.a, IM.na * 4));
	CK(hipMalloc(&IM.b, IM.nb * 4));
	CK(hipMalloc(&IM.all, IM.nall * 4));
	CK(hipMemcpy(IM.a, a.data(), IM.na * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(IM.b, b.data(), IM.nb * 4, hipMemcpyHostToDevice));
	CK(hipMemcpy(IM.all, all.data(), IM.nall * 4, hipMemcpyHostToDevice));
	IM.frames = frames;
	CK(hipMalloc(&IM.first, frames * 4));
	CK(hipMemcpy(IM.first, first.data(), frames * 4, hipMemcpyHostToDevice));
	CK(hipMalloc(&IM.res, frames * 16));
	CK(hipMalloc(&IM.tup, frames * 44));
	CK(hipMalloc(&IM.verd, frames));
	CK(hipMalloc(&C.out, 64));
	const double ga = IM.na * 64 / 1e9, gbb = IM.nb * 64 / 1e9, gp = lines * 64 / 1e9;
	printf("imix pool %.3f GB (%zu lines), A %.3f GB (%.2f lines/frame), B %.3f GB\n",
	       gp, (size_t)lines, ga, (double)IM.na / frames, gbb);
	for (int rep = 0; rep < 2; rep++)
		for (int grid : {2048, 8192}) {
			C.grid = grid;
			float t;
			t = time_it(run_pool, 0, 10);
			printf("grid %5d pool_seq  %.4f ms %7.1f GB/s\n", grid, t, gp / t * 1e3);
			t = time_it(run_lall<4>, 0, 10);
			printf("grid %5d list_all  %.4f ms %7.1f GB/s\n", grid, t, gp / t * 1e3);
			t = time_it(run_la<2>, 0, 10);
			printf("grid %5d A u2      %.4f ms %7.1f GB/s\n", grid, t, ga / t * 1e3);
			t = time_it(run_la<4>, 0, 10);
			printf("grid %5d A u4      %.4f ms %7.1f GB/s\n", grid, t, ga / t * 1e3);
			t = time_it(run_lb<4>, 0, 10);
			printf("grid %5d B u4      %.4f ms %7.1f GB/s\n", grid, t, gbb / t * 1e3);
			t = time_it(run_lsplit<4>, 0, 10);
			printf("grid %5d A|B split %.4f ms %7.1f GB/s\n", grid, t, gp / t * 1e3);
			const double gh = frames * 128 / 1e9, gw = frames * 61 / 1e9;
			headw_write = 0;
			t = time_it(run_headw, 0, 10);
			printf("grid %5d head      %.4f ms %7.1f GB/s (128 B a frame)\n", grid, t, gh / t * 1e3);
			headw_write = 1;
			t = time_it(run_headw, 0, 10);
			printf("grid %5d head+out  %.4f ms %7.1f GB/s (128 B read, 61 B written)\n", grid, t,
			       (gh + gw) / t * 1e3);
		}
	return 0;
}

/*
 * The bulk pass's record stores (argument "rec"): 16 M 16-byte records
 * written whole (the tile loop), then 16 bytes at a sorted 42 % of them
 * (one store a record, as the bulk pass writes its frames' records), or
 * the 64-byte aligned groups holding those records written whole: whether
 * a lone 16-byte store costs its ECC word's read-modify-write.
 */
__global__ __launch_bounds__(256) void k_rec_all(uint4 *rec, size_t n)
{
	for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
		rec[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ __launch_bounds__(256) void k_rec_some(uint4 *rec, const uint32_t *idx, size_t m,
						  int group)
{
	for (size_t k = blockIdx.x * 256ull + threadIdx.x; k < m; k += (size_t)gridDim.x * 256) {
		const uint32_t i = idx[k];
		if (group) {
			uint4 *g = rec + (i & ~3u);
			for (int j = 0; j < 4; j++)
				g[j] = make_uint4(i, (uint32_t)j, 5, 6);
		} else {
			rec[i] = make_uint4(i, 4, 5, 6);
		}
	}
}

static int rec_main()
{
	const size_t n = 16ull << 20;
	uint4 *rec;
	CK(hipMalloc(&rec, n * 16));
	std::vector<uint32_t> idx;
	uint64_t s = 0x5EED0003ull;
	for (size_t i = 0; i < n; i++) {
		s ^= s << 13; s ^= s >> 7; s ^= s << 17;
		if ((s >> 32) % 12 >= 7)   /* the 570 / 1500-byte frames of IMIX */
			idx.push_back((uint32_t)i);
	}
	uint32_t *d_idx;
	CK(hipMalloc(&d_idx, idx.size() * 4));
	CK(hipMemcpy(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
	hipEvent_t e0, e1, e2;
	CK(hipEventCreate(&e0));
	CK(hipEventCreate(&e1));
	CK(hipEventCreate(&e2));
	printf("records %zu, rewritten %zu (%.1f %%)\n", n, idx.size(), 100.0 * idx.size() / n);
	/* "cold": 2 GiB read between the two phases, so that the records'
	 * lines have left the L2 and the Infinity Cache, as in a launch */
	const size_t fl16 = (2ull << 30) / 16;
	uint4 *fl;
	CK(hipMalloc(&fl, fl16 * 16));
	CK(hipMemset(fl, 1, fl16 * 16));
	uint32_t *o;
	CK(hipMalloc(&o, 64));
	for (int rep = 0; rep < 4; rep++)
		for (int group = 0; group < 2; group++) {
			const bool cold = rep >= 2;
			CK(hipDeviceSynchronize());
			CK(hipEventRecord(e0, 0));
			hipLaunchKernelGGL(k_rec_all, dim3(8192), dim3(256), 0, 0, rec, n);
			if (cold)
				hipLaunchKernelGGL(k_read<false>, dim3(8192), dim3(256), 0, 0, fl, fl16, o);
			CK(hipEventRecord(e1, 0));
			hipLaunchKernelGGL(k_rec_some, dim3(8192), dim3(256), 0, 0, rec, d_idx,
					   idx.size(), group);
			CK(hipEventRecord(e2, 0));
			CK(hipEventSynchronize(e2));
			float a, b;
			CK(hipEventElapsedTime(&a, e0, e1));
			CK(hipEventElapsedTime(&b, e1, e2));
			printf("%s all-records%s %.4f ms, then %s %.4f ms (%zu B stored)\n",
			       cold ? "cold" : "warm", cold ? "+2GiB read" : "", a,
			       group ? "their 64-B groups whole" : "16 B a record  ", b,
			       idx.size() * (group ? 64 : 16));
		}
	return 0;
}

int main(int argc, char **argv)
{
	if (argc > 1 && !strcmp(argv[1], "rec"))
		return rec_main();
	if (argc > 1 && !strcmp(argv[1], "imix"))
		return imix_main();
	if (argc > 1 && !strcmp(argv[1], "bulk"))
		return bulk_main();
	if (argc > 1 && !strcmp(argv[1], "stride"))
		return stride_main();
	if (argc > 1 && !strcmp(argv[1], "syn"))
		return syn_main();
	const bool pair_only = argc > 1 && !strcmp(argv[1], "pair");
	const size_t frames = 16ull << 20;
	C.frames = frames;
	C.n16 = frames * 64 / 16;              /* 1 GiB */
	CK(hipMalloc(&C.a, C.n16 * 16));
	CK(hipMalloc(&C.b, C.n16 * 16));
	CK(hipMalloc(&C.desc, frames * 16));
	CK(hipMalloc(&C.res, frames * 16));
	CK(hipMalloc(&C.tup, frames * 16));
	CK(hipMalloc(&C.verd, frames));
	CK(hipMalloc(&C.out, 64));
	CK(hipMemset(C.a, 1, C.n16 * 16));
	CK(hipMemset(C.desc, 2, frames * 16));
	{
		/* real packed descriptors for the LDS-DMA kernel */
		uint4 *h = (uint4 *)malloc(frames * 16);
		for (size_t i = 0; i < frames; i++)
			h[i] = make_uint4((uint32_t)(i * 64), (uint32_t)((i * 64) >> 32), 64, 0);
		CK(hipMalloc(&descs_real, frames * 16));
		CK(hipMemcpy(descs_real, h, frames * 16, hipMemcpyHostToDevice));
		free(h);
	}
	const int grids[] = {1024, 2048, 4096, 8192};
	for (int gi = 0; gi < 4; gi++) {
		if (argc > 1 && !pair_only && gi < 2) continue;
		C.grid = grids[gi];
		const double gb = C.n16 * 16 / 1e9;
		float t;
		if (pair_only) {
			const double mb = frames * 113.0 / 1e9;
			for (int rep = 0; rep < 2; rep++) {
				t = time_it(run_mix<false, 1>, 0, 20);
				printf("grid %5d rx_mix        %7.1f GB/s  %.4f ms\n", C.grid, mb / t * 1e3, t);
				t = time_it(run_pair<0>, 0, 20);
				printf("grid %5d pair_byte     %7.1f GB/s  %.4f ms\n", C.grid, mb / t * 1e3, t);
				t = time_it(run_pair<1>, 0, 20);
				printf("grid %5d pair_noverd   %7.1f GB/s  %.4f ms (of the same 113 B)\n", C.grid, mb / t * 1e3, t);
				t = time_it(run_pair<2>, 0, 20);
				printf("grid %5d pair_line     %7.1f GB/s  %.4f ms\n", C.grid, mb / t * 1e3, t);
				t = time_it(run_pair<3>, 0, 20);
				printf("grid %5d pair_contig   %7.1f GB/s  %.4f ms\n", C.grid, mb / t * 1e3, t);
				t = time_it(run_lds, 0, 20);
				printf("grid %5d rx_lds        %7.1f GB/s  %.4f ms\n", C.grid, mb / t * 1e3, t);
			}
			continue;
		}
		t = time_it(run_read, 0, 20);
		printf("grid %5d read      %7.1f GB/s\n", C.grid, gb / t * 1e3);
		t = time_it(run_read_nt, 0, 20);
		printf("grid %5d read_nt   %7.1f GB/s\n", C.grid, gb / t * 1e3);
		t = time_it(run_write, 0, 20);
		printf("grid %5d write     %7.1f GB/s\n", C.grid, gb / t * 1e3);
		t = time_it(run_copy, 0, 20);
		printf("grid %5d copy      %7.1f GB/s\n", C.grid, gb / t * 1e3);
		const double mixb = frames * 113.0 / 1e9;
		t = time_it(run_mix<false, 1>, 0, 20);
		printf("grid %5d rx_mix    %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_mix<true, 1>, 0, 20);
		printf("grid %5d rx_mix_nt %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_mix<false, 2>, 0, 20);
		printf("grid %5d rx_mix_u2 %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_mix<true, 2>, 0, 20);
		printf("grid %5d rx_mix_nt_u2 %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_lds, 0, 20);
		printf("grid %5d rx_lds       %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_direct<false, 1>, 0, 20);
		printf("grid %5d rx_direct    %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_direct<true, 1>, 0, 20);
		printf("grid %5d rx_direct_nt %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
		t = time_it(run_direct<true, 2>, 0, 20);
		printf("grid %5d rx_direct_nt_u2 %7.1f GB/s  %.4f ms\n", C.grid, mixb / t * 1e3, t);
	}
	return 0;
}
