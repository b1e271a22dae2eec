// SPDX-License-Identifier: GPL-2.0
/*
 * xdpgpu.cpp - host side of the C ABI in include/xdpgpu.h.
 *
 * A context owns one device, two HIP streams (two in-flight RX batches), a
 * device mirror of the registered host UMEM and per-block counter slots.
 * The host path copies the UMEM runs a batch touches into the slot's device
 * mirror (no kernel ever reads or writes host memory), the descriptors,
 * launches the RX kernel and copies verdicts/results/tuples back.
 */
#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include <algorithm>
#include <atomic>
#include <initializer_list>
#include <utility>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <thread>

#include <sched.h>
#include <sys/mman.h>

#include "xdpgpu.h"
#include "xdpgpu_internal.h"
#include "nat64_state.h"

#include <time.h>

using namespace xdpgpu;

namespace {

constexpr uint32_t kSlots = 2;
constexpr uint32_t kDefaultMaxBatch = 1u << 20;

/* The host threads of XDPGPU_CFG_HOST_COMPACT: a fork-join pool, the
 * calling thread being thread 0.  run(f) calls f(t) for t in [0, size())
 * and returns when every call has. */
class HostPool {
public:
	/* as many of the n threads as the system gives (at least the
	 * caller's): a failed thread creation must not cross the C ABI */
	explicit HostPool(unsigned n)
	{
		for (unsigned t = 1; t < n; t++) {
			try {
				th_.emplace_back([this, t] { loop(t); });
			} catch (...) {
				break;
			}
			n_ = t + 1;
		}
	}
	~HostPool()
	{
		{
			std::lock_guard<std::mutex> lk(mu_);
			stop_ = true;
			gen_++;
		}
		cv_.notify_all();
		for (std::thread &t : th_)
			t.join();
	}
	unsigned size() const { return n_; }
	void run(const std::function<void(unsigned)> &f)
	{
		if (n_ == 1) {
			f(0);
			return;
		}
		{
			std::lock_guard<std::mutex> lk(mu_);
			job_ = &f;
			left_ = n_ - 1;
			gen_++;
		}
		cv_.notify_all();
		f(0);
		std::unique_lock<std::mutex> lk(mu_);
		done_.wait(lk, [this] { return left_ == 0; });
		job_ = nullptr;
	}

private:
	void loop(unsigned t)
	{
		uint64_t seen = 0;
		std::unique_lock<std::mutex> lk(mu_);
		for (;;) {
			cv_.wait(lk, [&] { return gen_ != seen; });
			seen = gen_;
			if (stop_)
				return;
			const std::function<void(unsigned)> *f = job_;
			lk.unlock();
			(*f)(t);
			lk.lock();
			if (--left_ == 0)
				done_.notify_one();
		}
	}
	unsigned n_ = 1;
	std::vector<std::thread> th_;
	std::mutex mu_;
	std::condition_variable cv_, done_;
	const std::function<void(unsigned)> *job_ = nullptr;
	unsigned left_ = 0;
	uint64_t gen_ = 0;
	bool stop_ = false;
};

struct Slot {
	hipStream_t stream = nullptr;
	hipEvent_t done = nullptr;
	unsigned long long *d_stats = nullptr; /* kStatSlots * CNT_SLOT */
	xdpgpu_desc *d_desc = nullptr;
	uint8_t *d_verdict = nullptr;
	xdpgpu_result *d_res = nullptr;
	uint8_t *d_tup = nullptr;
	uint32_t *d_xlist = nullptr;  /* exception list (fast -> generic kernel) */
	uint4 *d_ylist = nullptr;     /* exception payload sums (generic -> bulk) */
	uint64_t xcap = 0;
	uint32_t *d_xcount = nullptr;
	/* xdp_rx_db_kernel's shared-tile claim counters (RxArgs.steal): two
	 * sets, the next launch's zeroed by the current one */
	uint32_t *d_steal = nullptr;
	uint32_t steal_set = 0;
	/* host path: this slot's device mirror of the registered UMEM (one
	 * per slot, so two batches in flight never share mirror bytes) */
	uint8_t *d_mirror = nullptr;
	uint64_t mirror_cap = 0;
	/* XDPGPU_CFG_HOST_COMPACT: the batch's pieces packed by the host
	 * threads (page-locked), their device copy, and each frame's piece
	 * offset in 16-byte units (host and device) */
	uint8_t *h_pack = nullptr;
	uint8_t *d_pack = nullptr;
	uint64_t pack_cap = 0;
	uint32_t *h_poff = nullptr;
	uint32_t *d_poff = nullptr;
	uint64_t poff_cap = 0;
	/* echo write-back as compact records (UMEM not mapped) */
	EchoRec *d_erec = nullptr;
	EchoRec *h_erec = nullptr;
	uint32_t *d_ecnt = nullptr;
	uint32_t *h_ecnt = nullptr;          /* pinned */
	uint64_t erec_cap = 0;
	bool echo_pending = false;
	/* ordering of the slot's scratch (deferral lists, counts, counters,
	 * fragment buffers) between launches on different streams: the event
	 * recorded after the last launch that used it, on scr_last; after a
	 * launch on the slot's own stream it is recorded only when another
	 * stream comes (scr_lazy: the own stream lives as long as the slot,
	 * and a caller's stream may not) */
	hipEvent_t scr_ev = nullptr;
	hipStream_t scr_last = nullptr;
	bool scr_lazy = false;
	bool busy = false;
	/* a device batch (xdpgpu_submit_dev) enqueued since the last wait */
	bool dev_pending = false;
	/* pending host copies for xdpgpu_wait() */
	uint32_t n = 0;
};

} // namespace

struct xdpgpu_ctx {
	xdpgpu_cfg cfg;
	uint32_t max_blocks = kMaxRxBlocks;
	Slot slot[kSlots];
	/* registered host UMEM */
	uint8_t *h_umem = nullptr;
	uint64_t umem_size = 0;
	/* the UMEM is page-locked by a registration this context holds a
	 * reference on (hostreg_acquire): the base of that registration */
	bool pinned = false;
	uintptr_t reg_key = 0;
	/* aligned-mode chunk size (a power of two) when register_umem gave
	 * one, else 0: the host path then copies rows of chunks */
	uint32_t chunk = 0;
	uint32_t chunk_shift = 0;
	/* XDPGPU_CFG_UMEM_GATHER on a chunked UMEM: its GPU mapping (the
	 * gather kernel's source), else null */
	const uint8_t *d_hview = nullptr;
	/* the bytes the gather kernels read (device counter, added in by
	 * xdpgpu_host_stats) */
	unsigned long long *d_gbytes = nullptr;
	/* XDPGPU_CFG_HOST_COMPACT's threads (made on first use) */
	HostPool *hpool = nullptr;
	uint32_t host_threads = 0;     /* 0: default_host_threads() */
	/* host-path copy accounting (xdpgpu_host_stats) */
	struct xdpgpu_host_stats hstats{};
	/* XDPGPU_CFG_TIMING: 4 events per recorded launch */
	hipEvent_t *tev = nullptr;
	/* nat64 translator (xdpgpu_nat64_setup) */
	bool nat64 = false;
	xdpgpu_nat64_cfg ncfg;
	Nat64V6Bucket *d_v6map = nullptr;
	Nat64V4Bucket *d_v4map = nullptr;
	uint32_t nb = 0;           /* buckets of each table (device copy) */
	std::vector<xdpgpu_nat64_map> nstat;   /* the static entries */
	Nat64State nst;            /* host copy and the dynamic allocator */
	bool ndyn = false;         /* xdpgpu_nat64_dynamic */
	uint64_t nclock = 0;       /* batch clock, 0: CLOCK_MONOTONIC */
	/* dynamic state: the frames a batch lists, and the commit pass */
	uint32_t *d_midx = nullptr;
	uint4 *d_msrc = nullptr;
	uint32_t *d_mcnt = nullptr;            /* [0] listed, [1] committed */
	uint32_t *d_mov = nullptr;             /* [cap] order, then [cap] v4 */
	uint64_t mcap = 0;
	Nat64Patch *d_patch = nullptr;
	uint64_t pcap = 0;
	unsigned long long *d_spread = nullptr;   /* synproxy SYN-ACK counters */
	uint32_t tn = 0;
	char err[256];
};

static int set_err(xdpgpu_ctx *ctx, int rc, const char *fmt, ...)
{
	if (ctx) {
		va_list ap;
		va_start(ap, fmt);
		vsnprintf(ctx->err, sizeof(ctx->err), fmt, ap);
		va_end(ap);
	}
	return rc;
}

#define HIP_TRY(ctx, call)                                                   \
	do {                                                                 \
		hipError_t e_ = (call);                                      \
		if (e_ != hipSuccess)                                        \
			return set_err((ctx), -EIO, "%s: %s", #call,         \
				       hipGetErrorString(e_));               \
	} while (0)

static uint32_t tuple_bytes(uint32_t fmt)
{
	return fmt == XDPGPU_TUPLE_NET ? 44u : fmt == XDPGPU_TUPLE_V4 ? 16u : 0u;
}

extern "C" {

int xdpgpu_abi_version(void)
{
	return XDPGPU_ABI_VERSION;
}

int xdpgpu_device_count(void)
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess)
		return 0;
	return n;
}

const char *xdpgpu_last_error(xdpgpu_ctx *ctx)
{
	return ctx ? ctx->err : "no context";
}

/* Host staging of the compaction: ordinary write-back memory (2 MiB
 * aligned, advised for huge pages) that is then page-locked for the copy
 * engine, so the host threads write it through their caches. */
static void *staging_alloc(uint64_t bytes)
{
	const uint64_t sz = (bytes + (2u << 20) - 1) & ~(uint64_t)((2u << 20) - 1);
	void *p = nullptr;
	if (posix_memalign(&p, 2u << 20, sz))
		return nullptr;
	(void)madvise(p, sz, MADV_HUGEPAGE);
	memset(p, 0, sz);   /* fault the pages in before they are locked */
	if (hipHostRegister(p, sz, hipHostRegisterDefault) != hipSuccess) {
		(void)hipGetLastError();
		free(p);
		return nullptr;
	}
	return p;
}

static void staging_free(void *p)
{
	if (!p)
		return;
	if (hipHostUnregister(p) != hipSuccess)
		(void)hipGetLastError();
	free(p);
}

static void free_slot(Slot &s)
{
	if (s.d_stats)
		(void)hipFree(s.d_stats);
	if (s.d_desc)
		(void)hipFree(s.d_desc);
	if (s.d_verdict)
		(void)hipFree(s.d_verdict);
	if (s.d_res)
		(void)hipFree(s.d_res);
	if (s.d_tup)
		(void)hipFree(s.d_tup);
	if (s.d_xlist)
		(void)hipFree(s.d_xlist);
	if (s.d_xcount)
		(void)hipFree(s.d_xcount);
	if (s.d_steal)
		(void)hipFree(s.d_steal);
	if (s.d_ylist)
		(void)hipFree(s.d_ylist);
	(void)hipFree(s.d_mirror);
	(void)hipFree(s.d_pack);
	(void)hipFree(s.d_poff);
	staging_free(s.h_pack);
	staging_free(s.h_poff);
	(void)hipFree(s.d_erec);
	(void)hipFree(s.d_ecnt);
	if (s.h_ecnt)
		(void)hipHostFree(s.h_ecnt);
	free(s.h_erec);
	if (s.scr_ev)
		(void)hipEventDestroy(s.scr_ev);
	if (s.done)
		(void)hipEventDestroy(s.done);
	if (s.stream)
		(void)hipStreamDestroy(s.stream);
	s = Slot();
}

/* Host registrations of UMEMs, process-wide and counted.  Several RX
 * queues share one UMEM (the reference's sockets on one xsk_umem,
 * af_xdp_user.c:1542-1611), so several contexts register the same memory;
 * HIP keeps one registration per range, and the first hipHostUnregister
 * would tear it down under the others (their copies would lose the
 * pinning, and XDPGPU_CFG_UMEM_GATHER's device view would dangle).  A
 * context takes a reference on the registration that covers its range, or
 * makes one; the last reference unregisters.  Memory the caller pinned
 * (xdpgpu_host_alloc, or its own registration) cannot be registered again:
 * the context then holds nothing and the caller owns the pinning. */
struct HostReg {
	uint64_t size;
	uint32_t refs;
};
static std::mutex g_regmu;
static std::map<uintptr_t, HostReg> g_regs;

static bool hostreg_acquire(void *base, uint64_t size, uintptr_t *key)
{
	std::lock_guard<std::mutex> lk(g_regmu);
	const uintptr_t b = (uintptr_t)base;
	auto it = g_regs.upper_bound(b);
	if (it != g_regs.begin()) {
		--it;
		if (b >= it->first && b + size <= it->first + it->second.size) {
			it->second.refs++;
			*key = it->first;
			return true;
		}
	}
	if (hipHostRegister(base, size, hipHostRegisterDefault) != hipSuccess) {
		(void)hipGetLastError();
		return false;
	}
	g_regs[b] = HostReg{size, 1};
	*key = b;
	return true;
}

static void hostreg_release(uintptr_t key)
{
	std::lock_guard<std::mutex> lk(g_regmu);
	auto it = g_regs.find(key);
	if (it == g_regs.end() || --it->second.refs)
		return;
	if (hipHostUnregister((void *)key) != hipSuccess)
		(void)hipGetLastError();
	g_regs.erase(it);
}

/* Diagnostic for the tests: the live registrations' reference counts
 * summed over those covering p (0: none). */
int xdpgpu_host_pin_refs(const void *p)
{
	std::lock_guard<std::mutex> lk(g_regmu);
	const uintptr_t b = (uintptr_t)p;
	int refs = 0;
	for (const auto &r : g_regs)
		if (b >= r.first && b < r.first + r.second.size)
			refs += (int)r.second.refs;
	return refs;
}

/* Per-queue counters: the live contexts, and the counters of finished ones
 * by queue (xdpgpu_queue_stats). */
static std::mutex g_qmu;
static std::vector<xdpgpu_ctx *> g_live;
static std::map<uint32_t, struct xdpgpu_stats> g_retired;

static void add_stats(struct xdpgpu_stats &to, const struct xdpgpu_stats &s)
{
	to.frames += s.frames;
	to.bytes += s.bytes;
	for (int v = 0; v < XDPGPU_NUM_VERDICTS; v++)
		to.verdict[v] += s.verdict[v];
	to.l3_bad += s.l3_bad;
	to.l4_bad += s.l4_bad;
	to.l4_absent += s.l4_absent;
	to.frag += s.frag;
}

int xdpgpu_queue_stats(uint32_t queue_id, struct xdpgpu_stats *out)
{
	if (!out)
		return -EINVAL;
	memset(out, 0, sizeof(*out));
	std::lock_guard<std::mutex> lk(g_qmu);
	auto it = g_retired.find(queue_id);
	if (it != g_retired.end())
		add_stats(*out, it->second);
	for (xdpgpu_ctx *c : g_live) {
		if (c->cfg.queue_id != queue_id)
			continue;
		struct xdpgpu_stats s;
		const int rc = xdpgpu_stats(c, &s);
		if (rc)
			return rc;
		add_stats(*out, s);
	}
	return 0;
}

void xdpgpu_fini(xdpgpu_ctx *ctx)
{
	if (!ctx)
		return;
	{
		std::lock_guard<std::mutex> lk(g_qmu);
		auto it = std::find(g_live.begin(), g_live.end(), ctx);
		if (it != g_live.end()) {
			g_live.erase(it);
			struct xdpgpu_stats s;
			if (xdpgpu_stats(ctx, &s) == 0)
				add_stats(g_retired[ctx->cfg.queue_id], s);
		}
	}
	(void)hipSetDevice(ctx->cfg.device);
	(void)hipDeviceSynchronize();
	for (uint32_t i = 0; i < kSlots; i++)
		free_slot(ctx->slot[i]);
	delete ctx->hpool;
	if (ctx->d_gbytes)
		(void)hipFree(ctx->d_gbytes);
	if (ctx->tev) {
		for (uint32_t i = 0; i < 4 * XDPGPU_TIMING_MAX; i++)
			if (ctx->tev[i])
				(void)hipEventDestroy(ctx->tev[i]);
		delete[] ctx->tev;
	}
	if (ctx->d_v6map)
		(void)hipFree(ctx->d_v6map);
	if (ctx->d_v4map)
		(void)hipFree(ctx->d_v4map);
	for (void *p : {(void *)ctx->d_midx, (void *)ctx->d_msrc, (void *)ctx->d_mcnt,
			(void *)ctx->d_mov, (void *)ctx->d_patch, (void *)ctx->d_spread})
		if (p)
			(void)hipFree(p);
	if (ctx->pinned)
		hostreg_release(ctx->reg_key);
	delete ctx;
}

int xdpgpu_init(const xdpgpu_cfg *cfg, xdpgpu_ctx **out)
{
	if (!cfg || !out)
		return -EINVAL;
	if (cfg->window != 0 && cfg->window != 64 && cfg->window != 128)
		return -EINVAL;
	if (cfg->tuple_fmt > XDPGPU_TUPLE_NET)
		return -EINVAL;
	int ndev = xdpgpu_device_count();
	if (ndev <= 0)
		return -ENODEV;
	if (cfg->device < 0 || cfg->device >= ndev)
		return -EINVAL;

	xdpgpu_ctx *ctx = new (std::nothrow) xdpgpu_ctx();
	if (!ctx)
		return -ENOMEM;
	ctx->cfg = *cfg;
	if (!ctx->cfg.max_batch)
		ctx->cfg.max_batch = kDefaultMaxBatch;
	ctx->err[0] = 0;

	int rc = 0;
	do {
		hipDeviceProp_t prop;
		if (hipSetDevice(cfg->device) != hipSuccess ||
		    hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) {
			rc = set_err(ctx, -EIO, "hipSetDevice(%d) failed", cfg->device);
			break;
		}
		ctx->max_blocks = std::min<uint32_t>(kMaxRxBlocks,
			(uint32_t)prop.multiProcessorCount * 8u);
		for (uint32_t i = 0; i < kSlots && !rc; i++) {
			Slot &s = ctx->slot[i];
			size_t stat_bytes = (size_t)kStatSlots * CNT_SLOT * 8;
			if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
			    hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
			    hipEventCreateWithFlags(&s.scr_ev, hipEventDisableTiming) != hipSuccess ||
			    hipMalloc(&s.d_stats, stat_bytes) != hipSuccess ||
			    hipMemset(s.d_stats, 0, stat_bytes) != hipSuccess)
				rc = set_err(ctx, -ENOMEM, "slot %u allocation failed", i);
		}
		/* the counter memsets ran on the null stream, which does not
		 * order against the slots' non-blocking streams */
		if (!rc && hipDeviceSynchronize() != hipSuccess)
			rc = set_err(ctx, -EIO, "hipDeviceSynchronize failed");
		if (!rc && (cfg->flags & XDPGPU_CFG_TIMING)) {
			ctx->tev = new (std::nothrow) hipEvent_t[4 * XDPGPU_TIMING_MAX]();
			if (!ctx->tev) {
				rc = set_err(ctx, -ENOMEM, "timing events");
				break;
			}
			for (uint32_t i = 0; i < 4 * XDPGPU_TIMING_MAX && !rc; i++)
				if (hipEventCreate(&ctx->tev[i]) != hipSuccess)
					rc = set_err(ctx, -ENOMEM, "timing event %u", i);
		}
	} while (0);
	if (rc) {
		xdpgpu_fini(ctx);
		return rc;
	}
	{
		std::lock_guard<std::mutex> lk(g_qmu);
		g_live.push_back(ctx);
	}
	*out = ctx;
	return 0;
}

/* Drop the registered UMEM: the slots' mirrors and the host pinning. */
static void release_umem(xdpgpu_ctx *ctx)
{
	(void)hipDeviceSynchronize();
	for (uint32_t i = 0; i < kSlots; i++) {
		Slot &s = ctx->slot[i];
		(void)hipFree(s.d_mirror);
		s.d_mirror = nullptr;
		s.mirror_cap = 0;
	}
	if (ctx->pinned)
		hostreg_release(ctx->reg_key);
	ctx->pinned = false;
	ctx->reg_key = 0;
	ctx->h_umem = nullptr;
	ctx->d_hview = nullptr;
	ctx->umem_size = 0;
}

/* A slot's device mirror of the registered UMEM (+64: 16-byte loads of a
 * frame's last chunk stay inside it). */
static int ensure_mirror(xdpgpu_ctx *ctx, Slot &s)
{
	if (s.d_mirror && s.mirror_cap >= ctx->umem_size + 64)
		return 0;
	(void)hipFree(s.d_mirror);
	s.d_mirror = nullptr;
	s.mirror_cap = 0;
	if (hipMalloc(&s.d_mirror, ctx->umem_size + 64) != hipSuccess)
		return set_err(ctx, -ENOMEM, "device UMEM mirror of %llu bytes",
			       (unsigned long long)ctx->umem_size);
	s.mirror_cap = ctx->umem_size + 64;
	return 0;
}

int xdpgpu_register_umem(xdpgpu_ctx *ctx, void *base, uint64_t size,
			 uint32_t chunk_size, uint32_t headroom, uint32_t flags)
{
	if (!ctx || !base || !size)
		return -EINVAL;
	if (!(flags & XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG) && chunk_size &&
	    (chunk_size & (chunk_size - 1)))
		return set_err(ctx, -EINVAL, "chunk_size %u not a power of two",
			       chunk_size);
	if (headroom && chunk_size && headroom >= chunk_size)
		return -EINVAL;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	for (uint32_t i = 0; i < kSlots; i++)
		if (ctx->slot[i].busy)
			return set_err(ctx, -EBUSY, "slot %u in flight", i);
	release_umem(ctx);
	ctx->h_umem = (uint8_t *)base;
	ctx->umem_size = size;
	ctx->chunk = 0;
	ctx->chunk_shift = 0;
	if (!(flags & XDPGPU_UMEM_UNALIGNED_CHUNK_FLAG) && chunk_size >= 64) {
		ctx->chunk = chunk_size;
		while ((1u << ctx->chunk_shift) < chunk_size)
			ctx->chunk_shift++;
	}
	/* pin the caller's UMEM for the copy engines (pageable memory still
	 * works, only slower).  No kernel writes it: every batch's frames go
	 * into the slot's device mirror and the echo replies come back as
	 * compact records (the host memory faults of rounds
	 * 2-3 all followed kernels that read and wrote this UMEM through its
	 * GPU mapping, with LDS-DMA and non-temporal loads).  Only the
	 * opt-in gather (XDPGPU_CFG_UMEM_GATHER, chunked UMEMs) reads it
	 * there, with plain loads. */
	ctx->pinned = hostreg_acquire(base, size, &ctx->reg_key);
	if ((ctx->cfg.flags & XDPGPU_CFG_UMEM_GATHER) && ctx->chunk) {
		/* memory pinned here or by the caller (xdpgpu_host_alloc) */
		void *p = nullptr;
		if (hipHostGetDevicePointer(&p, base, 0) == hipSuccess && p) {
			if (!ctx->d_gbytes) {
				if (hipMalloc(&ctx->d_gbytes, sizeof(*ctx->d_gbytes)) != hipSuccess) {
					release_umem(ctx);
					return set_err(ctx, -ENOMEM, "gather byte counter");
				}
				HIP_TRY(ctx, hipMemset(ctx->d_gbytes, 0, sizeof(*ctx->d_gbytes)));
			}
			ctx->d_hview = (const uint8_t *)p;
		} else {
			(void)hipGetLastError();
		}
	}

	/* slot 0's mirror now, so that a size the device cannot hold fails
	 * here; slot 1's on its first batch */
	const int rc = ensure_mirror(ctx, ctx->slot[0]);
	if (rc) {
		release_umem(ctx);
		return rc;
	}
	return 0;
}

static int ensure_slot_buffers(xdpgpu_ctx *ctx, Slot &s, uint32_t n)
{
	int rc = ensure_mirror(ctx, s);
	if (rc)
		return rc;
	if (s.d_desc)
		return 0;
	uint32_t cap = ctx->cfg.max_batch;
	uint32_t tb = tuple_bytes(ctx->cfg.tuple_fmt);
	if (hipMalloc(&s.d_desc, (size_t)cap * sizeof(xdpgpu_desc)) != hipSuccess ||
	    hipMalloc(&s.d_verdict, (size_t)cap) != hipSuccess ||
	    hipMalloc(&s.d_res, (size_t)cap * sizeof(xdpgpu_result)) != hipSuccess ||
	    (tb && hipMalloc(&s.d_tup, (size_t)cap * tb) != hipSuccess))
		return set_err(ctx, -ENOMEM, "batch buffers for %u descriptors", cap);
	(void)n;
	return 0;
}

/* Deferred-frame list scratch for a launch of n frames (any grid up to
 * kMaxRxBlocks): two lists (exception, bulk) of per-wave regions of whole
 * tiles, xcap entries each, and their per-wave counts. */
static int ensure_xlist(xdpgpu_ctx *ctx, Slot &s, uint32_t n)
{
	/* the frames, as many more for xdp_rx_db_kernel's shared tiles
	 * (launch_db: a block's region holds its own tiles and up to twice its
	 * share of the shared ones, up to the whole batch), and per-block
	 * slack */
	const uint64_t need = 3ull * n + 64ull * 40 * kMaxRxBlocks + 1024;
	/* per-wave exception, bulk and deferred-payload counts */
	const size_t cbytes = (size_t)kMaxRxBlocks * 4 * 3 * sizeof(uint32_t);
	if (!s.d_xcount && (hipMalloc(&s.d_xcount, cbytes) != hipSuccess ||
			    hipMemset(s.d_xcount, 0, cbytes) != hipSuccess ||
			    hipDeviceSynchronize() != hipSuccess))
		return set_err(ctx, -ENOMEM, "exception counts");
	const size_t sbytes = 2ull * kStealHeads * kStealStride * sizeof(uint32_t);
	if (!s.d_steal && (hipMalloc(&s.d_steal, sbytes) != hipSuccess ||
			   hipMemset(s.d_steal, 0, sbytes) != hipSuccess ||
			   hipDeviceSynchronize() != hipSuccess)) {
		(void)hipFree(s.d_steal);
		s.d_steal = nullptr;
		return set_err(ctx, -ENOMEM, "shared-tile counters");
	}
	if (s.xcap >= need)
		return 0;
	if (s.d_xlist || s.d_ylist) {
		(void)hipDeviceSynchronize();
		(void)hipFree(s.d_xlist);
		(void)hipFree(s.d_ylist);
		s.d_xlist = nullptr;
		s.d_ylist = nullptr;
		s.xcap = 0;
	}
	if (hipMalloc(&s.d_xlist, 2 * need * sizeof(uint32_t)) != hipSuccess ||
	    hipMalloc(&s.d_ylist, need * sizeof(uint4)) != hipSuccess)
		return set_err(ctx, -ENOMEM, "deferral lists of %llu entries",
			       (unsigned long long)need);
	s.xcap = need;
	return 0;
}

/* A launch on `stream` that uses slot s's scratch waits for the previous
 * launch that used it when that one went to another stream (a caller's
 * stream for xdpgpu_process_dev / xdpgpu_nat64_dev, the slot's own for
 * xdpgpu_submit); scratch_leave marks the new owner. */
static int scratch_enter(xdpgpu_ctx *ctx, Slot &s, hipStream_t stream)
{
	if (s.scr_last && s.scr_last != stream) {
		if (s.scr_lazy) {
			/* everything enqueued on the slot's own stream so far,
			 * the last launch included */
			HIP_TRY(ctx, hipEventRecord(s.scr_ev, s.scr_last));
			s.scr_lazy = false;
		}
		HIP_TRY(ctx, hipStreamWaitEvent(stream, s.scr_ev, 0));
	}
	return 0;
}

/* (an event record after every launch cost 5 us between back-to-back
 * launches on one stream: config 2 0.3100/0.3132 vs 0.3185/0.3168 ms per
 * step without it, alternating processes) */
static int scratch_leave(xdpgpu_ctx *ctx, Slot &s, hipStream_t stream)
{
	s.scr_lazy = stream == s.stream;
	if (!s.scr_lazy)
		HIP_TRY(ctx, hipEventRecord(s.scr_ev, stream));
	s.scr_last = stream;
	return 0;
}

/* Host wait for the slot's last scratch user. */
static int scratch_sync(xdpgpu_ctx *ctx, Slot &s)
{
	if (!s.scr_last)
		return 0;
	if (s.scr_lazy) {
		HIP_TRY(ctx, hipEventRecord(s.scr_ev, s.scr_last));
		s.scr_lazy = false;
	}
	HIP_TRY(ctx, hipEventSynchronize(s.scr_ev));
	return 0;
}

/* bytes a frame for the automatic window (cfg.window 0): the caller's
 * UMEM over the batch (device path), or the batch's own mean frame length
 * (host path, whose descriptors the library reads) */
static int enqueue_rx(xdpgpu_ctx *ctx, Slot &s, uint8_t *d_umem, uint64_t usize,
		      const xdpgpu_desc *d_desc, uint32_t n, uint8_t *d_verdict,
		      xdpgpu_result *d_res, uint8_t *d_tup, hipStream_t stream,
		      uint64_t per_frame = 0)
{
	int rc = ensure_xlist(ctx, s, n);
	if (rc)
		return rc;
	RxArgs a;
	memset(&a, 0, sizeof(a));
	a.umem = d_umem;
	a.usize = usize;
	a.desc = d_desc;
	a.n = n;
	a.tuple_fmt = d_tup ? ctx->cfg.tuple_fmt : XDPGPU_TUPLE_NONE;
	a.verdict = d_verdict;
	a.res = d_res;
	a.tup = d_tup;
	a.flags = ctx->cfg.flags;
	a.initval = ctx->cfg.jhash_initval;
	a.stats = (ctx->cfg.flags & XDPGPU_CFG_STATS) ? s.d_stats : nullptr;
	a.xlist = s.d_xlist;
	a.xcount = s.d_xcount;
	a.blist = s.d_xlist + s.xcap;
	a.bcount = s.d_xcount + kMaxRxBlocks * 4;
	a.ylist = s.d_ylist;
	a.ycount = s.d_xcount + kMaxRxBlocks * 4 * 2;
	a.ydefer = !((ctx->cfg.tune >> 8) & 1);
	a.force_generic = (ctx->cfg.tune >> 9) & 1;
	a.frags = (ctx->cfg.flags & XDPGPU_CFG_FRAGS) ? 1u : 0u;
	a.xcap = s.xcap;
	a.steal = s.d_steal;
	a.steal_set = s.steal_set;
	/* shared tiles, in 16ths of the batch (cfg.tune bit 21: none).
	 * Config 2, one box, one process: none 0.3435 ms, 8 0.3284, 12
	 * 0.3226, 14 0.3227, 16 0.331 (tools/gpu_ab_steal.sh) */
	a.steal_16ths = (ctx->cfg.tune >> 21) & 1 ? 0u : 12u;
	/* the header window: as configured, or (0) 128 bytes for a batch of
	 * at least 128 bytes a frame (frames longer than 64 bytes then read
	 * their first line once), else 64 */
	if (!per_frame)
		per_frame = n ? usize / n : 0;
	a.win = ctx->cfg.window ? ctx->cfg.window : (per_frame >= 128 ? 128u : 64u);

	rc = scratch_enter(ctx, s, stream);
	if (rc)
		return rc;
	hipEvent_t *ev = nullptr;
	if (ctx->tev && ctx->tn < XDPGPU_TIMING_MAX)
		ev = ctx->tev + 4 * ctx->tn++;
	if (a.frags) {
		/* multi-buffer packets: the broken ones finished first, then
		 * (after the RX kernel, which skips their descriptors) every
		 * complete packet read in place as one frame */
		FragArgs f;
		memset(&f, 0, sizeof(f));
		f.umem = d_umem;
		f.usize = usize;
		f.desc = d_desc;
		f.n = n;
		f.verdict = d_verdict;
		f.res = d_res;
		f.tup = d_tup;
		f.tb = d_tup ? tuple_bytes(ctx->cfg.tuple_fmt) : 0;
		f.stats = a.stats;
		HIP_TRY(ctx, launch_frag_count(f, stream));
	}
	HIP_TRY(ctx, launch_rx(a, ctx->max_blocks, stream, ctx->cfg.tune, ev));
	/* the launch zeroed the other counter set: the next one uses it */
	s.steal_set ^= 1;
	if (a.frags)
		HIP_TRY(ctx, launch_rx_packets(a, ctx->max_blocks, stream));
	return scratch_leave(ctx, s, stream);
}

int xdpgpu_kernel_times(xdpgpu_ctx *ctx, xdpgpu_ktimes *out)
{
	if (!ctx || !out)
		return -EINVAL;
	memset(out, 0, sizeof(*out));
	if (!ctx->tev)
		return set_err(ctx, -EINVAL, "context made without XDPGPU_CFG_TIMING");
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	for (uint32_t k = 0; k < ctx->tn; k++) {
		/* one RX launch is one kernel: its two events (e[2], e[3] are
		 * the struct's old exception and bulk pairs, never recorded) */
		hipEvent_t *e = ctx->tev + 4 * k;
		float t;
		HIP_TRY(ctx, hipEventSynchronize(e[1]));
		HIP_TRY(ctx, hipEventElapsedTime(&t, e[0], e[1]));
		out->fast_ms += t;
		out->total_ms += t;
	}
	out->launches = ctx->tn;
	ctx->tn = 0;
	return 0;
}

/* Every buffer a *_dev call hands a kernel must be device memory: no
 * kernel of the library dereferences host memory (pinned or mapped host
 * memory read or written through its GPU mapping is what the host-memory
 * faults of rounds 2-3 had in common).  Each pointer is
 * queried on every call, nothing is remembered: a freed device range can
 * come back as host memory at the same address (profiles/r04_va_probe*),
 * and a query costs well under a microsecond next to a launch.  Null
 * pointers (optional outputs) are skipped. */
static int check_dev(xdpgpu_ctx *ctx, const char *what, const void *p)
{
	if (!p)
		return 0;
	hipPointerAttribute_t at;
	memset(&at, 0, sizeof(at));
	if (hipPointerGetAttributes(&at, p) != hipSuccess) {
		(void)hipGetLastError();
		return set_err(ctx, -EINVAL, "%s %p is not device memory", what, p);
	}
	if (at.type != hipMemoryTypeDevice && !at.isManaged)
		return set_err(ctx, -EINVAL, "%s %p is host memory (type %d): the kernels "
			       "read and write device memory only", what, p, (int)at.type);
	return 0;
}

static int check_dev_all(xdpgpu_ctx *ctx, std::initializer_list<std::pair<const char *,
			 const void *>> ptrs)
{
	for (const auto &w : ptrs)
		if (int rc = check_dev(ctx, w.first, w.second))
			return rc;
	return 0;
}

int xdpgpu_process_dev(xdpgpu_ctx *ctx, void *d_umem, uint64_t umem_size,
		       const xdpgpu_desc *d_descs, uint32_t n,
		       uint8_t *d_verdict, xdpgpu_result *d_res, void *d_tuples,
		       void *stream)
{
	if (!ctx || !d_umem || !d_descs || !d_verdict)
		return -EINVAL;
	if (n == 0)
		return 0;
	int rc = check_dev_all(ctx, {{"UMEM", d_umem}, {"descriptors", d_descs},
				     {"verdicts", d_verdict}, {"results", d_res},
				     {"tuples", d_tuples}});
	if (rc)
		return rc;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	return enqueue_rx(ctx, ctx->slot[0], (uint8_t *)d_umem, umem_size,
			  d_descs, n, d_verdict, d_res, (uint8_t *)d_tuples, st);
}

/* The device-resident RX loop with two batches in flight: slot `slot`'s
 * stream and scratch, so that the other slot's launch can take the CUs
 * this one leaves while its last tiles finish (one block per CU: the next
 * launch's block starts on a CU as soon as this one's has left it). */
int xdpgpu_submit_dev(xdpgpu_ctx *ctx, uint32_t slot, void *d_umem, uint64_t umem_size,
		      const xdpgpu_desc *d_descs, uint32_t n, uint8_t *d_verdict,
		      xdpgpu_result *d_res, void *d_tuples)
{
	if (!ctx || slot >= kSlots || !d_umem || !d_descs || !d_verdict)
		return -EINVAL;
	Slot &s = ctx->slot[slot];
	if (s.busy)
		return set_err(ctx, -EBUSY, "slot %u has a host batch in flight", slot);
	if (n == 0)
		return 0;
	int rc = check_dev_all(ctx, {{"UMEM", d_umem}, {"descriptors", d_descs},
				     {"verdicts", d_verdict}, {"results", d_res},
				     {"tuples", d_tuples}});
	if (rc)
		return rc;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	s.dev_pending = true;
	return enqueue_rx(ctx, s, (uint8_t *)d_umem, umem_size, d_descs, n, d_verdict, d_res,
			  (uint8_t *)d_tuples, s.stream);
}

void *xdpgpu_slot_stream(xdpgpu_ctx *ctx, uint32_t slot)
{
	if (!ctx || slot >= kSlots)
		return nullptr;
	return (void *)ctx->slot[slot].stream;
}

/* ---- nat64 ---- */

/* Buckets of the static tables: 4 slots each, 3 entries per bucket on
 * average, so that an overflow into the next bucket is rare. */
static uint32_t nat64_buckets(uint32_t n)
{
	return n < 3 ? 1u : (n + 2) / 3;
}

/* (re)allocate the device tables for the host copy's size and upload it */
static int nat64_upload(xdpgpu_ctx *ctx)
{
	const uint32_t nb = ctx->nst.buckets();
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	if (nb != ctx->nb || !ctx->d_v6map) {
		if (ctx->d_v6map)
			(void)hipFree(ctx->d_v6map);
		if (ctx->d_v4map)
			(void)hipFree(ctx->d_v4map);
		ctx->d_v6map = nullptr;
		ctx->d_v4map = nullptr;
		ctx->nb = 0;
		if (hipMalloc(&ctx->d_v6map, (size_t)nb * sizeof(Nat64V6Bucket)) != hipSuccess ||
		    hipMalloc(&ctx->d_v4map, (size_t)nb * sizeof(Nat64V4Bucket)) != hipSuccess)
			return set_err(ctx, -ENOMEM, "nat64 tables of %u buckets", nb);
		ctx->nb = nb;
	}
	HIP_TRY(ctx, hipMemcpy(ctx->d_v6map, ctx->nst.v6().data(),
			       (size_t)nb * sizeof(Nat64V6Bucket), hipMemcpyHostToDevice));
	HIP_TRY(ctx, hipMemcpy(ctx->d_v4map, ctx->nst.v4().data(),
			       (size_t)nb * sizeof(Nat64V4Bucket), hipMemcpyHostToDevice));
	return 0;
}

int xdpgpu_nat64_setup(xdpgpu_ctx *ctx, const xdpgpu_nat64_cfg *cfg,
		       const xdpgpu_nat64_map *map, uint32_t nmap)
{
	if (!ctx || !cfg || (nmap && !map))
		return -EINVAL;
	const uint32_t pl = cfg->v6_plen;
	if (pl != 32 && pl != 40 && pl != 48 && pl != 56 && pl != 64 && pl != 96)
		return set_err(ctx, -EINVAL, "v6 prefix length %u (nat64.c:118)", pl);
	if (cfg->direction > XDPGPU_NAT64_EGRESS || cfg->allow_plen > 128 ||
	    (cfg->v4_prefix & ~cfg->v4_mask) || nmap > (1u << 30))
		return -EINVAL;
	ctx->nat64 = false;
	ctx->ndyn = false;
	ctx->nstat.assign(map, map + nmap);
	ctx->nst.v4_prefix = cfg->v4_prefix;
	ctx->nst.v4_mask = cfg->v4_mask;
	ctx->nst.cap = 0;
	ctx->nst.build(ctx->nstat, nat64_buckets(nmap));
	const int rc = nat64_upload(ctx);
	if (rc)
		return rc;
	ctx->ncfg = *cfg;
	ctx->nat64 = true;
	return 0;
}

int xdpgpu_nat64_dynamic(xdpgpu_ctx *ctx, const xdpgpu_nat64_dyn *dyn)
{
	if (!ctx)
		return -EINVAL;
	if (!ctx->nat64)
		return set_err(ctx, -EINVAL, "xdpgpu_nat64_setup not called");
	uint32_t cap = 0;
	if (dyn) {
		/* num_addr (nat64.c:396), the size of all three maps */
		const uint32_t top = ctx->ncfg.v4_prefix | ~ctx->ncfg.v4_mask;
		if (~ctx->ncfg.v4_mask < 3)
			return set_err(ctx, -EINVAL, "v4 pool %#x/%#x has no dynamic addresses",
				       ctx->ncfg.v4_prefix, ctx->ncfg.v4_mask);
		cap = top - ctx->ncfg.v4_prefix - 2;
		if (cap > (1u << 26))
			return set_err(ctx, -E2BIG, "v4 pool of %u addresses", cap);
	}
	ctx->nat64 = false;
	ctx->nst.cap = cap;
	ctx->nst.timeout_ns = dyn ? dyn->timeout_ns : 0;
	ctx->nst.next_addr = dyn ? dyn->next_addr : 1;
	ctx->nclock = dyn ? dyn->now_ns : 0;
	const uint32_t nmap = (uint32_t)ctx->nstat.size();
	ctx->nst.build(ctx->nstat, nat64_buckets(std::max(nmap, cap)));
	const int rc = nat64_upload(ctx);
	if (rc)
		return rc;
	ctx->ndyn = dyn != nullptr;
	ctx->nat64 = true;
	return 0;
}

int xdpgpu_nat64_clock(xdpgpu_ctx *ctx, uint64_t now_ns)
{
	if (!ctx)
		return -EINVAL;
	ctx->nclock = now_ns;
	return 0;
}

int xdpgpu_nat64_direction(xdpgpu_ctx *ctx, uint32_t direction)
{
	if (!ctx || direction > XDPGPU_NAT64_EGRESS)
		return -EINVAL;
	if (!ctx->nat64)
		return set_err(ctx, -EINVAL, "xdpgpu_nat64_setup not called");
	ctx->ncfg.direction = direction;
	return 0;
}

static int nat64_devtab(xdpgpu_ctx *ctx, std::vector<Nat64V6Bucket> &out)
{
	out.resize(ctx->nb);
	HIP_TRY(ctx, hipMemcpy(out.data(), ctx->d_v6map, (size_t)ctx->nb * sizeof(Nat64V6Bucket),
			       hipMemcpyDeviceToHost));
	return 0;
}

int xdpgpu_nat64_state(xdpgpu_ctx *ctx, xdpgpu_nat64_entry *out, uint32_t max, uint32_t *n,
		       xdpgpu_nat64_dyn *dyn, uint32_t *queue, uint32_t qmax, uint32_t *nq)
{
	if (!ctx || (max && !out) || (qmax && !queue))
		return -EINVAL;
	if (!ctx->nat64)
		return set_err(ctx, -EINVAL, "xdpgpu_nat64_setup not called");
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	for (uint32_t i = 0; i < kSlots; i++)
		HIP_TRY(ctx, hipStreamSynchronize(ctx->slot[i].stream));
	std::vector<Nat64V6Bucket> dev;
	int rc = nat64_devtab(ctx, dev);
	if (rc)
		return rc;
	std::vector<xdpgpu_nat64_entry> all;
	ctx->nst.entries(all, &dev);
	if (n)
		*n = (uint32_t)all.size();
	for (uint32_t k = 0; k < max && k < all.size(); k++)
		out[k] = all[k];
	if (dyn) {
		memset(dyn, 0, sizeof(*dyn));
		dyn->timeout_ns = ctx->nst.timeout_ns;
		dyn->next_addr = ctx->nst.next_addr;
		dyn->now_ns = ctx->nclock;
	}
	const std::deque<uint32_t> &q = ctx->nst.queue();
	if (nq)
		*nq = (uint32_t)q.size();
	for (uint32_t k = 0; k < qmax && k < q.size(); k++)
		queue[k] = q[k];
	return 0;
}

/* the dynamic-state commit of one ingress batch (see xdpgpu.h): the
 * frames the kernels listed, in frame order through alloc_new_state on the
 * host, the changed table slots to the device, then the listed frames
 * again through the general kernel with their addresses */
static int nat64_commit(xdpgpu_ctx *ctx, Nat64Args a, uint64_t now, hipStream_t st)
{
	uint32_t m = 0;
	HIP_TRY(ctx, hipMemcpyAsync(&m, ctx->d_mcnt, 4, hipMemcpyDeviceToHost, st));
	HIP_TRY(ctx, hipStreamSynchronize(st));
	if (!m)
		return 0;
	if (m > a.n)
		return set_err(ctx, -EIO, "nat64: %u listed frames in a batch of %u", m, a.n);
	std::vector<uint32_t> idx(m);
	std::vector<uint4> src(m);
	HIP_TRY(ctx, hipMemcpyAsync(idx.data(), ctx->d_midx, (size_t)m * 4,
				    hipMemcpyDeviceToHost, st));
	HIP_TRY(ctx, hipMemcpyAsync(src.data(), ctx->d_msrc, (size_t)m * 16,
				    hipMemcpyDeviceToHost, st));
	HIP_TRY(ctx, hipStreamSynchronize(st));
	std::vector<uint32_t> sidx, ov;
	std::vector<Nat64Patch> patches;
	int err = 0;
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	ctx->nst.commit(idx.data(), src.data(), m, now,
			[ctx](std::vector<Nat64V6Bucket> &t) { return nat64_devtab(ctx, t); },
			sidx, ov, patches, err);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	if (getenv("XDPGPU_NAT64_TRACE")) {
		uint32_t shot = 0;
		for (uint32_t v : ov)
			shot += !v;
		fprintf(stderr, "nat64 commit: %u listed, %u failed, %zu patches, %.3f ms\n", m,
			shot, patches.size(),
			(t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) / 1e6);
	}
	if (err)
		return err;
	if (patches.size() > ctx->pcap) {
		if (ctx->d_patch)
			(void)hipFree(ctx->d_patch);
		ctx->d_patch = nullptr;
		ctx->pcap = 0;
		if (hipMalloc(&ctx->d_patch, patches.size() * sizeof(Nat64Patch)) != hipSuccess)
			return set_err(ctx, -ENOMEM, "nat64 patches");
		ctx->pcap = patches.size();
	}
	const uint32_t reg = (m + 63) & ~63u;
	/* stream-ordered; the host vectors live until the final synchronize */
	if (!patches.empty())
		HIP_TRY(ctx, hipMemcpyAsync(ctx->d_patch, patches.data(),
					    patches.size() * sizeof(Nat64Patch),
					    hipMemcpyHostToDevice, st));
	HIP_TRY(ctx, hipMemcpyAsync(ctx->d_mov, sidx.data(), (size_t)m * 4,
				    hipMemcpyHostToDevice, st));
	HIP_TRY(ctx, hipMemcpyAsync(ctx->d_mov + ctx->mcap, ov.data(), (size_t)m * 4,
				    hipMemcpyHostToDevice, st));
	HIP_TRY(ctx, hipMemcpyAsync(ctx->d_mcnt + 1, &m, 4, hipMemcpyHostToDevice, st));
	HIP_TRY(ctx, launch_nat64_patch(ctx->d_v6map, ctx->d_v4map, ctx->d_patch,
					(uint32_t)patches.size(), st));
	a.fast = 0;
	a.xlist = ctx->d_mov;
	a.xcount = ctx->d_mcnt + 1;
	a.nregions = 1;
	a.xregion = reg;
	a.ov = ctx->d_mov + ctx->mcap;
	HIP_TRY(ctx, launch_nat64(a, ctx->max_blocks, st));
	HIP_TRY(ctx, hipStreamSynchronize(st));
	return 0;
}

int xdpgpu_nat64_dev(xdpgpu_ctx *ctx, void *d_umem, uint64_t umem_size,
		     const xdpgpu_desc *d_descs, uint32_t n, uint8_t *d_action,
		     xdpgpu_desc *d_out, void *stream)
{
	if (!ctx || !d_umem || !d_descs || !d_action || !d_out)
		return -EINVAL;
	if (!ctx->nat64)
		return set_err(ctx, -EINVAL, "xdpgpu_nat64_setup not called");
	if (n == 0)
		return 0;
	if (int rc0 = check_dev_all(ctx, {{"UMEM", d_umem}, {"descriptors", d_descs},
					  {"actions", d_action}, {"output descriptors", d_out}}))
		return rc0;
	Nat64Args a;
	memset(&a, 0, sizeof(a));
	a.umem = (uint8_t *)d_umem;
	a.usize = umem_size;
	a.desc = d_descs;
	a.n = n;
	a.action = d_action;
	a.out = d_out;
	a.cfg = ctx->ncfg;
	a.v6map = ctx->d_v6map;
	a.v6nb = ctx->nb;
	const bool dyn = ctx->ndyn && ctx->ncfg.direction == XDPGPU_NAT64_INGRESS;
	uint64_t now = 0;
	if (dyn) {
		/* one instant per batch (bpf_ktime_get_ns, CLOCK_MONOTONIC) */
		now = ctx->nclock;
		if (!now) {
			struct timespec ts;
			clock_gettime(CLOCK_MONOTONIC, &ts);
			now = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
		}
		if (n > ctx->mcap) {
			for (void *p : {(void *)ctx->d_midx, (void *)ctx->d_msrc,
					(void *)ctx->d_mov})
				if (p)
					(void)hipFree(p);
			ctx->d_midx = nullptr;
			ctx->d_msrc = nullptr;
			ctx->d_mov = nullptr;
			ctx->mcap = 0;
			const uint64_t cap = ((uint64_t)n + 63) & ~63ull;
			if (hipMalloc(&ctx->d_midx, cap * 4) != hipSuccess ||
			    hipMalloc(&ctx->d_msrc, cap * 16) != hipSuccess ||
			    hipMalloc(&ctx->d_mov, cap * 8) != hipSuccess)
				return set_err(ctx, -ENOMEM, "nat64 miss lists of %u", n);
			ctx->mcap = cap;
		}
		if (!ctx->d_mcnt && hipMalloc(&ctx->d_mcnt, 16) != hipSuccess)
			return set_err(ctx, -ENOMEM, "nat64 miss count");
		a.dyn = 1;
		a.now = now;
		a.thr = now - ctx->nst.timeout_ns;
		a.miss_idx = ctx->d_midx;
		a.miss_src = ctx->d_msrc;
		a.miss_cnt = ctx->d_mcnt;
	}
	a.v4map = ctx->d_v4map;
	a.v4nb = ctx->nb;
	/* the fast kernels cover both directions under a /96 prefix; they
	 * share slot 0's deferral-list scratch with the RX path (a context
	 * runs one launch sequence at a time) */
	a.fast = ctx->ncfg.v6_plen == 96;
	a.diag = (ctx->cfg.tune >> 12) & 3;
	if (a.fast) {
		int rc = ensure_xlist(ctx, ctx->slot[0], n);
		if (rc)
			return rc;
		a.xlist = ctx->slot[0].d_xlist;
		a.xcount = ctx->slot[0].d_xcount;
		a.xcap = ctx->slot[0].xcap;
		/* shared tiles (cfg.tune bit 14: none): 12/16 of the batch */
		a.steal = ctx->slot[0].d_steal;
		a.steal_set = ctx->slot[0].steal_set;
		a.steal_16ths = (ctx->cfg.tune >> 14) & 1 ? 0u : 12u;
		for (int k = 0; k < 4; k++) {
			uint8_t m[4], w[4];
			for (int j = 0; j < 4; j++) {
				const uint32_t bit0 = 8 * (4 * k + j);
				const uint32_t pl = ctx->ncfg.allow_plen;
				const uint32_t nb = pl <= bit0 ? 0 : pl - bit0 >= 8 ? 8 : pl - bit0;
				m[j] = (uint8_t)(nb ? (0xff00u >> nb) & 0xff : 0);
				w[j] = ctx->ncfg.allow_prefix[4 * k + j] & m[j];
			}
			memcpy(&a.allow_m[k], m, 4);
			memcpy(&a.allow_w[k], w, 4);
		}
		memcpy(a.pref_w, ctx->ncfg.v6_prefix, 12);
	}
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	/* the shared-tile heads and the dynamic-state miss list are the
	 * context's: ordered after their last user on another stream */
	int rc = scratch_enter(ctx, ctx->slot[0], st);
	if (rc)
		return rc;
	if (dyn)
		HIP_TRY(ctx, hipMemsetAsync(ctx->d_mcnt, 0, 16, st));
	HIP_TRY(ctx, launch_nat64(a, ctx->max_blocks, st));
	/* the fast kernel zeroed the other counter set (as the RX launch) */
	if (a.fast)
		ctx->slot[0].steal_set ^= 1;
	rc = scratch_leave(ctx, ctx->slot[0], st);
	if (rc)
		return rc;
	return dyn ? nat64_commit(ctx, a, now, st) : 0;
}

int xdpgpu_synproxy_dev(xdpgpu_ctx *ctx, void *d_umem, uint64_t umem_size,
			const xdpgpu_desc *d_descs, uint32_t n, const xdpgpu_synproxy_cfg *cfg,
			uint8_t *d_verdict, xdpgpu_desc *d_out, uint64_t *d_synacks, void *stream)
{
	if (!ctx || !d_umem || !d_descs || !cfg || !d_verdict || !d_out)
		return -EINVAL;
	if (n == 0)
		return 0;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	if (int rc0 = check_dev_all(ctx, {{"UMEM", d_umem}, {"descriptors", d_descs},
					  {"verdicts", d_verdict}, {"output descriptors", d_out},
					  {"SYN-ACK count", d_synacks}}))
		return rc0;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	if (d_synacks && !ctx->d_spread) {
		/* the SYN-ACK counters, zeroed once: each launch's sum kernel
		 * clears them (launches of one context are stream-ordered) */
		const size_t bytes = (size_t)synproxy_spread_words() * 8;
		if (hipMalloc(&ctx->d_spread, bytes) != hipSuccess)
			return set_err(ctx, -ENOMEM, "synproxy counters");
		HIP_TRY(ctx, hipMemset(ctx->d_spread, 0, bytes));
	}
	/* the counters are the context's: a launch on another stream waits
	 * for the last launch that used them (its sum kernel reads and
	 * clears them), as the context's launches are ordered (xdpgpu.h) */
	int rc = scratch_enter(ctx, ctx->slot[0], st);
	if (rc)
		return rc;
	HIP_TRY(ctx, launch_synproxy((uint8_t *)d_umem, umem_size, d_descs, n, *cfg, d_verdict,
				     d_out, (unsigned long long *)d_synacks, ctx->d_spread, st));
	return scratch_leave(ctx, ctx->slot[0], st);
}

int xdpgpu_ceiling_dev(xdpgpu_ctx *ctx, const void *d_umem, uint64_t umem_size,
		       const xdpgpu_desc *d_descs, uint32_t n, uint8_t *d_verdict,
		       void *d_res, void *d_tuples, void *stream)
{
	if (!ctx || !d_umem || !d_descs || !d_verdict || !d_res || !d_tuples)
		return -EINVAL;
	if (n == 0)
		return 0;
	RxArgs a;
	memset(&a, 0, sizeof(a));
	a.umem = (uint8_t *)d_umem;
	a.usize = umem_size;
	a.desc = d_descs;
	a.n = n;
	a.verdict = d_verdict;
	a.res = (xdpgpu_result *)d_res;
	a.tup = (uint8_t *)d_tuples;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_ceiling(a, rx_grid_blocks(n, ctx->max_blocks), st));
	return 0;
}

/* The UMEM bytes a batch reads, as at most kMaxRuns runs of nearby frames
 * (gaps up to kRunGap bytes are copied along): one run for a batch of
 * consecutive frames, two for a batch that wraps round a cyclic fill ring,
 * found in descriptor order.  A batch scattered over the UMEM (more runs
 * than that in descriptor order: a recycled fill ring) is sorted by
 * address and merged with the smallest gap (kRunGap, x4, ...) that leaves
 * at most kMaxRuns runs, so that its copies stay few and close to the
 * bytes it names.  [lo, hi) is the span of all of them; used the bytes the
 * descriptors name.  +1 byte per frame: udp_csum's odd over-read. */
struct Run {
	uint64_t lo, hi;
};
constexpr uint64_t kRunGap = 4096;
constexpr size_t kMaxRuns = 64;

static void batch_runs(const xdpgpu_ctx *ctx, const xdpgpu_desc *descs,
		       uint32_t n, std::vector<Run> &runs, uint64_t &lo,
		       uint64_t &hi, uint64_t &used)
{
	runs.clear();
	lo = UINT64_MAX;
	hi = 0;
	used = 0;
	bool scattered = false;
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t eff = (descs[i].addr & ((1ull << 48) - 1)) +
				     (descs[i].addr >> 48);
		if (eff >= ctx->umem_size)
			continue;
		uint64_t end = eff + descs[i].len + 1;
		if (end > ctx->umem_size)
			end = ctx->umem_size;
		lo = std::min(lo, eff);
		hi = std::max(hi, end);
		used += descs[i].len;
		if (scattered)
			continue;
		if (!runs.empty() && eff >= runs.back().lo &&
		    eff <= runs.back().hi + kRunGap) {
			runs.back().hi = std::max(runs.back().hi, end);
			continue;
		}
		if (runs.size() == kMaxRuns) {
			scattered = true;
			continue;
		}
		runs.push_back({eff, end});
	}
	if (!scattered)
		return;
	std::vector<Run> fr;
	fr.reserve(n);
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t eff = (descs[i].addr & ((1ull << 48) - 1)) +
				     (descs[i].addr >> 48);
		if (eff < ctx->umem_size)
			fr.push_back({eff, std::min<uint64_t>(eff + descs[i].len + 1,
							     ctx->umem_size)});
	}
	std::sort(fr.begin(), fr.end(), [](const Run &x, const Run &y) { return x.lo < y.lo; });
	for (uint64_t gap = kRunGap;; gap *= 4) {
		runs.clear();
		for (const Run &r : fr) {
			if (!runs.empty() && r.lo <= runs.back().hi + gap)
				runs.back().hi = std::max(runs.back().hi, r.hi);
			else
				runs.push_back(r);
		}
		if (runs.size() <= kMaxRuns)
			return;
	}
}

/* Chunked UMEMs (aligned mode, register_umem's chunk_size; the reference's
 * geometry is 4 KiB chunks, af_xdp_user.c:56-57, xdpsock.c:133, with each
 * frame at its chunk's headroom): the bytes a batch names are one window
 * [off_lo, off_hi) of each chunk it uses, the same offsets in every chunk
 * (the kernel's XDP_PACKET_HEADROOM plus the UMEM headroom, plus the
 * frame).  They go over as rows: runs of consecutive chunk indices c0..c1
 * (gaps of up to kRowGap unused chunks copied along), one pitched copy per
 * run, pitch = the chunk, width = the window.  A 64 B frame in a 4 KiB
 * chunk then moves its own line, where the span copy of batch_runs moves
 * the whole chunk.  False when the rows do not pay (the window is half the
 * chunk or more: frames fill their chunks) or do not hold (a frame whose
 * udp_csum over-read byte lies in the next chunk): the caller copies
 * spans. */
struct Rows {
	uint64_t c0, c1;
};
constexpr uint64_t kRowGap = 8;

static bool batch_rows(const xdpgpu_ctx *ctx, const xdpgpu_desc *descs, uint32_t n,
		       std::vector<Rows> &rows, uint64_t &off_lo, uint64_t &off_hi,
		       uint64_t &used)
{
	rows.clear();
	used = 0;
	if (!ctx->chunk)
		return false;
	const uint64_t mask = ctx->chunk - 1;
	const uint32_t sh = ctx->chunk_shift;
	off_lo = UINT64_MAX;
	off_hi = 0;
	bool scattered = false;
	for (uint32_t i = 0; i < n; i++) {
		const uint64_t eff = descs[i].addr;
		/* an offset field in aligned mode: decoded as the kernel decodes
		 * it (addr>>48 added), by the span path */
		if (eff >> 48)
			return false;
		if (eff >= ctx->umem_size)
			continue;
		const uint64_t off = eff & mask;
		const uint64_t end = off + descs[i].len + 1;
		if (end > ctx->chunk)
			return false;
		off_lo = std::min(off_lo, off);
		off_hi = std::max(off_hi, end);
		used += descs[i].len;
		if (scattered)
			continue;
		const uint64_t c = eff >> sh;
		if (!rows.empty() && c >= rows.back().c0 && c <= rows.back().c1 + kRowGap) {
			rows.back().c1 = std::max(rows.back().c1, c);
			continue;
		}
		if (rows.size() == kMaxRuns) {
			scattered = true;
			continue;
		}
		rows.push_back({c, c});
	}
	if (off_hi <= off_lo || 2 * (off_hi - off_lo) > ctx->chunk) {
		/* (an empty window: no frame in the UMEM; rows: none to copy) */
		if (off_hi <= off_lo) {
			rows.clear();
			return true;
		}
		return false;
	}
	if (!scattered)
		return true;
	std::vector<uint64_t> cs;
	cs.reserve(n);
	for (uint32_t i = 0; i < n; i++)
		if (descs[i].addr < ctx->umem_size)
			cs.push_back(descs[i].addr >> sh);
	std::sort(cs.begin(), cs.end());
	cs.erase(std::unique(cs.begin(), cs.end()), cs.end());
	for (uint64_t gap = kRowGap;; gap *= 4) {
		rows.clear();
		for (uint64_t c : cs) {
			if (!rows.empty() && c <= rows.back().c1 + gap)
				rows.back().c1 = c;
			else
				rows.push_back({c, c});
		}
		if (rows.size() <= kMaxRuns)
			return true;
	}
}

/* XDPGPU_CFG_UMEM_GATHER: the RX launch's window wants the batch's mean
 * frame length (xdpgpu.h: a performance choice, the outputs are the same
 * whatever the window), which a sample of up to 4096 descriptors gives;
 * the gather itself needs no pass over the batch on the host (its bytes are
 * counted on the device). */
static uint64_t sampled_used(const xdpgpu_desc *descs, uint32_t n)
{
	const uint32_t step = n > 4096 ? n / 4096 : 1;
	uint64_t sum = 0, cnt = 0;
	for (uint32_t i = 0; i < n; i += step, cnt++)
		sum += descs[i].len;
	return cnt ? sum * n / cnt : 0;
}

/* The device view of a page-locked host array (hipHostMalloc'd or
 * registered), else null (pageable memory) */
static const void *host_view(const void *p)
{
	hipPointerAttribute_t at;
	memset(&at, 0, sizeof(at));
	if (hipPointerGetAttributes(&at, p) != hipSuccess) {
		(void)hipGetLastError();
		return nullptr;
	}
	if (at.type != hipMemoryTypeHost || !at.devicePointer)
		return nullptr;
	/* p may lie inside the allocation: the same offset from the device
	 * view of the host pointer the attributes name */
	if (at.hostPointer && (const char *)p >= (const char *)at.hostPointer)
		return (const char *)at.devicePointer +
		       ((const char *)p - (const char *)at.hostPointer);
	return at.devicePointer;
}

/* XDPGPU_CFG_UMEM_GATHER: the gather kernel moves the batch's frame bytes
 * into the slot's mirror.  hdesc: the descriptors' device view when the
 * caller's array is page-locked; the kernel then also writes their device
 * copy (s.d_desc), so that no descriptor copy waits on the copy engine
 * behind the other slot's output copies (rocprof timeline,
 * profiles/r05_gather: one engine runs every copy in order, and a
 * descriptor upload queued behind the previous batch's results kept the
 * next gather from starting).  Otherwise s.d_desc was uploaded first.
 * (The two slots' gathers run at once; one stream for both, the gathers
 * back to back, held each slot's kernels behind the other slot's gather:
 * 226 vs 239 M frames/s.) */
static int gather_batch(xdpgpu_ctx *ctx, Slot &s, uint32_t n, const xdpgpu_desc *hdesc)
{
	GatherArgs g;
	memset(&g, 0, sizeof(g));   /* poff null: the pieces at their UMEM offsets */
	g.src = ctx->d_hview;
	g.mirror = s.d_mirror;
	g.usize = ctx->umem_size;
	g.desc = s.d_desc;
	g.hdesc = hdesc;
	g.n = n;
	g.over_all = (ctx->cfg.flags & XDPGPU_CFG_FRAGS) ? 1u : 0u;
	g.nbytes = ctx->d_gbytes;
	HIP_TRY(ctx, launch_umem_gather(g, s.stream));
	ctx->hstats.umem_copies++;
	ctx->hstats.umem_gathers++;
	return 0;
}

/* XDPGPU_CFG_HOST_COMPACT's default thread count: XDPGPU_HOST_THREADS, else
 * the CPUs this process may run on (affinity set, cgroup v2 CPU quota), at
 * most 16. */
static unsigned default_host_threads()
{
	if (const char *e = getenv("XDPGPU_HOST_THREADS")) {
		const int v = atoi(e);
		if (v > 0)
			return (unsigned)std::min(v, 64);
	}
	unsigned n = 1;
	cpu_set_t set;
	CPU_ZERO(&set);
	if (sched_getaffinity(0, sizeof(set), &set) == 0)
		n = std::max(1, CPU_COUNT(&set));
	if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
		char q[32];
		long long period = 0;
		if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") && period > 0)
			n = std::min<unsigned>(n, (unsigned)std::max(1LL, atoll(q) / period));
		fclose(f);
	}
	return std::min(n, 16u);
}

static HostPool *host_pool(xdpgpu_ctx *ctx)
{
	if (!ctx->hpool)
		ctx->hpool = new (std::nothrow) HostPool(ctx->host_threads ? ctx->host_threads
								: default_host_threads());
	return ctx->hpool;
}

/* Page-locked and device staging of a slot for `bytes` packed bytes and n
 * piece offsets (grown by a quarter more than asked; the slot is idle). */
static int ensure_pack(xdpgpu_ctx *ctx, Slot &s, uint64_t bytes, uint32_t n)
{
	if (s.pack_cap < bytes + 64) {
		const uint64_t cap = bytes + bytes / 4 + 64;
		(void)hipFree(s.d_pack);
		staging_free(s.h_pack);
		s.d_pack = nullptr;
		s.h_pack = nullptr;
		s.pack_cap = 0;
		if (!(s.h_pack = (uint8_t *)staging_alloc(cap)) ||
		    hipMalloc(&s.d_pack, cap) != hipSuccess)
			return set_err(ctx, -ENOMEM, "compaction staging of %llu bytes",
				       (unsigned long long)cap);
		s.pack_cap = cap;
	}
	if (s.poff_cap < n) {
		const uint64_t cap = (uint64_t)n + n / 4 + 64;
		(void)hipFree(s.d_poff);
		staging_free(s.h_poff);
		s.d_poff = nullptr;
		s.h_poff = nullptr;
		s.poff_cap = 0;
		if (!(s.h_poff = (uint32_t *)staging_alloc(cap * 4)) ||
		    hipMalloc(&s.d_poff, cap * 4) != hipSuccess)
			return set_err(ctx, -ENOMEM, "compaction offsets");
		s.poff_cap = cap;
	}
	return 0;
}

/* XDPGPU_CFG_HOST_COMPACT: the host threads pack the batch's pieces, the
 * bytes umem_gather_kernel would read for each frame ([eff & ~15,
 * round_up(end, 16)) clamped to the UMEM, end = eff + len + udp_csum's
 * over-read byte where it can count), into the slot's page-locked staging
 * buffer at 16-byte aligned offsets, in descriptor order: a first pass
 * sizes each thread's share of the descriptors, a second copies it (the
 * reference's frames sit one per 4 KiB chunk, af_xdp_user.c:56-57, so each
 * copy is one or two cache lines from its own page; the source of the
 * frame eight ahead is prefetched).  Then one transfer of the packed bytes
 * and their offsets, and the gather kernel in its packed form puts each
 * piece at its UMEM offset of the slot's mirror. */
static int compact_batch(xdpgpu_ctx *ctx, Slot &s, const xdpgpu_desc *descs, uint32_t n,
			 uint64_t &used)
{
	HostPool *pool = host_pool(ctx);
	if (!pool)
		return set_err(ctx, -ENOMEM, "host threads");
	struct timespec ts0, ts1;
	clock_gettime(CLOCK_MONOTONIC, &ts0);
	const unsigned T = pool->size();
	const uint64_t usize = ctx->umem_size;
	const uint32_t over_all = (ctx->cfg.flags & XDPGPU_CFG_FRAGS) ? 1u : 0u;
	const uint8_t *umem = ctx->h_umem;
	/* frame d's piece [lo, hi) of the UMEM; false: it names no bytes */
	auto piece = [usize, over_all](const xdpgpu_desc &d, uint64_t &lo, uint64_t &hi) {
		const uint64_t eff = (d.addr & ((1ull << 48) - 1)) + (d.addr >> 48);
		if (eff >= usize || (uint64_t)d.len > usize - eff)
			return false;
		uint64_t end = eff + d.len + ((over_all | d.len) & 1);
		if (end > usize)
			end = usize;
		lo = eff & ~15ull;
		hi = std::min<uint64_t>((end + 15) & ~15ull, usize);
		return true;
	};
	/* The batch in kParts parts of T shares each; one fork-join of the
	 * threads for the whole batch (a wake-up of the pool can cost more
	 * than a part on a loaded host): every thread sizes its shares,
	 * thread 0 sums them into offsets (and grows the staging),
	 * then each part is packed and, once all of its shares are in, the
	 * calling thread (thread 0) issues its transfer, under the packing of
	 * the next part by the others.  (A 512 K batch of 64-byte frames:
	 * ≈ 0.9 ms of packing on 16 threads beside 0.9 ms of transfer.) */
	constexpr unsigned kParts = 4;
	const unsigned S = kParts * T;
	auto share = [n, S](unsigned k) { return (uint32_t)((uint64_t)n * k / S); };
	std::vector<uint64_t> base(S + 1, 0), lens(S, 0);
	std::atomic<unsigned> sized{0}, ready{0};
	std::atomic<unsigned> packed[kParts];
	for (unsigned q = 0; q < kParts; q++)
		packed[q].store(0, std::memory_order_relaxed);
	int rc = 0;
	uint64_t total = 0;
	uint64_t pack_ns = 0;
	auto spin = [](const std::atomic<unsigned> &v, unsigned want) {
		while (v.load(std::memory_order_acquire) < want)
			__builtin_ia32_pause();
	};
	pool->run([&](unsigned t) {
		for (unsigned q = 0; q < kParts; q++) {
			const unsigned k = q * T + t;
			uint64_t b = 0, l = 0;
			for (uint32_t i = share(k); i < share(k + 1); i++) {
				uint64_t lo, hi;
				if (piece(descs[i], lo, hi)) {
					b += (hi - lo + 15) & ~15ull;
					l += descs[i].len;
				}
			}
			base[k + 1] = b;
			lens[k] = l;
		}
		sized.fetch_add(1, std::memory_order_acq_rel);
		if (t == 0) {
			/* thread 0 (the caller's, whose HIP device is the
			 * context's): offsets once every share is sized, then the
			 * staging */
			spin(sized, T);
			used = 0;
			for (unsigned k = 0; k < S; k++) {
				base[k + 1] += base[k];
				used += lens[k];
			}
			total = base[S];
			if (total / 16 > UINT32_MAX)
				rc = set_err(ctx, -E2BIG, "batch of %llu packed bytes",
					     (unsigned long long)total);
			else
				rc = ensure_pack(ctx, s, total, n);
			ready.store(1, std::memory_order_release);
		}
		spin(ready, 1);
		if (rc)
			return;
		uint8_t *dst = s.h_pack;
		uint32_t *poff = s.h_poff;
		for (unsigned q = 0; q < kParts; q++) {
			const unsigned k = q * T + t;
			const uint32_t i1 = share(k + 1);
			uint64_t o = base[k];
			for (uint32_t i = share(k); i < i1; i++) {
				if (i + 8 < i1) {
					const xdpgpu_desc &f = descs[i + 8];
					const uint64_t e = (f.addr & ((1ull << 48) - 1)) + (f.addr >> 48);
					if (e < usize) {
						__builtin_prefetch(umem + e);
						__builtin_prefetch(umem + std::min(e + 64, usize - 1));
					}
				}
				uint64_t lo, hi;
				if (!piece(descs[i], lo, hi)) {
					poff[i] = 0;
					continue;
				}
				memcpy(dst + o, umem + lo, hi - lo);
				poff[i] = (uint32_t)(o >> 4);
				o += (hi - lo + 15) & ~15ull;
			}
			packed[q].fetch_add(1, std::memory_order_acq_rel);
			if (t)
				continue;
			/* thread 0: the part's transfer once every share is in */
			spin(packed[q], T);
			clock_gettime(CLOCK_MONOTONIC, &ts1);
			pack_ns += (uint64_t)(ts1.tv_sec - ts0.tv_sec) * 1000000000ull +
				   (uint64_t)ts1.tv_nsec - (uint64_t)ts0.tv_nsec;
			const uint64_t b0 = base[q * T], b1 = base[(q + 1) * T];
			if (b1 > b0 && !rc &&
			    hipMemcpyAsync(s.d_pack + b0, s.h_pack + b0, b1 - b0,
					   hipMemcpyHostToDevice, s.stream) != hipSuccess)
				rc = set_err(ctx, -EIO, "compaction transfer: %s",
					     hipGetErrorString(hipGetLastError()));
			clock_gettime(CLOCK_MONOTONIC, &ts0);
		}
	});
	if (rc)
		return rc;
	ctx->hstats.compact_ns += pack_ns;
	HIP_TRY(ctx, hipMemcpyAsync(s.d_poff, s.h_poff, (size_t)n * 4, hipMemcpyHostToDevice,
				    s.stream));
	GatherArgs g;
	memset(&g, 0, sizeof(g));
	g.src = s.d_pack;
	g.mirror = s.d_mirror;
	g.usize = usize;
	g.desc = s.d_desc;
	g.hdesc = nullptr;
	g.n = n;
	g.over_all = over_all;
	g.nbytes = nullptr;
	g.poff = s.d_poff;
	HIP_TRY(ctx, launch_umem_gather(g, s.stream));
	ctx->hstats.umem_h2d_bytes += total;
	ctx->hstats.desc_h2d_bytes += (uint64_t)n * 4;
	ctx->hstats.umem_copies++;
	ctx->hstats.umem_compacted++;
	return 0;
}

int xdpgpu_host_threads(xdpgpu_ctx *ctx, uint32_t n)
{
	if (!ctx)
		return -EINVAL;
	for (uint32_t i = 0; i < kSlots; i++)
		if (ctx->slot[i].busy)
			return set_err(ctx, -EBUSY, "slot %u in flight", i);
	const unsigned want = n ? std::min(n, 64u) : default_host_threads();
	if (!ctx->hpool || ctx->hpool->size() != want) {
		delete ctx->hpool;
		ctx->hpool = new (std::nothrow) HostPool(want);
		if (!ctx->hpool)
			return set_err(ctx, -ENOMEM, "host threads");
	}
	ctx->host_threads = n;
	return (int)ctx->hpool->size();
}

/* Copy a batch's frames into the slot's mirror: rows of chunks where they
 * pay (batch_rows), else spans (batch_runs).  Sets used (the bytes the
 * descriptors name) and adds the copy's bytes to the host stats. */
static int copy_batch(xdpgpu_ctx *ctx, Slot &s, const xdpgpu_desc *descs, uint32_t n,
		      uint64_t &used)
{
	std::vector<Rows> rows;
	uint64_t off_lo = 0, off_hi = 0;
	uint64_t bytes = 0, copies = 0;
	if (batch_rows(ctx, descs, n, rows, off_lo, off_hi, used)) {
		const uint64_t chunk = ctx->chunk, w = off_hi - off_lo;
		const uint32_t sh = ctx->chunk_shift;
		for (const Rows &r : rows) {
			uint64_t c1 = r.c1;
			/* a last chunk cut short by the UMEM's end: its row alone,
			 * clamped (the host UMEM is never read past its size) */
			if ((c1 << sh) + off_hi > ctx->umem_size) {
				const uint64_t a = (c1 << sh) + off_lo;
				if (a < ctx->umem_size) {
					HIP_TRY(ctx, hipMemcpyAsync(s.d_mirror + a, ctx->h_umem + a,
								    ctx->umem_size - a,
								    hipMemcpyHostToDevice, s.stream));
					bytes += ctx->umem_size - a;
					copies++;
				}
				if (c1 == r.c0)
					continue;
				c1--;
			}
			const uint64_t a = (r.c0 << sh) + off_lo, h = c1 - r.c0 + 1;
			if (h == 1)
				HIP_TRY(ctx, hipMemcpyAsync(s.d_mirror + a, ctx->h_umem + a, w,
							    hipMemcpyHostToDevice, s.stream));
			else
				HIP_TRY(ctx, hipMemcpy2DAsync(s.d_mirror + a, chunk, ctx->h_umem + a,
							      chunk, w, h, hipMemcpyHostToDevice,
							      s.stream));
			bytes += w * h;
			copies++;
		}
	} else {
		std::vector<Run> runs;
		uint64_t lo, hi;
		batch_runs(ctx, descs, n, runs, lo, hi, used);
		for (const Run &r : runs) {
			HIP_TRY(ctx, hipMemcpyAsync(s.d_mirror + r.lo, ctx->h_umem + r.lo, r.hi - r.lo,
						    hipMemcpyHostToDevice, s.stream));
			bytes += r.hi - r.lo;
			copies++;
		}
	}
	ctx->hstats.umem_h2d_bytes += bytes;
	ctx->hstats.umem_copies += copies;
	return 0;
}

int xdpgpu_host_stats(xdpgpu_ctx *ctx, struct xdpgpu_host_stats *out)
{
	if (!ctx || !out)
		return -EINVAL;
	*out = ctx->hstats;
	if (ctx->d_gbytes) {
		/* the gather kernels' bytes, counted on the device (batches
		 * still in flight may not be in yet) */
		unsigned long long b = 0;
		HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
		HIP_TRY(ctx, hipMemcpy(&b, ctx->d_gbytes, sizeof(b), hipMemcpyDeviceToHost));
		out->umem_h2d_bytes += b;
	}
	return 0;
}

int xdpgpu_submit(xdpgpu_ctx *ctx, uint32_t slot, const xdpgpu_desc *descs,
		  uint32_t n, uint8_t *verdict, xdpgpu_result *res,
		  void *tuples)
{
	if (!ctx || slot >= kSlots || !descs || !verdict)
		return -EINVAL;
	if (!ctx->h_umem)
		return set_err(ctx, -EINVAL, "no UMEM registered");
	if (n > ctx->cfg.max_batch)
		return -E2BIG;
	Slot &s = ctx->slot[slot];
	if (s.busy)
		return set_err(ctx, -EBUSY, "slot %u in flight", slot);
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	int rc = ensure_slot_buffers(ctx, s, n);
	if (rc)
		return rc;
	s.n = n;
	s.echo_pending = false;
	if (n == 0)
		return 0;

	/* the frames go to this slot's own mirror: a batch in flight on the
	 * other slot never sees them, whatever the two batches' addresses */
	uint64_t used = 0;
	const bool compact = ctx->cfg.flags & XDPGPU_CFG_HOST_COMPACT;
	const bool gather = !compact && ctx->d_hview != nullptr;
	if (gather)
		used = sampled_used(descs, n);
	const xdpgpu_desc *hdesc =
		gather ? (const xdpgpu_desc *)host_view(descs) : nullptr;
	if (!hdesc)
		HIP_TRY(ctx, hipMemcpyAsync(s.d_desc, descs, (size_t)n * sizeof(*descs),
					    hipMemcpyHostToDevice, s.stream));
	rc = compact ? compact_batch(ctx, s, descs, n, used)
	     : gather ? gather_batch(ctx, s, n, hdesc) : copy_batch(ctx, s, descs, n, used);
	if (rc)
		return rc;
	const bool echo = ctx->cfg.flags & XDPGPU_CFG_ICMP6_ECHO;
	uint8_t *d_tup = (tuples && ctx->cfg.tuple_fmt) ? s.d_tup : nullptr;
	/* the mean frame length picks the window (xdpgpu.h: 128 bytes when
	 * the frames average at least 128) */
	rc = enqueue_rx(ctx, s, s.d_mirror, ctx->umem_size, s.d_desc, n, s.d_verdict,
			res ? s.d_res : nullptr, d_tup, s.stream,
			std::max<uint64_t>(used / n, 1));
	ctx->hstats.batches++;
	ctx->hstats.frames += n;
	ctx->hstats.desc_h2d_bytes += (uint64_t)n * sizeof(*descs);
	ctx->hstats.out_d2h_bytes += (uint64_t)n * (1 + (res ? sizeof(*res) : 0) +
						     (d_tup ? tuple_bytes(ctx->cfg.tuple_fmt) : 0));
	if (rc)
		return rc;
	/* echo replies were written in the mirror: only the TX frames' first
	 * bytes go back to the host UMEM (SURVEY §8b ownership) */
	if (echo) {
		EchoArgs e;
		memset(&e, 0, sizeof(e));
		e.mirror = s.d_mirror;
		e.usize = ctx->umem_size;
		e.desc = s.d_desc;
		e.verdict = s.d_verdict;
		e.n = n;
		{
			if (s.erec_cap < n) {
				HIP_TRY(ctx, hipStreamSynchronize(s.stream));
				(void)hipFree(s.d_erec);
				free(s.h_erec);
				s.d_erec = nullptr;
				s.h_erec = nullptr;
				s.erec_cap = 0;
				const uint64_t cap = std::max<uint64_t>(n, 4096);
				s.h_erec = (EchoRec *)malloc(cap * sizeof(EchoRec));
				if (!s.h_erec ||
				    hipMalloc(&s.d_erec, cap * sizeof(EchoRec)) != hipSuccess)
					return set_err(ctx, -ENOMEM, "echo records");
				s.erec_cap = cap;
			}
			if (!s.d_ecnt &&
			    (hipMalloc(&s.d_ecnt, sizeof(uint32_t)) != hipSuccess ||
			     hipHostMalloc((void **)&s.h_ecnt, sizeof(uint32_t), 0) != hipSuccess))
				return set_err(ctx, -ENOMEM, "echo record count");
			HIP_TRY(ctx, hipMemsetAsync(s.d_ecnt, 0, sizeof(uint32_t), s.stream));
			e.rec = s.d_erec;
			e.nrec = s.d_ecnt;
			s.echo_pending = true;
		}
		HIP_TRY(ctx, launch_echo_writeback(e, s.stream));
		if (s.echo_pending)
			HIP_TRY(ctx, hipMemcpyAsync(s.h_ecnt, s.d_ecnt, sizeof(uint32_t),
						    hipMemcpyDeviceToHost, s.stream));
	}
	HIP_TRY(ctx, hipMemcpyAsync(verdict, s.d_verdict, n,
				    hipMemcpyDeviceToHost, s.stream));
	if (res)
		HIP_TRY(ctx, hipMemcpyAsync(res, s.d_res, (size_t)n * sizeof(*res),
					    hipMemcpyDeviceToHost, s.stream));
	if (d_tup)
		HIP_TRY(ctx, hipMemcpyAsync(tuples, d_tup,
					    (size_t)n * tuple_bytes(ctx->cfg.tuple_fmt),
					    hipMemcpyDeviceToHost, s.stream));
	HIP_TRY(ctx, hipEventRecord(s.done, s.stream));
	s.busy = true;
	return 0;
}

int xdpgpu_wait(xdpgpu_ctx *ctx, uint32_t slot)
{
	if (!ctx || slot >= kSlots)
		return -EINVAL;
	Slot &s = ctx->slot[slot];
	if (s.dev_pending) {
		s.dev_pending = false;
		HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
		HIP_TRY(ctx, hipStreamSynchronize(s.stream));
	}
	if (!s.busy)
		return 0;
	s.busy = false;
	HIP_TRY(ctx, hipEventSynchronize(s.done));
	if (s.echo_pending) {
		/* compact echo records: scatter each TX frame's first bytes */
		s.echo_pending = false;
		const uint32_t m = *s.h_ecnt;
		if (m) {
			HIP_TRY(ctx, hipMemcpyAsync(s.h_erec, s.d_erec, (size_t)m * sizeof(EchoRec),
						    hipMemcpyDeviceToHost, s.stream));
			HIP_TRY(ctx, hipStreamSynchronize(s.stream));
			for (uint32_t k = 0; k < m; k++)
				memcpy(ctx->h_umem + s.h_erec[k].eff, s.h_erec[k].b,
				       s.h_erec[k].len);
		}
	}
	return 0;
}

void *xdpgpu_host_alloc(uint64_t size)
{
	void *p = nullptr;
	if (!size || hipHostMalloc(&p, size, hipHostMallocPortable) != hipSuccess)
		return nullptr;
	return p;
}

void xdpgpu_host_free(void *p)
{
	if (p)
		(void)hipHostFree(p);
}

int xdpgpu_process(xdpgpu_ctx *ctx, const xdpgpu_desc *descs, uint32_t n,
		   uint8_t *verdict, xdpgpu_result *res, void *tuples)
{
	int rc = xdpgpu_submit(ctx, 0, descs, n, verdict, res, tuples);
	if (rc)
		return rc;
	return xdpgpu_wait(ctx, 0);
}

int xdpgpu_sync(xdpgpu_ctx *ctx, void *stream)
{
	if (!ctx)
		return -EINVAL;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	if (stream) {
		HIP_TRY(ctx, hipStreamSynchronize((hipStream_t)stream));
		return 0;
	}
	for (uint32_t i = 0; i < kSlots; i++)
		HIP_TRY(ctx, hipStreamSynchronize(ctx->slot[i].stream));
	return 0;
}

int xdpgpu_stats(xdpgpu_ctx *ctx, struct xdpgpu_stats *out)
{
	if (!ctx || !out)
		return -EINVAL;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	HIP_TRY(ctx, hipDeviceSynchronize());
	memset(out, 0, sizeof(*out));
	static thread_local unsigned long long host[kStatSlots * CNT_SLOT];
	for (uint32_t i = 0; i < kSlots; i++) {
		HIP_TRY(ctx, hipMemcpy(host, ctx->slot[i].d_stats, sizeof(host),
				       hipMemcpyDeviceToHost));
		for (uint32_t b = 0; b < kStatSlots; b++) {
			const unsigned long long *c = host + (size_t)b * CNT_SLOT;
			out->frames += c[CNT_FRAMES];
			out->bytes += c[CNT_BYTES];
			for (int v = 0; v < XDPGPU_NUM_VERDICTS; v++)
				out->verdict[v] += c[CNT_VERDICT0 + v];
			out->l3_bad += c[CNT_L3_BAD];
			out->l4_bad += c[CNT_L4_BAD];
			out->l4_absent += c[CNT_L4_ABSENT];
			out->frag += c[CNT_FRAG];
		}
	}
	return 0;
}

int xdpgpu_stats_reset(xdpgpu_ctx *ctx)
{
	if (!ctx)
		return -EINVAL;
	HIP_TRY(ctx, hipSetDevice(ctx->cfg.device));
	HIP_TRY(ctx, hipDeviceSynchronize());
	for (uint32_t i = 0; i < kSlots; i++)
		HIP_TRY(ctx, hipMemset(ctx->slot[i].d_stats, 0,
				       (size_t)kStatSlots * CNT_SLOT * 8));
	HIP_TRY(ctx, hipDeviceSynchronize());
	return 0;
}

int xdpgpu_jhash_dev(xdpgpu_ctx *ctx, const void *d_keys, uint32_t key_len,
		     uint32_t key_stride, uint32_t n, uint32_t initval,
		     uint32_t *d_out, void *stream)
{
	if (!ctx || (!d_keys && n) || (!d_out && n) || key_stride < key_len)
		return -EINVAL;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_jhash((const uint8_t *)d_keys, key_len, key_stride,
				  n, initval, d_out, st));
	return 0;
}

int xdpgpu_jhash2_dev(xdpgpu_ctx *ctx, const uint32_t *d_words, uint32_t nwords,
		      uint32_t word_stride, uint32_t n, uint32_t initval,
		      uint32_t *d_out, void *stream)
{
	if (!ctx || (!d_words && n && nwords) || (!d_out && n) || word_stride < nwords)
		return -EINVAL;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_jhash_words(d_words, nwords, word_stride, n, initval, 0, d_out,
					st));
	return 0;
}

int xdpgpu_jhash_nwords_dev(xdpgpu_ctx *ctx, const uint32_t *d_words, uint32_t nwords,
			    uint32_t word_stride, uint32_t n, uint32_t initval,
			    uint32_t *d_out, void *stream)
{
	if (!ctx || nwords < 1 || nwords > 3 || (!d_words && n) || (!d_out && n) ||
	    word_stride < nwords)
		return -EINVAL;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_jhash_words(d_words, nwords, word_stride, n, initval, nwords,
					d_out, st));
	return 0;
}

int xdpgpu_ip_fast_csum_dev(xdpgpu_ctx *ctx, const void *d_hdrs,
			    uint32_t hdr_stride, uint32_t n, uint16_t *d_out,
			    void *stream)
{
	if (!ctx || (!d_hdrs && n) || (!d_out && n) || hdr_stride < 60)
		return -EINVAL;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_ip_fast_csum((const uint8_t *)d_hdrs, hdr_stride, n,
					 d_out, st));
	return 0;
}

int xdpgpu_hints_dev(xdpgpu_ctx *ctx, const void *d_umem, uint64_t umem_size,
		     const xdpgpu_desc *d_descs, uint32_t n, uint32_t rx_time_btf_id,
		     uint32_t mark_btf_id, xdpgpu_hints *d_out, void *stream)
{
	if (!ctx || (n && (!d_umem || !d_descs || !d_out)))
		return -EINVAL;
	if (n == 0)
		return 0;
	if (int rc0 = check_dev_all(ctx, {{"UMEM", d_umem}, {"descriptors", d_descs},
					  {"hints", d_out}}))
		return rc0;
	hipStream_t st = stream ? (hipStream_t)stream : ctx->slot[0].stream;
	HIP_TRY(ctx, launch_hints((const uint8_t *)d_umem, umem_size, d_descs, n,
				  rx_time_btf_id, mark_btf_id, d_out, st));
	return 0;
}

} // extern "C"
