// SPDX-License-Identifier: GPL-2.0
/*
 * nat64_state.h - host side of the nat64 state tables (v6_state_map,
 * v4_reversemap and reclaimed_addrs, nat64-bpf/nat64_kern.c:17-46).
 *
 * The host keeps the authoritative copy of the tables' keys, values and
 * bucket words and the dynamic allocator's state (config.next_addr, the
 * reclaim queue, the insertion order); the device copy is what the kernels
 * probe, and it owns last_seen between commits (a hit stamps it).  A
 * commit takes the frames a batch listed (a miss, or a hit on a timed-out
 * entry) in frame order and replays alloc_new_state (:576-622) for each,
 * producing the IPv4 address every frame gets (0: SHOT) and the changed
 * table slots as patches for the device copy.
 */
#ifndef XDPGPU_NAT64_STATE_H
#define XDPGPU_NAT64_STATE_H

#include <deque>
#include <functional>
#include <map>
#include <vector>

#include "xdpgpu.h"
#include "xdpgpu_internal.h"

namespace xdpgpu {

class Nat64State {
public:
	/* Rebuild: `nb` buckets, the static entries (static_conf, last_seen
	 * 0) in order, a repeated key keeping its last value. */
	void build(const std::vector<xdpgpu_nat64_map> &statics, uint32_t nb);

	uint32_t buckets() const { return nb_; }
	const std::vector<Nat64V6Bucket> &v6() const { return v6_; }
	const std::vector<Nat64V4Bucket> &v4() const { return v4_; }

	/* dynamic allocation parameters (nat64_config, nat64.h:6-12) */
	uint32_t v4_prefix = 0, v4_mask = 0;
	uint64_t timeout_ns = 0, next_addr = 1;
	uint32_t cap = 0;                 /* num_addr (nat64.c:396) */

	/* The commit of one batch at time `now`.  idx/src: the listed frames
	 * (any order); out: the frames in order (sidx) and their addresses
	 * (ov); patches: the changed device slots.  devtab fills a copy of
	 * the device v6 table (last_seen), asked for at most once. */
	void commit(const uint32_t *idx, const uint4 *src, uint32_t m, uint64_t now,
		    const std::function<int(std::vector<Nat64V6Bucket> &)> &devtab,
		    std::vector<uint32_t> &sidx, std::vector<uint32_t> &ov,
		    std::vector<Nat64Patch> &patches, int &err);

	/* entries in insertion order, last_seen from `dev` (the device copy)
	 * where non-null */
	void entries(std::vector<xdpgpu_nat64_entry> &out,
		     const std::vector<Nat64V6Bucket> *dev) const;
	const std::deque<uint32_t> &queue() const { return queue_; }

private:
	bool find6(const uint32_t (&w)[4], uint32_t &slot) const;
	bool find4(uint32_t v4, uint32_t &slot) const;
	bool put6(const uint32_t (&w)[4], uint32_t v4, bool stat, uint64_t ls, uint32_t &slot);
	void put4(uint32_t v4, const uint32_t (&w)[4]);
	void erase6(uint32_t slot);
	void erase4(uint32_t slot);
	void touch(uint32_t table, uint32_t bucket, uint32_t slot);
	uint32_t reclaim(uint64_t now,
			 const std::function<int(std::vector<Nat64V6Bucket> &)> &devtab,
			 int &err);
	void push(uint32_t v4);

	uint32_t nb_ = 0;
	std::vector<Nat64V6Bucket> v6_;
	std::vector<Nat64V4Bucket> v4_;
	uint32_t count_ = 0;              /* v6 entries */
	std::map<uint64_t, uint32_t> order_;   /* insertion seq -> v6 slot */
	std::map<uint64_t, uint32_t> dorder_;  /* the same, dynamic entries */
	uint64_t cursor_ = 0;   /* per commit: the dynamic entries before this
				 * seq were seen not timed out (they stay so) */
	std::vector<uint64_t> seq_;            /* v6 slot -> insertion seq */
	uint64_t next_seq_ = 0;
	std::deque<uint32_t> queue_;           /* reclaimed_addrs, FIFO */
	/* per commit: the v6 slots written (their last_seen is the host's),
	 * the device copy, the touched slots as patch keys */
	std::vector<uint32_t> touched_;
	uint32_t epoch_ = 0;
	std::vector<Nat64V6Bucket> dev_;
	bool have_dev_ = false;
	std::map<uint64_t, uint32_t> pmap_;    /* (table, bucket, slot) */
};

} // namespace xdpgpu

#endif
