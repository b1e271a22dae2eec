// SPDX-License-Identifier: GPL-2.0
/*
 * nat64_state.cpp - the nat64 state tables on the host and the in-order
 * commit of dynamic allocations (see nat64_state.h).
 *
 * Reference: nat64-bpf/nat64_kern.c alloc_new_state (:576-622),
 * reclaim_v4_addr (:563-574), check_item (:543-561), the lookup and
 * last_seen refresh of nat64_handle_v6 (:809-828); map sizes nat64.c:396-401.
 */
#include "nat64_state.h"

#include <string.h>

#include <algorithm>

namespace xdpgpu {

static inline uint32_t home6(const uint32_t (&w)[4], uint32_t nb)
{
	return nat64_home(nat64_slot_hash(w[0], w[1], w[2], w[3]), nb);
}

static inline uint32_t home4(uint32_t v4, uint32_t nb)
{
	return nat64_home(nat64_slot_hash(v4, 0, 0, 0), nb);
}

void Nat64State::build(const std::vector<xdpgpu_nat64_map> &statics, uint32_t nb)
{
	nb_ = nb ? nb : 1;
	v6_.assign(nb_, Nat64V6Bucket());
	v4_.assign(nb_, Nat64V4Bucket());
	memset(v6_.data(), 0, (size_t)nb_ * sizeof(Nat64V6Bucket));
	memset(v4_.data(), 0, (size_t)nb_ * sizeof(Nat64V4Bucket));
	seq_.assign((size_t)nb_ * 4, 0);
	touched_.assign((size_t)nb_ * 4, 0);
	order_.clear();
	dorder_.clear();
	queue_.clear();
	count_ = 0;
	next_seq_ = 0;
	epoch_ = 0;
	for (const xdpgpu_nat64_map &e : statics) {
		uint32_t w[4], slot;
		memcpy(w, e.v6, 16);
		put6(w, e.v4, true, 0, slot);
		put4(e.v4, w);
	}
	pmap_.clear();
}

bool Nat64State::find6(const uint32_t (&w)[4], uint32_t &slot) const
{
	uint32_t b = home6(w, nb_);
	for (uint32_t p = 0; p < nb_; p++) {
		const Nat64V6Bucket &B = v6_[b];
		for (uint32_t j = 0; j < 4; j++) {
			if (((B.meta >> j) & 1) && B.key[j].x == w[0] && B.key[j].y == w[1] &&
			    B.key[j].z == w[2] && B.key[j].w == w[3]) {
				slot = b * 4 + j;
				return true;
			}
		}
		if (!(B.meta & kNat64Ovf))
			return false;
		b = b + 1 == nb_ ? 0 : b + 1;
	}
	return false;
}

bool Nat64State::find4(uint32_t v4, uint32_t &slot) const
{
	uint32_t b = home4(v4, nb_);
	for (uint32_t p = 0; p < nb_; p++) {
		const Nat64V4Bucket &B = v4_[b];
		for (uint32_t j = 0; j < 4; j++) {
			if (((B.meta >> j) & 1) && B.key[j] == v4) {
				slot = b * 4 + j;
				return true;
			}
		}
		if (!(B.meta & kNat64Ovf))
			return false;
		b = b + 1 == nb_ ? 0 : b + 1;
	}
	return false;
}

void Nat64State::touch(uint32_t table, uint32_t bucket, uint32_t slot)
{
	pmap_[(uint64_t)table << 40 | (uint64_t)bucket << 3 | slot] = 1;
}

/* an update of an existing key keeps its place; a new key takes the first
 * free slot from its home bucket on, marking the full buckets it passes */
bool Nat64State::put6(const uint32_t (&w)[4], uint32_t v4, bool stat, uint64_t ls,
		      uint32_t &slot)
{
	if (find6(w, slot)) {
		Nat64V6Bucket &B = v6_[slot >> 2];
		B.val[slot & 3] = v4;
		B.last_seen[slot & 3] = ls;
		B.meta = (B.meta & ~(1u << (8 + (slot & 3)))) | (stat ? 1u << (8 + (slot & 3)) : 0);
		if (stat)
			dorder_.erase(seq_[slot]);
		else
			dorder_[seq_[slot]] = slot;
		touch(0, slot >> 2, slot & 3);
		return true;
	}
	uint32_t b = home6(w, nb_);
	for (uint32_t p = 0; p < nb_; p++) {
		Nat64V6Bucket &B = v6_[b];
		const uint32_t fr = ~B.meta & 0xf;
		if (fr) {
			const uint32_t j = (uint32_t)__builtin_ctz(fr);
			B.key[j] = make_uint4(w[0], w[1], w[2], w[3]);
			B.val[j] = v4;
			B.last_seen[j] = ls;
			B.meta |= 1u << j;
			if (stat)
				B.meta |= 1u << (8 + j);
			slot = b * 4 + j;
			seq_[slot] = next_seq_;
			if (!stat)
				dorder_[next_seq_] = slot;
			order_[next_seq_++] = slot;
			count_++;
			touch(0, b, j);
			return true;
		}
		if (!(B.meta & kNat64Ovf)) {
			B.meta |= kNat64Ovf;
			touch(0, b, 4);
		}
		b = b + 1 == nb_ ? 0 : b + 1;
	}
	return false;
}

void Nat64State::put4(uint32_t v4, const uint32_t (&w)[4])
{
	uint32_t slot;
	if (find4(v4, slot)) {
		v4_[slot >> 2].val[slot & 3] = make_uint4(w[0], w[1], w[2], w[3]);
		touch(1, slot >> 2, slot & 3);
		return;
	}
	uint32_t b = home4(v4, nb_);
	for (uint32_t p = 0; p < nb_; p++) {
		Nat64V4Bucket &B = v4_[b];
		const uint32_t fr = ~B.meta & 0xf;
		if (fr) {
			const uint32_t j = (uint32_t)__builtin_ctz(fr);
			B.key[j] = v4;
			B.val[j] = make_uint4(w[0], w[1], w[2], w[3]);
			B.meta |= 1u << j;
			touch(1, b, j);
			return;
		}
		if (!(B.meta & kNat64Ovf)) {
			B.meta |= kNat64Ovf;
			touch(1, b, 4);
		}
		b = b + 1 == nb_ ? 0 : b + 1;
	}
}

void Nat64State::erase6(uint32_t slot)
{
	Nat64V6Bucket &B = v6_[slot >> 2];
	const uint32_t j = slot & 3;
	B.meta &= ~(1u << j | 1u << (8 + j));
	order_.erase(seq_[slot]);
	dorder_.erase(seq_[slot]);
	count_--;
	touch(0, slot >> 2, j);
}

void Nat64State::erase4(uint32_t slot)
{
	v4_[slot >> 2].meta &= ~(1u << (slot & 3));
	touch(1, slot >> 2, slot & 3);
}

/* bpf_map_push_elem on the queue of num_addr entries: -E2BIG when full */
void Nat64State::push(uint32_t v4)
{
	if (queue_.size() < cap)
		queue_.push_back(v4);
}

/* reclaim_v4_addr (nat64_kern.c:563-574): a queued address, else one
 * timed-out dynamic entry (check_item, :543-561: deleted from both maps,
 * its address queued; one entry at a time), else none.  The reference
 * walks v6_state_map in its hash order; this build walks insertion order. */
uint32_t Nat64State::reclaim(uint64_t now,
			     const std::function<int(std::vector<Nat64V6Bucket> &)> &devtab,
			     int &err)
{
	if (!queue_.empty()) {
		const uint32_t v = queue_.front();
		queue_.pop_front();
		return v;
	}
	/* static entries are never reclaimed: the walk covers the dynamic
	 * ones, from the commit's cursor (the entries before it were seen
	 * not timed out at this `now`, and an entry only leaves that state
	 * by a later batch) */
	const uint64_t thr = now - timeout_ns;   /* u64, as the reference */
	for (auto it = dorder_.lower_bound(cursor_); it != dorder_.end(); ++it) {
		const uint32_t slot = it->second, b = slot >> 2, j = slot & 3;
		cursor_ = it->first;
		uint64_t ls;
		if (touched_[slot] == epoch_) {
			ls = v6_[b].last_seen[j];
		} else {
			if (!have_dev_) {
				const int rc = devtab(dev_);
				if (rc) {
					err = rc;
					return 0;
				}
				have_dev_ = true;
			}
			ls = dev_[b].last_seen[j];
		}
		if (ls < thr) {
			const uint32_t v4 = v6_[b].val[j];
			uint32_t s4;
			erase6(slot);            /* invalidates it: leave the loop */
			if (find4(v4, s4))
				erase4(s4);
			push(v4);
			break;
		}
	}
	if (queue_.empty())
		return 0;
	const uint32_t v = queue_.front();
	queue_.pop_front();
	return v;
}

void Nat64State::commit(const uint32_t *idx, const uint4 *src, uint32_t m, uint64_t now,
			const std::function<int(std::vector<Nat64V6Bucket> &)> &devtab,
			std::vector<uint32_t> &sidx, std::vector<uint32_t> &ov,
			std::vector<Nat64Patch> &patches, int &err)
{
	err = 0;
	if (++epoch_ == 0) {
		std::fill(touched_.begin(), touched_.end(), 0u);
		epoch_ = 1;
	}
	have_dev_ = false;
	cursor_ = 0;
	pmap_.clear();
	std::vector<std::pair<uint32_t, uint32_t>> ord(m);
	for (uint32_t k = 0; k < m; k++)
		ord[k] = {idx[k], k};
	std::sort(ord.begin(), ord.end());
	sidx.resize(m);
	ov.resize(m);
	const uint32_t max_v4 = (v4_prefix | ~v4_mask) - 1;
	for (uint32_t q = 0; q < m && !err; q++) {
		const uint4 s = src[ord[q].second];
		const uint32_t w[4] = {s.x, s.y, s.z, s.w};
		sidx[q] = ord[q].first;
		uint32_t slot;
		if (find6(w, slot)) {
			/* present (an earlier frame made it, or timed out but
			 * not reclaimed): refresh last_seen, :821-823 */
			v6_[slot >> 2].last_seen[slot & 3] = now;
			touched_[slot] = epoch_;
			touch(0, slot >> 2, slot & 3);
			ov[q] = v6_[slot >> 2].val[slot & 3];
			continue;
		}
		/* alloc_new_state: the next pool address, else a reclaimed one */
		uint32_t src_v4 = 0;
		const uint32_t next_v4 = v4_prefix + (uint32_t)next_addr;
		if (next_v4 >= max_v4) {
			src_v4 = reclaim(now, devtab, err);
		} else {
			next_addr++;
			src_v4 = next_v4;
		}
		ov[q] = 0;
		if (!src_v4)
			continue;
		if (count_ >= cap) {         /* v6_state_map full: -E2BIG */
			push(src_v4);
			continue;
		}
		put6(w, src_v4, false, now, slot);
		touched_[slot] = epoch_;
		uint32_t s4;
		if (find4(src_v4, s4)) {     /* v4_reversemap NOEXIST fails */
			erase6(slot);
			push(src_v4);
			continue;
		}
		put4(src_v4, w);
		ov[q] = src_v4;
	}
	patches.clear();
	patches.reserve(pmap_.size());
	for (const auto &kv : pmap_) {
		const uint32_t table = (uint32_t)(kv.first >> 40);
		const uint32_t b = (uint32_t)((kv.first >> 3) & ((1ull << 37) - 1));
		const uint32_t j = (uint32_t)(kv.first & 7);
		Nat64Patch p;
		memset(&p, 0, sizeof(p));
		p.table = table;
		p.bucket = b;
		p.slot = j;
		if (table == 0) {
			p.meta = v6_[b].meta;
			if (j < 4) {
				p.k6 = v6_[b].key[j];
				p.v4 = v6_[b].val[j];
				p.last_seen = v6_[b].last_seen[j];
			}
		} else {
			p.meta = v4_[b].meta;
			if (j < 4) {
				p.v4 = v4_[b].key[j];
				p.k6 = v4_[b].val[j];
			}
		}
		patches.push_back(p);
	}
}

void Nat64State::entries(std::vector<xdpgpu_nat64_entry> &out,
			 const std::vector<Nat64V6Bucket> *dev) const
{
	out.clear();
	out.reserve(order_.size());
	for (const auto &kv : order_) {
		const uint32_t b = kv.second >> 2, j = kv.second & 3;
		xdpgpu_nat64_entry e;
		memset(&e, 0, sizeof(e));
		memcpy(e.v6, &v6_[b].key[j], 16);
		e.v4 = v6_[b].val[j];
		e.static_conf = (v6_[b].meta >> (8 + j)) & 1;
		e.last_seen = dev ? (*dev)[b].last_seen[j] : v6_[b].last_seen[j];
		out.push_back(e);
	}
}

} // namespace xdpgpu
