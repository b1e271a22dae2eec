# SPDX-License-Identifier: GPL-2.0
"""nat64 dynamic state: alloc_new_state, reclaim_v4_addr and
check_item (nat64-bpf/nat64_kern.c:543-622), the last_seen refresh of
nat64_handle_v6 (:809-828) and the map sizes of nat64.c:396-401.

CPU: the oracle's restatement (oracle/nat64_oracle.c, oracle_nat64_dyn)
against allocation sequences written down here from the reference's code:
pool order from next_addr = 1, a hit keeping its address, exhaustion at
(prefix | ~mask) - 1, reclaim of one timed-out entry at a time in the
reclaimed_addrs FIFO, static entries never reclaimed, the v6_state_map
capacity (num_addr, -E2BIG) and the v4_reversemap NOEXIST failure both
pushing the address back, and the u64 wrap of now - timeout_ns.  The
reference is a BPF program with no runnable harness here: these sequences
are builder-written expectations ("parity unpinned" at the reference level,
DESIGN.md §2); the order in which the reference's hash-map walk finds a
timed-out entry is the kernel's hash order, which this build fixes as
insertion order.

GPU: xdpgpu_nat64_dev with dynamic state, over several batches with the
clock advancing, bit-exact against the oracle: actions, output descriptors,
the UMEM after, and the state (entries in insertion order with last_seen,
next_addr, the reclaim queue).
"""
import ipaddress

import numpy as np
import pytest

import frames as F
import oracle
import xdpgpu
from test_nat64 import (EG, IN, NOSTATE, REDIR, SHOT, a4, a6, icmp6, ocfg, place, tcp,
                        udp, v4, v6)

T_OUT = 7200 * 10**9            # nat64.c default timeout (7200 s)
NOW0 = 10**13                   # a clock past the timeout (no u64 wrap)


def src(k):
    """the k-th source of the allowed /64 (2001:db8:1:2::/64)"""
    return a6(f"2001:db8:1:2::{k + 0x1000:x}")


def pool_cfg(direction=IN, mask_bits=16):
    cfg, _ = xdpgpu.nat64_pool_config(direction, 0)
    cfg.v4_mask = (0xFFFFFFFF << (32 - mask_bits)) & 0xFFFFFFFF
    return cfg


def v4s(x):
    return int(ipaddress.IPv4Address(x))


def dyn_frames(srcs, kinds=None):
    """one ingress frame per source: UDP, TCP or an echo request"""
    out = []
    for k, s in enumerate(srcs):
        kind = (kinds or "u")[k % len(kinds or "u")]
        if kind == "u":
            out.append(v6(udp(), 17, src=s))
        elif kind == "t":
            out.append(v6(tcp(), 6, src=s))
        elif kind == "e":
            out.append(v6(icmp6(128, 0, b"\x12\x34\x00\x01"), 58, src=s))
        elif kind == "v":        # VLAN-tagged: the general kernel
            out.append(v6(udp(), 17, src=s, tags=((0x8100, 5),)))
        elif kind == "b":        # ICMPv6 type the translator drops after the state
            out.append(v6(icmp6(135, 0), 58, src=s))
    return out


def srcaddr(fr_out):
    """IPv4 source of a translated (ingress) frame"""
    return int.from_bytes(bytes(fr_out[26:30]), "big")


def run(st, srcs, now, kinds=None):
    umem, descs = place(dyn_frames(srcs, kinds))
    u = umem.copy()
    act, out = st.run(u, descs, now)
    got = []
    for k in range(len(srcs)):
        if act[k] == REDIR:
            o = out[k]
            got.append(srcaddr(u[o["addr"]:o["addr"] + o["len"]]))
        else:
            got.append(int(act[k]) << 32)
    return got, act


def ostate(cfg, smap=(), timeout=T_OUT, next_addr=1):
    m = np.zeros(len(smap), xdpgpu.NAT64_MAP_DTYPE)
    for k, (s6, s4) in enumerate(smap):
        m[k]["v6"] = np.frombuffer(s6, np.uint8)
        m[k]["v4"] = s4
    return oracle.Nat64State(ocfg(cfg), m, timeout, next_addr), m


P = v4s("10.99.0.0")
SHOT_ = SHOT << 32


# ------------------------------------------------------------------ CPU tests
def test_oracle_first_sight_order():
    st, _ = ostate(pool_cfg())
    got, _ = run(st, [src(1), src(2), src(1), src(3), src(2)], NOW0)
    assert got == [P + 1, P + 2, P + 1, P + 3, P + 2]
    ent, nxt, q = st.state()
    assert nxt == 4 and len(q) == 0
    assert [int(e["v4"]) for e in ent] == [P + 1, P + 2, P + 3]
    assert all(int(e["last_seen"]) == NOW0 and not e["static_conf"] for e in ent)
    # a later batch refreshes last_seen of the sources it sees only
    run(st, [src(2)], NOW0 + 5)
    ent, _, _ = st.state()
    assert [int(e["last_seen"]) for e in ent] == [NOW0, NOW0 + 5, NOW0]


def test_oracle_exhaustion_and_reclaim():
    # /29: num_addr = 7 - 0 - 2 = 5, addresses .1-.5; .6 = max_v4 is never given
    cfg = pool_cfg(mask_bits=29)
    st, _ = ostate(cfg)
    got, _ = run(st, [src(k) for k in range(1, 7)], NOW0)
    assert got == [P + 1, P + 2, P + 3, P + 4, P + 5, SHOT_]   # nothing timed out
    ent, nxt, q = st.state()
    assert nxt == 6 and len(ent) == 5 and len(q) == 0
    # past the timeout: src 6 reclaims the first inserted entry (src 1);
    # src 1 then needs a new one and reclaims src 2's; src 3 is seen (kept)
    t1 = NOW0 + T_OUT + 1
    got, _ = run(st, [src(6), src(3), src(1), src(2)], t1)
    assert got == [P + 1, P + 3, P + 2, P + 4]
    ent, nxt, q = st.state()
    assert nxt == 6 and len(q) == 0
    assert [(bytes(e["v6"]), int(e["v4"])) for e in ent] == [
        (src(3), P + 3), (src(5), P + 5), (src(6), P + 1), (src(1), P + 2), (src(2), P + 4)]
    # exactly at the threshold (last_seen == now - timeout) is not timed out
    got, _ = run(st, [src(7)], NOW0 + T_OUT + T_OUT + 1)
    assert got == [P + 5]          # src 5 (last seen NOW0) goes, the others stay


def test_oracle_static_never_reclaimed():
    cfg = pool_cfg(mask_bits=29)
    st, _ = ostate(cfg, [(src(100), P + 5)])
    got, _ = run(st, [src(1), src(2), src(3), src(4)], NOW0)
    # with the static entry the table holds num_addr = 5 entries
    assert got == [P + 1, P + 2, P + 3, P + 4]
    got, _ = run(st, [src(5)], NOW0)
    # next .5: v6_state_map holds num_addr = 5 entries already -> -E2BIG
    assert got == [SHOT_]
    ent, nxt, q = st.state()
    assert nxt == 6 and list(q) == [P + 5]
    # much later, pool exhausted: every allocation pops the queued .5, finds
    # v6_state_map full and pushes it back; the walk is never reached
    t1 = NOW0 + 2 * T_OUT
    got, _ = run(st, [src(6), src(6)], t1)
    assert got == [SHOT_, SHOT_]
    ent, _, q = st.state()
    assert list(q) == [P + 5] and len(ent) == 5
    assert ent[0]["static_conf"] == 1 and bytes(ent[0]["v6"]) == src(100)


def test_oracle_reversemap_collision():
    # a static entry holds .2: the dynamic allocation of .2 fails at the
    # v4_reversemap insert, the v6 entry is removed and .2 queued
    cfg = pool_cfg(mask_bits=24)
    st, _ = ostate(cfg, [(src(100), P + 2)])
    got, _ = run(st, [src(1), src(2), src(3)], NOW0)
    assert got == [P + 1, SHOT_, P + 3]
    ent, nxt, q = st.state()
    assert nxt == 4 and list(q) == [P + 2] and len(ent) == 3


def test_oracle_timeout_wrap():
    # now < timeout: now - timeout_ns wraps (u64), every dynamic entry is
    # timed out at once
    cfg = pool_cfg(mask_bits=29)
    st, _ = ostate(cfg)
    got, _ = run(st, [src(k) for k in range(1, 8)], 1000)
    assert got == [P + 1, P + 2, P + 3, P + 4, P + 5, P + 1, P + 2]


def test_oracle_state_before_rewrite_failure():
    # the state is made before the ICMPv6 rewrite fails (nat64_kern.c:809-848)
    st, _ = ostate(pool_cfg())
    got, act = run(st, [src(1), src(2)], NOW0, kinds="bu")
    assert act[0] == SHOT and got[1] == P + 2
    ent, _, _ = st.state()
    assert [int(e["v4"]) for e in ent] == [P + 1, P + 2]


def test_oracle_egress_uses_dynamic_entries():
    cfg = pool_cfg()
    st, _ = ostate(cfg)
    run(st, [src(1), src(2)], NOW0)
    eg = pool_cfg(EG)
    st.cfg = ocfg(eg)
    umem, descs = place([v4(udp(), 17, dst=(P + 2).to_bytes(4, "big")),
                         v4(udp(), 17, dst=(P + 9).to_bytes(4, "big"))])
    act, out = st.run(umem, descs, NOW0 + 1)
    assert list(act) == [REDIR, SHOT]
    fr = umem[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    assert fr[38:54] == src(2)
    ent, _, _ = st.state()
    assert [int(e["last_seen"]) for e in ent] == [NOW0, NOW0]   # egress does not refresh


# ------------------------------------------------------------------ GPU tests
class GpuNat64:
    """xdpgpu_nat64_dev with dynamic state over device buffers"""

    def __init__(self, cfg, smap, timeout, next_addr=1):
        self.g = xdpgpu.XdpGpu(0)
        self.g.nat64_setup(cfg, smap)
        self.g.nat64_dynamic(timeout, next_addr)

    def run(self, umem, descs, now, direction=IN):
        import torch
        n = len(descs)
        dev = "cuda:0"
        d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
        d_umem[:umem.nbytes].copy_(torch.from_numpy(umem))
        d_desc = torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8)).to(dev)
        d_act = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
        d_out = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
        self.g.nat64_direction(direction)
        self.g.nat64_clock(now)
        self.g.nat64_dev(d_umem, umem.nbytes, d_desc, n, d_act, d_out,
                         torch.cuda.current_stream())
        torch.cuda.synchronize()
        return (d_act.cpu().numpy(), d_out.cpu().numpy().view(xdpgpu.DESC_DTYPE),
                d_umem.cpu().numpy()[:umem.nbytes])

    def close(self):
        self.g.close()


def same_state(g, o, what):
    ge, gn, gq = g.g.nat64_state()
    oe, on, oq = o.state()
    assert gn == on, f"{what}: next_addr {gn} != {on}"
    assert np.array_equal(gq, oq), f"{what}: queue {gq[:8]} != {oq[:8]}"
    assert len(ge) == len(oe), f"{what}: {len(ge)} entries != {len(oe)}"
    bad = np.nonzero(ge != oe)[0]
    assert len(bad) == 0, f"{what}: entries differ at {bad[:8]}: {ge[bad[:2]]} vs {oe[bad[:2]]}"


def batch_pool(rng, nsrc, n, kinds, skew=0):
    """n frames from nsrc sources, random order, mixed shapes, padded to the
    fast kernel's 64-byte minimum"""
    ks = rng.integers(1, nsrc + 1, n)
    frames = []
    for k in ks:
        kind = kinds[rng.integers(0, len(kinds))]
        fr = dyn_frames([src(int(k))], kind)[0]
        frames.append(fr + bytes(max(0, 96 - len(fr))))
    return place(frames, skew=skew)


def compare_batches(cfg, smap_list, timeout, batches, what):
    from test_nat64 import assert_nat64_same
    o, m = ostate(cfg, smap_list, timeout)
    g = GpuNat64(cfg, m, timeout)
    try:
        for b, (umem, descs, now, direction) in enumerate(batches):
            c = ocfg(cfg)
            c.direction = direction
            o.cfg = c
            u = umem.copy()
            wa, wo = o.run(u, descs, now)
            got = g.run(umem, descs, now, direction)
            assert_nat64_same(got, (wa, wo, u), f"{what} batch {b}")
            same_state(g, o, f"{what} batch {b}")
    finally:
        g.close()
        o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kinds", ["u", "utev", "utebv"])
def test_gpu_dyn_sequences(kinds):
    """small pool (/27: 29 addresses) under 60 sources: allocation,
    exhaustion, failures, reclaim across batches as the clock advances"""
    rng = np.random.default_rng(0x5EED0D0)
    cfg = pool_cfg(mask_bits=27)
    batches = []
    t = NOW0
    for b in range(6):
        umem, descs = batch_pool(rng, 60, 700, kinds, skew=8 if b % 3 == 2 else 0)
        batches.append((umem, descs, t, IN))
        t += T_OUT // 2 + 1
    compare_batches(cfg, [(src(200), P + 7)], T_OUT, batches, f"seq/{kinds}")


@pytest.mark.gpu
def test_gpu_dyn_scripted():
    """the CPU scripts above, on the GPU"""
    cfg = pool_cfg(mask_bits=29)
    seqs = [([src(k) for k in range(1, 7)], NOW0),
            ([src(6), src(3), src(1), src(2)], NOW0 + T_OUT + 1),
            ([src(7)], NOW0 + 2 * T_OUT + 1)]
    batches = []
    for s, t in seqs:
        umem, descs = place([fr + bytes(max(0, 96 - len(fr))) for fr in dyn_frames(s)])
        batches.append((umem, descs, t, IN))
    compare_batches(cfg, [], T_OUT, batches, "scripted")


@pytest.mark.gpu
def test_gpu_dyn_wrap_and_egress():
    """now < timeout (u64 wrap) with repeats inside one batch, then egress
    to the dynamic addresses with the shared tables"""
    rng = np.random.default_rng(7)
    cfg = pool_cfg(mask_bits=28)
    umem, descs = batch_pool(rng, 40, 500, "ut")
    frames = [v4(udp(), 17, dst=(P + k).to_bytes(4, "big")) for k in range(1, 20)]
    eu, ed = place([fr + bytes(max(0, 96 - len(fr))) for fr in frames])
    compare_batches(cfg, [], T_OUT, [(umem, descs, 1000, IN), (eu, ed, 2000, EG)],
                    "wrap/egress")


@pytest.mark.gpu
def test_gpu_dyn_large():
    """a 1 M-frame batch from 2000 sources over a /16 with 200 static
    entries (the fast kernel's path, with its shared tiles: 64 tiles per
    CU), then the same frames past the timeout (every dynamic entry timed
    out: all listed, all hits)"""
    rng = np.random.default_rng(11)
    cfg = pool_cfg(mask_bits=16)
    n, nsrc = 1 << 20, 2000
    ks = rng.integers(1, nsrc + 1, n)
    base = dyn_frames([src(1)], "u")[0]
    fr0 = base + bytes(max(0, 96 - len(base)))
    stride = 128
    umem = np.zeros(n * stride + 256, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    tmpl = np.frombuffer(fr0, np.uint8)
    umem[64:64 + n * stride].reshape(n, stride)[:, :len(fr0)] = tmpl
    descs["addr"] = np.arange(n, dtype=np.uint64) * stride + 64
    descs["len"] = len(fr0)
    # per-frame source: rewrite the last 16 bits of the source and fix the
    # UDP checksum incrementally (ones' complement of the difference)
    lo = (ks + 0x1000).astype(np.uint32)
    offs = descs["addr"].astype(np.int64)
    old = int.from_bytes(src(1)[14:16], "big")
    umem[offs + 14 + 22] = (lo >> 8).astype(np.uint8)
    umem[offs + 14 + 23] = (lo & 0xff).astype(np.uint8)
    c = umem[offs + 54 + 6].astype(np.uint32) << 8 | umem[offs + 54 + 7]
    s = (~c & 0xffff) + (~np.uint32(old) & 0xffff) + lo
    s = (s & 0xffff) + (s >> 16)
    s = (s & 0xffff) + (s >> 16)
    c2 = ~s & 0xffff
    c2[c2 == 0] = 0xffff
    umem[offs + 54 + 6] = (c2 >> 8).astype(np.uint8)
    umem[offs + 54 + 7] = (c2 & 0xff).astype(np.uint8)
    statics = [(src(50000 + k), P + 40000 + k) for k in range(200)]
    compare_batches(cfg, statics, T_OUT,
                    [(umem, descs, NOW0, IN), (umem, descs, NOW0 + T_OUT + 1, IN)],
                    "large")
