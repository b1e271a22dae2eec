# SPDX-License-Identifier: GPL-2.0
"""nat64 ICMP-error inner-header translation, the opt-in
XDPGPU_NAT64_F_ICMP_INNER (include/xdpgpu.h).

The reference leaves the IP header inside an ICMP error untranslated (the
FIXMEs at nat64-bpf/nat64_kern.c:438 and :736), so there is no reference
output to pin this against: every translated frame here is compared byte
for byte with a frame built in this file from RFC 7915 §4.3/§5.3 and the
outer field rules of nat64_handle_v4/_v6, with every checksum (outer IPv4
header, inner IPv4 header, ICMPv4 message, ICMPv6 message over its pseudo
header) recomputed in full (tests/golden/frames.py arithmetic), not updated
incrementally as the oracle and the GPU do.  The GPU is then bit-exact
against the oracle (actions, descriptors, UMEM), static and dynamic state.
"""
import struct

import numpy as np
import pytest

import frames as F
import oracle
import xdpgpu
from test_nat64 import (DST4, DST6, EG, IN, OK, REDIR, SHOT, SRC4, SRC6, a4, a6,
                        assert_nat64_same, gpu_nat64, icmp4, icmp6, ocfg, parse_l2, place,
                        run_oracle, v4, v6, v6hdr)

INNER = xdpgpu.NAT64_F_ICMP_INNER
HOST6, HOST4 = SRC6, DST4             # 2001:db8:1:2::5 <-> 10.99.0.5 (static map)
PEER6, PEER4 = DST6, a4("198.51.100.5")
ROUTER4 = SRC4                        # 198.51.100.7
PREF = a6("64:ff9b::")


def static4(addr6):
    """the pool config's static map: 2001:db8:1:2::k <-> 10.99.0.0 + k"""
    assert addr6[:8] == a6("2001:db8:1:2::")[:8]
    return struct.pack(">I", 0x0A630000 + int.from_bytes(addr6[8:], "big"))


def static6(addr4):
    k = int.from_bytes(addr4, "big") - 0x0A630000
    return a6("2001:db8:1:2::")[:8] + k.to_bytes(8, "big")


def embed(addr4):
    return PREF[:12] + addr4


def be16(b):
    return struct.unpack(">H", b)[0]


def csum_ip(h):
    return h[:10] + F.le16(~F.fold(F.ones_sum(h[:10] + b"\0\0" + h[12:])) & 0xFFFF) + h[12:]


# ------------------------------------------------------------ frame builders
def udp_seg(src, dst, v6_=True, n=24):
    seg = F.udp(5353, 33434, bytes(range(9, 9 + n)))
    c = F.l4_csum6(src, dst, 17, seg) if v6_ else F.l4_csum4(src, dst, 17, seg)
    return F.set_csum(seg, 6, c)


def tcp_seg(n=12):
    return F.tcp(443, 40001, bytes(range(1, 1 + n)))


def inner6(nh=17, seg=None, src=PEER6, dst=HOST6, hop=57, tc=0, plen=None, pre=b""):
    """the IPv6 packet an ICMPv6 error quotes (as the IPv6 host got it)"""
    if seg is None:
        seg = udp_seg(src, dst)
    return v6hdr(len(pre) + len(seg) if plen is None else plen, nh, src, dst, hop=hop,
                 tc=tc) + pre + seg


def inner4(proto=17, seg=None, src=HOST4, dst=PEER4, ttl=61, tos=0, options=b"", frag=0,
           tot=None, version=4):
    """the IPv4 packet an ICMPv4 error quotes (as the translator sent it)"""
    if seg is None:
        seg = udp_seg(src, dst, v6_=False)
    h = F.ipv4(len(seg), proto, src, dst, ttl=ttl, options=options, frag_off=frag,
               version=version,
               tot_len=None if tot is None else tot)
    h = csum_ip(h[:1] + bytes([tos]) + h[2:])
    return h + seg


def err6(t, c, rest, inner, src=HOST6, dst=PEER6, **kw):
    return v6(icmp6(t, c, rest, body=inner), 58, src=src, dst=dst, **kw)


def err4(t, c, rest, inner, src=ROUTER4, dst=HOST4, **kw):
    return v4(icmp4(t, c, rest, body=inner), 1, src=src, dst=dst, **kw)


def ingress_cases():
    """(name, frame, action, (type, code, rest) of the ICMPv4 header)"""
    c = []
    full = inner6()
    c.append(("port_unreach", err6(1, 4, bytes(4), full), REDIR, (3, 3, bytes(4))))
    c.append(("host_unreach_quoted_part", err6(1, 0, bytes(4), inner6(plen=1200)[:56]),
              REDIR, (3, 1, bytes(4))))
    c.append(("time_exceeded_tcp", err6(3, 0, bytes(4), inner6(6, tcp_seg())), REDIR,
              (11, 0, bytes(4))))
    c.append(("toobig_1400", err6(2, 0, struct.pack(">I", 1400), inner6(tc=0xb8), tc=0x48),
              REDIR, (3, 4, struct.pack(">HH", 0, 1380))))
    c.append(("paramprob_ptr8", err6(4, 0, struct.pack(">I", 8), full), REDIR,
              (12, 0, bytes([12, 0, 0, 8]))))
    c.append(("paramprob_nh", err6(4, 1, bytes(4), full), REDIR, (3, 2, bytes(4))))
    echo = bytes([128, 0, 0, 0, 0x12, 0x34, 0, 9]) + b"ping" * 4
    echo = F.set_csum(echo, 2, F.l4_csum6(PEER6, HOST6, 58, echo))
    c.append(("quoted_echo", err6(1, 4, bytes(4), inner6(58, echo)), REDIR,
              (3, 3, bytes(4))))
    # a router's error about a packet for another (static) host
    c.append(("other_host", err6(3, 0, bytes(4), inner6(dst=a6("2001:db8:1:2::9"))), REDIR,
              (11, 0, bytes(4))))
    c.append(("vlan", err6(1, 4, bytes(4), full, tags=((0x8100, 7),)), REDIR,
              (3, 3, bytes(4))))
    c.append(("qinq", err6(1, 4, bytes(4), full, tags=((0x88A8, 7), (0x8100, 8))), REDIR,
              (3, 3, bytes(4))))
    c.append(("hop_tc", err6(1, 3, bytes(4), inner6(hop=1, tc=0x2c), hop=33, tc=0x10),
              REDIR, (3, 1, bytes(4))))
    # not translatable: dropped
    c.append(("inner_dst_unmapped",
              err6(1, 4, bytes(4), inner6(dst=a6("2001:db8:1:2::1:0"))), SHOT, None))
    c.append(("inner_src_outside",
              err6(1, 4, bytes(4), inner6(src=a6("64:ff9c::c633:6405"))), SHOT, None))
    c.append(("inner_ext_hdr",
              err6(1, 4, bytes(4), inner6(0, pre=bytes([17]) + F.ext_opts(1))), SHOT, None))
    c.append(("inner_version4", err6(1, 4, bytes(4), inner4()), SHOT, None))
    c.append(("inner_cut", err6(1, 4, bytes(4), full[:30]), SHOT, None))
    c.append(("untranslatable_code", err6(1, 5, bytes(4), full), SHOT, None))
    short = bytearray(err6(1, 4, bytes(4), full))
    short[18:20] = struct.pack(">H", 47)          # payload_len < 8 + 40
    c.append(("outer_plen_47", bytes(short), SHOT, None))
    # not errors: exactly as without the flag
    c.append(("echo_req", v6(icmp6(128, 0, b"\x12\x34\x00\x01"), 58), REDIR, "plain"))
    c.append(("udp", v6(udp_seg(HOST6, PEER6), 17), REDIR, "plain"))
    c.append(("ipv4", v4(udp_seg(ROUTER4, HOST4, False), 17), OK, None))
    return c


def egress_cases():
    """(name, frame, action, (type, code, rest) of the ICMPv6 header)"""
    c = []
    full = inner4()
    c.append(("port_unreach", err4(3, 3, bytes(4), full), REDIR, (1, 4, bytes(4))))
    c.append(("host_unreach_quoted_part", err4(3, 1, bytes(4), inner4(tot=1200)[:28]),
              REDIR, (1, 0, bytes(4))))
    c.append(("fragneeded_1400", err4(3, 4, struct.pack(">HH", 0, 1400), inner4(tos=0xb8),
                                      tos=0x48),
              REDIR, (2, 0, struct.pack(">I", 1420))))
    c.append(("paramprob_ptr12", err4(12, 0, bytes([12, 0, 0, 0]), full), REDIR,
              (4, 0, struct.pack(">I", 8))))
    c.append(("proto_unreach", err4(3, 2, bytes(4), inner4(6, tcp_seg())), REDIR,
              (4, 1, struct.pack(">I", 6))))
    c.append(("inner_options", err4(3, 3, bytes(4), inner4(options=b"\x01" * 4)), REDIR,
              (1, 4, bytes(4))))
    c.append(("inner_ihl15", err4(3, 3, bytes(4), inner4(options=b"\x01" * 40)), REDIR,
              (1, 4, bytes(4))))
    echo = bytes([8, 0, 0, 0, 0, 7, 0, 1]) + b"pong" * 4
    echo = F.set_csum(echo, 2, ~F.fold(F.ones_sum(echo)) & 0xFFFF)
    c.append(("quoted_echo", err4(3, 3, bytes(4), inner4(1, echo)), REDIR, (1, 4, bytes(4))))
    c.append(("inner_df", err4(3, 3, bytes(4), inner4(frag=0x4000, ttl=1)), REDIR,
              (1, 4, bytes(4))))
    c.append(("ttl_tos", err4(3, 3, bytes(4), inner4(tos=0x2c), ttl=3, tos=0x10), REDIR,
              (1, 4, bytes(4))))
    # not translatable: dropped
    c.append(("inner_mf", err4(3, 3, bytes(4), inner4(frag=0x2000)), SHOT, None))
    c.append(("inner_frag_off", err4(3, 3, bytes(4), inner4(frag=0x0001)), SHOT, None))
    c.append(("inner_src_unmapped",
              err4(3, 3, bytes(4), inner4(src=a4("10.99.255.254"))), SHOT, None))
    c.append(("inner_cut", err4(3, 3, bytes(4), full[:12]), SHOT, None))
    c.append(("inner_options_cut", err4(3, 3, bytes(4), inner4(options=b"\x01" * 8)[:24]),
              SHOT, None))
    c.append(("inner_version6", err4(3, 3, bytes(4), inner6()), SHOT, None))
    short = bytearray(err4(3, 3, bytes(4), full))
    short[16:18] = struct.pack(">H", 20 + 8 + 19)  # tot_len < 20 + 8 + IHL
    c.append(("outer_tot_47", bytes(short), SHOT, None))
    c.append(("time_exceeded", err4(11, 0, bytes(4), full), SHOT, None))   # the reference's
    c.append(("untranslatable_code", err4(3, 14, bytes(4), full), SHOT, None))
    # not errors
    c.append(("echo", v4(icmp4(8, 0, b"\x00\x07\x00\x01"), 1, dst=HOST4), REDIR, "plain"))
    c.append(("udp", v4(udp_seg(ROUTER4, HOST4, False), 17, dst=HOST4), REDIR, "plain"))
    return c


# -------------------------------------------------- independent expectations
def want_ingress(fr, icmp_hdr):
    """the translated frame, built from the RFC rules with full checksums"""
    _, l3 = parse_l2(fr)
    o = fr[l3:l3 + 40]
    i6 = fr[l3 + 48:l3 + 88]
    rest = fr[l3 + 88:]
    tc = lambda h: ((h[0] & 0x0F) << 4) | (h[1] >> 4)
    nh = i6[6]
    h4i = struct.pack(">BBHHHBBH4s4s", 0x45, tc(i6), (be16(i6[4:6]) + 20) & 0xFFFF, 0, 0x4000,
                      i6[7], 1 if nh == 58 else nh, 0, i6[8 + 12:8 + 16], static4(i6[24:40]))
    h4i = csum_ip(h4i)
    t, c, r = icmp_hdr
    msg = bytes([t, c, 0, 0]) + r + h4i + rest
    msg = F.set_csum(msg, 2, ~F.fold(F.ones_sum(msg)) & 0xFFFF)
    plen = be16(o[4:6])
    assert plen == len(fr) - l3 - 40
    h4 = struct.pack(">BBHHHBBH4s4s", 0x45, tc(o), plen, 0, 0x4000, o[7], 1, 0,
                     static4(o[8:24]), o[24 + 12:40])
    h4 = csum_ip(h4)
    assert len(h4 + msg) == plen
    return fr[:12] + b"\x08\x00" + fr[14:l3] + h4 + msg


def want_egress(fr, icmp_hdr):
    _, l3 = parse_l2(fr)
    o = fr[l3:l3 + 20]
    i4 = fr[l3 + 28:]
    ihl = (i4[0] & 0xF) * 4
    rest = i4[ihl:]
    v6b = lambda tos: bytes([0x60 | ((tos & 0x70) >> 4), (tos << 4) & 0xFF, 0, 0])
    h6i = (v6b(i4[1]) + struct.pack(">HBB", (be16(i4[2:4]) - ihl) & 0xFFFF,
                                     58 if i4[9] == 1 else i4[9], i4[8]) +
           static6(i4[12:16]) + embed(i4[16:20]))
    t, c, r = icmp_hdr
    msg = bytes([t, c, 0, 0]) + r + h6i + rest
    src, dst = embed(o[12:16]), static6(o[16:20])
    assert be16(o[2:4]) - 20 == len(fr) - l3 - 20
    msg = F.set_csum(msg, 2, F.l4_csum6(src, dst, 58, msg))
    h6 = v6b(o[1]) + struct.pack(">HBB", len(msg), 58, o[8]) + src + dst
    return fr[:12] + b"\x86\xdd" + fr[14:l3] + h6 + msg


def inner_cfg(direction):
    cfg, smap = xdpgpu.nat64_pool_config(direction)
    cfg.flags = INNER
    return cfg, smap


# ------------------------------------------------------------------ CPU tests
@pytest.mark.parametrize("direction", [IN, EG])
def test_oracle_inner_vs_full_recompute(direction):
    cases = ingress_cases() if direction == IN else egress_cases()
    umem, descs = place([c[1] for c in cases])
    cfg, smap = inner_cfg(direction)
    act, out, u = run_oracle(umem, descs, direction, cfg=cfg, smap=smap)
    plain = run_oracle(umem, descs, direction)
    for k, (name, fr, want, hdr) in enumerate(cases):
        assert act[k] == want, f"{name}: action {act[k]} != {want}"
        lo = int(descs[k]["addr"])
        if want != REDIR:
            assert out[k] == descs[k], name
            assert np.array_equal(u[lo - 64:lo + len(fr)], umem[lo - 64:lo + len(fr)]), name
            continue
        o = out[k]
        got = u[o["addr"]:o["addr"] + o["len"]].tobytes()
        if hdr == "plain":
            # not an error: the reference's translation, untouched by the flag
            assert plain[0][k] == REDIR and out[k] == plain[1][k], name
            assert got == plain[2][o["addr"]:o["addr"] + o["len"]].tobytes(), name
            continue
        exp = want_ingress(fr, hdr) if direction == IN else want_egress(fr, hdr)
        assert got == exp, f"{name}: {got.hex()} != {exp.hex()}"
        shift = len(fr) - len(exp)
        assert int(o["addr"]) == lo + shift and int(o["len"]) == len(exp)
        # without the flag the same frame is the reference's outer-only translation
        assert plain[0][k] == REDIR
        assert int(plain[1][k]["addr"]) == lo + (20 if direction == IN else -20)


def test_oracle_inner_flag_off_is_reference():
    """the flag clear: every case as nat64_kern.c does it (outer only)"""
    for direction, cases in ((IN, ingress_cases()), (EG, egress_cases())):
        umem, descs = place([c[1] for c in cases])
        cfg, smap = xdpgpu.nat64_pool_config(direction)
        cfg2, _ = xdpgpu.nat64_pool_config(direction)
        assert cfg.flags == 0
        a1 = run_oracle(umem, descs, direction, cfg=cfg, smap=smap)
        a2 = run_oracle(umem, descs, direction)
        for x, y in zip(a1, a2):
            assert np.array_equal(x, y)
        shift = 20 if direction == IN else -20
        for k in np.nonzero(a1[0] == REDIR)[0]:
            assert int(a1[1][k]["addr"]) == int(descs[k]["addr"]) + shift


def test_oracle_inner_headroom():
    """egress needs 20 + (40 - IHL) bytes of UMEM in front: 40 for IHL 20,
    36 for 24 (each frame first in its UMEM)"""
    frames = [err4(3, 3, bytes(4), inner4()), err4(3, 3, bytes(4), inner4(options=bytes(4))),
              v4(udp_seg(ROUTER4, HOST4, False), 17, dst=HOST4)]
    cfg, smap = inner_cfg(EG)
    for headroom, want in ((40, [REDIR] * 3), (39, [SHOT, REDIR, REDIR]),
                           (36, [SHOT, REDIR, REDIR]), (35, [SHOT, SHOT, REDIR])):
        for fr, w in zip(frames, want):
            umem, descs = place([fr], headroom=headroom)
            act, _, _ = run_oracle(umem, descs, EG, cfg=cfg, smap=smap)
            assert act[0] == w, headroom


def packed(frames, headroom):
    """frames back to back, each behind `headroom` bytes of its own (a
    packed UMEM: a frame's headroom follows the previous frame's end)"""
    stride = max(len(f) for f in frames) + headroom
    stride = (stride + 63) & ~63
    return place(frames, headroom=headroom + 64, stride=stride)


def test_oracle_inner_packed_headroom():
    """cfg.headroom bounds egress growth by each frame's own headroom, not
    the UMEM's start: in a packed pool a frame that would grow into the
    previous frame is TC_ACT_SHOT and the previous frame is untouched"""
    frames = [err4(3, 3, bytes(4), inner4()), err4(3, 3, bytes(4), inner4(options=bytes(4))),
              v4(udp_seg(ROUTER4, HOST4, False), 17, dst=HOST4)] * 3
    for hr, want in ((40, [REDIR] * 3), (36, [SHOT, REDIR, REDIR]), (24, [SHOT, SHOT, REDIR]),
                     (16, [SHOT, SHOT, SHOT])):
        umem, descs = packed(frames, hr)
        cfg, smap = inner_cfg(EG)
        cfg.headroom = hr
        act, out, u = run_oracle(umem, descs, EG, cfg=cfg, smap=smap)
        assert list(act) == want * 3, hr
        # nothing written below each frame's own headroom
        for k in range(len(descs)):
            lo = int(descs[k]["addr"]) - hr
            prev_end = int(descs[k - 1]["addr"]) + int(descs[k - 1]["len"]) if k else 0
            assert np.array_equal(u[prev_end:lo], umem[prev_end:lo]), (hr, k)
        # without the bound the same pool grows into the gap in front
        cfg.headroom = 0
        act0, _, _ = run_oracle(umem, descs, EG, cfg=cfg, smap=smap)
        assert list(act0) == [REDIR] * 9


def dyn_state(direction, smap=()):
    from test_nat64_dyn import T_OUT, ostate, pool_cfg
    cfg = pool_cfg(direction)
    cfg.flags = INNER
    return ostate(cfg, smap, T_OUT)


def test_oracle_inner_dynamic():
    """dynamic state: the quoted destination must be the error's own source
    (its entry); the outer source's state is made even when the quoted
    header then fails"""
    from test_nat64_dyn import NOW0, P, src
    st, _ = dyn_state(IN)
    frames = [err6(1, 4, bytes(4), inner6(dst=src(1)), src=src(1)),
              err6(1, 4, bytes(4), inner6(dst=src(1)), src=src(2)),
              err6(1, 4, bytes(4), inner6(dst=src(3)), src=src(3))]
    umem, descs = place(frames)
    u = umem.copy()
    act, out = st.run(u, descs, NOW0)
    assert list(act) == [REDIR, SHOT, REDIR]
    ent, nxt, _ = st.state()
    assert nxt == 4 and [int(e["v4"]) for e in ent] == [P + 1, P + 2, P + 3]
    fr = u[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    assert fr[14 + 28 + 16:14 + 28 + 20] == struct.pack(">I", P + 1)   # inner daddr
    st.close()


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("direction", [IN, EG])
@pytest.mark.parametrize("headroom,skew", [(64, 0), (64, 1), (40, 4), (48, 8), (36, 0)])
def test_gpu_inner_cases(direction, headroom, skew):
    cases = ingress_cases() if direction == IN else egress_cases()
    umem, descs = place([c[1] for c in cases], headroom=headroom, skew=skew)
    cfg, smap = inner_cfg(direction)
    want = run_oracle(umem, descs, direction, cfg=cfg, smap=smap)
    assert (want[0] == REDIR).sum() >= 8
    got = gpu_nat64(umem, descs, direction, cfg, smap)
    assert_nat64_same(got, want, f"inner/{direction}/{headroom}/{skew}")


@pytest.mark.gpu
@pytest.mark.parametrize("hr", [40, 36, 24, 16])
def test_gpu_inner_packed_headroom(hr):
    """cfg.headroom on the GPU (fast and general kernels) against the
    oracle: the frames packed, each behind hr bytes of its own"""
    frames = [c[1] for c in egress_cases()] + [v4(udp_seg(ROUTER4, HOST4, False), 17,
                                                  dst=HOST4)] * 8
    umem, descs = packed(frames, hr)
    cfg, smap = inner_cfg(EG)
    cfg.headroom = hr
    want = run_oracle(umem, descs, EG, cfg=cfg, smap=smap)
    got = gpu_nat64(umem, descs, EG, cfg, smap)
    assert_nat64_same(got, want, f"inner-packed/{hr}")


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [IN, EG])
def test_gpu_inner_mixed_pool(direction):
    """the flag on over a pool batch (fast kernel + general kernel) with
    the error cases spread through it"""
    kind = xdpgpu.POOL_NAT64 if direction == IN else xdpgpu.POOL_NAT64_V4
    umem, descs, _ = xdpgpu.pool_generate(50000, kind, 128, 0x5EED0004)
    cases = ingress_cases() if direction == IN else egress_cases()
    ue, de = place([c[1] for c in cases] * 40, headroom=64, stride=256)
    base = umem.nbytes
    umem = np.concatenate([umem, ue])
    de = de.copy()
    de["addr"] += base
    rng = np.random.default_rng(7)
    descs = np.concatenate([descs, de])[rng.permutation(len(descs) + len(de))]
    cfg, smap = inner_cfg(direction)
    want = run_oracle(umem, descs, direction, cfg=cfg, smap=smap)
    got = gpu_nat64(umem, descs, direction, cfg, smap)
    assert_nat64_same(got, want, f"inner-pool/{direction}")


@pytest.mark.gpu
def test_gpu_inner_dynamic():
    from test_nat64_dyn import NOW0, T_OUT, compare_batches, pool_cfg, src
    cfg = pool_cfg(IN, mask_bits=27)
    cfg.flags = INNER
    rng = np.random.default_rng(11)
    batches = []
    t = NOW0
    for b in range(4):
        frames = []
        for _ in range(300):
            k, j = int(rng.integers(1, 40)), int(rng.integers(1, 40))
            r = rng.integers(0, 3)
            if r == 0:
                frames.append(err6(1, 4, bytes(4), inner6(dst=src(k)), src=src(k)))
            elif r == 1:
                frames.append(err6(3, 0, bytes(4), inner6(dst=src(j)), src=src(k)))
            else:
                frames.append(v6(udp_seg(src(k), PEER6), 17, src=src(k)))
        umem, descs = place(frames)
        batches.append((umem, descs, t, IN))
        t += T_OUT // 2 + 1
    compare_batches(cfg, [(src(200), 0x0A630007)], T_OUT, batches, "inner-dyn")
