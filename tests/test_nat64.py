# SPDX-License-Identifier: GPL-2.0
"""nat64 (nat64-bpf/nat64_kern.c, BASELINE config 4).

CPU: the oracle (oracle/nat64_oracle.c) against the RFC 6052 address
vectors, against hand-built frames with the action nat64_kern.c gives them,
against the pool generator's intent, and every translated frame against a
full checksum recomputation written here (independent of the oracle's
incremental arithmetic).  GPU: xdpgpu_nat64_dev bit-exact against the
oracle (action, output descriptors, UMEM after) on the same inputs.
"""
import ipaddress
import struct

import numpy as np
import pytest

import frames as F
import oracle
import xdpgpu

IN, EG = xdpgpu.NAT64_INGRESS, xdpgpu.NAT64_EGRESS
OK, SHOT, REDIR, NOSTATE = (xdpgpu.TC_ACT_OK, xdpgpu.TC_ACT_SHOT,
                            xdpgpu.TC_ACT_REDIRECT, xdpgpu.NAT64_NO_STATE)


def a6(s):
    return ipaddress.IPv6Address(s).packed


def a4(s):
    return ipaddress.IPv4Address(s).packed


SRC6 = a6("2001:db8:1:2::5")          # mapped to 10.99.0.5 by the pool config
DST6 = a6("64:ff9b::c633:6405")       # 198.51.100.5
SRC4 = a4("198.51.100.7")
DST4 = a4("10.99.0.5")

# RFC 6052 section 2.4 examples: (prefix, plen, IPv4-embedded address) for 192.0.2.33
RFC6052 = [("2001:db8::", 32, "2001:db8:c000:221::"),
           ("2001:db8:100::", 40, "2001:db8:1c0:2:21::"),
           ("2001:db8:122::", 48, "2001:db8:122:c000:2:2100::"),
           ("2001:db8:122:300::", 56, "2001:db8:122:3c0:0:221::"),
           ("2001:db8:122:344::", 64, "2001:db8:122:344:c0:2:2100:0"),
           ("2001:db8:122:344::", 96, "2001:db8:122:344::192.0.2.33"),
           ("64:ff9b::", 96, "64:ff9b::192.0.2.33")]


def ocfg(cfg):
    return oracle.Nat64Cfg.from_buffer_copy(bytes(cfg))


# ------------------------------------------------------------- frame builders
def v6hdr(plen, nh, src=SRC6, dst=DST6, hop=64, tc=0, flow=0):
    return struct.pack(">IHBB16s16s", (6 << 28) | (tc << 20) | flow, plen, nh, hop,
                       src, dst)


def v6(seg, nh, src=SRC6, dst=DST6, fix=True, tags=(), **kw):
    chk = {17: 6, 6: 16, 58: 2}.get(nh)
    if fix and chk is not None:
        seg = F.set_csum(seg, chk, 0)
        seg = F.set_csum(seg, chk, F.l4_csum6(src, dst, nh, seg))
    return F.eth(F.ETH_P_IPV6, tags) + v6hdr(len(seg), nh, src, dst, **kw) + seg


def v4(seg, proto, src=SRC4, dst=DST4, tos=0, frag=0, options=b"", ttl=64):
    chk = {17: 6, 6: 16, 1: 2}.get(proto)
    if chk is not None:
        seg = F.set_csum(seg, chk, 0)
        if proto == 1:
            c = ~F.fold(F.ones_sum(seg)) & 0xFFFF
        else:
            c = F.l4_csum4(src, dst, proto, seg)
        seg = F.set_csum(seg, chk, c)
    h = F.ipv4(len(seg), proto, src, dst, ttl=ttl, options=options, frag_off=frag)
    h = h[:1] + bytes([tos]) + h[2:10] + b"\0\0" + h[12:]
    h = h[:10] + F.le16(~F.fold(F.ones_sum(h)) & 0xFFFF) + h[12:]
    return F.eth(F.ETH_P_IP) + h + seg


def udp(n=40, sport=1234):
    return F.udp(sport, 53, bytes(range(7, 7 + n)))


def tcp(n=32):
    return F.tcp(40000, 443, bytes(range(3, 3 + n)))


def icmp6(t, c, rest=b"\0\0\0\0", body=b"x" * 24):
    return bytes([t, c, 0, 0]) + rest + body


def icmp4(t, c, rest=b"\0\0\0\0", body=b"y" * 24):
    return bytes([t, c, 0, 0]) + rest + body


def ingress_cases():
    """(name, frame, expected action) for nat64_handle_v6."""
    c = []
    c.append(("udp", v6(udp(), 17, tc=0xb8, flow=0x12345), REDIR))
    c.append(("tcp", v6(tcp(), 6, hop=17), REDIR))
    seg = F.set_csum(udp(), 6, 0)
    c.append(("udp_csum0_kept", v6(seg, 17, fix=False), REDIR))
    c.append(("udp_odd", v6(udp(41), 17), REDIR))
    c.append(("echo_req", v6(icmp6(128, 0, b"\x12\x34\x00\x01"), 58), REDIR))
    c.append(("echo_rep", v6(icmp6(129, 0, b"\x12\x34\x00\x02"), 58), REDIR))
    for code, act in ((0, REDIR), (1, REDIR), (2, REDIR), (3, REDIR), (4, REDIR), (5, SHOT)):
        c.append((f"unreach_{code}", v6(icmp6(1, code), 58), act))
    c.append(("toobig_1500", v6(icmp6(2, 0, struct.pack(">I", 1500)), 58), REDIR))
    c.append(("toobig_10", v6(icmp6(2, 0, struct.pack(">I", 10)), 58), SHOT))
    c.append(("toobig_big", v6(icmp6(2, 0, struct.pack(">I", 0x20000)), 58), SHOT))
    c.append(("time_exceed", v6(icmp6(3, 1), 58), REDIR))
    for ptr, act in ((0, REDIR), (1, REDIR), (4, REDIR), (5, REDIR), (6, REDIR), (7, REDIR),
                     (8, REDIR), (23, REDIR), (24, REDIR), (39, REDIR), (40, SHOT), (2, SHOT)):
        c.append((f"paramprob_ptr{ptr}", v6(icmp6(4, 0, struct.pack(">I", ptr)), 58), act))
    c.append(("paramprob_c1", v6(icmp6(4, 1), 58), REDIR))
    c.append(("paramprob_c2", v6(icmp6(4, 2), 58), SHOT))
    c.append(("ndp_ns", v6(icmp6(135, 0), 58), SHOT))
    c.append(("icmp6_short", v6(b"\x80\0\0\0", 58, fix=False), SHOT))
    hop = bytes([17]) + F.ext_opts(1)
    c.append(("ext_hop", F.eth(F.ETH_P_IPV6) + v6hdr(8 + len(udp()), 0) + hop + udp(), SHOT))
    chain = b"".join(bytes([0]) + F.ext_opts(1) for _ in range(6))
    c.append(("ext_6_chain", F.eth(F.ETH_P_IPV6) + v6hdr(48 + 20, 0) + chain + b"\0" * 20, OK))
    c.append(("ext_trunc", F.eth(F.ETH_P_IPV6) + v6hdr(8, 0) + bytes([17, 3]), OK))
    c.append(("dst_out_of_prefix", v6(udp(), 17, dst=a6("64:ff9c::c633:6405")), OK))
    c.append(("dst_127", v6(udp(), 17, dst=a6("64:ff9b::7f00:1")), SHOT))
    c.append(("dst_0", v6(udp(), 17, dst=a6("64:ff9b::")), SHOT))
    c.append(("dst_224", v6(udp(), 17, dst=a6("64:ff9b::e001:101")), SHOT))
    c.append(("src_not_allowed", v6(udp(), 17, src=a6("2001:db8:1:3::5")), SHOT))
    c.append(("src_no_state", v6(udp(), 17, src=a6("2001:db8:1:2::1:0")), NOSTATE))
    bad = bytearray(v6(udp(), 17))
    bad[14] = 0x50
    c.append(("version5", bytes(bad), OK))
    c.append(("short_53", v6(udp(), 17)[:53], OK))
    c.append(("nonext_56", F.eth(F.ETH_P_IPV6) + v6hdr(2, 59) + b"\0\0", REDIR))
    c.append(("no_next_54", F.eth(F.ETH_P_IPV6) + v6hdr(0, 59), OK))
    c.append(("udp_trunc", v6(udp(), 17)[:60], REDIR))
    c.append(("vlan1", v6(udp(), 17, tags=((0x8100, 5),)), REDIR))
    c.append(("vlan2", v6(tcp(), 6, tags=((0x88A8, 5), (0x8100, 6))), REDIR))
    c.append(("ipv4_frame", v4(udp(), 17), OK))
    c.append(("arp", F.eth(F.ETH_P_ARP) + b"\0" * 28, OK))
    c.append(("runt", b"\x01" * 10, OK))
    return c


def egress_cases():
    """(name, frame, expected action) for nat64_handle_v4."""
    c = []
    c.append(("udp", v4(udp(), 17, tos=0xb8), REDIR))
    c.append(("tcp", v4(tcp(), 6, ttl=9), REDIR))
    c.append(("udp_csum0_kept", v4(udp(), 17)[:-len(udp())] + F.set_csum(udp(), 6, 0), REDIR))
    c.append(("echo", v4(icmp4(8, 0, b"\x00\x07\x00\x01"), 1), REDIR))
    c.append(("echo_rep", v4(icmp4(0, 0, b"\x00\x07\x00\x02"), 1), REDIR))
    for code in range(16):
        act = SHOT if code == 14 else REDIR
        rest = struct.pack(">HH", 0, 500 if code == 4 else 0)
        c.append((f"unreach_{code}", v4(icmp4(3, code, rest), 1), act))
    c.append(("fragneeded_1400", v4(icmp4(3, 4, struct.pack(">HH", 0, 1400)), 1), REDIR))
    for p, act in ((0, REDIR), (1, REDIR), (2, REDIR), (3, REDIR), (8, REDIR), (9, REDIR),
                   (12, REDIR), (15, REDIR), (16, REDIR), (19, REDIR), (4, SHOT), (20, SHOT)):
        c.append((f"paramprob_{p}", v4(icmp4(12, 0, bytes([p, 0, 0, 0])), 1), act))
    c.append(("paramprob_c1", v4(icmp4(12, 1), 1), SHOT))
    c.append(("time_exceeded", v4(icmp4(11, 0), 1), SHOT))
    c.append(("icmp_short", v4(b"\x08\0\0\0", 1), SHOT))
    c.append(("options", v4(udp(), 17, options=b"\x01\x01\x01\x01"), SHOT))
    c.append(("mf", v4(udp(), 17, frag=0x2000), SHOT))
    c.append(("df", v4(udp(), 17, frag=0x4000), REDIR))
    c.append(("frag_off", v4(udp(), 17, frag=0x0010), SHOT))
    c.append(("dst_outside", v4(udp(), 17, dst=a4("10.98.0.5")), OK))
    c.append(("dst_unmapped", v4(udp(), 17, dst=a4("10.99.255.254")), SHOT))
    c.append(("ipv6_frame", v6(udp(), 17), OK))
    c.append(("proto_gre", v4(b"\0" * 24, 47), REDIR))
    return c


def place(frames, headroom=64, stride=256, skew=0):
    umem = np.zeros(len(frames) * stride + 256, np.uint8)
    descs = np.zeros(len(frames), xdpgpu.DESC_DTYPE)
    for k, fr in enumerate(frames):
        off = k * stride + headroom + skew
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
        descs[k] = (off, len(fr), 0)
    return umem, descs


# ------------------------------------------------------ independent checking
def parse_l2(fr):
    pos, proto = 14, struct.unpack(">H", fr[12:14])[0]
    for _ in range(2):
        if proto not in (0x8100, 0x88A8) or pos + 4 > len(fr):
            break
        proto = struct.unpack(">H", fr[pos + 2:pos + 4])[0]
        pos += 4
    return proto, pos


def check_translated(fr, direction, l3=14):
    """Full recomputation: the translated frame's IP header (at l3, the
    original frame's L3 offset: nat64_kern.c rewrites eth->h_proto, so a
    tagged frame's TPID becomes the new EtherType) and L4 checksum verify
    (RFC 1071/768/2460 semantics, computed here)."""
    if direction == IN:
        h = fr[l3:l3 + 20]
        assert h[0] == 0x45 and F.fold(F.ones_sum(h)) == 0xFFFF
        tot = struct.unpack(">H", h[2:4])[0]
        proto, src, dst = h[9], h[12:16], h[16:20]
        seg = fr[l3 + 20:l3 + tot]
        if proto in (6, 17) and len(seg) >= (18 if proto == 6 else 8):
            c = struct.unpack("<H", seg[16:18] if proto == 6 else seg[6:8])[0]
            if not (proto == 17 and c == 0):
                assert F.fold(F.ones_sum(seg) + F.pseudo4(src, dst, proto, len(seg))) == 0xFFFF
        elif proto == 1:
            assert F.fold(F.ones_sum(seg)) == 0xFFFF
    else:
        h = fr[l3:l3 + 40]
        assert h[0] >> 4 == 6
        plen, nh = struct.unpack(">H", h[4:6])[0], h[6]
        src, dst = h[8:24], h[24:40]
        seg = fr[l3 + 40:l3 + 40 + plen]
        if nh in (6, 17, 58):
            off = {6: 16, 17: 6, 58: 2}[nh]
            c = struct.unpack("<H", seg[off:off + 2])[0]
            if not (nh == 17 and c == 0):
                assert F.fold(F.ones_sum(seg) + F.pseudo6(src, dst, nh, len(seg))) == 0xFFFF


def run_oracle(umem, descs, direction, nmap=65533, cfg=None, smap=None):
    if cfg is None:
        cfg, smap = xdpgpu.nat64_pool_config(direction, nmap)
    u = umem.copy()
    act, out = oracle.nat64(u, descs, ocfg(cfg), smap)
    return act, out, u


# ------------------------------------------------------------------ CPU tests
def test_rfc6052_vectors():
    v4a = a4("192.0.2.33")
    for pref, plen, want in RFC6052:
        got = oracle.v4addr_to_v6(v4a, a6(pref), plen)
        assert got == a6(want), (pref, plen)
        back = oracle.v6addr_to_v4(got, plen)
        assert back[0] == v4a and back[1] == a6(pref)
    assert oracle.v4addr_to_v6(v4a, a6("64:ff9b::"), 80) is None


@pytest.mark.parametrize("direction", [IN, EG])
def test_oracle_cases(direction):
    cases = ingress_cases() if direction == IN else egress_cases()
    umem, descs = place([c[1] for c in cases])
    act, out, u = run_oracle(umem, descs, direction)
    for k, (name, fr, want) in enumerate(cases):
        assert act[k] == want, f"{name}: action {act[k]} != {want}"
        if want == REDIR:
            o = out[k]
            shift = 20 if direction == IN else -20
            assert int(o["addr"]) == int(descs[k]["addr"]) + shift
            assert int(o["len"]) == int(descs[k]["len"]) - shift
            check_translated(u[o["addr"]:o["addr"] + o["len"]].tobytes(), direction,
                             parse_l2(fr)[1])
        else:
            assert out[k] == descs[k]
            lo = int(descs[k]["addr"])
            assert np.array_equal(u[lo - 20:lo + len(fr)], umem[lo - 20:lo + len(fr)]), name


def test_oracle_field_mapping():
    """tos / flow label / hop limit / length mapping of both directions."""
    cases = ingress_cases()
    umem, descs = place([cases[0][1]])
    act, out, u = run_oracle(umem, descs, IN)
    fr = u[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    # tc 0xb8 -> priority 0xb, flow_lbl[0] 0x81 -> tos = 0xb << 4 | 0x8
    assert fr[15] == 0xb8 and fr[14 + 8] == 64 and fr[12:14] == b"\x08\x00"
    assert fr[14 + 6:14 + 8] == b"\x40\x00" and fr[14 + 12:14 + 16] == a4("10.99.0.5")
    assert fr[14 + 16:14 + 20] == a4("198.51.100.5")
    eg = egress_cases()
    umem, descs = place([eg[0][1]])
    act, out, u = run_oracle(umem, descs, EG)
    fr = u[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    # tos 0xb8: priority (0xb8 & 0x70) >> 4 = 3, flow_lbl[0] = 0x80
    assert fr[14] == 0x63 and fr[15] == 0x80 and fr[12:14] == b"\x86\xdd"
    assert fr[14 + 8:14 + 24] == a6("64:ff9b::c633:6407") and fr[14 + 24:14 + 40] == SRC6


def test_oracle_headroom():
    umem, descs = place([egress_cases()[0][1]], headroom=10)
    act, _, _ = run_oracle(umem, descs, EG)
    assert act[0] == SHOT


@pytest.mark.parametrize("plen", [32, 40, 48, 56, 64, 96])
def test_oracle_prefix_lengths(plen):
    cfg, smap = xdpgpu.nat64_pool_config(IN, 16)
    pref = bytearray(a6("2001:db8:122:344::"))
    for k in range(plen // 8, 16):
        pref[k] = 0
    cfg.v6_prefix[:] = list(pref)
    cfg.v6_plen = plen
    dst = oracle.v4addr_to_v6(a4("192.0.2.33"), bytes(pref), plen)
    umem, descs = place([v6(udp(), 17, dst=dst)])
    act, out, u = run_oracle(umem, descs, IN, cfg=cfg, smap=smap)
    assert act[0] == REDIR
    fr = u[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    assert fr[30:34] == a4("192.0.2.33")
    check_translated(fr, IN)
    cfg.direction = EG
    umem, descs = place([v4(udp(), 17, src=a4("192.0.2.33"), dst=a4("10.99.0.3"))])
    act, out, u = run_oracle(umem, descs, EG, cfg=cfg, smap=smap)
    assert act[0] == REDIR
    fr = u[out[0]["addr"]:out[0]["addr"] + out[0]["len"]].tobytes()
    assert fr[22:38] == dst
    check_translated(fr, EG)


@pytest.mark.parametrize("kind,direction", [(xdpgpu.POOL_NAT64, IN), (xdpgpu.POOL_NAT64_V4, EG)])
def test_oracle_pool(kind, direction):
    umem, descs, expect = xdpgpu.pool_generate(20000, kind, 128, 0x5EED0004)
    act, out, u = run_oracle(umem, descs, direction)
    np.testing.assert_array_equal(act, expect)
    for k in np.nonzero(act == REDIR)[0][:4000]:
        o = out[k]
        check_translated(u[o["addr"]:o["addr"] + o["len"]].tobytes(), direction)


# ------------------------------------------------------------------ GPU tests
def gpu_nat64(umem, descs, direction, cfg=None, smap=None):
    import torch
    if cfg is None:
        cfg, smap = xdpgpu.nat64_pool_config(direction)
    n = len(descs)
    dev = "cuda:0"
    d_umem = torch.zeros(umem.nbytes + 64, dtype=torch.uint8, device=dev)
    d_umem[:umem.nbytes].copy_(torch.from_numpy(umem))
    d_desc = torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8)).to(dev)
    d_act = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    with xdpgpu.XdpGpu(0) as g:
        g.nat64_setup(cfg, smap)
        g.nat64_dev(d_umem, umem.nbytes, d_desc, n, d_act, d_out,
                    torch.cuda.current_stream())
        torch.cuda.synchronize()
    return (d_act.cpu().numpy(), d_out.cpu().numpy().view(xdpgpu.DESC_DTYPE),
            d_umem.cpu().numpy()[:umem.nbytes])


def assert_nat64_same(got, want, what):
    ga, go, gu = got
    wa, wo, wu = want
    bad = np.nonzero(ga != wa)[0]
    assert len(bad) == 0, f"{what}: action at {bad[:8]}: {ga[bad[:8]]} vs {wa[bad[:8]]}"
    bad = np.nonzero(go != wo)[0]
    assert len(bad) == 0, f"{what}: out desc at {bad[:8]}"
    bad = np.nonzero(gu != wu)[0]
    assert len(bad) == 0, f"{what}: UMEM differs at bytes {bad[:8]}"


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [IN, EG])
@pytest.mark.parametrize("skew", [0, 1, 4, 8])
def test_gpu_cases(direction, skew):
    cases = ingress_cases() if direction == IN else egress_cases()
    umem, descs = place([c[1] for c in cases], skew=skew)
    want = run_oracle(umem, descs, direction)
    got = gpu_nat64(umem, descs, direction)
    assert_nat64_same(got, want, f"cases/{direction}/{skew}")


@pytest.mark.gpu
@pytest.mark.parametrize("direction", [IN, EG])
@pytest.mark.parametrize("headroom", [64, 32, 24, 16])
def test_gpu_cases_padded(direction, headroom):
    """The cases padded to 96 bytes: the fast kernels' shapes (>= 64 bytes,
    16-byte aligned, at headroom 64 and 32); headroom 24 is unaligned and 16
    leaves an egress frame too little room, both for the slow kernel."""
    cases = ingress_cases() if direction == IN else egress_cases()
    frames = [c[1] + bytes(max(0, 96 - len(c[1]))) for c in cases]
    umem, descs = place(frames, headroom=headroom)
    want = run_oracle(umem, descs, direction)
    assert (want[0] == REDIR).sum() > len(cases) // 2
    got = gpu_nat64(umem, descs, direction)
    assert_nat64_same(got, want, f"padded/{direction}/{headroom}")


@pytest.mark.gpu
@pytest.mark.parametrize("plen", [32, 40, 48, 56, 64, 96])
def test_gpu_prefix_lengths(plen):
    cfg, smap = xdpgpu.nat64_pool_config(IN, 16)
    pref = bytearray(a6("2001:db8:122:344::"))
    for k in range(plen // 8, 16):
        pref[k] = 0
    cfg.v6_prefix[:] = list(pref)
    cfg.v6_plen = plen
    dst = oracle.v4addr_to_v6(a4("192.0.2.33"), bytes(pref), plen)
    umem, descs = place([v6(udp(), 17, dst=dst), v6(tcp(), 6, dst=dst)])
    assert_nat64_same(gpu_nat64(umem, descs, IN, cfg, smap),
                      run_oracle(umem, descs, IN, cfg=cfg, smap=smap), f"plen{plen}")
    cfg.direction = EG
    umem, descs = place([v4(udp(), 17, src=a4("192.0.2.33"), dst=a4("10.99.0.3"))])
    assert_nat64_same(gpu_nat64(umem, descs, EG, cfg, smap),
                      run_oracle(umem, descs, EG, cfg=cfg, smap=smap), f"plen{plen}/eg")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,direction,n,kw", [
    (xdpgpu.POOL_NAT64, IN, 1 << 20, {}),
    # config 4 at full size (the bench leg's pool): every frame
    pytest.param(xdpgpu.POOL_NAT64, IN, 16 << 20, {}, id="config4-16M"),
    (xdpgpu.POOL_NAT64, IN, 100000, dict(headroom=4, stride=256)),
    (xdpgpu.POOL_NAT64_V4, EG, 1 << 20, {}),
    (xdpgpu.POOL_NAT64_V4, EG, 100000, dict(headroom=21, stride=192)),
])
def test_gpu_pool(kind, direction, n, kw):
    umem, descs, expect = xdpgpu.pool_generate(n, kind, 128, 0x5EED0004, **kw)
    want = run_oracle(umem, descs, direction)
    np.testing.assert_array_equal(want[0], expect)
    assert_nat64_same(gpu_nat64(umem, descs, direction), want, f"pool/{kind}")
