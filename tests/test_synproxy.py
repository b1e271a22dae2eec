# SPDX-License-Identifier: GPL-2.0
"""SYN proxy (xdp-synproxy/xdp_synproxy_kern.c): the TCP
checksum verify and recompute path and the SYN-ACK rewrite.

CPU: the oracle (oracle/synproxy_oracle.c) against frames built here with
the action the reference program gives them, and every SYN-ACK against an
independent restatement written here: addresses and ports swapped, ack =
seq + 1, the option layout of tcp_mkoptions (:480-510), the timestamp
cookie of tscookie_init (:274-308), the values map (:310-330), and the IP
and TCP checksums recomputed from scratch (RFC 1071/793/2460).  The cookie
itself is build-defined (include/xdpgpu.h; the kernel's is outside the
transform): "parity unpinned" at the reference level, DESIGN.md.

GPU: xdpgpu_synproxy_dev bit-exact against the oracle (verdicts, output
descriptors, the UMEM after, the SYN-ACK count) on the cases at several
alignments and on random SYN/ACK/other pools.
"""
import struct

import numpy as np
import pytest

import frames as F
import oracle
import xdpgpu

ABORTED, DROP, PASS, TX = 0, 1, 2, 3
V4S, V4D = bytes([192, 0, 2, 10]), bytes([198, 51, 100, 20])
V6S = bytes.fromhex("20010db8000000000000000000000a0a")
V6D = bytes.fromhex("20010db8000000000000000000001414")
NOW = 1_700_000_123_456_789_012
KEY = 0x5EED5EED


def cfg(values=0, ports=(80, 443), tailroom=256, now=NOW, key=KEY):
    c = xdpgpu.SynproxyCfg()
    c.values = values
    for k, p in enumerate(ports):
        c.ports[k] = p
    c.now_ns = now
    c.tailroom = tailroom
    c.cookie_key = key
    return c


def opts(mss=1460, sack=True, ts=0x11223344, ws=7):
    o = b""
    if mss is not None:
        o += struct.pack(">BBH", 2, 4, mss)
    if sack:
        o += b"\x04\x02"
    if ts is not None:
        o += struct.pack(">BBII", 8, 10, ts, 0)
    if ws is not None:
        o += b"\x01" + struct.pack(">BBB", 3, 3, ws)
    while len(o) % 4:
        o += b"\x00"
    return o


def tcpseg(sport=40000, dport=80, seq=0x01020304, ack=0, flags=0x02, o=b"", payload=b""):
    doff = 5 + len(o) // 4
    return struct.pack(">HHIIBBHHH", sport, dport, seq, ack, doff << 4, flags, 0xFFFF, 0,
                       0) + o + payload


def v4syn(seg, src=V4S, dst=V4D, frag=0x4000, ipopts=b"", bad_ip=False, csum_len=None,
          tos=0x10, ident=0x4242):
    """IPv4 + TCP; the TCP checksum over the segment (or its first csum_len
    bytes, as the reference's header-only check sees it)"""
    n = len(seg) if csum_len is None else csum_len
    c = ~F.fold(F.ones_sum(F.set_csum(seg, 16, 0)[:n]) + F.pseudo4(src, dst, 6, n)) & 0xFFFF
    seg = F.set_csum(seg, 16, c)
    h = F.ipv4(len(seg), 6, src, dst, options=ipopts, frag_off=frag, ident=ident,
               bad_csum=bad_ip)
    h = h[:1] + bytes([tos]) + h[2:10] + b"\0\0" + h[12:]
    cs = ~F.fold(F.ones_sum(h)) & 0xFFFF
    if bad_ip:
        cs ^= 0x0F0F
    h = h[:10] + F.le16(cs) + h[12:]
    return F.eth(F.ETH_P_IP) + h + seg


def v6syn(seg, src=V6S, dst=V6D, nh=6):
    c = ~F.fold(F.ones_sum(F.set_csum(seg, 16, 0)) + F.pseudo6(src, dst, 6, len(seg))) & 0xFFFF
    seg = F.set_csum(seg, 16, c)
    h = struct.pack(">IHBB16s16s", (6 << 28) | (0x2e << 20) | 0x12345, len(seg), nh, 50,
                    src, dst)
    return F.eth(F.ETH_P_IPV6) + h + seg


def cookie(frame, v6):
    """the build-defined cookie (include/xdpgpu.h) for a SYN frame"""
    ip = 14
    w = [0] * 9
    if v6:
        for i in range(4):
            w[i] = struct.unpack_from("<I", frame, ip + 8 + 4 * i)[0]
            w[4 + i] = struct.unpack_from("<I", frame, ip + 24 + 4 * i)[0]
        tcp = ip + 40
    else:
        w[0] = struct.unpack_from("<I", frame, ip + 12)[0]
        w[4] = struct.unpack_from("<I", frame, ip + 16)[0]
        tcp = ip + (frame[ip] & 15) * 4
    sp, dp, seq = struct.unpack_from(">HHI", frame, tcp)
    w[8] = sp << 16 | dp
    key = oracle.buf(struct.pack("<9I", *w))     # jhash2: pinned against jhash.h
    h = oracle.lib().oracle_jhash2(key, 9, (KEY + NOW // 60_000_000_000) & 0xFFFFFFFF)
    return (h + seq) & 0xFFFFFFFF


def expect_synack(frame, v6, mss=None, wscale=7, ttl=64, client=None):
    """Independent restatement of the SYN-ACK the reference writes."""
    ip = 14
    tcp = ip + (40 if v6 else (frame[ip] & 15) * 4)
    sp, dp, seq = struct.unpack_from(">HHI", frame, tcp)
    fl = frame[tcp + 13]
    mss = mss if mss is not None else (1440 if v6 else 1460)
    c = client or {}
    o = struct.pack(">BBH", 2, 4, mss)
    ece = False
    if c.get("ts") is not None:
        tsval = (NOW // 1_000_000) & 0xFFFFFFFF & ~0x3F
        tsval |= c.get("ws", 0xF) & 0xF
        if c.get("sack"):
            tsval |= 1 << 4
        if fl & 0xC0 == 0xC0:
            tsval |= 1 << 5
            ece = True
        o += (b"\x04\x02\x08\x0a" if c.get("sack") else b"\x01\x01\x08\x0a")
        o += struct.pack(">II", tsval, c["ts"])
        if (tsval & 0xF) != 0xF:
            o += struct.pack(">BBBB", 1, 3, 3, wscale)
    th = struct.pack(">HHIIBBHHH", dp, sp, cookie(frame, v6), (seq + 1) & 0xFFFFFFFF,
                     (5 + len(o) // 4) << 4, 0x12 | (0x40 if ece else 0), 0, 0, 0) + o
    if v6:
        src, dst = frame[ip + 24:ip + 40], frame[ip + 8:ip + 24]
        ck = ~F.fold(F.ones_sum(th) + F.pseudo6(src, dst, 6, len(th))) & 0xFFFF
        th = F.set_csum(th, 16, ck)
        ih = struct.pack(">IHBB16s16s", 0x60000000, len(th), 6, ttl, src, dst)
    else:
        src, dst = frame[ip + 16:ip + 20], frame[ip + 12:ip + 16]
        ck = ~F.fold(F.ones_sum(th) + F.pseudo4(src, dst, 6, len(th))) & 0xFFFF
        th = F.set_csum(th, 16, ck)
        frag = struct.unpack_from(">H", frame, ip + 6)[0]
        ih = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(th), 0, frag, ttl, 6, 0, src, dst)
        ih = ih[:10] + F.le16(~F.fold(F.ones_sum(ih)) & 0xFFFF) + ih[12:]
    return frame[6:12] + frame[0:6] + frame[12:14] + ih + th


def cases():
    """(name, frame, action, client options for the SYN-ACK check)"""
    full = dict(ts=0x11223344, sack=True, ws=7)
    c = []
    c.append(("v4_syn", v4syn(tcpseg(o=opts())), TX, full))
    c.append(("v6_syn", v6syn(tcpseg(o=opts())), TX, full))
    c.append(("v4_syn_nots", v4syn(tcpseg(o=opts(ts=None))), TX, {}))
    c.append(("v4_syn_noopts", v4syn(tcpseg()), TX, {}))
    c.append(("v4_syn_nows", v4syn(tcpseg(o=opts(ws=None))), TX, dict(ts=0x11223344, sack=True)))
    c.append(("v4_syn_ws15", v4syn(tcpseg(o=opts(ws=15))), TX, dict(ts=0x11223344, sack=True,
                                                                     ws=14)))
    c.append(("v4_syn_nosack", v4syn(tcpseg(o=opts(sack=False))), TX, dict(ts=0x11223344, ws=7)))
    c.append(("v4_syn_ecn", v4syn(tcpseg(flags=0xC2, o=opts())), TX, full))
    c.append(("v4_syn_ipopts", v4syn(tcpseg(o=opts()), ipopts=b"\x01\x01\x01\x00"), TX, full))
    c.append(("v4_syn_port443", v4syn(tcpseg(dport=443, o=opts())), TX, full))
    c.append(("v4_port_other", v4syn(tcpseg(dport=22, o=opts())), PASS, None))
    c.append(("v4_udp", F.v4_frame(17, F.udp(1, 80, b"x" * 20), frag_off=0x4000), PASS, None))
    c.append(("arp", F.eth(0x0806) + b"\0" * 28, PASS, None))
    c.append(("vlan", F.eth(F.ETH_P_IP, tags=((0x8100, 7),)) + v4syn(tcpseg())[14:], PASS, None))
    c.append(("v4_nodf", v4syn(tcpseg(), frag=0), DROP, None))
    c.append(("v4_mf", v4syn(tcpseg(), frag=0x6000), DROP, None))
    c.append(("v4_synack_in", v4syn(tcpseg(flags=0x12)), DROP, None))
    c.append(("v4_none", v4syn(tcpseg(flags=0x08)), DROP, None))
    c.append(("v4_synfin", v4syn(tcpseg(flags=0x03)), DROP, None))
    c.append(("v4_synrst", v4syn(tcpseg(flags=0x06)), DROP, None))
    c.append(("v4_bad_ip", v4syn(tcpseg(o=opts()), bad_ip=True), DROP, None))
    seg = tcpseg(o=opts())
    c.append(("v4_bad_tcp", v4syn(seg)[:-1] + bytes([v4syn(seg)[-1] ^ 1]), DROP, None))
    c.append(("v4_syn_payload", v4syn(tcpseg(o=opts(), payload=b"hello world!")), DROP, None))
    c.append(("v4_syn_payload_hdrsum",
              v4syn(tcpseg(o=opts(), payload=b"hello world!"), csum_len=20 + len(opts())),
              TX, full))
    c.append(("v4_short_tcp", v4syn(tcpseg())[:14 + 20 + 12], DROP, None))
    c.append(("v4_doff3", v4syn(tcpseg())[:46] + b"\x30" + v4syn(tcpseg())[47:], DROP, None))
    c.append(("v4_ihl4", v4syn(tcpseg())[:14] + b"\x44" + v4syn(tcpseg())[15:], DROP, None))
    c.append(("v6_other_nh", v6syn(tcpseg(), nh=17), PASS, None))
    c.append(("v6_synrst", v6syn(tcpseg(flags=0x06)), DROP, None))
    c.append(("runt", b"\x00" * 10, DROP, None))
    return c


def ack_frame(v6, good=True, rst=False):
    syn = (v6syn if v6 else v4syn)(tcpseg(o=opts()))
    ck = cookie(syn, v6)
    seq = 0x01020304 + 1
    a = ck + 1 if good else ck + 2
    return (v6syn if v6 else v4syn)(tcpseg(seq=seq, ack=a & 0xFFFFFFFF,
                                           flags=0x14 if rst else 0x10))


def place(frames, stride=256, headroom=64, skew=0):
    umem = np.zeros(len(frames) * stride + 512, np.uint8)
    descs = np.zeros(len(frames), xdpgpu.DESC_DTYPE)
    for k, fr in enumerate(frames):
        off = k * stride + headroom + skew
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
        umem[off + len(fr):off + len(fr) + 64] = 0xA5     # old bytes past the end
        descs[k] = (off, len(fr), 0)
    return umem, descs


# ------------------------------------------------------------------ CPU tests
def test_oracle_cases():
    cs = cases()
    umem, descs = place([c[1] for c in cs])
    u = umem.copy()
    v, out, n = oracle.synproxy(u, descs, cfg())
    for k, (name, fr, want, client) in enumerate(cs):
        assert v[k] == want, f"{name}: {v[k]} != {want}"
        a, ln = int(out[k]["addr"]), int(out[k]["len"])
        if want == TX:
            got = u[a:a + ln].tobytes()
            exp = expect_synack(fr, name.startswith("v6"), client=client)
            assert got == exp, f"{name}:\n{got.hex()}\n{exp.hex()}"
    assert n == sum(1 for c in cs if c[2] == TX)


def test_oracle_values_map():
    fr = v4syn(tcpseg(o=opts()))
    umem, descs = place([fr, v6syn(tcpseg(o=opts()))])
    vals = 1400 | (5 << 16) | (33 << 24) | (1300 << 32)
    v, out, _ = oracle.synproxy(umem, descs, cfg(values=vals))
    assert list(v) == [TX, TX]
    a, ln = int(out[0]["addr"]), int(out[0]["len"])
    assert umem[a:a + ln].tobytes() == expect_synack(
        fr, False, mss=1400, wscale=5, ttl=33, client=dict(ts=0x11223344, sack=True, ws=7))
    a6 = int(out[1]["addr"])
    assert struct.unpack_from(">H", umem, a6 + 14 + 40 + 22)[0] == 1300
    assert umem[a6 + 14 + 7] == 33


def test_oracle_ack_and_growth():
    frames = [ack_frame(False), ack_frame(True), ack_frame(False, good=False),
              ack_frame(False, rst=True)]
    umem, descs = place(frames)
    u = umem.copy()
    v, out, n = oracle.synproxy(u, descs, cfg())
    assert list(v) == [PASS, PASS, DROP, DROP] and n == 0
    for k, fr in enumerate(frames):
        a, ln = int(descs[k]["addr"]), len(fr)
        # grown by TCP_MAXLEN - 20 zeroed bytes (bpf_xdp_adjust_tail)
        assert int(out[k]["len"]) == ln + 40
        assert not u[a + ln:a + ln + 40].any()
        assert u[a:a + ln].tobytes() == fr
    # the previous minute's cookie still passes, two minutes back does not
    c1 = cfg(now=NOW + 60_000_000_000)
    c2 = cfg(now=NOW + 120_000_000_000)
    assert oracle.synproxy(umem.copy(), descs[:1], c1)[0][0] == PASS
    assert oracle.synproxy(umem.copy(), descs[:1], c2)[0][0] == DROP


def test_oracle_tailroom():
    fr = v4syn(tcpseg(o=opts()))      # doff 10: grows by 20
    umem, descs = place([fr])
    assert oracle.synproxy(umem.copy(), descs, cfg(tailroom=19))[0][0] == ABORTED
    assert oracle.synproxy(umem.copy(), descs, cfg(tailroom=20))[0][0] == TX
    # growth past the UMEM's end
    umem2 = np.zeros(64 + len(fr) + 10, np.uint8)
    umem2[64:64 + len(fr)] = np.frombuffer(fr, np.uint8)
    d2 = np.array([(64, len(fr), 0)], xdpgpu.DESC_DTYPE)
    assert oracle.synproxy(umem2, d2, cfg())[0][0] == ABORTED


# ------------------------------------------------------------------ GPU tests
def gpu_synproxy(umem, descs, c):
    import torch
    n = len(descs)
    dev = "cuda:0"
    d_umem = torch.from_numpy(umem.copy()).to(dev)
    d_desc = torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8)).to(dev)
    d_v = torch.full((n,), 0xEE, dtype=torch.uint8, device=dev)
    d_out = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    with xdpgpu.XdpGpu(0) as g:
        g.synproxy_dev(d_umem, umem.nbytes, d_desc, n, c, d_v, d_out, d_cnt,
                       torch.cuda.current_stream())
        torch.cuda.synchronize()
    return (d_v.cpu().numpy(), d_out.cpu().numpy().view(xdpgpu.DESC_DTYPE),
            d_umem.cpu().numpy(), int(d_cnt.item()))


def assert_same(umem, descs, c, what):
    u = umem.copy()
    wv, wo, wn = oracle.synproxy(u, descs, c)
    gv, go, gu, gn = gpu_synproxy(umem, descs, c)
    bad = np.nonzero(gv != wv)[0]
    assert len(bad) == 0, f"{what}: verdict at {bad[:8]}: {gv[bad[:8]]} vs {wv[bad[:8]]}"
    bad = np.nonzero(go != wo)[0]
    assert len(bad) == 0, f"{what}: out desc at {bad[:8]}"
    bad = np.nonzero(gu != u)[0]
    assert len(bad) == 0, f"{what}: UMEM differs at {bad[:8]}"
    assert gn == wn, f"{what}: {gn} SYN-ACKs vs {wn}"
    return wv


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [0, 1, 2, 4])
def test_gpu_cases(skew):
    cs = cases()
    frames = [c[1] for c in cs] + [ack_frame(False), ack_frame(True),
                                   ack_frame(False, good=False)]
    umem, descs = place(frames, skew=skew)
    v = assert_same(umem, descs, cfg(), f"cases/{skew}")
    assert (v == TX).sum() >= 10


@pytest.mark.gpu
def test_gpu_tailroom_and_values():
    frames = [v4syn(tcpseg(o=opts())), v6syn(tcpseg(o=opts())), ack_frame(True)]
    umem, descs = place(frames)
    for tr in (0, 19, 20, 40, 256):
        assert_same(umem, descs, cfg(tailroom=tr), f"tailroom {tr}")
    vals = 1400 | (5 << 16) | (33 << 24) | (1300 << 32)
    assert_same(umem, descs, cfg(values=vals), "values")


def random_pool(n, seed):
    rng = np.random.default_rng(seed)
    frames = []
    for _ in range(n):
        kind = rng.integers(0, 10)
        v6 = bool(rng.integers(0, 3) == 0)
        mk = v6syn if v6 else v4syn
        o = opts(mss=int(rng.integers(500, 9000)) if rng.integers(0, 4) else None,
                 sack=bool(rng.integers(0, 2)),
                 ts=int(rng.integers(0, 1 << 32)) if rng.integers(0, 4) else None,
                 ws=int(rng.integers(0, 16)) if rng.integers(0, 3) else None)
        sport = int(rng.integers(1024, 65536))
        seq = int(rng.integers(0, 1 << 32))
        if kind < 5:
            frames.append(mk(tcpseg(sport=sport, seq=seq, o=o,
                                    flags=0x02 | (0xC0 if kind == 4 else 0))))
        elif kind < 7:
            frames.append(ack_frame(v6, good=bool(rng.integers(0, 2))))
        elif kind == 7:
            frames.append(mk(tcpseg(sport=sport, dport=int(rng.integers(1, 1000)), o=o)))
        elif kind == 8:
            fr = bytearray(mk(tcpseg(sport=sport, seq=seq, o=o)))
            fr[int(rng.integers(14, len(fr)))] ^= 1 << int(rng.integers(0, 8))
            frames.append(bytes(fr))
        else:
            frames.append(F.v4_frame(17, F.udp(sport, 80, b"q" * int(rng.integers(0, 60))),
                                     frag_off=0x4000))
    return frames


@pytest.mark.gpu
@pytest.mark.parametrize("stride,skew", [(128, 0), (256, 3), (192, 16)])
def test_gpu_random_pool(stride, skew):
    frames = random_pool(20000, stride + skew)
    umem, descs = place(frames, stride=stride, headroom=0, skew=skew)
    v = assert_same(umem, descs, cfg(tailroom=stride - 100 - skew), f"pool/{stride}/{skew}")
    assert (v == TX).sum() > 1000 and (v == PASS).sum() > 1000 and (v == DROP).sum() > 500
