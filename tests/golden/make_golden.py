#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""TEST INFRASTRUCTURE: regenerate tests/golden/*.npz (run in the container
where /root/reference exists; the GPU box only reads the committed files).

* fixtures.npz - hand-built edge-case frames in one UMEM, their descriptors,
  and the expected outputs of the pipeline under three configurations.  The
  expected outputs come from the oracle (oracle/liboracle.so) and are only
  written after three independent checks pass for every frame:
    1. the hand-written expectation of each case below (verdict, offsets,
       protocol, VLAN depth, and the published golden checksums of the
       reference's own generated frames);
    2. every IPv4 header / TCP / UDP / ICMP checksum recomputed with the
       reference's lib_checksum.h compiled in place (oracle/_ref/libref.so);
       IPv6 pseudo-header sums with the independent frames.py arithmetic;
    3. every flow hash recomputed with the reference's include/jhash.h.
* csum_vectors.npz / jhash_vectors.npz - random inputs with the outputs of
  the reference functions themselves (do_csum, ip_fast_csum, udp_csum,
  csum_tcpudp_magic, jhash, jhash2, jhash_3words).

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import ctypes as C
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

import oracle  # noqa: E402
from frames import (ETH_P_8021AD, ETH_P_8021Q, ETH_P_ARP, ETH_P_IP,  # noqa: E402
                    ETH_P_IPV6, V6D, V6S, eth, ext_ah, ext_frag, ext_opts,
                    fold, icmp, ipv4, ipv6, l4_csum4, l4_csum6, ones_sum, set_csum, tcp,
                    udp, v4_frame, v6_frame)

ABORTED, DROP, PASS, TX, REDIRECT = 0, 1, 2, 3, 4
F_L3_OK, F_L4_OK, F_VLAN, F_IPV6, F_FRAG, F_L4_ABSENT, F_IP, F_L4 = (
    1, 2, 4, 8, 16, 32, 64, 128)

CFGS = {
    # name: (flags, initval, tuple_fmt)
    "verify": (0x1 | 0x4, 0, 1),
    "echo_net": (0x1 | 0x2 | 0x4, 0xDEADBEEF, 2),
    "noverify": (0x4, 1, 1),
}

XDPSOCK_60 = bytes.fromhex(
    "3cfdfe9e7f71ecb1d7983ac008004500002e000000004011527c0a0a0a100a0a"
    "0a2010001000001a0291123456781234567812345678123456781234")


def xdpsock_frame(size=64, vlan=False, pattern=0x12345678):
    """xdpsock gen_eth_hdr_data() restated (xdpsock.c:893-971); the golden
    checksums of the result are asserted against SURVEY.md §8c."""
    r = oracle.ref_lib()
    hdr_tags = ((ETH_P_8021Q, 1),) if vlan else ()
    l2 = size - 4
    l3 = 18 if vlan else 14
    ip_len = l2 - l3
    udp_len = ip_len - 20
    data = bytearray(udp_len - 8)
    pat = struct.pack(">I", pattern)
    for i in range(len(data)):
        data[i] = pat[i & 3]
    seg = udp(0x1000, 0x1000, bytes(data))
    return v4_frame(17, seg, src=bytes([10, 10, 10, 16]),
                    dst=bytes([10, 10, 10, 32]), tags=hdr_tags) + b"\0" * 4


def afxdp_user_frame():
    """af_xdp_user gen_base_pkt() (af_xdp_user.c:629-700), 64-byte size."""
    data = bytes(b"ABCD" * 5)[:18]
    seg = udp(0x1000, 0x1000, data)
    f = v4_frame(17, seg, src=bytes([192, 168, 44, 1]),
                 dst=bytes([192, 168, 44, 3]))
    return bytes.fromhex("bcee7bdac262245ebe57f164") + f[12:] + b"\0" * 4


def cases():
    """(name, frame, desc_len or None, expected verdict under 'verify',
    field expectations dict, placement)"""
    S4 = b"\x0a\x00\x00\x01"
    D4 = b"\x0a\x00\x00\x02"
    pay = bytes(range(40))
    out = []

    def add(name, frame, verdict, exp=None, length=None, place="std"):
        out.append((name, bytes(frame), length, verdict, exp or {}, place))

    # --- the reference's own generated frames, golden checksums
    f = xdpsock_frame()
    assert f[:60] == XDPSOCK_60, "xdpsock restatement drifted"
    add("xdpsock_default", f, REDIRECT,
        dict(l3_off=14, l4_off=34, l4_proto=17, l3_csum=0x7C52, l4_csum=0x9102,
             flags_set=F_IP | F_L3_OK | F_L4 | F_L4_OK), length=60)
    add("xdpsock_vlan", xdpsock_frame(vlan=True), REDIRECT,
        dict(l3_off=18, l4_off=38, nvlan=1, l3_csum=0x8052, l4_csum=0x456B,
             flags_set=F_VLAN | F_L4_OK), length=60)
    add("xdpsock_1500", xdpsock_frame(size=1500), REDIRECT,
        dict(l3_csum=0xE04C, l4_csum=0x922D, l4_len=1462), length=1496)
    add("afxdp_user_default", afxdp_user_frame(), REDIRECT,
        dict(l3_csum=0x6AA1, l4_csum=0x08B3), length=64)

    # --- Ethernet / VLAN (parsing_helpers.h:86-129)
    add("runt_13", f[:13], ABORTED)
    add("empty_len0", f, ABORTED, length=0)
    arp = eth(ETH_P_ARP) + bytes.fromhex("000108000604000100") + b"\x11" * 19
    add("arp", arp + b"\0" * 18, PASS)
    arp_vlan = eth(ETH_P_ARP, ((ETH_P_8021Q, 5),)) + b"\x22" * 28
    add("arp_vlan", arp_vlan + b"\0" * 14, PASS)
    seg = udp(1234, 80, pay[:20])
    add("qinq_udp", v4_frame(17, seg, tags=((ETH_P_8021AD, 100), (ETH_P_8021Q, 200))),
        REDIRECT, dict(l3_off=22, l4_off=42, nvlan=2, flags_set=F_VLAN | F_L4_OK))
    add("three_tags_not_ip",
        v4_frame(17, seg, tags=((ETH_P_8021AD, 1), (ETH_P_8021Q, 2), (ETH_P_8021Q, 3))),
        REDIRECT, dict(l3_off=22, nvlan=2, l4_proto=0, flags_clear=F_IP))
    add("vlan_truncated", eth(ETH_P_8021Q) + b"\x00", REDIRECT,
        dict(l3_off=14, nvlan=0, flags_clear=F_IP))
    add("unknown_ethertype", eth(0x88CC) + b"\x01" * 46, REDIRECT,
        dict(flags_clear=F_IP, l4_proto=0))

    # --- IPv4 (parsing_helpers.h:196-222)
    add("ipv4_version5", v4_frame(17, seg, version=5), ABORTED)
    add("ipv4_ihl4", v4_frame(17, seg, ihl=4), ABORTED)
    add("ipv4_hdr_truncated", v4_frame(17, seg)[:30], ABORTED)
    add("ipv4_ihl_past_end", v4_frame(17, seg, ihl=15)[:60], ABORTED)
    add("ipv4_totlen_past_end", v4_frame(17, seg, tot_len=200), ABORTED)
    add("ipv4_totlen_lt_hl", v4_frame(17, seg, tot_len=16), ABORTED)
    for nopt in (1, 4, 10):
        add(f"ipv4_options_{nopt}", v4_frame(17, seg, options=b"\x01" * (4 * nopt)),
            REDIRECT, dict(l4_off=34 + 4 * nopt, flags_set=F_L3_OK | F_L4_OK))
    add("ipv4_bad_csum", v4_frame(17, seg, bad_csum=True), DROP,
        dict(flags_clear=F_L3_OK, flags_set=F_L4_OK))
    add("ipv4_gre", v4_frame(47, b"\0" * 24), REDIRECT,
        dict(l4_proto=47, l4_off=34, flags_clear=F_L4 | F_L4_OK))
    add("ipv4_padding_after_totlen", v4_frame(17, seg) + b"\xee" * 30, REDIRECT,
        dict(l4_len=28))
    # fragments (build-defined: no L4 checksum; non-first has no L4 header)
    add("ipv4_frag_first", v4_frame(17, udp(1, 2, pay[:20], length=500), frag_off=0x2000,
                                    fix_l4=False), REDIRECT,
        dict(flags_set=F_FRAG | F_L4, flags_clear=F_L4_OK, l4_len=0))
    add("ipv4_frag_middle", v4_frame(17, pay[:32], frag_off=0x2000 | 100, fix_l4=False),
        REDIRECT, dict(flags_set=F_FRAG, flags_clear=F_L4))
    add("ipv4_frag_last", v4_frame(6, pay[:32], frag_off=50, fix_l4=False),
        REDIRECT, dict(flags_set=F_FRAG, flags_clear=F_L4))

    # --- UDP (parsing_helpers.h:272-290, lib_checksum.h:168-179)
    add("udp_bad_csum", v4_frame(17, seg)[:-1] + b"\x00", DROP,
        dict(flags_clear=F_L4_OK, flags_set=F_L3_OK))
    fz = v4_frame(17, seg)
    fz = fz[:40] + b"\0\0" + fz[42:]
    add("udp_csum_absent", fz, REDIRECT, dict(flags_set=F_L4_ABSENT | F_L4_OK))
    add("udp_len_lt_8", v4_frame(17, udp(1, 2, pay[:20], length=7), fix_l4=False),
        ABORTED)
    add("udp_len_past_ip", v4_frame(17, udp(1, 2, pay[:20], length=29), fix_l4=False),
        ABORTED)
    add("udp_hdr_truncated", v4_frame(17, pay[:6], fix_l4=False), ABORTED)
    useg = udp(1, 2, pay[:20], length=27)       # odd: over-read of byte 27
    useg = set_csum(useg, 6, l4_csum4(S4, D4, 17, useg[:27], overread=useg[27]))
    add("udp_odd_len_overread", v4_frame(17, useg, fix_l4=False), REDIRECT,
        dict(l4_len=27, flags_set=F_L4_OK))
    useg = udp(7, 9, pay[:19])                  # odd, ends at frame end
    fr = v4_frame(17, useg, overread=0xAB) + b"\xab"
    add("udp_odd_len_fcs_byte", fr, REDIRECT, dict(l4_len=27, flags_set=F_L4_OK),
        length=len(fr) - 1)

    # --- TCP (parsing_helpers.h:295-318)
    add("tcp_doff5", v4_frame(6, tcp(5555, 443, pay[:12])), REDIRECT,
        dict(l4_proto=6, l4_len=32, flags_set=F_L4_OK))
    add("tcp_doff15", v4_frame(6, tcp(5555, 443, pay[:3], doff=15)), REDIRECT,
        dict(l4_len=63, flags_set=F_L4_OK))
    add("tcp_doff4", v4_frame(6, tcp(1, 2, pay[:20], doff=4, options=b"")), ABORTED)
    add("tcp_doff_past_end", v4_frame(6, tcp(1, 2, b"", doff=8, options=b"\x01" * 8),
                                      fix_l4=False), ABORTED)
    add("tcp_truncated", v4_frame(6, tcp(1, 2, b"")[:12], fix_l4=False), ABORTED)
    tb = v4_frame(6, tcp(5555, 443, pay[:12]))
    add("tcp_bad_csum", tb[:50] + bytes([tb[50] ^ 0xFF]) + tb[51:], DROP)

    # --- ICMP
    add("icmp4_echo", v4_frame(1, icmp(8, 0, pay[:36])), REDIRECT,
        dict(l4_proto=1, flags_set=F_L4_OK))
    add("icmp4_odd", v4_frame(1, icmp(8, 0, pay[:35])), REDIRECT, dict(l4_len=39))
    add("icmp4_bad", v4_frame(1, icmp(8, 0, pay[:36]), fix_l4=False), DROP)
    add("icmp4_all_zero", v4_frame(1, b"\0" * 8, fix_l4=False), DROP,
        dict(l4_csum=0xFFFF))
    add("icmp4_truncated", v4_frame(1, b"\x08\x00\x00", fix_l4=False), ABORTED)

    # --- IPv6 (parsing_helpers.h:139-194), NDP (af_xdp_kern.c:114-148)
    for t in (133, 134, 135, 136, 137):
        add(f"ndp_{t}", v6_frame(58, icmp(t, 0, b"\0" * 20)), PASS)
    add("icmp6_132", v6_frame(58, icmp(132, 0, b"\0" * 20)), REDIRECT)
    add("icmp6_138", v6_frame(58, icmp(138, 0, b"\0" * 20)), REDIRECT)
    add("icmp6_echo_req", v6_frame(58, icmp(128, 0, pay[:32])), REDIRECT,
        dict(l4_proto=58, l4_off=54, flags_set=F_IPV6 | F_L4_OK))
    add("icmp6_truncated", v6_frame(58, b"\x80\x00\x00\x00", fix_l4=False), ABORTED)
    add("ndp_bad_csum_still_pass", v6_frame(58, icmp(135, 0, b"\1" * 20), fix_l4=False),
        PASS)
    add("udp6", v6_frame(17, udp(53, 5353, pay[:30])), REDIRECT,
        dict(l4_off=54, l4_len=38, flags_set=F_IPV6 | F_L4_OK | F_L3_OK))
    add("udp6_odd", v6_frame(17, udp(53, 5353, pay[:31])), REDIRECT, dict(l4_len=39))
    add("udp6_zero_csum", v6_frame(17, udp(53, 5353, pay[:30]), fix_l4=False), DROP)
    add("tcp6", v6_frame(6, tcp(22, 40000, pay[:17], doff=6)), REDIRECT,
        dict(l4_proto=6))
    add("ipv6_version4", v6_frame(17, udp(1, 2, pay[:8]))[:14] + b"\x40" +
        v6_frame(17, udp(1, 2, pay[:8]))[15:], ABORTED)
    add("ipv6_truncated", v6_frame(17, udp(1, 2, pay[:8]))[:50], ABORTED)
    add("ipv6_plen_past_end", v6_frame(17, udp(1, 2, pay[:8]), payload_len=300), ABORTED)
    nonext = eth(ETH_P_IPV6) + ipv6(0, 59, V6S, V6D)
    add("ipv6_no_next_exact", nonext, ABORTED)          # opt_hdr check past end
    add("ipv6_no_next_padded", nonext + b"\0\0", REDIRECT,
        dict(l4_proto=59, l4_off=54, flags_clear=F_L4))
    exts_all = [(0, ext_opts(1)), (60, ext_opts(2)), (43, ext_opts(1)),
                (51, ext_ah(1)), (135, ext_opts(1))]
    for k in range(1, 6):
        add(f"ipv6_ext_{k}", v6_frame(17, udp(9, 10, pay[:12]), exts=exts_all[:k]),
            REDIRECT, dict(l4_proto=17, flags_set=F_L4_OK))
    six = exts_all + [(60, ext_opts(1))]
    add("ipv6_ext_6_exhausted", v6_frame(17, udp(9, 10, pay[:12]), exts=six), ABORTED)
    add("ipv6_ext_truncated", v6_frame(17, udp(9, 10, b""), exts=[(0, ext_opts(4))])[:70],
        ABORTED)
    add("ipv6_frag_first", v6_frame(17, udp(9, 10, pay[:24], length=900),
                                    exts=[(44, ext_frag(0, True))], fix_l4=False),
        REDIRECT, dict(flags_set=F_FRAG | F_L4, flags_clear=F_L4_OK, l4_off=62))
    add("ipv6_frag_later", v6_frame(17, pay[:24], exts=[(44, ext_frag(100, False))],
                                    fix_l4=False),
        REDIRECT, dict(flags_set=F_FRAG, flags_clear=F_L4))
    add("ndp_in_later_fragment", v6_frame(58, icmp(135, 0, b"\0" * 8),
                                          exts=[(44, ext_frag(3, False))], fix_l4=False),
        PASS)
    add("ipv6_vlan_tcp_deep_check",
        v6_frame(6, tcp(1000, 2000, bytes(range(200)) * 7, doff=15),
                 tags=((ETH_P_8021Q, 7),)), REDIRECT,
        dict(l3_off=18, l4_off=58, flags_set=F_L4_OK))
    add("ipv6_ext_deep_l4",
        v6_frame(17, udp(3, 4, pay[:30]), exts=[(0, ext_opts(2)), (60, ext_opts(2))],
                 tags=((ETH_P_8021AD, 1), (ETH_P_8021Q, 2))), REDIRECT,
        dict(l3_off=22, l4_off=94, flags_set=F_L4_OK))

    # --- deep IPv4 header past a 64-byte window
    add("qinq_ipv4_ihl15", v4_frame(17, udp(5, 6, pay[:20]), options=b"\x01" * 40,
                                    tags=((ETH_P_8021AD, 1), (ETH_P_8021Q, 2))),
        REDIRECT, dict(l3_off=22, l4_off=82, flags_set=F_L3_OK | F_L4_OK))
    add("qinq_ipv4_ihl15_bad", v4_frame(17, udp(5, 6, pay[:20]), options=b"\x01" * 40,
                                        tags=((ETH_P_8021AD, 1), (ETH_P_8021Q, 2)),
                                        bad_csum=True), DROP)

    # --- big frames (payload past the header window, cooperative sums)
    big = bytes((i * 7 + 3) & 0xFF for i in range(9000))
    add("udp_1500", v4_frame(17, udp(1, 2, big[:1458])) + b"\0" * 4, REDIRECT,
        dict(l4_len=1466, flags_set=F_L4_OK))
    add("udp_1500_bad", v4_frame(17, udp(1, 2, big[:1458]))[:-3] + b"\0\0\0", DROP)
    add("tcp_jumbo_9000", v4_frame(6, tcp(1, 2, big[:8900])), REDIRECT,
        dict(flags_set=F_L4_OK))
    add("udp6_4000_odd", v6_frame(17, udp(1, 2, big[:3999])), REDIRECT,
        dict(l4_len=4007, flags_set=F_L4_OK))
    add("icmp4_1200_odd", v4_frame(1, icmp(0, 0, big[:1197])), REDIRECT,
        dict(l4_len=1201, flags_set=F_L4_OK))

    # --- placement / descriptor edge cases
    add("xdpsock_odd_addr", f, REDIRECT, dict(l3_csum=0x7C52, l4_csum=0x9102),
        length=60, place="odd")
    add("xdpsock_addr_4mod16", f, REDIRECT, dict(l3_csum=0x7C52), length=60,
        place="four")
    add("udp_1500_odd_addr", v4_frame(17, udp(1, 2, big[:1458])), REDIRECT,
        dict(flags_set=F_L4_OK), place="odd")
    add("xdpsock_unaligned_encoded", f, REDIRECT, dict(l3_csum=0x7C52), length=60,
        place="encoded")
    add("desc_out_of_bounds", f, ABORTED, length=60, place="oob")
    add("desc_len_past_umem", f, ABORTED, length=60, place="straddle")
    useg = udp(7, 9, pay[:19])
    last = v4_frame(17, useg, overread=0)
    add("udp_odd_overread_past_umem", last, REDIRECT, dict(l4_len=27, flags_set=F_L4_OK),
        place="end")
    return out


def layout(cs):
    """Place every frame in one UMEM; returns umem, descs."""
    placed = []
    off = 0
    end_case = None
    for idx, (name, frame, length, _, _, place) in enumerate(cs):
        L = len(frame) if length is None else length
        if place == "end":
            end_case = idx
            placed.append(None)
            continue
        shift = {"odd": 1, "four": 4, "encoded": 0}.get(place, 0)
        start = off + shift
        placed.append((start, L, place))
        off = (start + len(frame) + 64 + 127) & ~127
    # the 'end' frame is last in memory: its over-read byte is past the UMEM
    name, frame, length, _, _, _ = cs[end_case]
    start = off
    placed[end_case] = (start, len(frame), "end")
    size = start + len(frame)
    umem = np.zeros(size, np.uint8)
    descs = np.zeros(len(cs), oracle.DESC_DTYPE)
    for idx, (name, frame, length, _, _, place) in enumerate(cs):
        start, L, place = placed[idx]
        if place in ("oob", "straddle"):
            umem[start:start + len(frame)] = np.frombuffer(frame, np.uint8)
            descs[idx]["addr"] = size + 4096 if place == "oob" else size - 10
            descs[idx]["len"] = L
            continue
        umem[start:start + len(frame)] = np.frombuffer(frame, np.uint8)
        if place == "encoded":
            base = start & ~0xFFF
            descs[idx]["addr"] = ((start - base) << 48) | base
        else:
            descs[idx]["addr"] = start
        descs[idx]["len"] = L
    return umem, descs


def check_against_reference(cs, umem, descs, verdict, res, tup_net):
    """Independent checks 1-3 (see module docstring)."""
    r = oracle.ref_lib()
    assert r is not None, "oracle/_ref/libref.so required (run where /root/reference exists)"
    fails = []
    for i, (name, frame, length, want_v, exp, place) in enumerate(cs):
        v = int(verdict[i])
        rr = res[i]
        if v != want_v:
            fails.append(f"{name}: verdict {v} != expected {want_v}")
            continue
        for k in ("l3_off", "l4_off", "l4_proto", "nvlan", "l4_len", "l3_csum", "l4_csum"):
            if k in exp and int(rr[k]) != exp[k]:
                fails.append(f"{name}: {k} {int(rr[k]):#x} != {exp[k]:#x}")
        fl = int(rr["flags"])
        if "flags_set" in exp and (fl & exp["flags_set"]) != exp["flags_set"]:
            fails.append(f"{name}: flags {fl:#x} lack {exp['flags_set']:#x}")
        if "flags_clear" in exp and (fl & exp["flags_clear"]):
            fails.append(f"{name}: flags {fl:#x} have {exp['flags_clear']:#x}")
        if v in (ABORTED, PASS):
            if any(int(rr[k]) for k in rr.dtype.names):
                fails.append(f"{name}: non-zero record for verdict {v}")
            continue
        addr = int(descs[i]["addr"])
        eff = (addr & ((1 << 48) - 1)) + (addr >> 48)
        p = bytes(umem[eff:eff + int(descs[i]["len"]) + 1])
        l3 = int(rr["l3_off"])
        # 2. IPv4 header checksum with the reference's ip_fast_csum
        if (fl & F_IP) and not (fl & F_IPV6):
            hl = (p[l3] & 0xF) * 4
            h = bytearray(p[l3:l3 + hl])
            h[10] = h[11] = 0
            hb = oracle.buf(bytes(h))
            want = r.ref_ip_fast_csum(hb, hl // 4)
            if want != int(rr["l3_csum"]):
                fails.append(f"{name}: l3_csum {int(rr['l3_csum']):#x} != ref {want:#x}")
            ok = r.ref_ip_fast_csum(oracle.buf(p[l3:l3 + hl]), hl // 4) == 0
            if ok != bool(fl & F_L3_OK):
                fails.append(f"{name}: L3_OK flag disagrees with reference")
        # 2. L4 checksum
        ln = int(rr["l4_len"])
        if ln:
            l4 = int(rr["l4_off"])
            proto = int(rr["l4_proto"])
            chk = {17: 6, 6: 16, 1: 2, 58: 2}[proto]
            seg = bytearray(umem[eff + l4:eff + l4 + ln + 1].tobytes())
            if len(seg) < ln + 1:
                seg += b"\0"          # over-read past the UMEM reads as 0
            seg[chk] = seg[chk + 1] = 0
            if not (fl & F_IPV6) and proto != 1:
                sa = struct.unpack("<I", p[l3 + 12:l3 + 16])[0]
                da = struct.unpack("<I", p[l3 + 16:l3 + 20])[0]
                want = r.ref_udp_csum(sa, da, ln, proto, oracle.buf(bytes(seg)))
            elif not (fl & F_IPV6):
                want = ~r.ref_do_csum(oracle.buf(bytes(seg[:ln])), ln) & 0xFFFF
            else:
                want = l4_csum6(p[l3 + 8:l3 + 24], p[l3 + 24:l3 + 40], proto,
                                bytes(seg[:ln]))
                body = r.ref_do_csum(oracle.buf(bytes(seg[:ln])), ln)
                s = body + ones_sum(p[l3 + 8:l3 + 40]) + \
                    ones_sum(struct.pack(">I", ln)) + ones_sum(struct.pack(">I", proto))
                if (~fold(s) & 0xFFFF) != want:
                    fails.append(f"{name}: ipv6 pseudo arithmetic disagrees")
            if want != int(rr["l4_csum"]):
                fails.append(f"{name}: l4_csum {int(rr['l4_csum']):#x} != ref {want:#x}")
        # (the flow hash is pinned against the reference jhash by the
        # caller, at the initval the NET-tuple run used)
    return fails


def random_vectors():
    r = oracle.ref_lib()
    rng = np.random.default_rng(0x60D)
    # do_csum over random (offset, length) slices of a random buffer
    buf = rng.integers(0, 256, 4096, dtype=np.uint8)
    raw = C.create_string_buffer(buf.tobytes(), 4096 + 16)
    base = C.addressof(raw)
    offs = rng.integers(0, 8, 2000).astype(np.uint32)
    lens = rng.integers(0, 1600, 2000).astype(np.uint32)
    lens[:16] = np.arange(16)
    dc = np.array([r.ref_do_csum(base + int(o), int(n)) for o, n in zip(offs, lens)],
                  np.uint32)
    # ip_fast_csum over random 20..60 byte headers
    ihl = rng.integers(5, 16, 500).astype(np.uint32)
    hdrs = rng.integers(0, 256, (500, 60), dtype=np.uint8)
    hdrs[:, 0] = (0x40 | ihl).astype(np.uint8)
    ipc = np.array([r.ref_ip_fast_csum(oracle.buf(hdrs[k].tobytes()), int(ihl[k]))
                    for k in range(500)], np.uint16)
    # udp_csum with odd and even lengths (over-read byte included in data)
    ul = rng.integers(8, 1500, 500).astype(np.uint32)
    udata = rng.integers(0, 256, (500, 1502), dtype=np.uint8)
    sa = rng.integers(0, 2 ** 32, 500, dtype=np.uint64).astype(np.uint32)
    da = rng.integers(0, 2 ** 32, 500, dtype=np.uint64).astype(np.uint32)
    pr = rng.choice([6, 17], 500).astype(np.uint8)
    uc = np.array([r.ref_udp_csum(int(sa[k]), int(da[k]), int(ul[k]), int(pr[k]),
                                  oracle.buf(udata[k].tobytes())) for k in range(500)],
                  np.uint16)
    # csum_tcpudp_magic / csum_fold on random words
    sums = rng.integers(0, 2 ** 32, 500, dtype=np.uint64).astype(np.uint32)
    mg = np.array([r.ref_csum_tcpudp_magic(int(sa[k]), int(da[k]), int(ul[k]),
                                           int(pr[k]), int(sums[k]))
                   for k in range(500)], np.uint16)
    cf = np.array([r.ref_csum_fold(int(s)) for s in sums], np.uint16)
    np.savez_compressed(os.path.join(HERE, "csum_vectors.npz"), buf=buf, offs=offs,
                        lens=lens, do_csum=dc, ihl=ihl, hdrs=hdrs, ip_fast_csum=ipc,
                        udp_len=ul, udp_data=udata, saddr=sa, daddr=da, proto=pr,
                        udp_csum=uc, sums=sums, tcpudp_magic=mg, csum_fold=cf)

    # jhash over random keys of length 0..64 and the word variants
    klen = np.concatenate([np.arange(65), rng.integers(0, 65, 1000)]).astype(np.uint32)
    keys = rng.integers(0, 256, (len(klen), 64), dtype=np.uint8)
    iv = rng.integers(0, 2 ** 32, len(klen), dtype=np.uint64).astype(np.uint32)
    iv[:65] = 0
    jh = np.array([r.ref_jhash(oracle.buf(keys[k].tobytes()), int(klen[k]), int(iv[k]))
                   for k in range(len(klen))], np.uint32)
    wl = rng.integers(0, 17, 500).astype(np.uint32)
    jh2 = np.array([r.ref_jhash2(oracle.buf(keys[k].tobytes()), int(wl[k]), int(iv[k]))
                    for k in range(500)], np.uint32)
    w3 = rng.integers(0, 2 ** 32, (500, 3), dtype=np.uint64).astype(np.uint32)
    j3 = np.array([r.ref_jhash_3words(int(a), int(b), int(c), int(v))
                   for (a, b, c), v in zip(w3, iv[:500])], np.uint32)
    j2 = np.array([r.ref_jhash_2words(int(a), int(b), int(v))
                   for (a, b, _), v in zip(w3, iv[:500])], np.uint32)
    j1 = np.array([r.ref_jhash_1word(int(a), int(v))
                   for (a, _, _), v in zip(w3, iv[:500])], np.uint32)
    np.savez_compressed(os.path.join(HERE, "jhash_vectors.npz"), klen=klen, keys=keys,
                        initval=iv, jhash=jh, wlen=wl, jhash2=jh2, words3=w3,
                        jhash_3words=j3, jhash_2words=j2, jhash_1word=j1)


def main():
    oracle.build()
    cs = cases()
    umem, descs = layout(cs)
    names = [c[0] for c in cs]
    assert len(set(names)) == len(names)
    out = {"umem": umem, "descs": descs.view(np.uint8)}
    for cname, (flags, iv, fmt) in CFGS.items():
        um = umem.copy()
        v, res, tup, st = oracle.process(um, descs, flags, iv, fmt)
        out[f"{cname}_verdict"] = v
        out[f"{cname}_res"] = res.view(np.uint8)
        out[f"{cname}_tup"] = tup
        out[f"{cname}_umem_after"] = um
        out[f"{cname}_stats"] = np.array(
            [st["frames"], st["bytes"], *st["verdict"], st["l3_bad"], st["l4_bad"],
             st["l4_absent"], st["frag"]], np.uint64)
    # hash pinning: rerun with NET tuples at the 'verify' initval
    um = umem.copy()
    v, res, tup_net, _ = oracle.process(um, descs, 0x5, 0, 2)
    fails = check_against_reference(cs, umem, descs, v, res, tup_net)
    r = oracle.ref_lib()
    for i, name in enumerate(names):
        if v[i] in (ABORTED, PASS):
            continue
        key = tup_net[i * 44:(i + 1) * 44].tobytes()
        want = r.ref_jhash(oracle.buf(key), 44, 0)
        if want != int(res[i]["hash"]):
            fails.append(f"{name}: hash {int(res[i]['hash']):#x} != ref jhash {want:#x}")
    # echo: the rewritten frame must be the ICMPv6 reply with a valid csum
    ev = out["echo_net_verdict"]
    ie = names.index("icmp6_echo_req")
    if ev[ie] != TX:
        fails.append("icmp6_echo_req not TX under echo")
    if fails:
        print("\n".join(fails))
        raise SystemExit(f"{len(fails)} golden checks failed")
    np.savez_compressed(os.path.join(HERE, "fixtures.npz"), **out)
    with open(os.path.join(HERE, "fixtures.json"), "w") as f:
        json.dump({"names": names, "cfgs": {k: list(v) for k, v in CFGS.items()},
                   "expected_verdict_verify": [c[3] for c in cs]}, f, indent=1)
    random_vectors()
    print(f"wrote {len(cs)} fixture frames, csum and jhash vectors")


if __name__ == "__main__":
    main()
