# SPDX-License-Identifier: GPL-2.0
"""TEST INFRASTRUCTURE: a tiny, independent frame builder for fixtures.

Builds Ethernet/VLAN/IPv4/IPv6/UDP/TCP/ICMP frames with RFC 1071 checksums
computed here in plain Python (independent of oracle/ and of the product),
so fixtures cross-check three separate statements of the arithmetic: this
file, oracle/xdp_oracle.c and the reference headers (oracle/_ref).
"""
from __future__ import annotations

import struct

ETH_P_IP, ETH_P_IPV6, ETH_P_ARP = 0x0800, 0x86DD, 0x0806
ETH_P_8021Q, ETH_P_8021AD = 0x8100, 0x88A8

DMAC = bytes.fromhex("3cfdfe9e7f71")
SMAC = bytes.fromhex("ecb1d7983ac0")


def ones_sum(data: bytes) -> int:
    """Sum of little-endian 16-bit words (odd tail byte zero padded)."""
    if len(data) & 1:
        data = data + b"\0"
    s = 0
    for i in range(0, len(data), 2):
        s += data[i] | (data[i + 1] << 8)
    return s


def fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def le16(v: int) -> bytes:
    return struct.pack("<H", v & 0xFFFF)


def eth(ethertype: int, tags=(), dmac=DMAC, smac=SMAC) -> bytes:
    """tags: sequence of (tpid, tci)."""
    b = dmac + smac
    for tpid, tci in tags:
        b += struct.pack(">HH", tpid, tci)
    return b + struct.pack(">H", ethertype)


def ipv4(payload_len: int, proto: int, src: bytes, dst: bytes, ttl=64,
         options: bytes = b"", frag_off: int = 0, ident: int = 0,
         tot_len: int | None = None, version: int = 4, ihl: int | None = None,
         bad_csum: bool = False) -> bytes:
    assert len(options) % 4 == 0
    hl = 20 + len(options)
    if ihl is None:
        ihl = hl // 4
    if tot_len is None:
        tot_len = hl + payload_len
    h = struct.pack(">BBHHHBBH4s4s", (version << 4) | ihl, 0, tot_len, ident,
                    frag_off, ttl, proto, 0, src, dst) + options
    c = ~fold(ones_sum(h)) & 0xFFFF
    if bad_csum:
        c ^= 0x0F0F
    return h[:10] + le16(c) + h[12:]


def ipv6(payload_len: int, nexthdr: int, src: bytes, dst: bytes,
         hop_limit=64, version: int = 6) -> bytes:
    return struct.pack(">IHBB16s16s", version << 28, payload_len, nexthdr,
                       hop_limit, src, dst)


def pseudo4(src: bytes, dst: bytes, proto: int, length: int) -> int:
    """lib_checksum.h csum_tcpudp_nofold pseudo-header terms (LE)."""
    return (struct.unpack("<I", src)[0] + struct.unpack("<I", dst)[0] +
            ((proto + length) << 8))


def pseudo6(src: bytes, dst: bytes, proto: int, length: int) -> int:
    s = ones_sum(src) + ones_sum(dst)
    s += ones_sum(struct.pack(">I", length)) + ones_sum(struct.pack(">I", proto))
    return s


def l4_csum4(src: bytes, dst: bytes, proto: int, seg: bytes,
             overread: int = 0) -> int:
    """udp_csum() semantics: odd length takes the next byte as high half."""
    data = seg + (bytes([overread]) if len(seg) & 1 else b"")
    return ~fold(ones_sum(data) + pseudo4(src, dst, proto, len(seg))) & 0xFFFF


def l4_csum6(src: bytes, dst: bytes, proto: int, seg: bytes) -> int:
    return ~fold(ones_sum(seg) + pseudo6(src, dst, proto, len(seg))) & 0xFFFF


def udp(sport: int, dport: int, payload: bytes, length: int | None = None) -> bytes:
    if length is None:
        length = 8 + len(payload)
    return struct.pack(">HHHH", sport, dport, length, 0) + payload


def tcp(sport: int, dport: int, payload: bytes, doff: int = 5,
        options: bytes | None = None) -> bytes:
    if options is None:
        options = b"\x01" * (doff * 4 - 20)
    return (struct.pack(">HHIIBBHHH", sport, dport, 0x01020304, 0x0A0B0C0D,
                        doff << 4, 0x18, 0xFFFF, 0, 0) + options + payload)


def icmp(typ: int, code: int, rest: bytes) -> bytes:
    return bytes([typ, code, 0, 0]) + rest


def set_csum(seg: bytes, off: int, value: int) -> bytes:
    return seg[:off] + le16(value) + seg[off + 2:]


def v4_frame(l4proto: int, seg: bytes, src=b"\x0a\x00\x00\x01",
             dst=b"\x0a\x00\x00\x02", tags=(), options=b"", frag_off=0,
             fix_l4=True, overread: int = 0, **ipkw) -> bytes:
    """Ethernet + IPv4 + segment with correct checksums unless told not to."""
    chk = {17: 6, 6: 16, 1: 2}.get(l4proto)
    if fix_l4 and chk is not None:
        seg = set_csum(seg, chk, 0)
        if l4proto == 1:
            c = ~fold(ones_sum(seg)) & 0xFFFF
        else:
            c = l4_csum4(src, dst, l4proto, seg, overread)
        seg = set_csum(seg, chk, c)
    return (eth(ETH_P_IP, tags) +
            ipv4(len(seg), l4proto, src, dst, options=options,
                 frag_off=frag_off, **ipkw) + seg)


V6S = bytes.fromhex("20010db8000000000000000000000001")
V6D = bytes.fromhex("20010db8000000000000000000000002")


def v6_frame(l4proto: int, seg: bytes, exts=(), src=V6S, dst=V6D, tags=(),
             fix_l4=True, payload_len: int | None = None) -> bytes:
    """exts: list of (type, body_bytes) written in order; the chain's last
    next-header is l4proto."""
    chk = {17: 6, 6: 16, 58: 2}.get(l4proto)
    if fix_l4 and chk is not None:
        seg = set_csum(seg, chk, 0)
        seg = set_csum(seg, chk, l4_csum6(src, dst, l4proto, seg))
    ext_bytes = b""
    types = [t for t, _ in exts]
    for k, (t, body) in enumerate(exts):
        nxt = types[k + 1] if k + 1 < len(types) else l4proto
        ext_bytes += bytes([nxt]) + body
    first = types[0] if types else l4proto
    plen = len(ext_bytes) + len(seg) if payload_len is None else payload_len
    return eth(ETH_P_IPV6, tags) + ipv6(plen, first, src, dst) + ext_bytes + seg


def ext_opts(n8: int = 1) -> bytes:
    """HOP/DST/ROUTING/MH body (after the next-header byte): hdrlen + pad."""
    body = bytes([n8 - 1]) + b"\x01" + bytes([n8 * 8 - 4]) + b"\0" * (n8 * 8 - 4)
    return body


def ext_ah(hdrlen: int = 1) -> bytes:
    """AH: total (hdrlen+2)*4 bytes."""
    total = (hdrlen + 2) * 4
    return bytes([hdrlen]) + b"\0" * (total - 2)


def ext_frag(offset8: int, more: bool, ident: int = 0x1234) -> bytes:
    return b"\0" + struct.pack(">HI", (offset8 << 3) | (1 if more else 0), ident)
