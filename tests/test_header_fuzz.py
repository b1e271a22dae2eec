# SPDX-License-Identifier: GPL-2.0
"""Header fuzz: frames of the fast and quick shapes (IPv4 UDP/TCP/ICMP,
IPv6 UDP/TCP/ICMPv6 incl. NDP, ARP, 0..2 VLAN tags) with one header field at
a time set to a random or boundary value (EtherType, version/IHL, tot_len,
fragment bits, protocol, UDP length, TCP data offset, ICMPv6 type, IPv6
payload length and next header) or the descriptor length cut, so that every
branch of the tile loop's classification (fast, bulk, quick ABORTED/PASS,
exception) meets frames on both sides of its conditions.  The HIP path
against the oracle, bit-exact: verdicts, records, tuples, UMEM, counters
(CPU: the generator's own checks)."""
import os
import sys

import numpy as np
import pytest

import oracle
import xdpgpu

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
import frames as F  # noqa: E402


def _base(rng):
    tags = [(0x8100 if rng.random() < 0.8 else 0x88A8, int(rng.integers(0, 4096)))
            for _ in range(int(rng.choice([0, 0, 0, 1, 2])))]
    plen = int(rng.choice([0, 1, 7, 18, 30, 60, 61, 100, 500]))
    pay = rng.integers(0, 256, plen, dtype=np.uint8).tobytes()
    k = rng.random()
    if k < 0.35:
        return F.v4_frame(17, F.udp(int(rng.integers(1, 65536)), 53, pay), tags=tags)
    if k < 0.55:
        return F.v4_frame(6, F.tcp(1234, 80, pay, doff=int(rng.integers(5, 9))), tags=tags)
    if k < 0.62:
        return F.v4_frame(1, F.icmp(8, 0, b"\x12\x34\x00\x01" + pay), tags=tags)
    if k < 0.70:
        arp = bytes([0, 1, 8, 0, 6, 4, 0, 1]) + bytes(20)
        return F.eth(0x0806, tags) + arp + bytes(int(rng.integers(0, 30)))
    if k < 0.80:
        return F.v6_frame(17, F.udp(4000, 53, pay), tags=tags)
    if k < 0.88:
        return F.v6_frame(6, F.tcp(4000, 443, pay, doff=int(rng.integers(5, 9))), tags=tags)
    t = int(rng.choice([128, 129, 133, 134, 135, 136, 137, 1, 3]))
    return F.v6_frame(58, F.icmp(t, 0, b"\0\0\0\0" + pay), tags=tags)


def _mutate(fr: bytes, rng) -> bytes:
    """One field of the frame set to a random or boundary value."""
    b = bytearray(fr)
    n = 0
    while len(b) >= n + 18 and b[12 + n:14 + n] in (b"\x81\x00", b"\x88\xa8"):
        n += 4
    l3 = 14 + n
    et = bytes(b[12 + n:14 + n])
    field = int(rng.integers(0, 10))
    if field == 0 and len(b) > 14:
        b[12 + n:14 + n] = rng.choice([b"\x08\x00", b"\x86\xdd", b"\x08\x06", b"\x81\x00",
                                        b"\x12\x34"])
    elif et == b"\x08\x00" and len(b) >= l3 + 20:
        if field == 1:
            b[l3] = int(rng.choice([0x45, 0x44, 0x40, 0x46, 0x4F, 0x55, 0x35, 0x65]))
        elif field == 2:
            tot = int(rng.choice([0, 19, 20, 21, 28, len(b) - l3, len(b) - l3 + 1, 65535,
                                  int(rng.integers(0, 2000))]))
            b[l3 + 2:l3 + 4] = tot.to_bytes(2, "big")
        elif field == 3:
            b[l3 + 6:l3 + 8] = int(rng.choice([0x2000, 0x4000, 0x0001, 0x6001, 0x1fff,
                                               0x3fff])).to_bytes(2, "big")
        elif field == 4:
            b[l3 + 9] = int(rng.choice([1, 6, 17, 0, 58, 255]))
        elif field == 5 and len(b) >= l3 + 28 and b[l3 + 9] == 17:
            ul = int(rng.choice([0, 7, 8, 9, len(b) - l3 - 20, len(b) - l3 - 19, 4000]))
            b[l3 + 24:l3 + 26] = ul.to_bytes(2, "big")
        elif field == 6 and len(b) >= l3 + 34 and b[l3 + 9] == 6:
            b[l3 + 32] = int(rng.integers(0, 16)) << 4
    elif et == b"\x86\xdd" and len(b) >= l3 + 40:
        if field == 1:
            b[l3] = int(rng.choice([0x60, 0x40, 0x70, 0x00])) | (b[l3] & 0x0F)
        elif field == 2:
            pl = int(rng.choice([0, 7, 8, 20, len(b) - l3 - 40, len(b) - l3 - 39, 1500]))
            b[l3 + 4:l3 + 6] = pl.to_bytes(2, "big")
        elif field == 4:
            b[l3 + 6] = int(rng.choice([17, 6, 58, 0, 43, 44, 59]))
        elif field == 7 and len(b) >= l3 + 41 and b[l3 + 6] == 58:
            b[l3 + 40] = int(rng.choice([128, 129, 132, 133, 137, 138, 135]))
        elif field == 6 and len(b) >= l3 + 53 and b[l3 + 6] == 6:
            b[l3 + 52] = int(rng.integers(0, 16)) << 4
    if field == 8:
        b = b[:int(rng.integers(0, len(b) + 1))]
    elif field == 9:
        b = b[:int(rng.choice([0, 1, 13, 14, 15, 17, 18, 21, 33, 34, 41, 42, 53, 54, 61,
                               62, 63, 64]))]
    return bytes(b)


def fuzz_pool(seed: int, n: int, align: int = 16):
    rng = np.random.default_rng(seed)
    blobs = []
    for _ in range(n):
        fr = _base(rng)
        if rng.random() < 0.7:
            fr = _mutate(fr, rng)
        if rng.random() < 0.3:
            fr += rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes()
        blobs.append(fr)
    offs, o = [], 0
    for fr in blobs:
        # mostly aligned (16 bytes: the fast and quick shapes; 128: a
        # 128-byte window's second half staged), some not
        o = (o + align - 1) & ~(align - 1) if rng.random() < 0.9 else o + int(rng.integers(1, 16))
        offs.append(o)
        o += max(len(fr), 1)
    umem = np.zeros(o + 64, np.uint8)
    for off, fr in zip(offs, blobs):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    descs = np.zeros(n, xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr in blobs]
    return umem, descs


def test_fuzz_pool_covers_every_class():
    """The pool reaches every verdict and the quick shapes (CPU)."""
    umem, descs = fuzz_pool(5, 6000)
    v, _, _, st = oracle.process(umem.copy(), descs, 0x5, 0, 1)
    counts = np.bincount(v, minlength=5)
    assert all(counts[k] > 50 for k in (xdpgpu.ABORTED, xdpgpu.DROP, xdpgpu.PASS,
                                        xdpgpu.REDIRECT)), counts
    assert (descs["len"] < 14).sum() > 20


@pytest.mark.gpu
@pytest.mark.parametrize("seed,window,align", [(1, 64, 16), (2, 64, 16), (3, 64, 16),
                                               (4, 128, 128), (5, 128, 128), (6, 128, 16)])
def test_fuzz_vs_oracle(seed, window, align):
    """Mutated headers against the oracle; with 128-byte windows the
    frames mostly start a 128-byte line, so that the second half is staged
    and the read-time range parse (read_tile_w2) sees the mutations too."""
    torch = pytest.importorskip("torch")
    from test_gpu_parity import assert_same, oracle_stats_match, run_dev
    umem, descs = fuzz_pool(seed, 20000, align)
    for flags, iv, fmt in ((0x5, 0, 1), (0x7, 0x9E3779B9, 2), (0x4, 3, 0)):
        ou = umem.copy()
        ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
        v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, 0)
        assert_same((v, res, tup, um), (ov, ores, otup, ou),
                    f"fuzz{seed}/w{window}/{flags:#x}/{fmt}")
        oracle_stats_match(st, ost)
    del torch
