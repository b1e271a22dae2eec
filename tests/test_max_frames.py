# SPDX-License-Identifier: GPL-2.0
"""Maximum-size frames: IPv4 tot_len 65535 and IPv6 payload_len 65535, the
largest checksum ranges lib_checksum.h's udp_csum/tcp_csum
(AF_XDP-interaction/lib_checksum.h) and the IPv6 pseudo header of
xdp_synproxy_kern.c can be asked to cover.  All-0xFF payloads drive the
bulk kernel's 32-bit sum of 16-bit halves to its largest value (the range
is < 64 KiB + 64 B, xdp_rx.hip bulk_batch), zero payloads the other end;
odd lengths take the over-read byte, the last frame ends at the UMEM end.

CPU: the oracle's verdicts and counters on frames built with correct,
corrupted and absent checksums.  GPU: every RX variant against the oracle."""
import numpy as np
import pytest

import frames as F
import oracle
import xdpgpu

V4_MAX = 65535 - 20          # IPv4 payload at tot_len 65535
V6_MAX = 65535               # IPv6 payload_len


def max_pool(seed=5):
    """Frames at 16-byte aligned offsets with random gaps; returns umem,
    descs and, per frame, 'ok' / 'bad' / 'absent' as built."""
    rng = np.random.default_rng(seed)
    ff, zero = b"\xff" * 65536, b"\0" * 65536
    rnd = rng.integers(0, 256, 65536, dtype=np.uint8).tobytes()
    built = [
        (F.v4_frame(17, F.udp(1, 53, ff[:V4_MAX - 8])), "ok"),
        (F.v4_frame(6, F.tcp(2, 80, ff[:V4_MAX - 20])), "ok"),
        (F.v4_frame(17, F.udp(3, 53, zero[:V4_MAX - 8])), "ok"),
        (F.v4_frame(17, F.udp(4, 53, rnd[:V4_MAX - 8]), tags=[(0x8100, 5)] * 2), "ok"),
        (F.v4_frame(6, F.tcp(5, 80, rnd[:V4_MAX - 32], doff=8)), "ok"),
        (F.v4_frame(17, F.udp(6, 53, ff[:V4_MAX - 9])), "ok"),
        (F.v6_frame(17, F.udp(7, 53, ff[:V6_MAX - 9])), "ok"),
        (F.v6_frame(6, F.tcp(8, 80, ff[:V6_MAX - 21])), "ok"),
        (F.v6_frame(17, F.udp(9, 53, rnd[:V6_MAX - 8])), "ok"),
        (F.v6_frame(17, F.udp(10, 53, zero[:V6_MAX - 8])), "ok"),
    ]
    # corrupted copies: one payload byte flipped in the middle
    for k in (0, 1, 6, 8):
        b = bytearray(built[k][0])
        b[len(b) // 2] ^= 0x5A
        built.append((bytes(b), "bad"))
    # UDP over IPv4 with no checksum (zero: absent)
    seg = F.set_csum(F.udp(11, 53, ff[:V4_MAX - 8]), 6, 0)
    built.append((F.v4_frame(17, seg, fix_l4=False), "absent"))
    # last: odd IPv4 UDP length ending at the UMEM end (over-read is zero)
    built.append((F.v4_frame(17, F.udp(12, 53, ff[:V4_MAX - 9])), "ok"))
    offs, o = [], 0
    for fr, _ in built:
        o += 16 * int(rng.integers(0, 4))
        offs.append(o)
        o = (o + len(fr) + 15) & ~15
    umem = np.zeros(offs[-1] + len(built[-1][0]), np.uint8)
    for off, (fr, _) in zip(offs, built):
        umem[off:off + len(fr)] = np.frombuffer(fr, np.uint8)
    descs = np.zeros(len(built), xdpgpu.DESC_DTYPE)
    descs["addr"] = offs
    descs["len"] = [len(fr) for fr, _ in built]
    return umem, descs, [k for _, k in built]


def test_oracle_max_frames():
    umem, descs, kind = max_pool()
    v, _, _, st = oracle.process(umem.copy(), descs, 0x5, 0, 1)
    kind = np.array(kind)
    assert (v[kind == "bad"] == xdpgpu.DROP).all()
    assert not (v[kind != "bad"] == xdpgpu.DROP).any()
    assert not (v == xdpgpu.ABORTED).any()
    assert st["l4_bad"] == (kind == "bad").sum()
    assert st["l4_absent"] == (kind == "absent").sum()
    assert st["bytes"] == int(descs["len"].sum())


@pytest.mark.gpu
def test_gpu_max_frames_vs_oracle():
    pytest.importorskip("torch")
    from test_gpu_parity import VARIANTS, assert_same, oracle_stats_match, run_dev
    umem, descs, _ = max_pool()
    for tune, window in VARIANTS:
        for flags, iv, fmt in ((0x5, 0, 1), (0x7, 0x9E3779B9, 2), (0x4, 7, 1)):
            ou = umem.copy()
            ov, ores, otup, ost = oracle.process(ou, descs, flags, iv, fmt)
            print(f"max frames: tune {tune:#x} window {window} flags {flags:#x}", flush=True)
            v, res, tup, um, st = run_dev(umem, descs, flags, iv, fmt, window, tune)
            assert_same((v, res, tup, um), (ov, ores, otup, ou),
                        f"max/{tune:#x}/{window}/{flags:#x}")
            oracle_stats_match(st, ost)
